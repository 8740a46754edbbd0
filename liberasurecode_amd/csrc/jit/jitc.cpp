// jitc.cpp -- ecamd_jitc: compiles one generated HIP kernel source to a gfx950 code object with
// hiprtc, in its own process.  libecamd (hip/ecamd_jit.hip) starts it as a child process, so a
// compile never shares a process with the GPU work and can outlive (or be abandoned by) its
// parent harmlessly; the result is written to <out>.tmp.<pid> and renamed to <out>, so readers
// only ever see a whole code object.  This program never touches the GPU.
//
//   ecamd_jitc <source.hip> <out.co>      exit 0 on success
#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <unistd.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

int main(int argc, char** argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s <source.hip> <out.co>\n", argv[0]);
        return 2;
    }
    std::ifstream in(argv[1]);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string src = ss.str();
    if (src.empty()) return 2;
    hiprtcProgram prog = nullptr;
    if (hiprtcCreateProgram(&prog, src.c_str(), "ecamd_bitslice.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return 1;
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    if (hiprtcCompileProgram(prog, 3, opts) != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        std::fprintf(stderr, "ecamd_jitc: compile failed:\n%s\n", log.c_str());
        return 1;
    }
    size_t n = 0;
    if (hiprtcGetCodeSize(prog, &n) != HIPRTC_SUCCESS || n == 0) return 1;
    std::string code(n, '\0');
    if (hiprtcGetCode(prog, &code[0]) != HIPRTC_SUCCESS) return 1;
    hiprtcDestroyProgram(&prog);
    const std::string tmp = std::string(argv[2]) + ".tmp." + std::to_string(getpid());
    {
        std::ofstream out(tmp, std::ios::binary);
        out.write(code.data(), static_cast<std::streamsize>(code.size()));
        if (!out) return 1;
    }
    return std::rename(tmp.c_str(), argv[2]) == 0 ? 0 : 1;
}
