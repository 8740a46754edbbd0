// jitc.cpp -- ecamd_jitc: builds the bitsliced kernel for one coefficient matrix (host/bitslice.cpp:
// XOR network, then HIP source) and compiles it to a gfx950 code object with hiprtc, in its own
// process.  libecamd (hip/ecamd_jit.hip) starts it as a child process, so neither the network
// search nor the compile runs on a caller's thread or shares a process with the GPU work, and a
// parent that exits abandons it harmlessly.  The code object is written to <out>.tmp.<pid> and
// renamed to <out>, so readers only ever see a whole one; the request file is removed once read,
// and with ECAMD_JIT_KEEP_SOURCE=1 the generated source lands beside the code object as
// <out minus .co>.hip for inspection.  This program never touches the GPU.
//
//   ecamd_jitc <request> <out.co> [arch]   request: bitslice_request() text; arch: the target GPU
//                                          (the parent passes its device's, default gfx950);
//                                          exit 0 on success
#include <hip/hiprtc.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "bitslice.hpp"

namespace {

bool write_whole(const std::string& path, const std::string& bytes)
{
    const std::string tmp = path + ".tmp." + std::to_string(getpid());
    {
        std::ofstream out(tmp, std::ios::binary);
        out.write(bytes.data(), static_cast<std::streamsize>(bytes.size()));
        if (!out) return false;
    }
    return std::rename(tmp.c_str(), path.c_str()) == 0;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc != 3 && argc != 4) {
        std::fprintf(stderr, "usage: %s <request> <out.co> [arch]\n", argv[0]);
        return 2;
    }
    std::string arch = argc == 4 && argv[3][0] ? argv[3] : "gfx950";
    for (char ch : arch)
        if (!std::isalnum(static_cast<unsigned char>(ch))) {
            std::fprintf(stderr, "ecamd_jitc: bad arch %s\n", argv[3]);
            return 2;
        }
    std::ifstream in(argv[1]);
    std::stringstream ss;
    ss << in.rdbuf();
    std::vector<int> coeff;
    int R = 0, K = 0, cap = 0, depth = 0;
    bool copy = false, crc = false, crc_lane = false, crc_nib = false, wave = false, budget2 = false;
    int crc_pos = 1;
    std::vector<int> shifts;
    int prefetch = 0;
    ecamd::BsOcc occ;
    int crc_wave = 0;
    if (!ecamd::bitslice_parse_request(ss.str(), coeff, R, K, cap, depth, &copy, &crc, &crc_pos, &crc_lane,
                                       &crc_nib, &wave, &budget2, &shifts, &prefetch, &occ, &crc_wave)) {
        std::fprintf(stderr, "ecamd_jitc: bad request %s\n", argv[1]);
        return 2;
    }
    ecamd::BitsliceStyle style;  // lazy / barrier: experiments only, the parent's cache key does not see them
    style.copy_through = copy;
    style.crc = crc;
    style.crc_pos = crc_pos;
    style.crc_lane = crc_lane;
    style.crc_nib = crc_nib;
    style.threads = wave ? 64 : occ.threads ? occ.threads : 256;
    style.crc_wave = crc_wave & 15;
    style.crc_mix = (crc_wave & 16) != 0;
    style.crc_mb = 4 - ((crc_wave >> 5) & 3);
    style.crc_l1 = (crc_wave >> 7) & 1;
    style.waves = wave || crc_wave ? occ.wmin : 0;  // one-wave forms: the request's occupancy (0: by R)
    style.waves_max = wave || crc_wave ? occ.wmax : 0;
    style.input_barrier = (wave || crc_wave) && occ.barrier;
    style.in_shift = shifts;
    style.prefetch = prefetch;
    if (const char* v = std::getenv("ECAMD_BS_WPE")) style.waves = std::atoi(v);  // experiment only
    if (const char* v = std::getenv("ECAMD_BS_WPE_MAX")) style.waves_max = std::atoi(v);  // experiment only
    if (const char* v = std::getenv("ECAMD_BS_LAZY")) style.lazy_temps = std::atoi(v) != 0;
    if (const char* v = std::getenv("ECAMD_BS_BARRIER")) style.input_barrier = std::atoi(v) != 0;
    if (const char* v = std::getenv("ECAMD_BS_RLANE")) style.realign_lane = std::atoi(v) != 0;
    if (const char* v = std::getenv("ECAMD_BS_DPPRED")) style.dpp_reduce = std::atoi(v) != 0;  // A/B only
    std::remove(argv[1]);
    const std::string src = ecamd::bitslice_source(ecamd::bitslice_network(coeff, R, K, cap), depth, style);
    std::string out(argv[2]);
    const char* keep = std::getenv("ECAMD_JIT_KEEP_SOURCE");
    if (keep && std::atoi(keep) && out.size() > 3 && out.compare(out.size() - 3, 3, ".co") == 0)
        write_whole(out.substr(0, out.size() - 3) + ".hip", src);

    hiprtcProgram prog = nullptr;
    if (hiprtcCreateProgram(&prog, src.c_str(), "ecamd_bitslice.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return 1;
    const std::string arch_opt = "--offload-arch=" + arch;
    const char* opts[] = {arch_opt.c_str(), "-O3", "-std=c++17"};
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
    return write_whole(out, code) ? 0 : 1;
}
