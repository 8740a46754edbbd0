// ecamd_jit.hip -- run-time specialised bitsliced GF(2^16) kernels (host/bitslice.hpp).
//
// The XOR network of a bitsliced map depends on every coefficient, so its kernel is generated for
// the matrix and compiled with hiprtc (loaded with dlopen: without it the LDS-table kernels simply
// keep running).  Compilation takes a few seconds and runs on a background thread the first time
// a matrix is seen; launches use the LDS-table kernel until the code object is ready (knob
// "bitslice" = 1, the default), or wait for it (= 2; tests, bench); ecamd_bitslice_wait() waits for
// every pending compile.  Code objects are cached per matrix, modules per device.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../host/bitslice.hpp"
#include "ecamd.h"
#include "ecamd_internal.hpp"

namespace ecamd {
namespace {

struct Rtc {
    hiprtcResult (*create)(hiprtcProgram*, const char*, const char*, int, const char* const*,
                           const char* const*) = nullptr;
    hiprtcResult (*compile)(hiprtcProgram, int, const char* const*) = nullptr;
    hiprtcResult (*code_size)(hiprtcProgram, size_t*) = nullptr;
    hiprtcResult (*code)(hiprtcProgram, char*) = nullptr;
    hiprtcResult (*log_size)(hiprtcProgram, size_t*) = nullptr;
    hiprtcResult (*log)(hiprtcProgram, char*) = nullptr;
    hiprtcResult (*destroy)(hiprtcProgram*) = nullptr;
    bool ok = false;
};

const Rtc& rtc()
{
    static Rtc r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"libhiprtc.so.7", "libhiprtc.so", "/opt/rocm/lib/libhiprtc.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (!h) return;
#define SYM(f, n) r.f = reinterpret_cast<decltype(r.f)>(dlsym(h, n))
        SYM(create, "hiprtcCreateProgram");
        SYM(compile, "hiprtcCompileProgram");
        SYM(code_size, "hiprtcGetCodeSize");
        SYM(code, "hiprtcGetCode");
        SYM(log_size, "hiprtcGetProgramLogSize");
        SYM(log, "hiprtcGetProgramLog");
        SYM(destroy, "hiprtcDestroyProgram");
#undef SYM
        r.ok = r.create && r.compile && r.code_size && r.code && r.destroy;
    });
    return r;
}

// Code object of the kernel for one network ("" when the compile failed).
std::string compile_network(const std::string& src)
{
    const Rtc& r = rtc();
    if (!r.ok) return {};
    hiprtcProgram prog = nullptr;
    if (r.create(&prog, src.c_str(), "ecamd_bitslice.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return {};
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    std::string out;
    if (r.compile(prog, 3, opts) == HIPRTC_SUCCESS) {
        size_t n = 0;
        if (r.code_size(prog, &n) == HIPRTC_SUCCESS && n > 0) {
            out.resize(n);
            if (r.code(prog, &out[0]) != HIPRTC_SUCCESS) out.clear();
        }
    } else if (r.log_size && r.log) {
        size_t n = 0;
        r.log_size(prog, &n);
        std::string log(n, '\0');
        if (n) r.log(prog, &log[0]);
        std::fprintf(stderr, "libecamd: bitslice kernel compile failed:\n%s\n", log.c_str());
    }
    r.destroy(&prog);
    return out;
}

struct BsEntry {
    std::vector<int> coeff;
    int R = 0, K = 0;
    int cap = 0;  // shared temporaries allowed in the network (fewer: fewer registers)
    int gen = 0;  // bumped when the network is rebuilt
    std::shared_future<std::string> code;
    std::mutex mu;
    std::map<int, hipFunction_t> fn;  // per device; nullptr: unusable there
    std::vector<hipModule_t> modules;
};

// Temporaries per input: 40 fits the register file at 2 waves per SIMD for the C5 networks
// (252 VGPRs, no scratch); a network that spills is rebuilt once with 16.
constexpr int kCapFirst = 40;
constexpr int kCapRetry = 16;

void start_compile(BsEntry& e)
{
    const BitsliceNet net = bitslice_network(e.coeff, e.R, e.K, e.cap);
    e.code = std::async(std::launch::async, compile_network, bitslice_source(net)).share();
    e.gen++;
}

std::mutex g_jit_mu;
std::map<std::vector<int>, std::shared_ptr<BsEntry>> g_jit;

}  // namespace

// Kernel for the R x K matrix on `dev`: nullptr while compiling (wait = false) or when the
// bitsliced form is unavailable; starts the compile the first time the matrix is seen.
hipFunction_t bitslice_function(int dev, const std::vector<int>& coeff, int R, int K, bool wait)
{
    if (R <= 0 || R > kBsMaxR || K <= 0 || K > kBsMaxK || !rtc().ok) return nullptr;
    std::vector<int> key = {R, K};
    key.insert(key.end(), coeff.begin(), coeff.end());
    std::shared_ptr<BsEntry> e;
    {
        std::lock_guard<std::mutex> lk(g_jit_mu);
        if (g_jit.size() >= 1024 && !g_jit.count(key)) g_jit.clear();  // bound; in-use entries live on
        auto& slot = g_jit[key];
        if (!slot) {
            slot = std::make_shared<BsEntry>();
            slot->coeff = coeff;
            slot->R = R;
            slot->K = K;
            slot->cap = kCapFirst;
            start_compile(*slot);
        }
        e = slot;
    }
    for (;;) {
        std::shared_future<std::string> code;
        int gen = 0;
        {
            std::lock_guard<std::mutex> lk(e->mu);
            auto it = e->fn.find(dev);
            if (it != e->fn.end()) return it->second;
            code = e->code;
            gen = e->gen;
        }
        if (!wait && code.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return nullptr;
        const std::string& co = code.get();
        std::lock_guard<std::mutex> lk(e->mu);
        if (e->gen != gen) continue;  // rebuilt meanwhile by another thread
        auto it = e->fn.find(dev);
        if (it != e->fn.end()) return it->second;
        hipFunction_t fn = nullptr;
        int spill = 0;
        if (!co.empty()) {
            hipModule_t mod = nullptr;
            if (hipModuleLoadData(&mod, co.data()) == hipSuccess) {
                e->modules.push_back(mod);
                if (hipModuleGetFunction(&fn, mod, "ecamd_bs_kernel") != hipSuccess) fn = nullptr;
                if (fn && hipFuncGetAttribute(&spill, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, fn) == hipSuccess &&
                    spill > 0)
                    fn = nullptr;  // a spilling network runs slower than the LDS tables
            }
            (void)hipGetLastError();
        }
        if (!fn && spill > 0 && e->cap > kCapRetry) {  // rebuild with fewer temporaries
            e->cap = kCapRetry;
            start_compile(*e);
            e->fn.clear();
            continue;
        }
        e->fn[dev] = fn;
        return fn;
    }
}

int bitslice_launch(hipFunction_t fn, const BsArgs& args, int grid, hipStream_t st)
{
    BsArgs a = args;
    void* params[] = {&a};
    const hipError_t e = hipModuleLaunchKernel(fn, static_cast<unsigned>(grid), 1, 1, 256, 1, 1, 0, st,
                                               params, nullptr);
    if (e != hipSuccess)
        return dev_fail(ECAMD_EHIP, "hipModuleLaunchKernel(bitslice): %s", hipGetErrorString(e));
    return 0;
}

}  // namespace ecamd

extern "C" int ecamd_bitslice_wait(void)
{
    std::vector<std::shared_ptr<ecamd::BsEntry>> all;
    {
        std::lock_guard<std::mutex> lk(ecamd::g_jit_mu);
        for (auto& kv : ecamd::g_jit) all.push_back(kv.second);
    }
    int failed = 0;
    for (auto& e : all) {
        std::shared_future<std::string> code;
        {
            std::lock_guard<std::mutex> lk(e->mu);
            code = e->code;
        }
        if (code.get().empty()) failed++;
    }
    return failed;
}

extern "C" int ecamd_bitslice_available(void) { return ecamd::rtc().ok ? 1 : 0; }
