// probe_api.hip -- C ABI of libecamd_probe.so (include/ecamd_probe.h): bandwidth and lookup-engine
// probes used by bench.py (live copy-peak denominator) and tools/ sweeps.  Kept out of libecamd.so
// so the codec library carries no experiment code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <vector>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "ecamd_probe.h"
#include "probe.hpp"

using namespace ecamd;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) return fail(-5, "%s: %s", #expr, hipGetErrorString(e_));     \
    } while (0)

int ensure_device(int* dev)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(-19, "no HIP device");
    HIP_TRY(hipGetDevice(dev));
    return 0;
}

int cu_count(int dev)
{
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
        cus = 256;
    return cus;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" {

const char* ecamd_probe_last_error(void) { return g_err.c_str(); }

int ecamd_probe_stream_copy(void* dst, const void* src, int64_t bytes, void* stream)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    if (!aligned16(dst) || !aligned16(src) || bytes % 16)
        return fail(-22, "stream copy needs 16-byte aligned pointers and size");
    hipLaunchKernelGGL(stream_copy_kernel, dim3(cu_count(dev) * 8), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<uint4*>(dst),
                       static_cast<const uint4*>(src), bytes / 16);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_probe_bw(int kind, int unroll, int wgs_per_cu, void* dst, const void* src,
                         int64_t bytes, void* stream)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    static uint32_t* sink = nullptr;
    if (!sink) HIP_TRY(hipMalloc(&sink, 1024 * sizeof(uint32_t)));
    dim3 grid(cu_count(dev) * std::max(1, wgs_per_cu)), block(256);
    hipStream_t st = static_cast<hipStream_t>(stream);
    auto* d = static_cast<uint8_t*>(dst);
    auto* s = static_cast<const uint8_t*>(src);
    switch (unroll) {
    case 1: hipLaunchKernelGGL(bw_probe_kernel<1>, grid, block, 0, st, d, s, bytes, kind, sink); break;
    case 4: hipLaunchKernelGGL(bw_probe_kernel<4>, grid, block, 0, st, d, s, bytes, kind, sink); break;
    default: hipLaunchKernelGGL(bw_probe_kernel<8>, grid, block, 0, st, d, s, bytes, kind, sink); break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_probe_copy_tiles(int threads, void* dst, const void* src, int64_t bytes, void* stream)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    if (threads != 64 && threads != 128 && threads != 256) return fail(-22, "copy tiles: threads 64 / 128 / 256");
    const int64_t tile = static_cast<int64_t>(threads) * 16;
    if (bytes < tile || bytes % tile || bytes / tile >= (int64_t{1} << 31)) return fail(-22, "copy tiles: bytes");
    static uint32_t* sink = nullptr;
    if (!sink) HIP_TRY(hipMalloc(&sink, 1024 * sizeof(uint32_t)));
    hipLaunchKernelGGL(bw_probe_kernel<1>, dim3(static_cast<unsigned>(bytes / tile)), dim3(threads), 0,
                       static_cast<hipStream_t>(stream), static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src),
                       bytes, 0, sink);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_probe_lookup(int mode, int wgs_per_cu, int iters, const void* d_table, void* stream)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    static uint32_t* sink = nullptr;
    if (!sink) HIP_TRY(hipMalloc(&sink, 64));
    const dim3 grid(cu_count(dev) * std::max(1, wgs_per_cu)), block(256);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const auto* t = static_cast<const uint4*>(d_table);
    switch (mode) {
    case 0: hipLaunchKernelGGL(lookup_probe_kernel<0>, grid, block, 0, st, t, iters, sink); break;
    case 1: hipLaunchKernelGGL(lookup_probe_kernel<1>, grid, block, 0, st, t, iters, sink); break;
    case 2: hipLaunchKernelGGL(lookup_probe_kernel<2>, grid, block, 0, st, t, iters, sink); break;
    case 3: hipLaunchKernelGGL(lookup_probe_kernel<3>, grid, block, 0, st, t, iters, sink); break;
    case 4: hipLaunchKernelGGL(lookup_probe_kernel<4>, grid, block, 0, st, t, iters, sink); break;
    default: hipLaunchKernelGGL(lookup_probe_kernel<5>, grid, block, 0, st, t, iters, sink); break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_probe_launch(int mode, const void* d_src, int bytes, void* stream)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    if (bytes < 0 || bytes > 64 * 1024 || bytes % 16) return fail(-22, "launch probe: bytes 0..64 KiB, multiple of 16");
    static uint32_t* sink = nullptr;
    if (!sink) HIP_TRY(hipMalloc(&sink, 64));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const auto* s = static_cast<const uint8_t*>(d_src);
    const size_t lds = static_cast<size_t>(bytes);
    switch (mode) {
    case 0: hipLaunchKernelGGL((launch_probe_kernel<0, 0>), dim3(1), dim3(256), 0, st, sink, s, bytes); break;
    case 1: hipLaunchKernelGGL((launch_probe_kernel<1, 0>), dim3(1), dim3(256), lds, st, sink, s, bytes); break;
    case 2: hipLaunchKernelGGL((launch_probe_kernel<2, 0>), dim3(1), dim3(256), lds, st, sink, s, bytes); break;
    case 3: hipLaunchKernelGGL((launch_probe_kernel<0, 1024>), dim3(1), dim3(256), 0, st, sink, s, bytes); break;
    default: hipLaunchKernelGGL((launch_probe_kernel<0, 4096>), dim3(1), dim3(256), 0, st, sink, s, bytes); break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_probe_mix(int lp, int sp, int ch, int threads, int wgs_per_cu, void* base,
                          int64_t bs, int K, int R, int nstripes, void* stream)
{
    return ecamd_probe_mix2(lp, sp, ch, threads, wgs_per_cu, 0, 0, base, bs, K, R, nstripes, stream);
}

int ecamd_probe_mix2(int lp, int sp, int ch, int threads, int wgs_per_cu, int order,
                           int wave_contig, void* base, int64_t bs, int K, int R, int nstripes,
                           void* stream)
{
    return ecamd_probe_mix3(lp, sp, ch, threads, wgs_per_cu, order, wave_contig, base, bs, K, R, nstripes,
                            nullptr, stream);
}

int ecamd_probe_mix3(int lp, int sp, int ch, int threads, int wgs_per_cu, int order, int wave_contig,
                     void* base, int64_t bs, int K, int R, int nstripes, const int* frag, void* stream)
{
    return ecamd_probe_mix4(lp, sp, ch, threads, std::max(1, wgs_per_cu), -order - 1, wave_contig, base, bs, K, R,
                            nstripes, frag, stream);
}

// cap_per_cu < 0 carries mix3's tile order (-order - 1) with no cap; >= 0 is the per-CU cap (order 0)
int ecamd_probe_mix4(int lp, int sp, int ch, int threads, int wgs_per_cu, int cap_per_cu, int wave_contig,
                     void* base, int64_t bs, int K, int R, int nstripes, const int* frag, void* stream)
{
    const int order = cap_per_cu < 0 ? -cap_per_cu - 1 : 0;
    const int cap = cap_per_cu < 0 ? 0 : cap_per_cu;
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    if (ch != 1 && ch != 2 && ch != 4) return fail(-22, "mix probe: ch must be 1, 2 or 4");
    if (ch == 4 && threads > 256) return fail(-22, "mix probe: ch 4 runs at most 256 threads");
    if (threads < 64 || threads > 1024 || threads % 64) return fail(-22, "mix probe: threads");
    const int64_t span = static_cast<int64_t>(threads) * 16 * ch;
    const int64_t sstride = bs * (K + R);
    if (K < 1 || R < 0 || K + R > 64 || bs % span || !aligned16(base) || sstride >= (1ll << 31) || nstripes < 1)
        return fail(-22, "mix probe: bad shape");
    MixArgs a{static_cast<uint8_t*>(base), sstride, static_cast<int>(bs), K, R, 0, 0, order,
              wave_contig != 0, {}};
    for (int i = 0; i < K + R; i++) {
        a.frag[i] = frag ? frag[i] : i;
        if (a.frag[i] < 0 || a.frag[i] >= K + R) return fail(-22, "mix probe: fragment slot out of range");
    }
    a.tiles_per_stripe = static_cast<uint32_t>(bs / span);
    a.ntiles = a.tiles_per_stripe * static_cast<uint32_t>(nstripes);
    const int grid = wgs_per_cu <= 0 ? static_cast<int>(a.ntiles)
                                     : static_cast<int>(std::min<int64_t>(
                                           a.ntiles, static_cast<int64_t>(cu_count(dev)) * wgs_per_cu));
    const size_t lds = cap > 0 ? (static_cast<size_t>(160 * 1024) / static_cast<size_t>(cap)) & ~size_t(511) : 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    bool launched = false;
#define ECAMD_MIX(LP, SP)                                                                           \
    if (!launched && lp == LP && sp == SP) {                                                        \
        if (ch == 1)                                                                                \
            hipLaunchKernelGGL((mix_probe_kernel<LP, SP, 1>), dim3(grid), dim3(threads), lds, st, a); \
        else if (ch == 2)                                                                           \
            hipLaunchKernelGGL((mix_probe_kernel<LP, SP, 2>), dim3(grid), dim3(threads), lds, st, a); \
        else                                                                                        \
            hipLaunchKernelGGL((mix_probe_kernel<LP, SP, 4>), dim3(grid), dim3(threads), lds, st, a); \
        launched = true;                                                                            \
    }
    ECAMD_MIX_POLICIES(ECAMD_MIX)
#undef ECAMD_MIX
    if (!launched) return fail(-22, "mix probe: policy pair (%d, %d) not instantiated", lp, sp);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_probe_valu(int op, int wgs_per_cu, int iters, void* stream)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    static uint32_t* sink = nullptr;
    if (!sink) HIP_TRY(hipMalloc(&sink, 64));
    const dim3 grid(cu_count(dev) * std::max(1, wgs_per_cu)), block(256);
    hipStream_t st = static_cast<hipStream_t>(stream);
    switch (op) {
    case 0: hipLaunchKernelGGL(valu_probe_kernel<0>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 1: hipLaunchKernelGGL(valu_probe_kernel<1>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 2: hipLaunchKernelGGL(valu_probe_kernel<2>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 3: hipLaunchKernelGGL(valu_probe_kernel<3>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 4: hipLaunchKernelGGL(valu_probe_kernel<4>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 5: hipLaunchKernelGGL(valu_probe_kernel<5>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 6: hipLaunchKernelGGL(valu_probe_kernel<6>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 8: hipLaunchKernelGGL(valu_probe_kernel<8>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 9: hipLaunchKernelGGL(valu_probe_kernel<9>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 10: hipLaunchKernelGGL(valu_probe_kernel<10>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    case 11: hipLaunchKernelGGL(valu_probe_kernel<11>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    default: hipLaunchKernelGGL(valu_probe_kernel<7>, grid, block, 0, st, iters, 0x9e37u, sink); break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_probe_unaligned(int mode, int shift, void* dst, const void* src, int64_t bytes, void* stream)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    if (mode < 0 || mode > 5 || shift < 0 || shift > 15 || bytes < 4096 || bytes % 4096 ||
        bytes / 4096 >= (int64_t{1} << 31) || !aligned16(dst) || !aligned16(src))
        return fail(-22, "unaligned probe: mode 0..5, shift 0..15, bytes a multiple of 4096, aligned buffers");
    const dim3 grid(static_cast<unsigned>(bytes / 4096)), block(256);
    hipStream_t st = static_cast<hipStream_t>(stream);
    auto* d = static_cast<uint8_t*>(dst);
    auto* s = static_cast<const uint8_t*>(src);
    switch (mode) {
    case 0: hipLaunchKernelGGL(unaligned_probe_kernel<0>, grid, block, 0, st, d, s, bytes, shift); break;
    case 1: hipLaunchKernelGGL(unaligned_probe_kernel<1>, grid, block, 0, st, d, s, bytes, shift); break;
    case 2: hipLaunchKernelGGL(unaligned_probe_kernel<2>, grid, block, 0, st, d, s, bytes, shift); break;
    case 3: hipLaunchKernelGGL(unaligned_probe_kernel<3>, grid, block, 0, st, d, s, bytes, shift); break;
    case 4: hipLaunchKernelGGL(unaligned_probe_kernel<4>, grid, block, 0, st, d, s, bytes, shift); break;
    default: hipLaunchKernelGGL(unaligned_probe_kernel<5>, grid, block, 0, st, d, s, bytes, shift); break;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}


int ecamd_probe_mailbox(int n, int payload, int idle_us, double* out_us)
{
    int dev = 0;
    int rc = ensure_device(&dev);
    if (rc) return rc;
    if (n < 1 || n > 100000 || payload < 0 || payload > 256 || idle_us < 1 || idle_us > 100000 || !out_us)
        return fail(-22, "mailbox probe: n 1..100000, payload 0..256, idle_us 1..100000");
    uint32_t* mb = nullptr;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&mb), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    for (int i = 0; i < 1024; i++) mb[i] = 0;
    hipStream_t st = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL(mailbox_probe_kernel, dim3(1), dim3(64), 0, st, mb, n, payload,
                       static_cast<uint64_t>(idle_us) * 100u);
    hipError_t le = hipGetLastError();
    std::vector<double> us;
    us.reserve(static_cast<size_t>(n));
    int failed = le != hipSuccess ? -5 : 0;
    // the first request waits for the wave to start: a generous bound, later ones idle_us
    for (int i = 1; i <= n && !failed; i++) {
        volatile uint32_t* ack = mb + 1;
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(mb, static_cast<uint32_t>(i), __ATOMIC_RELEASE);
        for (;;) {
            if (*ack == static_cast<uint32_t>(i)) break;
            const double el = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (el > (i == 1 ? 2e6 : static_cast<double>(idle_us))) {
                failed = -62;
                break;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        // a gap between requests, as between calls
        const auto g0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g0).count() < 2.0) {
        }
    }
    __atomic_store_n(mb + 2, 1u, __ATOMIC_RELEASE);  // stop: the wave exits at its next poll
    hipError_t se = hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
    (void)hipHostFree(mb);
    if (le != hipSuccess) return fail(-5, "mailbox probe launch: %s", hipGetErrorString(le));
    if (se != hipSuccess) return fail(-5, "mailbox probe sync: %s", hipGetErrorString(se));
    if (failed) return fail(failed, "mailbox probe: no ack within the bound");
    std::vector<double> s(us.begin() + 1, us.end());
    if (s.empty()) s = us;
    std::sort(s.begin(), s.end());
    double sum = 0;
    for (double v : s) sum += v;
    out_us[0] = sum / static_cast<double>(s.size());
    out_us[1] = s.front();
    out_us[2] = s[s.size() / 2];
    out_us[3] = s[s.size() * 9 / 10];
    return 0;
}

}  // extern "C"
