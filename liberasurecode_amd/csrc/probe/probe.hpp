// probe.hpp -- kernels of the measurement library libecamd_probe.so (include/ecamd_probe.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ecamd {

struct MixArgs {
    uint8_t* base;
    int64_t stripe_stride;
    int frag_stride;
    int K, R;
    uint32_t ntiles;
    uint32_t tiles_per_stripe;
    int order;        // 0: grid-stride tile order, 1: contiguous tile range per workgroup,
                      // 2: grid-stride with the fragment order rotated per tile
    int wave_contig;  // 1: a wave's CH chunks are contiguous (1 KiB apart)
    int frag[64];     // fragment slot of read i (0..K-1) and of write r (K+r): which slots are read
                      //   and which written (identity: reads first, then writes)
};

// (load policy, store policy) pairs instantiated for mix_probe_kernel; gfx950 cpol bits
// 1 = sc0, 2 = nt, 16 = sc1.
#define ECAMD_MIX_POLICIES(X) \
    X(0, 0) X(0, 2) X(0, 16) X(0, 18) X(0, 1) \
    X(2, 0) X(2, 2) X(2, 16) X(2, 18) X(2, 1) \
    X(1, 0) X(1, 2) X(16, 2) X(18, 2) X(3, 2) X(18, 18)
template <int LP, int SP, int CH>
__global__ void mix_probe_kernel(MixArgs a);

template <int MODE>
__global__ void lookup_probe_kernel(const uint4* __restrict__ table, int iters, uint32_t* sink);

template <int STAGE, int CODE>
__global__ void launch_probe_kernel(uint32_t* sink, const uint8_t* src, int bytes);

template <int U>
__global__ void bw_probe_kernel(uint8_t* dst, const uint8_t* src, int64_t bytes, int kind,
                                uint32_t* sink);
__global__ void mailbox_probe_kernel(uint32_t* mb, int n, int payload, uint64_t idle_ticks);
__global__ void stream_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, int64_t n);

template <int OP>
__global__ void valu_probe_kernel(int iters, uint32_t seed, uint32_t* sink);

template <int MODE>
__global__ void unaligned_probe_kernel(uint8_t* dst, const uint8_t* src, int64_t bytes, int shift);

}  // namespace ecamd
