// probe_bitslice.hip -- experiment: bitsliced GF(2^16) encode for C5 (k=20, m=8), the network
// generated from the reference generator by tools/gen_bitslice.py (build/bs_c5_net.inc).  No
// table lookups: each lane turns 32 words of each fragment into 16 bit planes (a 16x16 bit
// transpose per 16-bit half), XORs planes into 8 x 16 output planes, transposes back.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ecamd_isa.hpp"
#include "probe.hpp"

namespace ecamd {
namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#include "bs_c5_net.inc"

// (m & x) | (~m & y) in one op; written out because the compiler adds a redundant mask otherwise
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y)
{
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(x), "v"(y));
    return r;
}

// 16x16 bit transpose inside each 16-bit half of 16 dwords (an involution): plane of bit b ends
// in A[15 - b], word w (dword w/2, half w%2) at bit (15 - w/2) + 16*(w%2).
__device__ __forceinline__ void tr16(uint32_t (&A)[16])
{
#pragma unroll
    for (int k = 0; k < 8; k++) {  // 8-bit blocks: byte moves
        const uint32_t a = A[k], b = A[k + 8];
        A[k] = __builtin_amdgcn_perm(a, b, 0x07030501u);
        A[k + 8] = __builtin_amdgcn_perm(a, b, 0x06020400u);
    }
#pragma unroll
    for (int j = 4, m = 0x0F0F0F0F; j; j >>= 1, m ^= m << j) {
#pragma unroll
        for (int k = 0; k < 16; k = (k + j + 1) & ~j) {
            // the swap as two bit selects (v_bfi_b32): 2 shifts + 2 selects per pair
            const uint32_t a = A[k], b = A[k + j], mu = static_cast<uint32_t>(m);
            A[k] = bfi(mu, b >> j, a);
            A[k + j] = bfi(mu, b, a << j);
        }
    }
}

template <int V, int J>
__device__ __forceinline__ void bs_input(__amdgpu_buffer_rsrc_t r, int off, int fstride,
                                         uint32_t (&acc)[8][16])
{
    uint32_t P[16];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, J * fstride + off + c * 4096, 0, 2);
        P[4 * c + 0] = x[0];
        P[4 * c + 1] = x[1];
        P[4 * c + 2] = x[2];
        P[4 * c + 3] = x[3];
    }
    tr16(P);
    if constexpr (V == 8)
        bs_net_c8<J>(acc, P);
    else
        bs_net_c24<J>(acc, P);
    if constexpr (J + 1 < 20) bs_input<V, J + 1>(r, off, fstride, acc);
}

}  // namespace

// V: CSE temps per input (8 or 24); waves per SIMD the register budget aims for: 3 or 2
template <int V>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu(V == 8 ? 3 : 2, V == 8 ? 3 : 2)))
    bs_c5_encode_kernel(uint8_t* base, int64_t stripe_stride, int fstride, uint32_t ntiles,
                        uint32_t tiles_per_stripe)
{
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t s = t / tiles_per_stripe;
        const int off = static_cast<int>(t - s * tiles_per_stripe) * 16384 + threadIdx.x * 16;
        const auto r = __builtin_amdgcn_make_buffer_rsrc(base + static_cast<int64_t>(s) * stripe_stride, 0,
                                                         static_cast<int>(28 * fstride), 0x00020000);
        uint32_t acc[8][16];
#pragma unroll
        for (int o = 0; o < 8; o++)
#pragma unroll
            for (int p = 0; p < 16; p++) acc[o][p] = 0u;
        bs_input<V, 0>(r, off, fstride, acc);
#pragma unroll
        for (int o = 0; o < 8; o++) {
            tr16(acc[o]);
#pragma unroll
            for (int c = 0; c < 4; c++) {
                v4u v = {acc[o][4 * c], acc[o][4 * c + 1], acc[o][4 * c + 2], acc[o][4 * c + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(v, r, (20 + o) * fstride + off + c * 4096, 0, 2);
            }
        }
    }
}

template __global__ void bs_c5_encode_kernel<8>(uint8_t*, int64_t, int, uint32_t, uint32_t);
template __global__ void bs_c5_encode_kernel<24>(uint8_t*, int64_t, int, uint32_t, uint32_t);

}  // namespace ecamd
