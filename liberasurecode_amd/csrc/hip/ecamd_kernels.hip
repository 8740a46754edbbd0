// ecamd_kernels.hip -- gfx950 (MI355X / CDNA4) kernels for the erasure-code hot path.
//
// gf16_apply_kernel: out[r] = sum_j A[r][j] * in[j] over GF(2^16) on little-endian 16-bit words,
// for many independent stripes in one launch.  This is the GPU form of the reference's
// region_dot_product / region_multiply / region_xor (src/builtin/rs_vand/liberasurecode_rs_vand.c:
// 336-397), which encode, decode and reconstruct all reduce to (:399-558).
//
//   * HBM: every lane moves 16 B per fragment per tile (global_load_dwordx4), a wave covers a
//     contiguous 1 KiB of each fragment; inputs are read once and all outputs written once per
//     tile, so algorithmic traffic = (K + R) * blocksize per stripe.
//   * LDS: multiply-by-constant is GF(2)-linear, so c*x = T_lo[x & 0xff] ^ T_hi[x >> 8].  The
//     tables of one input pack all W outputs of the row group into one W*2-byte entry, so one
//     16-bit input word costs two ds_read_b{32,64,128} for every output at once (W = 2, 4, 8).
//     The whole image (K * 512 * 2W bytes) is staged into LDS once per workgroup; workgroups are
//     persistent and grid-stride over tiles, so the staging cost is amortised.
//   * Inputs are fetched one group of 4 fragments ahead of the lookups (software pipeline) so
//     each wave keeps >= 4 KiB of loads in flight while its LDS lookups run.
//
// xor_apply_kernel: out[r] = XOR of the inputs selected by mask[r] (flat-XOR HD codes,
// src/builtin/xor_codes/xor_code.c:141-207); pure streaming.
//
// splitmix_fill_kernel: synthetic fragment bytes (bench / tests), same stream as tests/ecdata.py.
//
// The device helpers live in ecamd_apply.hpp; gf16_stream_kernel -- the form every strided launch
// that fits it takes (buffer loads, unrolled inputs) -- in ecamd_stream.hpp, instantiated per
// output width in ecamd_stream_w{2,4,8}.hip.  gf16_apply_kernel below remains for pointer-table
// launches, more than 20 inputs per pass, offsets beyond 2 GiB and the nibble / ablation sweeps.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ecamd_isa.hpp"
#include "ecamd_kernels.hpp"

#include "ecamd_apply.hpp"

namespace ecamd {


template <int W, bool PTRS, bool NT, bool NIB, bool COPY>
__device__ __forceinline__ void gf16_apply_body(const ApplyArgs& a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int EB = 2 * W;
    const int tbytes = a.ncols * (NIB ? 64 : 512) * EB;
    for (int o = threadIdx.x * 16; o < tbytes; o += blockDim.x * 16)
        *reinterpret_cast<uint4*>(lds + o) = *reinterpret_cast<const uint4*>(a.tables + o);
    __syncthreads();

    const int64_t span = static_cast<int64_t>(blockDim.x) * 16;
    for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const uint32_t s = t / a.tiles_per_stripe;
        const int64_t off = static_cast<int64_t>(t - s * a.tiles_per_stripe) * span +
                            static_cast<int64_t>(threadIdx.x) * 16;
        const int64_t rem = a.bs - off;
        if (rem <= 0) continue;
        if (rem >= 16)
            apply_tile<W, PTRS, NT, NIB, COPY, false>(a, lds, s, off, 16);
        else
            apply_tile<W, PTRS, NT, NIB, COPY, true>(a, lds, s, off, static_cast<int>(rem));
    }
}

template <int W, bool PTRS, bool NT, bool NIB>
__global__ void __launch_bounds__(NIB ? 512 : 1024) gf16_apply_kernel(const ApplyArgs a)
{
    gf16_apply_body<W, PTRS, NT, NIB, false>(a);
}

// Framed encode (hip/ecamd_frame_api.hip): the k data inputs are read straight from the object
// and copied into their fragment payloads by the same launch that computes the parity.
template <int W>
__global__ void __launch_bounds__(1024) gf16_copy_apply_kernel(const ApplyArgs a)
{
    gf16_apply_body<W, false, true, false, true>(a);
}
template __global__ void gf16_copy_apply_kernel<2>(const ApplyArgs);
template __global__ void gf16_copy_apply_kernel<4>(const ApplyArgs);
template __global__ void gf16_copy_apply_kernel<8>(const ApplyArgs);


#define ECAMD_INST(W, P, N, B) \
    template __global__ void gf16_apply_kernel<W, P, N, B>(const ApplyArgs);
#define ECAMD_INST2(P, N, B) ECAMD_INST(2, P, N, B) ECAMD_INST(4, P, N, B) ECAMD_INST(8, P, N, B)
ECAMD_INST2(false, false, false) ECAMD_INST2(true, false, false)
ECAMD_INST2(false, true, false) ECAMD_INST2(true, true, false)
ECAMD_INST2(false, true, true) ECAMD_INST2(true, true, true)
#undef ECAMD_INST2
#undef ECAMD_INST

// ---------------------------------------------------------------- flat XOR ----

template <int W, bool PTRS, bool TAIL>
__device__ __forceinline__ void xor_tile(const ApplyArgs& a, uint32_t s, int64_t off, int rem)
{
    const int K = a.ncols;
    uint4 acc[W];
#pragma unroll
    for (int r = 0; r < W; r++) acc[r] = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < K; j++) {
        const uint8_t* p = in_frag<PTRS>(a, s, j) + off;
        const uint4 x = TAIL ? load_tail(p, rem) : load16(p);
#pragma unroll
        for (int r = 0; r < W; r++) {
            const uint32_t m = 0u - ((a.masks[r] >> j) & 1u);  // wave-uniform select
            acc[r].x ^= x.x & m;
            acc[r].y ^= x.y & m;
            acc[r].z ^= x.z & m;
            acc[r].w ^= x.w & m;
        }
    }
#pragma unroll
    for (int r = 0; r < W; r++) {
        if (r >= a.nrows) break;
        uint8_t* q = out_frag<PTRS>(a, s, r) + off;
        uint4 v = acc[r];
        if (a.accumulate) {
            uint4 prev = TAIL ? load_tail(q, rem) : load16(q);
            v.x ^= prev.x;
            v.y ^= prev.y;
            v.z ^= prev.z;
            v.w ^= prev.w;
        }
        if (TAIL)
            store_tail(q, v, rem);
        else
            *reinterpret_cast<uint4*>(q) = v;
    }
}

template <int W, bool PTRS>
__global__ void __launch_bounds__(256) xor_apply_kernel(const ApplyArgs a)
{
    const int64_t span = static_cast<int64_t>(blockDim.x) * 16;
    for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const uint32_t s = t / a.tiles_per_stripe;
        const int64_t off = static_cast<int64_t>(t - s * a.tiles_per_stripe) * span +
                            static_cast<int64_t>(threadIdx.x) * 16;
        const int64_t rem = a.bs - off;
        if (rem <= 0) continue;
        if (rem >= 16)
            xor_tile<W, PTRS, false>(a, s, off, 16);
        else
            xor_tile<W, PTRS, true>(a, s, off, static_cast<int>(rem));
    }
}

template __global__ void xor_apply_kernel<8, false>(const ApplyArgs);
template __global__ void xor_apply_kernel<8, true>(const ApplyArgs);

// xor_stream_kernel<KG>: the strided flat-XOR apply for up to 4*KG inputs in the form of
// gf16_stream_kernel (ecamd_stream.hpp): buffer loads on one resource per stripe, the loads of a
// group of 4 inputs unconditional (out-of-range offsets read zeros, no traffic), inputs unrolled.
// Output r accumulates input j under the wave-uniform mask bit j of masks[r]: one v_bitop3 per
// dword (acc ^ (x & m)), no branches.  COPY (framed flat-XOR encode, round 4): every input is also
// stored at copy_base + s*copy_stride + copy_off32[j] as it is loaded (object chunk -> data payload;
// the caller runs whole tiles only).
template <int KG, bool COPY>
__global__ void __launch_bounds__(256) xor_stream_kernel(const ApplyArgs a)
{
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const int cstride = static_cast<int>(blockDim.x) * 16;
    for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const uint32_t sl = t / a.tiles_per_stripe;
        const int64_t toff = static_cast<int64_t>(t - sl * a.tiles_per_stripe) * cstride;
        const uint32_t s = a.stripe_list ? static_cast<uint32_t>(a.stripe_list[sl]) : sl;
        const int64_t o64 = toff + static_cast<int64_t>(threadIdx.x) * 16;
        if (toff + cstride > a.bs) {  // last, partial tile of each fragment
            const int64_t rem = a.bs - o64;
            if (rem >= 16)
                xor_tile<8, false, false>(a, s, o64, 16);
            else if (rem > 0)
                xor_tile<8, false, true>(a, s, o64, static_cast<int>(rem));
            continue;
        }
        const int off = static_cast<int>(o64);
        const auto rin = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.in_base) + static_cast<int64_t>(s) * a.in_stride, 0,
            static_cast<int>(a.in_records), 0x00020000);
        const auto rout = __builtin_amdgcn_make_buffer_rsrc(
            a.out_base + static_cast<int64_t>(s) * a.out_stride, 0, static_cast<int>(a.out_records),
            0x00020000);
        v4 acc[8];
#pragma unroll
        for (int r = 0; r < 8; r++) acc[r] = v4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int g = 0; g < KG; g++) {
            v4 x[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int j = 4 * g + i;
                const int o = (j < a.ncols) ? a.in_off32[j] + off : static_cast<int>(0x80000000u);
                x[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, o, 0, 2);
            }
            if constexpr (COPY) {
                const auto rcopy = __builtin_amdgcn_make_buffer_rsrc(
                    a.copy_base + static_cast<int64_t>(s) * a.copy_stride, 0, static_cast<int>(a.copy_records), 0x00020000);
#pragma unroll
                for (int i = 0; i < 4; i++) {  // skipped inputs: an out-of-range offset, dropped
                    const int j = 4 * g + i;
                    const int o = (j < a.ncols && a.copy_off32[j] >= 0) ? a.copy_off32[j] + off
                                                                         : static_cast<int>(0x80000000u);
                    __builtin_amdgcn_raw_buffer_store_b128(x[i], rcopy, o, 0, 2);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int j = 4 * g + i;
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    if (r >= a.nrows) break;
                    const uint32_t msk = 0u - ((a.masks[r] >> j) & 1u);  // wave-uniform
#pragma unroll
                    for (int d = 0; d < 4; d++) acc[r][d] = xor_and(acc[r][d], x[i][d], msk);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 8; r++) {
            if (r >= a.nrows) break;
            const int o = a.out_off32[r] + off;
            v4 v = acc[r];
            if (a.accumulate) v ^= __builtin_amdgcn_raw_buffer_load_b128(rout, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(v, rout, o, 0, 2);
        }
    }
}

template __global__ void xor_stream_kernel<1, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<2, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<3, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<4, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<8, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<1, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<2, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<3, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<4, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<8, true>(const ApplyArgs);

// ---------------------------------------------------------------- synthetic data ----

__global__ void __launch_bounds__(256) splitmix_fill_kernel(FillArgs f)
{
    const int64_t words = (f.bs + 7) / 8;
    const int64_t total = words * f.nfrags * static_cast<int64_t>(f.nstripes);
    for (int64_t g = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; g < total;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = g % words;
        const int64_t fs = g / words;
        const int frag = static_cast<int>(fs % f.nfrags);
        const int64_t s = fs / f.nfrags;
        const uint64_t seed = f.seed_base ^ (static_cast<uint64_t>(s + f.stripe0) << 8) ^
                              static_cast<uint64_t>(frag);
        uint64_t z = seed + static_cast<uint64_t>(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        uint8_t* p = f.base + s * f.stripe_stride + frag * f.frag_stride + i * 8;
        const int64_t left = f.bs - i * 8;
        if (left >= 8) {
            *reinterpret_cast<uint64_t*>(p) = z;
        } else {
            for (int b = 0; b < left; b++) p[b] = static_cast<uint8_t>(z >> (8 * b));
        }
    }
}

}  // namespace ecamd
