// probe_kernels.hip -- measurement kernels of libecamd_probe.so (NOT part of the codec product):
// HBM ceilings (bw_probe_kernel, stream_copy_kernel), the codec's exact read/write pattern with no
// table work (mix_probe_kernel) and the LDS / L1 lookup engines (lookup_probe_kernel).  DESIGN.md
// §4 cites their numbers as the denominators the codec kernels are judged against.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "probe.hpp"

namespace ecamd {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ldnt(const uint8_t* p)
{
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void stnt(uint8_t* p, uint4 v)
{
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

}  // namespace



}  // namespace ecamd

namespace ecamd {

// Streaming copy at 16 B per lane, 4 chunks in flight, non-temporal: the measured HBM ceiling
// for one read + one write stream (DESIGN.md reports the roofline against it and the spec).
__global__ void __launch_bounds__(256) stream_copy_kernel(uint4* __restrict__ dst,
                                                          const uint4* __restrict__ src, int64_t n)
{
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        v4 a = __builtin_nontemporal_load(reinterpret_cast<const v4*>(src + i));
        v4 b = __builtin_nontemporal_load(reinterpret_cast<const v4*>(src + i + stride));
        v4 c = __builtin_nontemporal_load(reinterpret_cast<const v4*>(src + i + 2 * stride));
        v4 d = __builtin_nontemporal_load(reinterpret_cast<const v4*>(src + i + 3 * stride));
        __builtin_nontemporal_store(a, reinterpret_cast<v4*>(dst + i));
        __builtin_nontemporal_store(b, reinterpret_cast<v4*>(dst + i + stride));
        __builtin_nontemporal_store(c, reinterpret_cast<v4*>(dst + i + 2 * stride));
        __builtin_nontemporal_store(d, reinterpret_cast<v4*>(dst + i + 3 * stride));
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

}  // namespace ecamd

namespace ecamd {

// Bandwidth probes for DESIGN.md (not used by the codec): kind 0 copy, 1 read-only (XOR-reduce,
// one dword written per lane at the end), 2 write-only.  Each workgroup owns contiguous tiles of
// blockDim * 16 * U bytes; U loads per lane are in flight before any store.
template <int U>
__global__ void __launch_bounds__(256) bw_probe_kernel(uint8_t* dst, const uint8_t* src,
                                                       int64_t bytes, int kind, uint32_t* sink)
{
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const int64_t tile = static_cast<int64_t>(blockDim.x) * 16 * U;
    const int64_t ntiles = bytes / tile;
    v4 acc = {0u, 0u, 0u, 0u};
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = t * tile + static_cast<int64_t>(threadIdx.x) * 16;
        v4 r[U];
        if (kind != 2) {
#pragma unroll
            for (int u = 0; u < U; u++)
                r[u] = __builtin_nontemporal_load(reinterpret_cast<const v4*>(src + base + u * blockDim.x * 16));
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) r[u] = v4{static_cast<unsigned>(t), 1u, 2u, static_cast<unsigned>(u)};
        }
        if (kind == 1) {
#pragma unroll
            for (int u = 0; u < U; u++) acc ^= r[u];
        } else {
#pragma unroll
            for (int u = 0; u < U; u++)
                __builtin_nontemporal_store(r[u], reinterpret_cast<v4*>(dst + base + u * blockDim.x * 16));
        }
    }
    if (kind == 1 && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[threadIdx.x] = acc.x;
}

template __global__ void bw_probe_kernel<1>(uint8_t*, const uint8_t*, int64_t, int, uint32_t*);
template __global__ void bw_probe_kernel<4>(uint8_t*, const uint8_t*, int64_t, int, uint32_t*);
template __global__ void bw_probe_kernel<8>(uint8_t*, const uint8_t*, int64_t, int, uint32_t*);

// Codec-shaped streaming probe (sweeps only): the access pattern of gf16_apply_kernel on the
// strided [S][K+R][bs] layout -- K fragment reads, R fragment writes per tile, the same tile order
// and prefetch depth -- with no LDS work, and the cache policy of the buffer loads (LP) and stores
// (SP) as the aux immediate (gfx950 cpol: 1 = sc0, 2 = nt, 16 = sc1).  CH chunks of 16 B per lane
// per fragment, the chunks of one lane blockDim*16 bytes apart.
template <int LP, int SP, int CH>
__global__ void __launch_bounds__(CH == 4 ? 256 : 1024) mix_probe_kernel(MixArgs a)
{
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    // wave_contig: each wave covers CH KiB of a fragment contiguously (chunks 1 KiB apart);
    // otherwise the chunks of a lane are blockDim*16 bytes apart.  order 1: every workgroup
    // walks a contiguous range of tiles instead of striding over the grid.
    const int cstride = a.wave_contig ? 1024 : static_cast<int>(blockDim.x) * 16;
    const int lane_off = a.wave_contig
                             ? static_cast<int>(threadIdx.x / 64) * 1024 * CH + static_cast<int>(threadIdx.x % 64) * 16
                             : static_cast<int>(threadIdx.x) * 16;
    // order 2: grid-stride, but tile t reads its K fragments starting at fragment t % K and writes
    // its R outputs starting at t % R (rotated), so neighbouring tiles hit different fragments at once
    const bool contig = a.order == 1;
    const uint32_t per = (a.ntiles + gridDim.x - 1) / gridDim.x;
    const uint32_t t0 = contig ? blockIdx.x * per : blockIdx.x;
    const uint32_t t1 = contig ? min(a.ntiles, t0 + per) : a.ntiles;
    const uint32_t dt = contig ? 1u : gridDim.x;
    for (uint32_t t = t0; t < t1; t += dt) {
        const int rk = a.order == 2 ? static_cast<int>(t % static_cast<uint32_t>(a.K)) : 0;
        const int rr = a.order == 2 && a.R > 0 ? static_cast<int>(t % static_cast<uint32_t>(a.R)) : 0;
        auto rd = [&](int i) { return a.frag[i + rk < a.K ? i + rk : i + rk - a.K]; };
        const uint32_t s = t / a.tiles_per_stripe;
        const int off = static_cast<int>(t - s * a.tiles_per_stripe) * static_cast<int>(blockDim.x) * 16 * CH +
                        lane_off;
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
            a.base + static_cast<int64_t>(s) * a.stripe_stride, 0,
            static_cast<int>(a.stripe_stride), 0x00020000);
        v4 acc[CH];
#pragma unroll
        for (int c = 0; c < CH; c++) acc[c] = v4{0u, 0u, 0u, 0u};
        v4 cur[4][CH], nxt[4][CH];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int c = 0; c < CH; c++)
                cur[i][c] = (i < a.K) ? __builtin_amdgcn_raw_buffer_load_b128(
                                            rsrc, rd(i) * a.frag_stride + off + c * cstride, 0, LP)
                                      : v4{0u, 0u, 0u, 0u};
        for (int j0 = 0; j0 < a.K; j0 += 4) {
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int c = 0; c < CH; c++)
                    nxt[i][c] = (j0 + 4 + i < a.K)
                                    ? __builtin_amdgcn_raw_buffer_load_b128(
                                          rsrc, rd(j0 + 4 + i) * a.frag_stride + off + c * cstride, 0, LP)
                                    : v4{0u, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int c = 0; c < CH; c++) {
                    acc[c] ^= cur[i][c];
                    cur[i][c] = nxt[i][c];
                }
        }
        for (int r = 0; r < a.R; r++)
#pragma unroll
            for (int c = 0; c < CH; c++)
                __builtin_amdgcn_raw_buffer_store_b128(
                    acc[c] + static_cast<unsigned>(r), rsrc,
                    a.frag[a.K + (r + rr < a.R ? r + rr : r + rr - a.R)] * a.frag_stride + off + c * cstride, 0,
                    SP);
    }
}

#define ECAMD_MIX(LP, SP) \
    template __global__ void mix_probe_kernel<LP, SP, 1>(MixArgs); \
    template __global__ void mix_probe_kernel<LP, SP, 2>(MixArgs); \
    template __global__ void mix_probe_kernel<LP, SP, 4>(MixArgs);
ECAMD_MIX_POLICIES(ECAMD_MIX)
#undef ECAMD_MIX

}  // namespace ecamd

namespace ecamd {

// Table-lookup engine probe (sweeps only): random 16-byte lookups into 4 KiB tables, from LDS
// (MODE 0), from global memory through the CU's vector L1 (MODE 1), or half and half (MODE 2),
// 4 lookups per xorshift step; MODE 3 / 4: 16-entry (256 B, nibble-sized) tables from L1 / LDS;
// MODE 5: LDS byte tables and L1 16-entry tables half and half.  Prices the L1 as a second
// lookup engine beside the LDS.
template <int MODE>
__global__ void __launch_bounds__(256) lookup_probe_kernel(const uint4* __restrict__ table, int iters,
                                                           uint32_t* sink)
{
    __shared__ uint4 tab[1024];  // 4 tables x 256 entries x 16 B
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) tab[i] = table[i];
    __syncthreads();
    uint32_t x = 0x9e3779b9u ^ (blockIdx.x * 1024 + threadIdx.x) * 0x85ebca6bu;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int it = 0; it < iters; it++) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const bool nib = MODE == 3 || MODE == 4 || (MODE == 5 && !(b & 1));
            const uint32_t idx = nib ? b * 256 + ((x >> (8 * b)) & 0xfu) : b * 256 + ((x >> (8 * b)) & 0xffu);
            uint4 e;
            if (MODE == 0 || MODE == 4 || ((MODE == 2 || MODE == 5) && (b & 1)))
                e = tab[idx];
            else
                e = table[idx];
            acc.x ^= e.x;
            acc.y ^= e.y;
            acc.z ^= e.z;
            acc.w ^= e.w;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = acc.x;
}

template __global__ void lookup_probe_kernel<0>(const uint4*, int, uint32_t*);
template __global__ void lookup_probe_kernel<1>(const uint4*, int, uint32_t*);
template __global__ void lookup_probe_kernel<2>(const uint4*, int, uint32_t*);
template __global__ void lookup_probe_kernel<3>(const uint4*, int, uint32_t*);
template __global__ void lookup_probe_kernel<4>(const uint4*, int, uint32_t*);
template __global__ void lookup_probe_kernel<5>(const uint4*, int, uint32_t*);

}  // namespace ecamd

namespace ecamd {

// VALU issue-cost probe: each lane runs `iters` rounds of 8 independent chains of one
// instruction form (OP), so the SIMD sees back-to-back independent VALU work from every wave;
// cycles per wave-instruction = wall cycles x waves per SIMD / (iters x 8).  OP: 0 v_xor_b32,
// 1 v_bitop3_b32 (XOR3), 2 v_lshlrev_b32_sdwa (byte select), 3 v_bfe_u32, 4 v_and_b32,
// 5 v_perm_b32, 6 v_lshl_or_b32, 7 ds_read_b128 from a 16-entry table (conflict-free),
// 8 v_bfi_b32 (SGPR mask), 9 v_lshrrev_b32, 10 v_bitop3_b32 0xCA (select, SGPR mask),
// 11 v_alignbit_b32.
template <int OP>
__global__ void __launch_bounds__(256) valu_probe_kernel(int iters, uint32_t seed, uint32_t* sink)
{
    __shared__ uint4 tab[16];
    if (threadIdx.x < 16) tab[threadIdx.x] = make_uint4(threadIdx.x, seed, 3, 4);
    __syncthreads();
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = seed * (threadIdx.x + 1 + i);
    const uint32_t k = seed | 1u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t r;
            if constexpr (OP == 0) {
                asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(k));
            } else if constexpr (OP == 1) {
                asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a[i]), "v"(k), "v"(a[(i + 1) & 7]));
            } else if constexpr (OP == 2) {
                asm volatile("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                             : "=v"(r) : "v"(a[i]));
                r ^= 0;
            } else if constexpr (OP == 3) {
                asm volatile("v_bfe_u32 %0, %1, 8, 4" : "=v"(r) : "v"(a[i]));
            } else if constexpr (OP == 4) {
                asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(k));
            } else if constexpr (OP == 5) {
                asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a[i]), "v"(k), "v"(a[(i + 3) & 7]));
            } else if constexpr (OP == 6) {
                asm volatile("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(r) : "v"(a[i]), "v"(k));
            } else if constexpr (OP == 8) {
                asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(k), "v"(a[i]), "v"(a[(i + 3) & 7]));
            } else if constexpr (OP == 9) {
                asm volatile("v_lshrrev_b32 %0, 4, %1" : "=v"(r) : "v"(a[i]));
            } else if constexpr (OP == 10) {
                asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "s"(k), "v"(a[i]), "v"(a[(i + 3) & 7]));
            } else if constexpr (OP == 11) {
                asm volatile("v_alignbit_b32 %0, %1, %2, 4" : "=v"(r) : "v"(a[i]), "v"(a[(i + 3) & 7]));
            } else {
                uint4 v;
                asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((a[i] & 15u) * 16u));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                r = v.x;
            }
            a[i] = r;
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= a[i];
    if (x == 0x12345678u) sink[0] = x;
}
template __global__ void valu_probe_kernel<0>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<1>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<2>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<3>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<4>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<5>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<6>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<7>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<8>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<9>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<10>(int, uint32_t, uint32_t*);
template __global__ void valu_probe_kernel<11>(int, uint32_t, uint32_t*);

}  // namespace ecamd

namespace ecamd {

// Unaligned-copy probe (sweeps only): `bytes` copied in one-workgroup 4 KiB tiles (256 lanes x 16 B)
// between an aligned side and a side displaced by `shift` bytes -- what the framed copies and the
// copy-through codec see at object offsets j*bs when bs % 16 != 0.  MODE 0: both sides aligned
// (shift ignored); 1: 16-byte buffer loads at src + shift; 2: two aligned loads + v_alignbyte
// window; 3: one aligned load, the second chunk from the next lane (DPP wave_shl:1, lane 63 loads
// its own); 4: dword-aligned 16-byte load at floor4(src + shift) + one dword load, v_alignbyte;
// 5: aligned loads, 16-byte buffer stores at dst + shift (the join's side).
template <int MODE>
__global__ void __launch_bounds__(256) unaligned_probe_kernel(uint8_t* dst, const uint8_t* src, int64_t bytes,
                                                              int shift)
{
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const int64_t tile = 4096;
    const int64_t t = blockIdx.x;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src) + t * tile, 0, 4096 + 32, 0x00020000);
    const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + t * tile, 0, 4096 + 32, 0x00020000);
    const int off = static_cast<int>(threadIdx.x) * 16;
    v4 v;
    if (MODE == 0 || MODE == 5) {
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2);
    } else if (MODE == 1) {
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, off + shift, 0, 2);
    } else if (MODE == 2 || MODE == 3) {
        const int q = (off + shift) & ~15, d = shift & 15;
        const v4 lo = __builtin_amdgcn_raw_buffer_load_b128(rs, q, 0, 2);
        const bool last = (threadIdx.x & 63u) == 63u;
        v4 hi = __builtin_amdgcn_raw_buffer_load_b128(rs, MODE == 2 || last ? q + 16 : static_cast<int>(0x80000000u), 0, 2);
        if (MODE == 3) {
            auto shl1 = [](uint32_t x) {
                return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x130, 0xf, 0xf, false));
            };
            const v4 n = v4{shl1(lo.x), shl1(lo.y), shl1(lo.z), shl1(lo.w)};
            hi = last ? hi : n;
        }
        const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const int dw = d >> 2, by = d & 3;
        v4 o;
        switch (dw) {
        case 0: o = v4{w[0], w[1], w[2], w[3]}; break;
        case 1: o = v4{w[1], w[2], w[3], w[4]}; break;
        case 2: o = v4{w[2], w[3], w[4], w[5]}; break;
        default: o = v4{w[3], w[4], w[5], w[6]}; break;
        }
        if (by) {
            const uint32_t nx = dw == 0 ? w[4] : dw == 1 ? w[5] : dw == 2 ? w[6] : w[7];
            o = v4{__builtin_amdgcn_alignbyte(o.y, o.x, by), __builtin_amdgcn_alignbyte(o.z, o.y, by),
                   __builtin_amdgcn_alignbyte(o.w, o.z, by), __builtin_amdgcn_alignbyte(nx, o.w, by)};
        }
        v = o;
    } else {  // MODE 4
        const int a4 = (off + shift) & ~3, by = (off + shift) & 3;
        const v4 lo = __builtin_amdgcn_raw_buffer_load_b128(rs, a4, 0, 2);
        const uint32_t nx = __builtin_amdgcn_raw_buffer_load_b32(rs, by ? a4 + 16 : static_cast<int>(0x80000000u), 0, 2);
        v = by ? v4{__builtin_amdgcn_alignbyte(lo.y, lo.x, by), __builtin_amdgcn_alignbyte(lo.z, lo.y, by),
                    __builtin_amdgcn_alignbyte(lo.w, lo.z, by), __builtin_amdgcn_alignbyte(nx, lo.w, by)}
               : lo;
    }
    __builtin_amdgcn_raw_buffer_store_b128(v, rd, MODE == 5 ? off + shift : off, 0, 2);
    (void)bytes;
}

template __global__ void unaligned_probe_kernel<0>(uint8_t*, const uint8_t*, int64_t, int);
template __global__ void unaligned_probe_kernel<1>(uint8_t*, const uint8_t*, int64_t, int);
template __global__ void unaligned_probe_kernel<2>(uint8_t*, const uint8_t*, int64_t, int);
template __global__ void unaligned_probe_kernel<3>(uint8_t*, const uint8_t*, int64_t, int);
template __global__ void unaligned_probe_kernel<4>(uint8_t*, const uint8_t*, int64_t, int);
template __global__ void unaligned_probe_kernel<5>(uint8_t*, const uint8_t*, int64_t, int);

// One workgroup's fixed cost (per-call objects of a few KiB run one workgroup): STAGE 0 none,
// 1 `bytes` of a device buffer into LDS one 16-byte load per thread and round, 2 the same with 8
// loads in flight; CODE straight-line dependent VALU steps (≈8 bytes of code each) before the
// single store -- the cost of fetching a long kernel body into a cold instruction cache.
template <int STAGE, int CODE>
__global__ void __launch_bounds__(256) launch_probe_kernel(uint32_t* sink, const uint8_t* src, int bytes)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = static_cast<int>(threadIdx.x);
    if constexpr (STAGE == 1) {
        for (int o = tid * 16; o < bytes; o += 256 * 16)
            *reinterpret_cast<uint4*>(lds + o) = *reinterpret_cast<const uint4*>(src + o);
    } else if constexpr (STAGE == 2) {
        for (int o0 = tid * 16; o0 < bytes; o0 += 8 * 4096) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (o0 + u * 4096 < bytes) v[u] = *reinterpret_cast<const uint4*>(src + o0 + u * 4096);
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (o0 + u * 4096 < bytes) *reinterpret_cast<uint4*>(lds + o0 + u * 4096) = v[u];
        }
    }
    if constexpr (STAGE) __syncthreads();
    uint32_t x = STAGE ? *reinterpret_cast<const uint32_t*>(lds + tid * 4) : static_cast<uint32_t>(tid);
#pragma unroll
    for (int i = 0; i < CODE; i++) x = __builtin_amdgcn_alignbit(x, x ^ (0x9e3779b9u + i), i & 31) + (i * 0x85ebca6bu);
    if (tid == 0) sink[blockIdx.x] = x;
}
template __global__ void launch_probe_kernel<0, 0>(uint32_t*, const uint8_t*, int);
template __global__ void launch_probe_kernel<1, 0>(uint32_t*, const uint8_t*, int);
template __global__ void launch_probe_kernel<2, 0>(uint32_t*, const uint8_t*, int);
template __global__ void launch_probe_kernel<0, 1024>(uint32_t*, const uint8_t*, int);
template __global__ void launch_probe_kernel<0, 4096>(uint32_t*, const uint8_t*, int);


// Mailbox round trip (round 6, the resident-server question of DESIGN.md §10): one wave polls a word in
// pinned host memory (system-scope acquire loads, s_sleep between them) for request i = 1..n, optionally
// reads `payload` bytes of the mailbox after it (the argument block a server would fetch), and stores
// the ack word.  Every wave exits: after request n, when the host sets stop, or after idle_ticks of the
// 100 MHz constant clock (s_memrealtime) with no new request.
__global__ void __launch_bounds__(64) mailbox_probe_kernel(uint32_t* mb, int n, int payload, uint64_t idle_ticks)
{
    const int lane = static_cast<int>(threadIdx.x);
    uint32_t sum = 0;
    for (int i = 1; i <= n; i++) {
        uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool got = false;
        for (;;) {
            const uint32_t seq = __hip_atomic_load(mb, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            const uint32_t stop = __hip_atomic_load(mb + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (stop) break;
            if (seq == static_cast<uint32_t>(i)) {
                got = true;
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
            __builtin_amdgcn_s_sleep(1);
        }
        if (!got) break;
        if (payload > 0 && lane * 4 < payload)
            sum += __hip_atomic_load(mb + 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        sum = __builtin_amdgcn_readfirstlane(sum);
        if (lane == 0) {
            __hip_atomic_store(mb + 3, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
            __hip_atomic_store(mb + 1, static_cast<uint32_t>(i), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

}  // namespace ecamd
