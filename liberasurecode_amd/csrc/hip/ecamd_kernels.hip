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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ecamd_isa.hpp"
#include "ecamd_kernels.hpp"

namespace ecamd {

namespace {

__device__ __forceinline__ uint4 load16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 stream_load16(const uint8_t* p)
{
    if constexpr (NT) {
        u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *reinterpret_cast<const uint4*>(p);
    }
}

template <bool NT>
__device__ __forceinline__ void stream_store16(uint8_t* p, uint4 v)
{
    if constexpr (NT) {
        u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
    } else {
        *reinterpret_cast<uint4*>(p) = v;
    }
}

// Partial 16-byte chunk at the end of a fragment: bytes [0, rem) of p, zero filled.
__device__ __forceinline__ uint4 load_tail(const uint8_t* p, int rem)
{
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; i++) {
        uint32_t b = (i < rem) ? static_cast<uint32_t>(p[i]) : 0u;
        w[i >> 2] |= b << (8 * (i & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_tail(uint8_t* p, uint4 v, int rem)
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; i++)
        if (i < rem) p[i] = static_cast<uint8_t>(w[i >> 2] >> (8 * (i & 3)));
}

template <bool PTRS>
__device__ __forceinline__ const uint8_t* in_frag(const ApplyArgs& a, uint32_t s, int j)
{
    if constexpr (PTRS)
        return a.in_ptrs[static_cast<int64_t>(s) * a.in_stride + a.in_off[j]];
    else
        return a.in_base + static_cast<int64_t>(s) * a.in_stride + a.in_off[j];
}

template <bool PTRS>
__device__ __forceinline__ uint8_t* out_frag(const ApplyArgs& a, uint32_t s, int r)
{
    if constexpr (PTRS)
        return a.out_ptrs[static_cast<int64_t>(s) * a.out_stride + a.out_off[r]];
    else
        return a.out_base + static_cast<int64_t>(s) * a.out_stride + a.out_off[r];
}

// One LDS table entry of D dwords (D = W/2): ds_read_b32 / b64 / b128.
template <int D>
__device__ __forceinline__ void lds_entry(const uint8_t* p, uint32_t (&e)[D])
{
    if constexpr (D == 1) {
        e[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (D == 2) {
        uint2 v = *reinterpret_cast<const uint2*>(p);
        e[0] = v.x;
        e[1] = v.y;
    } else {
        uint4 v = *reinterpret_cast<const uint4*>(p);
        e[0] = v.x;
        e[1] = v.y;
        e[2] = v.z;
        e[3] = v.w;
    }
}

// acc[w] ^= T_lo[j][lo(x_w)] ^ T_hi[j][hi(x_w)] for the 8 words of one 16-byte chunk.
template <int W>
__device__ __forceinline__ void mac_chunk(const uint8_t* tl, uint4 x, uint32_t (&acc)[8][W / 2])
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    const uint8_t* th = tl + 256 * EB;
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const uint32_t v = xs[w >> 1] >> ((w & 1) * 16);
        uint32_t e0[D], e1[D];
        lds_entry<D>(tl + (v & 0xffu) * EB, e0);
        lds_entry<D>(th + ((v >> 8) & 0xffu) * EB, e1);
#pragma unroll
        for (int d = 0; d < D; d++) acc[w][d] = xor3(acc[w][d], e0[d], e1[d]);
    }
}

constexpr int log2i(int v) { return v <= 1 ? 0 : 1 + log2i(v / 2); }

// Nibble tables (host/tables.hpp build_nibble_tables): four conflict-free lookups per word.  The
// nibbles of a data dword are spread into bytes once; each table offset is then one SDWA shift.
template <int W, int H>
__device__ __forceinline__ void mac_word_nib(const uint8_t* t, uint32_t lo, uint32_t hi,
                                             uint32_t (&acc)[W / 2])
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    constexpr int S = log2i(EB);
    uint32_t e0[D], e1[D], e2[D], e3[D];
    lds_entry<D>(t + 0 * 16 * EB + byte_shl<2 * H, S>(lo), e0);      // bits 0-3 of the word
    lds_entry<D>(t + 1 * 16 * EB + byte_shl<2 * H, S>(hi), e1);      // bits 4-7
    lds_entry<D>(t + 2 * 16 * EB + byte_shl<2 * H + 1, S>(lo), e2);  // bits 8-11
    lds_entry<D>(t + 3 * 16 * EB + byte_shl<2 * H + 1, S>(hi), e3);  // bits 12-15
#pragma unroll
    for (int d = 0; d < D; d++) acc[d] = xor3(xor3(acc[d], e0[d], e1[d]), e2[d], e3[d]);
}

template <int W>
__device__ __forceinline__ void mac_chunk_nib(const uint8_t* t, uint4 x, uint32_t (&acc)[8][W / 2])
{
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo = xs[i] & 0x0f0f0f0fu, hi = (xs[i] >> 4) & 0x0f0f0f0fu;
        mac_word_nib<W, 0>(t, lo, hi, acc[2 * i]);
        mac_word_nib<W, 1>(t, lo, hi, acc[2 * i + 1]);
    }
}

template <int W, bool PTRS, bool NT, bool NIB, bool COPY, bool TAIL>
__device__ __forceinline__ void apply_tile(const ApplyArgs& a, const uint8_t* lds, uint32_t s,
                                           int64_t off, int rem)
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    const int K = a.ncols;
    uint32_t acc[8][D];
#pragma unroll
    for (int w = 0; w < 8; w++)
#pragma unroll
        for (int d = 0; d < D; d++) acc[w][d] = 0u;

    auto fetch = [&](int j) -> uint4 {
        const uint8_t* p = in_frag<PTRS>(a, s, j) + off;
        return TAIL ? load_tail(p, rem) : stream_load16<NT>(p);
    };
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = (i < K) ? fetch(i) : make_uint4(0, 0, 0, 0);
    for (int j0 = 0; j0 < K; j0 += 4) {
#pragma unroll
        for (int i = 0; i < 4; i++)
            nxt[i] = (j0 + 4 + i < K) ? fetch(j0 + 4 + i) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (j0 + i < K) {
                if constexpr (COPY) {  // copy-through: the input also lands in its own slot
                    if (a.copy_off[j0 + i] >= 0) {  // wave-uniform
                        uint8_t* c = a.copy_base + static_cast<int64_t>(s) * a.copy_stride +
                                     a.copy_off[j0 + i] + off;
                        if (TAIL)
                            store_tail(c, cur[i], rem);
                        else
                            stream_store16<NT>(c, cur[i]);
                    }
                }
                if constexpr (NIB)
                    mac_chunk_nib<W>(lds + static_cast<size_t>(j0 + i) * 64 * EB, cur[i], acc);
                else
                    mac_chunk<W>(lds + static_cast<size_t>(j0 + i) * 512 * EB, cur[i], acc);
            }
#pragma unroll
        for (int i = 0; i < 4; i++) cur[i] = nxt[i];
    }

#pragma unroll
    for (int r = 0; r < W; r++) {
        if (r >= a.nrows) break;
        uint32_t o[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const uint32_t A = acc[2 * d][r >> 1], B = acc[2 * d + 1][r >> 1];
            o[d] = (r & 1) ? ((A >> 16) | (B & 0xffff0000u)) : ((A & 0xffffu) | (B << 16));
        }
        uint4 v = make_uint4(o[0], o[1], o[2], o[3]);
        uint8_t* q = out_frag<PTRS>(a, s, r) + off;
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
            stream_store16<NT>(q, v);
    }
}

}  // namespace

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

// ------------------------------------------------------------ streaming form ----
// gf16_stream_kernel<W, KG, CH, PF>: the strided gf16 apply for up to 4*KG inputs, written so the
// HBM stream never stalls behind the table work:
//   * buffer loads/stores on one resource per stripe (32-bit offsets, no 64-bit address math);
//     the loads of a group of 4 inputs are unconditional -- an input index past ncols gets an
//     out-of-range offset, which the buffer unit answers with zeros and no memory traffic -- so
//     the code is straight-line and the next group's loads stay in flight (counted vmcnt) while
//     the current group's lookups run;
//   * inputs fully unrolled: each input's table base is a compile-time LDS offset and each
//     table index one SDWA byte-select shift (byte_shl), i.e. one VALU op per lookup;
//   * CH 16-byte chunks per lane per fragment (blockDim*16 bytes apart): CH*1 KiB per wave per
//     fragment in one tile;
//   * PF: the next group's loads issued before (true) or after (false) this group's lookups.
// Partial tiles at the end of a fragment go through apply_tile's byte-exact tail code.
namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int W, int J>
__device__ __forceinline__ void mac_chunk_imm(const uint8_t* lds, v4u x, uint32_t (&acc)[8][W / 2])
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    constexpr int S = log2i(EB);
    constexpr int TL = J * 512 * EB;
    constexpr int TH = TL + 256 * EB;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const uint32_t v = x[w >> 1];
        uint32_t e0[D], e1[D];
        if (w & 1) {
            lds_entry<D>(lds + TL + byte_shl<2, S>(v), e0);
            lds_entry<D>(lds + TH + byte_shl<3, S>(v), e1);
        } else {
            lds_entry<D>(lds + TL + byte_shl<0, S>(v), e0);
            lds_entry<D>(lds + TH + byte_shl<1, S>(v), e1);
        }
#pragma unroll
        for (int d = 0; d < D; d++) acc[w][d] = xor3(acc[w][d], e0[d], e1[d]);
    }
}

// Nibble tables (host/tables.cpp build_nibble_tables: per input 4 tables of 16 entries, table q
// for bits 4q..4q+3 of the word).  A 16-entry table of EB-byte entries spans 16*EB <= 256 bytes,
// one LDS bank row, so no lookup ever conflicts -- at twice the lookups of the byte tables.  The
// nibbles of a data dword are moved to scaled-index position once (L: low nibbles, H: high
// nibbles, each times EB), each lookup address is then one byte extract, the table base a
// compile-time offset.
template <int W, int J>
__device__ __forceinline__ void mac_chunk_nib_imm(const uint8_t* lds, v4u x, uint32_t (&acc)[8][W / 2])
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    constexpr int S = log2i(EB);
    constexpr uint32_t M = 0x0f0f0f0fu << S;
    constexpr int T = J * 64 * EB;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t L = (x[i] << S) & M;
        const uint32_t H = (S >= 4 ? (x[i] << (S - 4)) : (x[i] >> (4 - S))) & M;
#pragma unroll
        for (int h = 0; h < 2; h++) {  // word 2i+h = bytes 2h (bits 0-7), 2h+1 (bits 8-15)
            uint32_t e0[D], e1[D], e2[D], e3[D];
            lds_entry<D>(lds + T + 0 * 16 * EB + ((L >> (16 * h)) & 0xffu), e0);
            lds_entry<D>(lds + T + 1 * 16 * EB + ((H >> (16 * h)) & 0xffu), e1);
            lds_entry<D>(lds + T + 2 * 16 * EB + ((L >> (16 * h + 8)) & 0xffu), e2);
            lds_entry<D>(lds + T + 3 * 16 * EB + ((H >> (16 * h + 8)) & 0xffu), e3);
#pragma unroll
            for (int d = 0; d < D; d++)
                acc[2 * i + h][d] = xor3(xor3(acc[2 * i + h][d], e0[d], e1[d]), e2[d], e3[d]);
        }
    }
}

template <int W, int CH, int J, bool NIB>
__device__ __forceinline__ void input_mac(const ApplyArgs& a, const uint8_t* lds, const v4u (&x)[CH],
                                          uint32_t (&acc)[CH][8][W / 2])
{
    if (J < a.ncols) {  // wave-uniform
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if constexpr (NIB)
                mac_chunk_nib_imm<W, J>(lds, x[c], acc[c]);
            else
                mac_chunk_imm<W, J>(lds, x[c], acc[c]);
        }
    }
}

template <int W, int CH, int G, int KG>
__device__ __forceinline__ void load_group(const ApplyArgs& a, __amdgpu_buffer_rsrc_t rin, int off,
                                           int cstride, v4u (&x)[4][CH])
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int j = 4 * G + i;
        const int base = (j < a.ncols) ? a.in_off32[j] + off : static_cast<int>(0x80000000u);
#pragma unroll
        for (int c = 0; c < CH; c++)
            x[i][c] = __builtin_amdgcn_raw_buffer_load_b128(rin, base + c * cstride, 0, 2);
    }
}

// Group G's lookups; with PF the loads of group G+1 are issued before them (in flight during the
// lookups), without PF after them (each wave: load, wait, look up -- latency hidden by occupancy).
template <int W, int CH, int G, int KG, bool PF, bool NIB>
__device__ __forceinline__ void stream_group(const ApplyArgs& a, const uint8_t* lds,
                                             __amdgpu_buffer_rsrc_t rin, int off, int cstride,
                                             v4u (&cur)[4][CH], uint32_t (&acc)[CH][8][W / 2])
{
    v4u nxt[4][CH];
    if constexpr (PF && G + 1 < KG) load_group<W, CH, G + 1, KG>(a, rin, off, cstride, nxt);
    input_mac<W, CH, 4 * G + 0, NIB>(a, lds, cur[0], acc);
    input_mac<W, CH, 4 * G + 1, NIB>(a, lds, cur[1], acc);
    input_mac<W, CH, 4 * G + 2, NIB>(a, lds, cur[2], acc);
    input_mac<W, CH, 4 * G + 3, NIB>(a, lds, cur[3], acc);
    if constexpr (G + 1 < KG) {
        if constexpr (!PF) load_group<W, CH, G + 1, KG>(a, rin, off, cstride, nxt);
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int c = 0; c < CH; c++) cur[i][c] = nxt[i][c];
        stream_group<W, CH, G + 1, KG, PF, NIB>(a, lds, rin, off, cstride, cur, acc);
    }
}

}  // namespace

template <int W, int KG, int CH, bool PF, bool NIB>
__global__ void __launch_bounds__(1024) gf16_stream_kernel(const ApplyArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    const int tbytes = a.ncols * (NIB ? 64 : 512) * EB;
    for (int o = threadIdx.x * 16; o < tbytes; o += blockDim.x * 16)
        *reinterpret_cast<uint4*>(lds + o) = *reinterpret_cast<const uint4*>(a.tables + o);
    __syncthreads();

    const int cstride = static_cast<int>(blockDim.x) * 16;
    const int64_t span = static_cast<int64_t>(cstride) * CH;
    // tile_order 1: each workgroup walks its own contiguous range of tiles (a long sequential
    // run through each fragment); 0: tiles strided over the grid.
    const uint32_t per = (a.ntiles + gridDim.x - 1) / gridDim.x;
    const uint32_t t0 = a.tile_order ? blockIdx.x * per : blockIdx.x;
    const uint32_t t1 = a.tile_order ? min(a.ntiles, t0 + per) : a.ntiles;
    const uint32_t dt = a.tile_order ? 1u : gridDim.x;
    for (uint32_t t = t0; t < t1; t += dt) {
        const uint32_t s = t / a.tiles_per_stripe;
        const int64_t toff = static_cast<int64_t>(t - s * a.tiles_per_stripe) * span;
        if (toff + span > a.bs) {  // last, partial tile of each fragment
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const int64_t o = toff + c * cstride + static_cast<int64_t>(threadIdx.x) * 16;
                const int64_t rem = a.bs - o;
                if (rem >= 16)
                    apply_tile<W, false, true, NIB, false, false>(a, lds, s, o, 16);
                else if (rem > 0)
                    apply_tile<W, false, true, NIB, false, true>(a, lds, s, o, static_cast<int>(rem));
            }
            continue;
        }
        const int off = static_cast<int>(toff) + static_cast<int>(threadIdx.x) * 16;
        const auto rin = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.in_base) + static_cast<int64_t>(s) * a.in_stride, 0,
            static_cast<int>(a.in_records), 0x00020000);
        const auto rout = __builtin_amdgcn_make_buffer_rsrc(
            a.out_base + static_cast<int64_t>(s) * a.out_stride, 0, static_cast<int>(a.out_records),
            0x00020000);

        uint32_t acc[CH][8][D];
#pragma unroll
        for (int c = 0; c < CH; c++)
#pragma unroll
            for (int w = 0; w < 8; w++)
#pragma unroll
                for (int d = 0; d < D; d++) acc[c][w][d] = 0u;
        v4u cur[4][CH];
        load_group<W, CH, 0, KG>(a, rin, off, cstride, cur);
        stream_group<W, CH, 0, KG, PF, NIB>(a, lds, rin, off, cstride, cur, acc);

#pragma unroll
        for (int r = 0; r < W; r++) {
            if (r >= a.nrows) break;
#pragma unroll
            for (int c = 0; c < CH; c++) {
                v4u v;
#pragma unroll
                for (int d = 0; d < 4; d++) {
                    const uint32_t A = acc[c][2 * d][r >> 1], B = acc[c][2 * d + 1][r >> 1];
                    v[d] = (r & 1) ? ((A >> 16) | (B & 0xffff0000u)) : ((A & 0xffffu) | (B << 16));
                }
                const int o = a.out_off32[r] + off + c * cstride;
                if (a.accumulate) v ^= __builtin_amdgcn_raw_buffer_load_b128(rout, o, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(v, rout, o, 0, 2);  // nt
            }
        }
    }
}

#define ECAMD_STREAM_INST(W, KG, CH, PF, NIB) \
    template __global__ void gf16_stream_kernel<W, KG, CH, PF, NIB>(const ApplyArgs);
#define ECAMD_STREAM_KG(W, CH, PF, NIB)                                                   \
    ECAMD_STREAM_INST(W, 1, CH, PF, NIB) ECAMD_STREAM_INST(W, 2, CH, PF, NIB)             \
    ECAMD_STREAM_INST(W, 3, CH, PF, NIB) ECAMD_STREAM_INST(W, 4, CH, PF, NIB)             \
    ECAMD_STREAM_INST(W, 5, CH, PF, NIB)
ECAMD_STREAM_KG(2, 1, true, false) ECAMD_STREAM_KG(4, 1, true, false) ECAMD_STREAM_KG(8, 1, true, false)
ECAMD_STREAM_KG(2, 1, false, false) ECAMD_STREAM_KG(4, 1, false, false) ECAMD_STREAM_KG(8, 1, false, false)
ECAMD_STREAM_KG(2, 2, true, false) ECAMD_STREAM_KG(4, 2, true, false)
ECAMD_STREAM_KG(2, 2, false, false) ECAMD_STREAM_KG(4, 2, false, false)
ECAMD_STREAM_KG(2, 1, false, true) ECAMD_STREAM_KG(4, 1, false, true) ECAMD_STREAM_KG(8, 1, false, true)
#undef ECAMD_STREAM_KG
#undef ECAMD_STREAM_INST

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
