// ecamd_stream.hpp -- gf16_stream_kernel, the strided GF(2^16) apply used for every strided launch
// that fits it (definition; instantiated per output width in ecamd_stream_w{2,4,8}.hip so the
// variants compile in parallel).
#pragma once
#include "ecamd_apply.hpp"

namespace ecamd {

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

// Per-tile addressing shared by the helpers below: the input and copy-through resources of the
// stripe, this lane's byte offset in a fragment and the distance between its chunks.
struct StreamTile {
    __amdgpu_buffer_rsrc_t rin;
    __amdgpu_buffer_rsrc_t rcopy;
    int off;      // this lane's byte offset in a fragment
    int cstride;  // bytes between a lane's chunks
};

// Hybrid lookups (TM >= 2, 8-output passes): some table lookups of each group of 4 inputs are
// read through the vector L1 (plain global loads of the same image) instead of the LDS, so the
// two lookup engines work side by side -- random 16-byte lookups run ~5.4 per clock per CU from
// LDS and ~2 from L1 (tools/lookup_probe.py).  The L1 lookups are all issued at the start of the
// group and consumed after the other inputs' LDS lookups, so their latency overlaps LDS work.
// hyb_fetch: words 0..N-1 of input J's lo (HI = 0) or hi (HI = 1) byte table.
template <int W, int J, int HI, int N>
__device__ __forceinline__ void hyb_fetch(const uint8_t* gtab, v4u x, uint32_t (&e)[N][W / 2])
{
    constexpr int D = W / 2;
    constexpr int S = log2i(2 * W);
    constexpr int T = J * 512 * 2 * W + HI * 256 * 2 * W;
#pragma unroll
    for (int w = 0; w < N; w++) {
        const uint32_t v = x[w >> 1];
        if (w & 1)
            lds_entry<D>(gtab + T + byte_shl<2 + HI, S>(v), e[w]);
        else
            lds_entry<D>(gtab + T + byte_shl<0 + HI, S>(v), e[w]);
    }
}

// mac_chunk_imm with the first NL lo and NH hi lookups taken from registers (hyb_fetch).
template <int W, int J, int NL, int NH>
__device__ __forceinline__ void mac_chunk_mixed(const uint8_t* lds, v4u x, const uint32_t (&el)[NL ? NL : 1][W / 2],
                                                const uint32_t (&eh)[NH ? NH : 1][W / 2],
                                                uint32_t (&acc)[8][W / 2])
{
    constexpr int D = W / 2;
    constexpr int S = log2i(2 * W);
    constexpr int TL = J * 512 * 2 * W;
    constexpr int TH = TL + 256 * 2 * W;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const uint32_t v = x[w >> 1];
        uint32_t e0[D], e1[D];
        if (w < NL) {
#pragma unroll
            for (int d = 0; d < D; d++) e0[d] = el[w < NL ? w : 0][d];
        } else if (w & 1) {
            lds_entry<D>(lds + TL + byte_shl<2, S>(v), e0);
        } else {
            lds_entry<D>(lds + TL + byte_shl<0, S>(v), e0);
        }
        if (w < NH) {
#pragma unroll
            for (int d = 0; d < D; d++) e1[d] = eh[w < NH ? w : 0][d];
        } else if (w & 1) {
            lds_entry<D>(lds + TH + byte_shl<3, S>(v), e1);
        } else {
            lds_entry<D>(lds + TH + byte_shl<1, S>(v), e1);
        }
#pragma unroll
        for (int d = 0; d < D; d++) acc[w][d] = xor3(acc[w][d], e0[d], e1[d]);
    }
}

template <int W, int CH, int J, int TM>
__device__ __forceinline__ void input_mac(const ApplyArgs& a, const uint8_t* lds, const StreamTile& t,
                                          const v4u (&x)[CH], uint32_t (&acc)[CH][8][W / 2])
{
    if (J < a.ncols) {  // wave-uniform
        if (a.copy_records && a.copy_off32[J] >= 0) {  // copy-through: input J also lands in its slot
#pragma unroll
            for (int c = 0; c < CH; c++)
                __builtin_amdgcn_raw_buffer_store_b128(x[c], t.rcopy, a.copy_off32[J] + t.off + c * t.cstride,
                                                       0, 2);
        }
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if constexpr (TM == 1)
                mac_chunk_nib_imm<W, J>(lds, x[c], acc[c]);
            else
                mac_chunk_imm<W, J>(lds, x[c], acc[c]);
        }
    }
}

// The next lane's 16 bytes (DPP wave_shl:1; lane 63 gets zeros -- its caller loads its own).
__device__ __forceinline__ v4u next_lane16(const v4u& v)
{
    auto shl1 = [](uint32_t x) {
        return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x130, 0xf, 0xf, false));
    };
    return v4u{shl1(v[0]), shl1(v[1]), shl1(v[2]), shl1(v[3])};
}

// Bytes [d, d + 16) of the 32-byte pair (lo, hi), d wave-uniform (a scalar branch picks the
// dword shift, v_alignbyte the byte shift).
__device__ __forceinline__ v4u realign16(const v4u& lo, const v4u& hi, int d)
{
    const uint32_t w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    v4u o;
    uint32_t n;
    switch (d >> 2) {
    case 0: o = v4u{w[0], w[1], w[2], w[3]}; n = w[4]; break;
    case 1: o = v4u{w[1], w[2], w[3], w[4]}; n = w[5]; break;
    case 2: o = v4u{w[2], w[3], w[4], w[5]}; n = w[6]; break;
    default: o = v4u{w[3], w[4], w[5], w[6]}; n = w[7]; break;
    }
    const int by = d & 3;
    if (by)
        o = v4u{__builtin_amdgcn_alignbyte(o[1], o[0], by), __builtin_amdgcn_alignbyte(o[2], o[1], by),
                __builtin_amdgcn_alignbyte(o[3], o[2], by), __builtin_amdgcn_alignbyte(n, o[3], by)};
    return o;
}

// RA (realign): inputs at offsets that are not multiples of 16 (copy-through encode straight from
// objects whose chunks start at j*bs, e.g. Swift's bs = 104858) are read as the two aligned
// 16-byte chunks under each lane's window and realigned in registers: aligned loads instead of
// unaligned ones that straddle two chunks (the launcher sends the last 16 bytes of a fragment
// down the byte-exact tail path, so the second chunk never leaves the input).
template <int W, int CH, int G, int KG, bool RA = false>
__device__ __forceinline__ void load_group(const ApplyArgs& a, const StreamTile& t, v4u (&x)[4][CH])
{
    if constexpr (RA) {
        v4u y[4][CH];
        if (a.realign_dpp) {  // one aligned load per lane; the neighbour lane holds the next chunk
            const bool last = (threadIdx.x & 63u) == 63u;  // its next chunk is the next wave's: loaded in
#pragma unroll                                              // the same burst (other lanes: out of range)
            for (int i = 0; i < 4; i++) {
                const int j = 4 * G + i;
                const int base = (j < a.ncols) ? (a.in_off32[j] & ~15) + t.off : static_cast<int>(0x80000000u);
                const bool need = last && j < a.ncols && (a.in_off32[j] & 15);
#pragma unroll
                for (int c = 0; c < CH; c++) {
                    x[i][c] = __builtin_amdgcn_raw_buffer_load_b128(t.rin, base + c * t.cstride, 0, 2);
                    y[i][c] = __builtin_amdgcn_raw_buffer_load_b128(
                        t.rin, need ? base + c * t.cstride + 16 : static_cast<int>(0x80000000u), 0, 2);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int c = 0; c < CH; c++) {
                    const v4u n = next_lane16(x[i][c]);
                    y[i][c] = last ? y[i][c] : n;
                }
        } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int j = 4 * G + i;
            const int base = (j < a.ncols) ? (a.in_off32[j] & ~15) + t.off : static_cast<int>(0x80000000u);
#pragma unroll
            for (int c = 0; c < CH; c++) {
                x[i][c] = __builtin_amdgcn_raw_buffer_load_b128(t.rin, base + c * t.cstride, 0, 2);
                y[i][c] = __builtin_amdgcn_raw_buffer_load_b128(
                    t.rin, (j < a.ncols && (a.in_off32[j] & 15)) ? base + c * t.cstride + 16
                                                                 : static_cast<int>(0x80000000u), 0, 2);
            }
        }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int j = 4 * G + i;
            const int d = j < a.ncols ? a.in_off32[j] & 15 : 0;  // wave-uniform
            if (d)
#pragma unroll
                for (int c = 0; c < CH; c++) x[i][c] = realign16(x[i][c], y[i][c], d);
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int j = 4 * G + i;
        const int base = (j < a.ncols) ? a.in_off32[j] + t.off : static_cast<int>(0x80000000u);
#pragma unroll
        for (int c = 0; c < CH; c++)
            x[i][c] = __builtin_amdgcn_raw_buffer_load_b128(t.rin, base + c * t.cstride, 0, 2);
    }
}

// Group G's lookups; with PF the loads of group G+1 are issued before them (in flight during the
// lookups), without PF after them (each wave: load, wait, look up -- latency hidden by occupancy).
template <int W, int CH, int G, int KG, bool PF, int TM, bool RA = false>
__device__ __forceinline__ void stream_group(const ApplyArgs& a, const uint8_t* lds, const StreamTile& t,
                                             v4u (&cur)[4][CH], uint32_t (&acc)[CH][8][W / 2])
{
    v4u nxt[4][CH];
    if constexpr (PF && G + 1 < KG) load_group<W, CH, G + 1, KG, RA>(a, t, nxt);
    if constexpr (TM == 2 && CH == 1) {
        // input 0's hi table via L1 (12.5% of the lookups; taking 3/16 -- input 2's hi for words
        // 0..3, or input 0's lo for words 0..3 -- measured 12% slower than none: a 40 KiB table
        // footprint no longer fits the 32 KiB L1)
        uint32_t eh0[8][W / 2], dummy[1][W / 2];
        const bool live0 = 4 * G < a.ncols;
        if (live0) {
            hyb_fetch<W, 4 * G, 1, 8>(a.tables, cur[0][0], eh0);
            if (a.copy_records && a.copy_off32[4 * G] >= 0)
                __builtin_amdgcn_raw_buffer_store_b128(cur[0][0], t.rcopy, a.copy_off32[4 * G] + t.off, 0, 2);
        }
        input_mac<W, CH, 4 * G + 1, 0>(a, lds, t, cur[1], acc);
        input_mac<W, CH, 4 * G + 2, 0>(a, lds, t, cur[2], acc);
        input_mac<W, CH, 4 * G + 3, 0>(a, lds, t, cur[3], acc);
        if (live0) mac_chunk_mixed<W, 4 * G, 0, 8>(lds, cur[0][0], dummy, eh0, acc[0]);
    } else {
        input_mac<W, CH, 4 * G + 0, TM>(a, lds, t, cur[0], acc);
        input_mac<W, CH, 4 * G + 1, TM>(a, lds, t, cur[1], acc);
        input_mac<W, CH, 4 * G + 2, TM>(a, lds, t, cur[2], acc);
        input_mac<W, CH, 4 * G + 3, TM>(a, lds, t, cur[3], acc);
    }
    if constexpr (G + 1 < KG) {
        if constexpr (!PF) load_group<W, CH, G + 1, KG, RA>(a, t, nxt);
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int c = 0; c < CH; c++) cur[i][c] = nxt[i][c];
        stream_group<W, CH, G + 1, KG, PF, TM, RA>(a, lds, t, cur, acc);
    }
}

}  // namespace

template <int W, int KG, int CH, bool PF, bool NIB, int TM, bool RA = false>
__device__ __forceinline__ void gf16_stream_body(const ApplyArgs& a)
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
    // tile_order bit 0: each workgroup walks its own contiguous range of tiles (a long sequential
    // run through each fragment), else tiles strided over the grid; bit 1: XCD-grouped block ids
    // (workgroups are dispatched round-robin over the 8 XCDs, so block b runs on XCD b % 8; the
    // remap gives each XCD a contiguous 1/8 of the logical blocks).
    uint32_t bid = blockIdx.x;
    if ((a.tile_order & 2) && gridDim.x % 8 == 0) bid = (bid % 8) * (gridDim.x / 8) + bid / 8;
    const bool ranged = a.tile_order & 1;
    const uint32_t per = (a.ntiles + gridDim.x - 1) / gridDim.x;
    const uint32_t t0 = ranged ? bid * per : bid;
    const uint32_t t1 = ranged ? min(a.ntiles, t0 + per) : a.ntiles;
    const uint32_t dt = ranged ? 1u : gridDim.x;
    for (uint32_t t = t0; t < t1; t += dt) {
        const uint32_t sl = t / a.tiles_per_stripe;
        const int64_t toff = static_cast<int64_t>(t - sl * a.tiles_per_stripe) * span;
        const uint32_t s = a.stripe_list ? static_cast<uint32_t>(a.stripe_list[sl]) : sl;
        // last, partial tile of each fragment -- and, for objects shorter than the k payloads
        // (ApplyArgs::limited), every tile reaching past the shortest input's end: the byte-exact
        // per-chunk path reads zeros there
        // (RA: also the tile holding a fragment's last 16 bytes, whose second aligned chunk would
        // reach past the input)
        if (toff + span + (RA ? 16 : 0) > a.bs || (a.limited && toff + span + (RA ? 16 : 0) > a.min_len)) {
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const int64_t o = toff + c * cstride + static_cast<int64_t>(threadIdx.x) * 16;
                const int64_t rem = a.bs - o;
                // byte-exact chunk path (load_tail / store_tail take whole chunks in one access)
                const int rc = static_cast<int>(rem < 16 ? rem : 16);
                if (rem <= 0) {
                } else if (a.copy_records) {  // copy-through launches (framed encode / decode-join)
                    apply_tile<W, false, true, NIB, true, true>(a, lds, s, o, rc);
                } else {
                    apply_tile<W, false, true, NIB, false, true>(a, lds, s, o, rc);
                }
            }
            continue;
        }
        const int off = static_cast<int>(toff) + static_cast<int>(threadIdx.x) * 16;
        StreamTile tile;
        tile.rin = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.in_base) + static_cast<int64_t>(s) * a.in_stride, 0,
            static_cast<int>(a.in_records), 0x00020000);
        tile.rcopy = __builtin_amdgcn_make_buffer_rsrc(
            a.copy_base + static_cast<int64_t>(s) * a.copy_stride, 0, static_cast<int>(a.copy_records),
            0x00020000);
        tile.off = off;
        tile.cstride = cstride;
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
        load_group<W, CH, 0, KG, RA>(a, tile, cur);
        stream_group<W, CH, 0, KG, PF, TM, RA>(a, lds, tile, cur, acc);

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


template <int W, int KG, int CH, bool PF, bool NIB>
__global__ void __launch_bounds__(1024) gf16_stream_kernel(const ApplyArgs a)
{
    gf16_stream_body<W, KG, CH, PF, NIB, NIB ? 1 : 0>(a);
}

// Copy-through passes whose inputs start at offsets that are not multiples of 16 (RA above).
template <int W, int KG>
__global__ void __launch_bounds__(1024) gf16_realign_kernel(const ApplyArgs a)
{
    gf16_stream_body<W, KG, 1, false, false, 0, true>(a);
}

// 8-output passes with the hybrid LDS + L1 lookups (TM = 2), e.g. C5's 20 -> 8.
template <int KG>
__global__ void __launch_bounds__(1024) gf16_hybrid_kernel(const ApplyArgs a)
{
    gf16_stream_body<8, KG, 1, false, false, 2>(a);
}

// One group of 4 inputs of gf16_ptrs_stream_kernel: a buffer resource per fragment, loads
// unconditional (out-of-range offset past ncols), lookups at compile-time table offsets.
template <int W, int G, int KG>
__device__ __forceinline__ void ptrs_group(const ApplyArgs& a, const uint8_t* lds,
                                           const uint8_t* const (&ptr)[4 * KG], int off,
                                           uint32_t (&acc)[8][W / 2])
{
    v4u x[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int j = 4 * G + i;
        const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(ptr[j]), 0,
                                                         static_cast<int>(a.bs), 0x00020000);
        x[i] = __builtin_amdgcn_raw_buffer_load_b128(r, j < a.ncols ? off : static_cast<int>(0x80000000u), 0, 2);
    }
    if (4 * G + 0 < a.ncols) mac_chunk_imm<W, 4 * G + 0>(lds, x[0], acc);
    if (4 * G + 1 < a.ncols) mac_chunk_imm<W, 4 * G + 1>(lds, x[1], acc);
    if (4 * G + 2 < a.ncols) mac_chunk_imm<W, 4 * G + 2>(lds, x[2], acc);
    if (4 * G + 3 < a.ncols) mac_chunk_imm<W, 4 * G + 3>(lds, x[3], acc);
    if constexpr (G + 1 < KG) ptrs_group<W, G + 1, KG>(a, lds, ptr, off, acc);
}

// gf16_ptrs_stream_kernel<W, KG>: the pointer-table form (ecamd_map_apply_ptrs, heterogeneous
// decode batches): input j of stripe s is the fragment at in_ptrs[s*in_stride + in_off[j]], so
// every fragment gets its own buffer resource (base from a scalar load of the table, range = the
// fragment) and the same unconditional, unrolled loads / compile-time table offsets as above.
template <int W, int KG>
__global__ void __launch_bounds__(1024) gf16_ptrs_stream_kernel(const ApplyArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    const int tbytes = a.ncols * 512 * EB;
    for (int o = threadIdx.x * 16; o < tbytes; o += blockDim.x * 16)
        *reinterpret_cast<uint4*>(lds + o) = *reinterpret_cast<const uint4*>(a.tables + o);
    __syncthreads();

    const int span = static_cast<int>(blockDim.x) * 16;
    for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const uint32_t s = t / a.tiles_per_stripe;
        const int64_t toff = static_cast<int64_t>(t - s * a.tiles_per_stripe) * span;
        const int64_t o64 = toff + static_cast<int64_t>(threadIdx.x) * 16;
        // last, partial tile of each fragment -- and, for objects shorter than the k payloads
        // (ApplyArgs::limited), every tile reaching past the shortest input's end: the byte-exact
        // per-chunk path reads zeros there
        if (toff + span > a.bs || (a.limited && toff + span > a.min_len)) {
            const int64_t rem = a.bs - o64;
            if (rem >= 16)
                apply_tile<W, true, true, false, false, false>(a, lds, s, o64, 16);
            else if (rem > 0)
                apply_tile<W, true, true, false, false, true>(a, lds, s, o64, static_cast<int>(rem));
            continue;
        }
        const int off = static_cast<int>(o64);
        // every fragment pointer of the stripe up front: one burst of scalar loads, one wait
        const uint8_t* const* inp = a.in_ptrs + static_cast<int64_t>(s) * a.in_stride;
        uint8_t* const* outp = a.out_ptrs + static_cast<int64_t>(s) * a.out_stride;
        const uint8_t* ptr[4 * KG];
#pragma unroll
        for (int j = 0; j < 4 * KG; j++) ptr[j] = inp[a.in_off[j < a.ncols ? j : 0]];
        uint8_t* optr[W];
#pragma unroll
        for (int r = 0; r < W; r++) optr[r] = outp[a.out_off[r < a.nrows ? r : 0]];
        uint32_t acc[8][D];
#pragma unroll
        for (int w = 0; w < 8; w++)
#pragma unroll
            for (int d = 0; d < D; d++) acc[w][d] = 0u;
        ptrs_group<W, 0, KG>(a, lds, ptr, off, acc);
#pragma unroll
        for (int r = 0; r < W; r++) {
            if (r >= a.nrows) break;
            v4u v;
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t A = acc[2 * d][r >> 1], B = acc[2 * d + 1][r >> 1];
                v[d] = (r & 1) ? ((A >> 16) | (B & 0xffff0000u)) : ((A & 0xffffu) | (B << 16));
            }
            const auto ro = __builtin_amdgcn_make_buffer_rsrc(optr[r], 0, static_cast<int>(a.bs), 0x00020000);
            if (a.accumulate) v ^= __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 2);  // nt
        }
    }
}

}  // namespace ecamd

#define ECAMD_STREAM_INST(W, KG, CH, PF, NIB) \
    template __global__ void ecamd::gf16_stream_kernel<W, KG, CH, PF, NIB>(const ecamd::ApplyArgs);
#define ECAMD_HYBRID_KG \
    template __global__ void ecamd::gf16_hybrid_kernel<1>(const ecamd::ApplyArgs); \
    template __global__ void ecamd::gf16_hybrid_kernel<2>(const ecamd::ApplyArgs); \
    template __global__ void ecamd::gf16_hybrid_kernel<3>(const ecamd::ApplyArgs); \
    template __global__ void ecamd::gf16_hybrid_kernel<4>(const ecamd::ApplyArgs); \
    template __global__ void ecamd::gf16_hybrid_kernel<5>(const ecamd::ApplyArgs);
#define ECAMD_REALIGN_KG(W)                                                               \
    template __global__ void ecamd::gf16_realign_kernel<W, 1>(const ecamd::ApplyArgs);    \
    template __global__ void ecamd::gf16_realign_kernel<W, 2>(const ecamd::ApplyArgs);    \
    template __global__ void ecamd::gf16_realign_kernel<W, 3>(const ecamd::ApplyArgs);    \
    template __global__ void ecamd::gf16_realign_kernel<W, 4>(const ecamd::ApplyArgs);    \
    template __global__ void ecamd::gf16_realign_kernel<W, 5>(const ecamd::ApplyArgs);
#define ECAMD_PTRS_KG(W)                                                                  \
    template __global__ void ecamd::gf16_ptrs_stream_kernel<W, 1>(const ecamd::ApplyArgs);      \
    template __global__ void ecamd::gf16_ptrs_stream_kernel<W, 2>(const ecamd::ApplyArgs);      \
    template __global__ void ecamd::gf16_ptrs_stream_kernel<W, 3>(const ecamd::ApplyArgs);      \
    template __global__ void ecamd::gf16_ptrs_stream_kernel<W, 4>(const ecamd::ApplyArgs);      \
    template __global__ void ecamd::gf16_ptrs_stream_kernel<W, 5>(const ecamd::ApplyArgs);
#define ECAMD_STREAM_KG(W, CH, PF, NIB)                                                   \
    ECAMD_STREAM_INST(W, 1, CH, PF, NIB) ECAMD_STREAM_INST(W, 2, CH, PF, NIB)             \
    ECAMD_STREAM_INST(W, 3, CH, PF, NIB) ECAMD_STREAM_INST(W, 4, CH, PF, NIB)             \
    ECAMD_STREAM_INST(W, 5, CH, PF, NIB)
