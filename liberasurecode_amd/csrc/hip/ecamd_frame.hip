// ecamd_frame.hip -- on-device fragment framing for the device-resident path:
// the 80-byte fragment headers and the zlib-compatible payload / metadata CRC32 of the reference
// (src/erasurecode_postprocessing.c:37-93, src/erasurecode_helpers.c:463-496; wire format
// include/erasurecode.h fragment_header_t), plus the object <-> payload copies of
// prepare_fragments_for_encode (src/erasurecode_preprocessing.c:36-108) and fragments_to_string
// (:269-370).
//
// CRC32 of a payload (host/crc.hpp has the algebra) runs in two kernels:
//   crc_partial_kernel<B>  one wave per "span" of J KiB of one payload.  Lane l owns the 16-byte
//     pieces l, l+64, l+128, ... of the span (so every wave load is a coalesced 1 KiB), and keeps
//     state s = A^1024 s ^ r0(piece): r0(piece) is 128/B lookups of B-bit fields in LDS tables and
//     A^1024 (the 1008-byte gap to the lane's next piece, plus the piece) 32/B lookups.  A 6-level
//     shuffle butterfly (A^(16*2^t) tables) folds the 64 lane states into r0(span).  Spans are
//     aligned to the END of the payload's 16-byte body, so the first one is padded with leading
//     zeros, which do not change r0.
//   crc_finalize_kernel    one thread per payload: Horner over its spans with A^(J KiB), the last
//     len % 16 bytes through the byte table, crc = ~(A^len ~0 ^ r0), and -- when asked -- the
//     whole 80-byte header with its metadata checksum.
// Piece tables per dword: byte tables (4 KiB, random lookups conflict in the LDS banks) or nibble
// tables (16 entries span 16 distinct banks, so lookups never conflict, at twice the lookups and
// VALU work); crc_partial_kernel<MB, G> takes byte tables for the first MB dwords of a piece.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ecamd_crc_dev.hpp"
#include "ecamd_frame.hpp"
#include "ecamd_isa.hpp"

namespace ecamd {

using crcdev::lmap;
using crcdev::piece_r0;
using crcdev::piece_words;

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 nt_load16(const uint8_t* p)
{
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

__device__ __forceinline__ uint32_t byte_step(const uint32_t* T, uint32_t s, uint32_t b, int legacy)
{
    uint32_t sh = s >> 8;
    if (legacy && (s & 0x80000000u)) sh |= 0xff000000u;
    return T[(s ^ b) & 0xffu] ^ sh;
}

__device__ __forceinline__ const uint8_t* item_ptr(const CrcArgs& a, int64_t item)
{
    const int64_t s = item / a.nfrag;
    const int f = static_cast<int>(item - s * a.nfrag);
    return a.base + s * a.stripe_stride + f * a.frag_stride;
}

}  // namespace

// lane l takes lane l + N of its row of 16 (DPP row_shl; past the row's end: 0)
template <int N>
__device__ __forceinline__ uint32_t row_shl(uint32_t x)
{
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x100 + N, 0xf, 0xf, false));
}

template <int MB, int G, bool POS>
__global__ __launch_bounds__(512) void crc_partial_kernel(const CrcArgs a, const uint32_t* __restrict__ img,
                                                          uint32_t* __restrict__ partial)
{
    // POS: position tables -- piece u of a group of 4 has its own tables with the shift to the
    // group's last piece (A^(1024*(3-u))) folded in, so the lane state takes one A^4096 step per
    // 4 pieces instead of four A^1024 steps (a quarter of the serial lookup chain).
    constexpr int PW = piece_words(MB), PIECE = POS ? 4 * PW : PW;
    constexpr int FIELDS = (32 / G) << G, WORDS = PIECE + 7 * FIELDS;
    __shared__ uint32_t tab[WORDS];
    for (int i = threadIdx.x; i < WORDS; i += blockDim.x) tab[i] = img[i];
    __syncthreads();
    const uint32_t* gap = tab + PIECE;
    const int lane = threadIdx.x & 63;
    const int nw = blockDim.x >> 6;
    const int64_t total = static_cast<int64_t>(a.items) * a.nspans;
    const int64_t span = static_cast<int64_t>(a.J) * 1024;
    for (int64_t ws = static_cast<int64_t>(blockIdx.x) * nw + (threadIdx.x >> 6); ws < total;
         ws += static_cast<int64_t>(gridDim.x) * nw) {
        const int64_t item = ws / a.nspans;
        const int q = static_cast<int>(ws - item * a.nspans);
        const uint8_t* p = item_ptr(a, item) + a.payload_off;
        const int64_t start = a.body - static_cast<int64_t>(a.nspans - q) * span + lane * 16;
        uint32_t st = 0;
        // Two groups of 4 pieces in flight: group g+1 is loading while group g is looked up.  The
        // loads are unconditional buffer loads: a piece before the payload (the first span's
        // leading zeros) or past the span gets an out-of-range offset, which reads zeros with no
        // memory traffic, so the compiler can count the loads in flight (vmcnt(N), not vmcnt(0)).
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0,
                                                          static_cast<int>(a.body), 0x00020000);
        auto load4 = [&](int j, u32x4 (&v)[4]) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t off = start + static_cast<int64_t>(j + u) * 1024;
                const bool live = j + u < a.J && off >= 0;
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, live ? static_cast<int>(off)
                                                                      : static_cast<int>(0x80000000u),
                                                             0, 2);
            }
        };
        u32x4 cur[4], nxt[4];
        load4(0, cur);
        for (int j = 0; j < a.J; j += 4) {
            load4(j + 4, nxt);
            if constexpr (POS) {
                st = xor3(lmap<G>(gap, st), piece_r0<MB>(tab, cur[0]), piece_r0<MB>(tab + PW, cur[1])) ^
                     piece_r0<MB>(tab + 2 * PW, cur[2]) ^ piece_r0<MB>(tab + 3 * PW, cur[3]);
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) st = lmap<G>(gap, st) ^ piece_r0<MB>(tab, cur[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
        }
        // Lane l's state sits (63 - l) pieces before the span end: fold pairs, quads, ... -- inside
        // each row of 16 lanes by DPP row_shl (lane l takes lane l + 2^t; only the lanes that are
        // multiples of 2^(t+1) matter), then the 4 row values by v_readlane, folded on uniform values
        // (no ds_bpermute: the LDS serves the lookups; broadcast lookups do not conflict)
        st = lmap<G>(tab + PIECE + FIELDS * 1, st) ^ row_shl<1>(st);
        st = lmap<G>(tab + PIECE + FIELDS * 2, st) ^ row_shl<2>(st);
        st = lmap<G>(tab + PIECE + FIELDS * 3, st) ^ row_shl<4>(st);
        st = lmap<G>(tab + PIECE + FIELDS * 4, st) ^ row_shl<8>(st);
        const uint32_t r0 = __builtin_amdgcn_readlane(st, 0), r1 = __builtin_amdgcn_readlane(st, 16);
        const uint32_t r2 = __builtin_amdgcn_readlane(st, 32), r3 = __builtin_amdgcn_readlane(st, 48);
        const uint32_t s0 = lmap<G>(tab + PIECE + FIELDS * 5, r0) ^ r1, s1 = lmap<G>(tab + PIECE + FIELDS * 5, r2) ^ r3;
        st = lmap<G>(tab + PIECE + FIELDS * 6, s0) ^ s1;
        if (lane == 0) partial[ws] = st;
    }
}

#define ECAMD_CRC_INST(MB, G, POS) \
    template __global__ void crc_partial_kernel<MB, G, POS>(const CrcArgs, const uint32_t* __restrict__, \
                                                            uint32_t* __restrict__);
ECAMD_CRC_INST(4, 8, false) ECAMD_CRC_INST(0, 8, false) ECAMD_CRC_INST(0, 4, false)
ECAMD_CRC_INST(1, 8, false) ECAMD_CRC_INST(2, 8, false) ECAMD_CRC_INST(3, 8, false)
ECAMD_CRC_INST(4, 8, true) ECAMD_CRC_INST(0, 8, true) ECAMD_CRC_INST(1, 8, true)
ECAMD_CRC_INST(2, 8, true) ECAMD_CRC_INST(3, 8, true)
#undef ECAMD_CRC_INST

namespace {

template <int N>
__device__ __forceinline__ void put(uint8_t* h, int off, uint64_t v)
{
#pragma unroll
    for (int i = 0; i < N; ++i) h[off + i] = static_cast<uint8_t>(v >> (8 * i));
}

template <int N>
__device__ __forceinline__ uint32_t get(const uint8_t* h, int off)
{
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) v |= static_cast<uint32_t>(h[off + i]) << (8 * i);
    return v;
}

__device__ __forceinline__ uint32_t meta_crc(const uint32_t* T, const uint8_t* h, int legacy)
{
    uint32_t s = ~0u;
#pragma unroll
    for (int i = 0; i < kMetaBytes; ++i) s = byte_step(T, s, h[i], legacy);
    return ~s;
}

}  // namespace

__global__ void crc_finalize_kernel(const CrcArgs a, const uint32_t* __restrict__ img,
                                    const uint32_t* __restrict__ partial, uint32_t* __restrict__ crc_out,
                                    const HeaderArgs h)
{
    const int64_t item = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (item >= a.items) return;
    const uint32_t* span = img + a.span_off;
    const uint32_t* T = img + a.t_off;
    const uint8_t* frag = item_ptr(a, item);
    uint32_t crc = 0;
    if (a.nspans > 0) {
        uint32_t acc = 0;
        const uint32_t* pp = partial + item * a.nspans;
        for (int q = 0; q < a.nspans; ++q) {
            acc = span[acc & 0xff] ^ span[256 + ((acc >> 8) & 0xff)] ^
                  span[512 + ((acc >> 16) & 0xff)] ^ span[768 + (acc >> 24)] ^ pp[q];
        }
        const uint8_t* p = frag + a.payload_off;
        for (int64_t i = a.body; i < a.len; ++i) acc = byte_step(T, acc, p[i], a.legacy);
        if (a.tail_crc) {
            uint32_t sh = 0;
#pragma unroll
            for (int b = 0; b < 32; ++b) sh ^= (acc >> b & 1u) ? a.tail_cols[b] : 0u;
            acc = sh ^ ~a.tail_crc[item] ^ a.tail_c0;
        }
        crc = ~(a.c0 ^ acc);
        if (crc_out) crc_out[item] = crc;
    }
    if (!h.write) return;
    // add_fragment_metadata (src/erasurecode_postprocessing.c:37-69) on a zeroed header
    // (alloc_fragment_buffer, src/erasurecode_helpers.c:124-138).
    uint8_t hd[kHeaderBytes];
#pragma unroll
    for (int i = 0; i < kHeaderBytes; ++i) hd[i] = 0;
    const int f = static_cast<int>(item % a.nfrag);
    put<4>(hd, 0, static_cast<uint32_t>(h.idx0 + f));
    put<4>(hd, 4, h.size);
    put<4>(hd, 8, h.backend_meta_size);
    put<8>(hd, 12, h.orig_data_size);
    put<1>(hd, 20, h.chksum_type);
    if (h.chksum_type == kChksumCrc32) put<4>(hd, 21, crc);
    put<1>(hd, 54, h.backend_id);
    put<4>(hd, 55, h.backend_version);
    put<4>(hd, 59, kFragMagic);
    put<4>(hd, 63, h.libec_version);
    put<4>(hd, 67, meta_crc(T, hd, a.legacy));
    uint8_t* out = const_cast<uint8_t*>(frag);
#pragma unroll
    for (int c = 0; c < kHeaderBytes / 16; ++c) {
        uint4 v = make_uint4(get<4>(hd, 16 * c), get<4>(hd, 16 * c + 4), get<4>(hd, 16 * c + 8),
                             get<4>(hd, 16 * c + 12));
        *reinterpret_cast<uint4*>(out + 16 * c) = v;
    }
}

__global__ void crc_combine_kernel(const uint32_t* __restrict__ tiles, uint32_t* __restrict__ out,
                                   const uint32_t* __restrict__ span, int64_t items, int nf, int tps, int g)
{
    const int q = tps / g;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;  // item * q + r
    if (i >= items * q) return;
    const int64_t item = i / q;
    const int r = static_cast<int>(i - item * q);
    const int64_t s = item / nf;
    const int f = static_cast<int>(item - s * nf);
    const uint32_t* p = tiles + (s * tps + static_cast<int64_t>(r) * g) * nf + f;
    uint32_t acc = 0;
    for (int t = 0; t < g; ++t)
        acc = span[acc & 0xff] ^ span[256 + ((acc >> 8) & 0xff)] ^ span[512 + ((acc >> 16) & 0xff)] ^
              span[768 + (acc >> 24)] ^ p[static_cast<int64_t>(t) * nf];
    out[i] = acc;
}

// prepare_fragments_for_encode: data payload j of stripe s = object bytes [j*bs, (j+1)*bs), zero
// padded past the object's end (and through the 16-byte slack after the payload).
__global__ void frame_split_kernel(const SplitArgs a)
{
    const int64_t per_frag = (a.bs + 15) / 16;
    const int64_t total = per_frag * a.k * a.nstripes;
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < total;
         t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t sj = t / per_frag;
        const int64_t c = t - sj * per_frag;
        const int64_t s = sj / a.k;
        const int j = static_cast<int>(sj - s * a.k);
        const int64_t src_off = j * a.bs + c * 16;
        int64_t n = a.size - src_off;
        n = n < 0 ? 0 : n;
        n = n > a.bs - c * 16 ? a.bs - c * 16 : n;
        const uint8_t* src = a.obj + s * a.obj_stride + src_off;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (n >= 16 && a.aligned) {
            u32x4 w = nt_load16(src);
            v = make_uint4(w.x, w.y, w.z, w.w);
        } else if (n > 0) {
            uint32_t w[4] = {0, 0, 0, 0};
            for (int i = 0; i < (n < 16 ? n : 16); ++i) w[i >> 2] |= static_cast<uint32_t>(src[i]) << (8 * (i & 3));
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        uint8_t* dst = a.frags + s * a.stripe_stride + j * a.frag_stride + kHeaderBytes + c * 16;
        u32x4 o = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(dst));
    }
}

// Streaming forms of the two copies for objects / stripes whose offsets fit 32 bits: a tile is
// kCopyU x blockDim lanes x 16 B of one data fragment of one stripe (t -> stripe, fragment, tile: 32-bit
// index math once per tile), loads and stores are buffer ops on one resource per stripe with
// 32-bit offsets, and the unaligned side of the copy (object offset j*bs when bs % 16 != 0) takes
// unaligned 16-byte buffer accesses -- as the copy-through codec launch does -- instead of bytes.
// Only the chunk that straddles two payloads or the object's end goes byte by byte.
// kCopyU (template parameter of the two kernels below): chunks per lane and tile, 4 or 1.

__device__ __forceinline__ u32x4 window16(const u32x4& lo, const u32x4& hi, int dw, int by);

// prepare_fragments_for_encode, streaming: chunk c of payload j = object bytes [j*bs + 16c, +16),
// realigned in registers from the two aligned object chunks under it when j*bs % 16 != 0 (aligned
// loads and stores on both sides); the payload's last chunk, anything reaching past the object's
// end (zero padded) and a window whose second chunk would reach past the object go byte by byte.
// The next lane's 16 bytes (lane 63: whatever `own` is; the caller loads that lane's itself): a
// wave's consecutive lanes hold consecutive aligned chunks, so the second chunk under a realigned
// window is the neighbour's first -- one load per lane instead of two (DPP wave_shl:1, VALU only).
static __device__ __forceinline__ u32x4 next_lane16(const u32x4& v)
{
    auto shl1 = [](uint32_t x) {
        return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x130, 0xf, 0xf, false));
    };
    return u32x4{shl1(v.x), shl1(v.y), shl1(v.z), shl1(v.w)};
}

// the low n bytes of x (n <= 0: none, n >= 4: all)
__device__ __forceinline__ uint32_t keep_bytes(uint32_t x, int n)
{
    return n >= 4 ? x : n <= 0 ? 0u : x & ((1u << (8 * n)) - 1u);
}

// kDpp (knob frame_copy_dpp): the realigning path takes each lane's second aligned chunk from its
// neighbour lane (next_lane16) and only the last lane of a wave loads its own.
template <int kCopyU, bool kDpp>
__global__ void __launch_bounds__(256) frame_split_stream_kernel(const SplitArgs a)
{
    const uint32_t T = blockDim.x;  // lanes per tile (64 / 128 / 256)
    const uint32_t per_frag = static_cast<uint32_t>((a.bs + 15) / 16);  // payload chunks
    const uint32_t cfrom = static_cast<uint32_t>(a.from >> 4);           // first chunk copied
    const uint32_t tpf = (per_frag - cfrom + T * kCopyU - 1) / (T * kCopyU);
    const uint32_t ntiles = tpf * static_cast<uint32_t>(a.k) * static_cast<uint32_t>(a.nstripes);
    const int bs = static_cast<int>(a.bs);
    const int size = static_cast<int>(a.size);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t sj = t / tpf;
        const uint32_t tc = t - sj * tpf;
        const uint32_t s = sj / static_cast<uint32_t>(a.k);
        const int j = static_cast<int>(sj - s * static_cast<uint32_t>(a.k));
        const int lo = j * bs;
        const int delta = lo & 15, dw = delta >> 2, by = delta & 3;
        const auto robj = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.obj) + static_cast<int64_t>(s) * a.obj_stride, 0, size, 0x00020000);
        uint8_t* pay = a.frags + static_cast<int64_t>(s) * a.stripe_stride + j * a.frag_stride + kHeaderBytes;
        const auto rpay = __builtin_amdgcn_make_buffer_rsrc(pay, 0, static_cast<int>(per_frag * 16), 0x00020000);
        u32x4 v0[kCopyU], v1[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const int c = static_cast<int>(cfrom + (tc * kCopyU + u) * T + threadIdx.x);
            const int src = lo + c * 16;
            const int q = src >> 4;
            // the window lies inside the object (the payload's last, partial chunk included)
            const bool fast = src + 16 <= size && (delta == 0 || (q << 4) + 32 <= size);
            if (kDpp && delta) {  // every lane's aligned chunk (past the object: zeros), the neighbour's next;
                // the wave's last lane loads its own second chunk in the same burst (the other lanes'
                // offsets are out of range: no memory access)
                v0[u] = __builtin_amdgcn_raw_buffer_load_b128(robj, q << 4, 0, 2);
                v1[u] = __builtin_amdgcn_raw_buffer_load_b128(
                    robj, (threadIdx.x & 63u) == 63u ? (q << 4) + 16 : static_cast<int>(0x80000000u), 0, 2);
            } else {
                v0[u] = __builtin_amdgcn_raw_buffer_load_b128(robj, fast ? q << 4 : static_cast<int>(0x80000000u), 0, 2);
                v1[u] = __builtin_amdgcn_raw_buffer_load_b128(
                    robj, fast && delta ? (q << 4) + 16 : static_cast<int>(0x80000000u), 0, 2);
            }
        }
        if (kDpp && delta) {
            const bool last = (threadIdx.x & 63u) == 63u;
#pragma unroll
            for (int u = 0; u < kCopyU; ++u) {
                const u32x4 n = next_lane16(v0[u]);
                v1[u] = last ? v1[u] : n;
            }
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const int c = static_cast<int>(cfrom + (tc * kCopyU + u) * T + threadIdx.x);
            if (c >= static_cast<int>(per_frag)) continue;
            const int src = lo + c * 16;
            const int q = src >> 4;
            u32x4 v;
            const bool in_obj = src + 16 <= size && (delta == 0 || (q << 4) + 32 <= size);
            if (c * 16 + 16 <= bs && in_obj) {
                v = delta ? window16(v0[u], v1[u], dw, by) : v0[u];
            } else if (in_obj) {  // the payload's last, partial chunk inside the object:
                // its window masked to the payload's bs - 16c bytes (the rest is zero padding)
                v = delta ? window16(v0[u], v1[u], dw, by) : v0[u];
                const int n = bs - c * 16;
                v = u32x4{keep_bytes(v.x, n), keep_bytes(v.y, n - 4), keep_bytes(v.z, n - 8), keep_bytes(v.w, n - 12)};
            } else {  // ragged end: bytes, zero padded
                int n = size - src;
                n = n < 0 ? 0 : n;
                n = n > bs - c * 16 ? bs - c * 16 : n;
                const uint8_t* p = a.obj + static_cast<int64_t>(s) * a.obj_stride + src;
                uint32_t w[4] = {0, 0, 0, 0};
                for (int i = 0; i < (n < 16 ? n : 16); ++i) w[i >> 2] |= static_cast<uint32_t>(p[i]) << (8 * (i & 3));
                v = u32x4{w[0], w[1], w[2], w[3]};
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, rpay, c * 16, 0, 2);
        }
    }
}
template __global__ void frame_split_stream_kernel<1, false>(const SplitArgs);
template __global__ void frame_split_stream_kernel<4, false>(const SplitArgs);
template __global__ void frame_split_stream_kernel<1, true>(const SplitArgs);
template __global__ void frame_split_stream_kernel<4, true>(const SplitArgs);

// Bytes [d, d + 16) of the 32-byte pair (lo, hi), d = 4 * dw + by wave-uniform: v_alignbyte on
// the dword pairs (realigns an unaligned 16-byte window from two aligned loads).
__device__ __forceinline__ u32x4 window16(const u32x4& lo, const u32x4& hi, int dw, int by)
{
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    u32x4 o;
    switch (dw) {  // wave-uniform
    case 0: o = u32x4{w[0], w[1], w[2], w[3]}; break;
    case 1: o = u32x4{w[1], w[2], w[3], w[4]}; break;
    case 2: o = u32x4{w[2], w[3], w[4], w[5]}; break;
    default: o = u32x4{w[3], w[4], w[5], w[6]}; break;
    }
    if (by) {
        const uint32_t n = dw == 0 ? w[4] : dw == 1 ? w[5] : dw == 2 ? w[6] : w[7];
        o = u32x4{__builtin_amdgcn_alignbyte(o.y, o.x, by), __builtin_amdgcn_alignbyte(o.z, o.y, by),
                  __builtin_amdgcn_alignbyte(o.w, o.z, by), __builtin_amdgcn_alignbyte(n, o.w, by)};
    }
    return o;
}

// fragments_to_string, streaming: payload j fills object bytes [lo, hi) = [j*bs, min((j+1)*bs,
// size)).  Every aligned 16-byte object chunk has ONE owner: payload j writes chunks
// [floor(lo/16), e) with e = floor(hi/16) below the object's end (a chunk straddling payloads j and
// j+1 belongs to j+1) and ceil(size/16) for the last payload.  A chunk wholly inside [lo, hi) is an
// aligned store of payload bytes [p, p + 16) (p = 16ch - lo), realigned in registers from the two
// aligned payload chunks under it when bs % 16 != 0 (Swift's 1 MiB segments at k = 10: bs = 104858);
// the payload rows are read up to their 16-byte-rounded length, which the fragment layout reserves.
// The straddling chunk is an ordinary lane too (round 4): its first load fetches the last 16 bytes
// of payload j-1 (one unaligned load, same instruction as every lane's -- the loads address the
// whole stripe) and its second the first chunk of payload j, so the same realignment merges them,
// with no dependent loads after the burst.  Only the object's final partial chunk goes byte by byte,
// so nothing is written outside [0, size).  Needs bs >= 32 (the host falls back to frame_join_kernel).
// tile_align (knob frame_join_align): a payload's tiles start at object chunks that are multiples of
// the tile (T x kCopyU chunks), so every workgroup's stores cover whole aligned object lines; the
// lanes before the payload's first chunk idle.
template <int kCopyU, bool kDpp>
__global__ void __launch_bounds__(256) frame_join_stream_kernel(const JoinArgs a, int k, int tile_align)
{
    const uint32_t T = blockDim.x;  // lanes per tile (64 / 128 / 256)
    const int bs = static_cast<int>(a.bs);
    const int bs16 = (bs + 15) & ~15;
    const int size = static_cast<int>(a.size);
    const int fs = static_cast<int>(a.frag_stride);
    const uint32_t per_frag = static_cast<uint32_t>(bs / 16 + 2 + (tile_align ? T * kCopyU - 1 : 0));
    const uint32_t tpf = (per_frag + T * kCopyU - 1) / (T * kCopyU);
    const uint32_t ntiles = tpf * static_cast<uint32_t>(k) * static_cast<uint32_t>(a.nstripes);
    constexpr int kOut = static_cast<int>(0x80000000u);  // out of range: no memory access, zeros
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t sj = t / tpf;
        const uint32_t tc = t - sj * tpf;
        const uint32_t s = sj / static_cast<uint32_t>(k);
        const int j = static_cast<int>(sj - s * static_cast<uint32_t>(k));
        const int lo = j * bs;
        const int hi = lo + bs < size ? lo + bs : size;
        if (hi <= lo) continue;  // payload past the object's end (wave-uniform)
        const int c0 = lo >> 4, c1 = hi < size ? hi >> 4 : (size + 15) >> 4;
        const int cb = tile_align ? c0 & ~static_cast<int>(T * kCopyU - 1) : c0;  // the tiles' first chunk
        if (cb + static_cast<int>(tc * kCopyU * T) >= c1) continue;  // an aligned payload's spare last tile
        const int delta = (16 - (lo & 15)) & 15;  // p mod 16 for every chunk of this payload
        const int dw = delta >> 2, by = delta & 3;
        const uint8_t* stripe = a.frags + static_cast<int64_t>(s) * a.stripe_stride;
        const uint8_t* pay = stripe + j * fs + kHeaderBytes;
        const int pay_off = j * fs + kHeaderBytes;  // payload j in the stripe (32-bit: copy_fits32)
        const auto rstr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(stripe), 0,
                                                            (k - 1) * fs + kHeaderBytes + bs16, 0x00020000);
        uint8_t* ob = a.obj + static_cast<int64_t>(s) * a.obj_stride;
        const auto robj = __builtin_amdgcn_make_buffer_rsrc(ob, 0, size, 0x00020000);
        u32x4 v0[kCopyU], v1[kCopyU];
        bool strad[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const int ch = cb + static_cast<int>((tc * kCopyU + u) * T + threadIdx.x);
            const int q = ((ch << 4) - lo) >> 4;  // aligned payload chunk under the window's start
            // the chunk payloads j-1 and j share: its window is (last 16 bytes of j-1 || chunk 0 of j)
            strad[u] = delta && j > 0 && ch == c0 && (c0 << 4) + 16 <= hi;
            const bool fast = ((ch << 4) >= lo || strad[u]) && (ch << 4) + 16 <= hi;
            const int first = strad[u] ? pay_off - fs + bs - 16 : pay_off + (q << 4);
            if (kDpp && delta) {  // every lane's aligned chunk (before the payload row: zeros); the
                // wave's last lane loads its own second chunk in the same burst
                v0[u] = __builtin_amdgcn_raw_buffer_load_b128(rstr, q >= 0 || strad[u] ? first : kOut, 0, 2);
                v1[u] = __builtin_amdgcn_raw_buffer_load_b128(
                    rstr, (threadIdx.x & 63u) == 63u && q >= -1 ? pay_off + (q << 4) + 16 : kOut, 0, 2);
            } else {
                v0[u] = __builtin_amdgcn_raw_buffer_load_b128(rstr, fast ? first : kOut, 0, 2);
                v1[u] = __builtin_amdgcn_raw_buffer_load_b128(rstr, fast && delta ? pay_off + (q << 4) + 16 : kOut, 0,
                                                              2);
            }
        }
        if (kDpp && delta) {
            const bool last = (threadIdx.x & 63u) == 63u;
#pragma unroll
            for (int u = 0; u < kCopyU; ++u) {
                const u32x4 n = next_lane16(v0[u]);
                v1[u] = last ? v1[u] : n;
            }
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const int ch = cb + static_cast<int>((tc * kCopyU + u) * T + threadIdx.x);
            if (ch >= c1 || ch < c0) continue;  // (before c0: the idle lanes of an aligned first tile)
            const int A = ch << 4;
            if ((A >= lo || strad[u]) && A + 16 <= hi) {
                __builtin_amdgcn_raw_buffer_store_b128(delta ? window16(v0[u], v1[u], dw, by) : v0[u], robj, A, 0, 2);
                continue;
            }
            if (A < lo && A + 16 <= hi) continue;  // (not reached: the straddling chunk is stored above)
            // the object's final partial chunk (bytes before lo, if any, from payload j-1)
            const int b1 = A + 16 < hi ? A + 16 : hi;
            for (int b = A; b < b1; ++b) ob[b] = b < lo ? pay[b - lo - a.frag_stride + bs] : pay[b - lo];
        }
    }
}
template __global__ void frame_join_stream_kernel<1, false>(const JoinArgs, int, int);
template __global__ void frame_join_stream_kernel<4, false>(const JoinArgs, int, int);
template __global__ void frame_join_stream_kernel<1, true>(const JoinArgs, int, int);
template __global__ void frame_join_stream_kernel<4, true>(const JoinArgs, int, int);

// fragments_to_string: object bytes [0, size) = data payloads 0..k-1 concatenated.
__global__ void frame_join_kernel(const JoinArgs a)
{
    const int64_t per_obj = (a.size + 15) / 16;
    const int64_t total = per_obj * a.nstripes;
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < total;
         t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t s = t / per_obj;
        const int64_t o = (t - s * per_obj) * 16;
        const uint8_t* fr = a.frags + s * a.stripe_stride + kHeaderBytes;
        uint8_t* dst = a.obj + s * a.obj_stride + o;
        const int64_t n = a.size - o < 16 ? a.size - o : 16;
        if (n == 16 && a.aligned) {
            const int64_t j = o / a.bs;
            u32x4 w = nt_load16(fr + j * a.frag_stride + (o - j * a.bs));
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(dst));
        } else {
            for (int i = 0; i < n; ++i) {
                const int64_t b = o + i;
                const int64_t j = b / a.bs;
                dst[i] = fr[j * a.frag_stride + (b - j * a.bs)];
            }
        }
    }
}

// is_invalid_fragment_header / checksum verification (src/erasurecode.c:1050-1140): per fragment
// bit 0 bad magic, bit 1 metadata checksum (neither zlib nor legacy), bit 2 idx != slot, bit 3
// size != blocksize, bit 4 payload CRC32 mismatch (only when chksum_type says CRC32).
__global__ void frame_verify_kernel(const CrcArgs a, const uint32_t* __restrict__ img_zlib,
                                    const uint32_t* __restrict__ img_legacy,
                                    const uint32_t* __restrict__ crc, int64_t bs,
                                    uint32_t* __restrict__ status)
{
    const int64_t item = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (item >= a.items) return;
    const uint8_t* frag = item_ptr(a, item);
    uint8_t hd[kHeaderBytes];
#pragma unroll
    for (int c = 0; c < kHeaderBytes / 16; ++c) {
        uint4 v = *reinterpret_cast<const uint4*>(frag + 16 * c);
        put<4>(hd, 16 * c, v.x);
        put<4>(hd, 16 * c + 4, v.y);
        put<4>(hd, 16 * c + 8, v.z);
        put<4>(hd, 16 * c + 12, v.w);
    }
    uint32_t st = 0;
    if (get<4>(hd, 59) != kFragMagic) st |= 1u;
    const uint32_t stored = get<4>(hd, 67);
    if (stored != meta_crc(img_zlib + a.t_off, hd, 0) && stored != meta_crc(img_legacy + a.t_off, hd, 1))
        st |= 2u;
    if (get<4>(hd, 0) != static_cast<uint32_t>(item % a.nfrag)) st |= 4u;
    if (get<4>(hd, 4) != static_cast<uint32_t>(bs)) st |= 8u;
    if (hd[20] == kChksumCrc32 && crc && get<4>(hd, 21) != crc[item]) st |= 16u;
    status[item] = st;
}

}  // namespace ecamd
