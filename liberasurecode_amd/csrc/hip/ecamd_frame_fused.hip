// ecamd_frame_fused.hip -- liberasurecode_encode with CHKSUM_CRC32 for S objects resident in HBM,
// codec and payload checksums in ONE launch (reference: encode
// src/erasurecode.c:383-477, CRC src/erasurecode_helpers.c:463-496).
//
// gf16_frame_crc_kernel<W, KG> is the copy-through gf16_stream_kernel (the k data inputs read from
// the objects, stored into their payload slots, the parity written) that also folds every input
// and output 16-byte piece into a per-lane CRC32 state while the bytes are in registers, so the
// payloads are never re-read for their checksums (24 instead of 38 MiB of HBM traffic per C3
// stripe).  The checksum algebra is host/crc.hpp's: r0(X || Y) = A^|Y| r0(X) ^ r0(Y).
//   * Work unit = one contiguous range of `per` tiles of one stripe (a tile = blockDim*16 bytes of
//     every fragment); lane l of wave w sees the piece at tile*T + w*1024 + l*16 of each fragment,
//     one tile apart, so its state steps as s = A^T s ^ r0(piece) (T = tile bytes, one G=4 map).
//   * At the end of the unit a 6-level shuffle butterfly (A^(16*2^t)) folds the lanes of a wave,
//     the waves' states meet in LDS and one thread per fragment folds them with A^1024 (Horner),
//     giving r0 of the range; crc_finalize_kernel then runs Horner over the ranges of each
//     payload (A^(range bytes)) and writes the 80-byte headers, exactly as after crc_partial.
// Requirements (checked on the host, else the split path runs): one map pass (the k inputs and
// m outputs fit one launch), objects 16-byte aligned that fill the payloads exactly, and the
// payload size a multiple of the tile.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ecamd_crc_dev.hpp"
#include "ecamd_frame.hpp"
#include "ecamd_stream.hpp"

namespace ecamd {
namespace {

using crcdev::lmap;
using crcdev::piece_r0;

constexpr int kMap4 = 128;  // one G=4 field-table map (8 x 16 words)

// MB: byte tables for the first MB dwords of a piece, nibble tables for the rest (crcdev).
// NIB: the codec's own lookups on nibble tables (conflict-free, 1/8 of the LDS image) instead of
// byte tables -- the LDS array, not instruction issue, bounds this kernel.
template <int W, int G, int KG, int MB, bool NIB>
__device__ __forceinline__ void fused_group(const ApplyArgs& a, const uint8_t* lds, const uint32_t* ctab,
                                            const uint32_t* gap, const StreamTile& t,
                                            uint32_t (&acc)[8][W / 2], uint32_t (&st)[4 * KG + W])
{
    v4u x[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int j = 4 * G + i;
        const int base = (j < a.ncols) ? a.in_off32[j] + t.off : static_cast<int>(0x80000000u);
        x[i] = __builtin_amdgcn_raw_buffer_load_b128(t.rin, base, 0, 2);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int j = 4 * G + i;
        if (j < a.ncols) {  // wave-uniform
            __builtin_amdgcn_raw_buffer_store_b128(x[i], t.rcopy, a.copy_off32[j] + t.off, 0, 2);
            st[j] = lmap<4>(gap, st[j]) ^ piece_r0<MB>(ctab, x[i]);
        }
    }
    if constexpr (NIB) {
        if (4 * G + 0 < a.ncols) mac_chunk_nib_imm<W, 4 * G + 0>(lds, x[0], acc);
        if (4 * G + 1 < a.ncols) mac_chunk_nib_imm<W, 4 * G + 1>(lds, x[1], acc);
        if (4 * G + 2 < a.ncols) mac_chunk_nib_imm<W, 4 * G + 2>(lds, x[2], acc);
        if (4 * G + 3 < a.ncols) mac_chunk_nib_imm<W, 4 * G + 3>(lds, x[3], acc);
    } else {
        if (4 * G + 0 < a.ncols) mac_chunk_imm<W, 4 * G + 0>(lds, x[0], acc);
        if (4 * G + 1 < a.ncols) mac_chunk_imm<W, 4 * G + 1>(lds, x[1], acc);
        if (4 * G + 2 < a.ncols) mac_chunk_imm<W, 4 * G + 2>(lds, x[2], acc);
        if (4 * G + 3 < a.ncols) mac_chunk_imm<W, 4 * G + 3>(lds, x[3], acc);
    }
    if constexpr (G + 1 < KG) fused_group<W, G + 1, KG, MB, NIB>(a, lds, ctab, gap, t, acc, st);
}

}  // namespace

template <int W, int KG, int MB, bool NIB>
__global__ void __launch_bounds__(512) gf16_frame_crc_kernel(const ApplyArgs a, const FusedCrcArgs c)
{
    constexpr int kPieceWords = crcdev::piece_words(MB);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    constexpr int NS = 4 * KG + W;  // state slots: inputs 0 .. 4KG-1, outputs 4KG .. 4KG+W-1
    const int tbytes = a.ncols * (NIB ? 64 : 512) * EB;
    for (int o = threadIdx.x * 16; o < tbytes; o += blockDim.x * 16)
        *reinterpret_cast<uint4*>(lds + o) = *reinterpret_cast<const uint4*>(a.tables + o);
    uint32_t* ctab = reinterpret_cast<uint32_t*>(lds + tbytes);
    constexpr int cwords = kPieceWords + 8 * kMap4;  // pieces | gap | 6 levels | A^1024
    for (int i = threadIdx.x; i < cwords; i += blockDim.x) ctab[i] = c.img[i];
    uint32_t* xch = ctab + cwords;  // [wave][NS] lane-0 states of each wave
    __syncthreads();
    const uint32_t* gap = ctab + kPieceWords;
    const uint32_t* level = gap + kMap4;
    const uint32_t* a1024 = level + 6 * kMap4;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwaves = blockDim.x >> 6;
    const int cstride = static_cast<int>(blockDim.x) * 16;
    const uint32_t nstripes = a.ntiles / a.tiles_per_stripe;
    const uint32_t units = nstripes * c.q;

    for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {
        const uint32_t s = u / c.q;
        const uint32_t r = u - s * c.q;
        StreamTile tile;
        tile.rin = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.in_base) + static_cast<int64_t>(s) * a.in_stride, 0,
            static_cast<int>(a.in_records), 0x00020000);
        tile.rcopy = __builtin_amdgcn_make_buffer_rsrc(
            a.copy_base + static_cast<int64_t>(s) * a.copy_stride, 0, static_cast<int>(a.copy_records),
            0x00020000);
        tile.cstride = cstride;
        const auto rout = __builtin_amdgcn_make_buffer_rsrc(
            a.out_base + static_cast<int64_t>(s) * a.out_stride, 0, static_cast<int>(a.out_records),
            0x00020000);
        uint32_t st[NS];
#pragma unroll
        for (int f = 0; f < NS; f++) st[f] = 0u;
        for (int t = static_cast<int>(r) * c.per; t < static_cast<int>(r + 1) * c.per; t++) {
            tile.off = t * cstride + static_cast<int>(threadIdx.x) * 16;
            uint32_t acc[8][D];
#pragma unroll
            for (int w = 0; w < 8; w++)
#pragma unroll
                for (int d = 0; d < D; d++) acc[w][d] = 0u;
            fused_group<W, 0, KG, MB, NIB>(a, lds, ctab, gap, tile, acc, st);
#pragma unroll
            for (int o = 0; o < W; o++) {
                if (o >= a.nrows) break;
                v4u v;
#pragma unroll
                for (int d = 0; d < 4; d++) {
                    const uint32_t A = acc[2 * d][o >> 1], B = acc[2 * d + 1][o >> 1];
                    v[d] = (o & 1) ? ((A >> 16) | (B & 0xffff0000u)) : ((A & 0xffffu) | (B << 16));
                }
                __builtin_amdgcn_raw_buffer_store_b128(v, rout, a.out_off32[o] + tile.off, 0, 2);
                st[4 * KG + o] = lmap<4>(gap, st[4 * KG + o]) ^ piece_r0<MB>(ctab, v);
            }
        }
        // lanes of a wave -> the wave's 1 KiB segment end (the crc_partial_kernel butterfly)
#pragma unroll
        for (int f = 0; f < NS; f++) {
            const bool live = f < 4 * KG ? f < a.ncols : f - 4 * KG < a.nrows;
            if (!live) continue;  // wave-uniform
            uint32_t x = st[f];
#pragma unroll
            for (int l = 0; l < 6; ++l) x = lmap<4>(level + kMap4 * l, x) ^ __shfl_down(x, 1 << l, 64);
            if (lane == 0) xch[wave * NS + f] = x;
        }
        __syncthreads();
        // waves -> the range end: Horner with A^1024, one thread per fragment
        if (static_cast<int>(threadIdx.x) < NS) {
            const int f = threadIdx.x;
            const bool live = f < 4 * KG ? f < a.ncols : f - 4 * KG < a.nrows;
            if (live) {
                uint32_t v = 0u;
                for (int w = 0; w < nwaves; w++) v = lmap<4>(a1024, v) ^ xch[w * NS + f];
                const int frag = f < 4 * KG ? f : a.ncols + (f - 4 * KG);
                c.partial[(static_cast<int64_t>(s) * c.nfrag + frag) * c.q + r] = v;
            }
        }
        __syncthreads();
    }
}

#define ECAMD_FUSED_INST(W, MB, NIB)                                                                   \
    template __global__ void gf16_frame_crc_kernel<W, 1, MB, NIB>(const ApplyArgs, const FusedCrcArgs); \
    template __global__ void gf16_frame_crc_kernel<W, 2, MB, NIB>(const ApplyArgs, const FusedCrcArgs); \
    template __global__ void gf16_frame_crc_kernel<W, 3, MB, NIB>(const ApplyArgs, const FusedCrcArgs); \
    template __global__ void gf16_frame_crc_kernel<W, 4, MB, NIB>(const ApplyArgs, const FusedCrcArgs); \
    template __global__ void gf16_frame_crc_kernel<W, 5, MB, NIB>(const ApplyArgs, const FusedCrcArgs);
ECAMD_FUSED_INST(2, 1, false) ECAMD_FUSED_INST(4, 1, false) ECAMD_FUSED_INST(8, 1, false)
ECAMD_FUSED_INST(2, 4, false) ECAMD_FUSED_INST(4, 4, false) ECAMD_FUSED_INST(8, 4, false)
ECAMD_FUSED_INST(2, 4, true) ECAMD_FUSED_INST(4, 4, true) ECAMD_FUSED_INST(8, 4, true)
ECAMD_FUSED_INST(2, 1, true) ECAMD_FUSED_INST(4, 1, true) ECAMD_FUSED_INST(8, 1, true)
#undef ECAMD_FUSED_INST

}  // namespace ecamd
