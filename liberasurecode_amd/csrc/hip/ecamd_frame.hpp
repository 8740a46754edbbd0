// ecamd_frame.hpp -- argument blocks of the framing / CRC kernels (hip/ecamd_frame.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ecamd {

constexpr int kHeaderBytes = 80;           // sizeof(fragment_header_t), include/erasurecode.h
constexpr int kMetaBytes = 59;             // sizeof(fragment_metadata_t)
constexpr uint32_t kFragMagic = 0xb0c5ecc;  // LIBERASURECODE_FRAG_HEADER_MAGIC
constexpr uint8_t kChksumCrc32 = 2;        // CHKSUM_CRC32

// Items = nstripes * nfrag payloads; item (s, f) fragment at base + s*stripe_stride + f*frag_stride,
// its payload at + payload_off, len bytes (body = len & ~15 handled by the partial kernel).
struct CrcArgs {
    const uint8_t* base;
    int64_t stripe_stride;
    int64_t frag_stride;
    int64_t payload_off;
    int64_t len;
    int64_t body;
    int64_t items;
    int nfrag;
    int nspans;      // spans per item (0: no checksum, header only)
    int J;           // KiB per span
    int legacy;      // 1: liberasurecode_crc32_alt machine
    uint32_t c0;     // A^len(~0)
    uint32_t span_off;
    uint32_t t_off;
    // crc_finalize_kernel over ranges that end before the payload does: the CRC32 of the rest
    // (tail_crc[item], the checksum of the payload's last tail bytes) is folded in as
    // acc = A^tail(acc) ^ r0(tail), r0(tail) = ~tail_crc ^ tail_c0 (tail_c0 = A^tail(~0), tail_cols =
    // the 32 columns of A^tail); tail_crc null: the ranges end at `body`
    const uint32_t* tail_crc;
    uint32_t tail_c0;
    uint32_t tail_cols[32];
};

struct HeaderArgs {
    int write;
    int idx0;
    uint32_t size;
    uint32_t backend_meta_size;
    uint64_t orig_data_size;
    uint32_t backend_version;
    uint32_t libec_version;
    uint8_t chksum_type;
    uint8_t backend_id;
};

struct SplitArgs {
    const uint8_t* obj;
    int64_t obj_stride;
    int64_t size;
    uint8_t* frags;
    int64_t stripe_stride;
    int64_t frag_stride;
    int64_t bs;
    int k;
    int nstripes;
    int aligned;     // object base / stride / bs all 16-byte multiples
    int64_t from;    // streaming split only: payload bytes [from, bs) (a multiple of 16), 0 = all
};

struct JoinArgs {
    const uint8_t* frags;
    int64_t stripe_stride;
    int64_t frag_stride;
    int64_t bs;
    uint8_t* obj;
    int64_t obj_stride;
    int64_t size;
    int nstripes;
    int aligned;
};

// gf16_frame_crc_kernel (ecamd_frame_fused.hip): partial[(s*nfrag + f)*q + r] = r0 of range r
// (q ranges of `per` tiles per fragment) of fragment f of stripe s.
struct FusedCrcArgs {
    const uint32_t* img;  // [piece tables, MB = 1 | A^tile | A^(16*2^t), t < 6 | A^1024], G = 4 maps
    uint32_t* partial;
    int q;
    int per;
    int nfrag;
};

template <int MB, int G, bool POS>
__global__ void crc_partial_kernel(const CrcArgs a, const uint32_t* __restrict__ img,
                                   uint32_t* __restrict__ partial);
__global__ void crc_finalize_kernel(const CrcArgs a, const uint32_t* __restrict__ img,
                                    const uint32_t* __restrict__ partial,
                                    uint32_t* __restrict__ crc_out, const HeaderArgs h);
// The crc variant in one-wave tiles writes r0 of every fragment's 4 KiB tile, tile-major:
// tiles[(s * tps + t) * nf + f].  Range r of g consecutive tiles of payload item = s * nf + f:
// out[item * (tps / g) + r] = Horner over its tiles with A^4096 (span: its byte tables) -- the
// layout crc_finalize_kernel reads.
__global__ void crc_combine_kernel(const uint32_t* __restrict__ tiles, uint32_t* __restrict__ out,
                                   const uint32_t* __restrict__ span, int64_t items, int nf, int tps, int g);
__global__ void frame_split_kernel(const SplitArgs a);
__global__ void frame_join_kernel(const JoinArgs a);
// 32-bit-offset streaming forms (objects < 2 GiB, stripes < 2 GiB): tiles of 4 x 256 x 16 B
template <int kCopyU, bool kDpp>
__global__ void frame_split_stream_kernel(const SplitArgs a);
template <int kCopyU, bool kDpp>
__global__ void frame_join_stream_kernel(const JoinArgs a, int k, int tile_align);
__global__ void frame_verify_kernel(const CrcArgs a, const uint32_t* __restrict__ img_zlib,
                                    const uint32_t* __restrict__ img_legacy,
                                    const uint32_t* __restrict__ crc, int64_t bs,
                                    uint32_t* __restrict__ status);

}  // namespace ecamd
