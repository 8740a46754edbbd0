// ecamd_kernels.hpp -- kernel argument blocks shared by ecamd_kernels.hip and ecamd_device.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ecamd {

constexpr int kMaxCols = 80;      // inputs per launch: 80 * 512 * 4 B = 160 KiB of LDS at W = 2
constexpr int kMaxRows = 8;       // outputs per launch
constexpr int kLdsBytes = 163840; // gfx950: 160 KiB per workgroup

struct ApplyArgs {
    const uint8_t* tables;            // split-table image (gf16) -- unused by xor
    const uint8_t* in_base;           // strided form
    uint8_t* out_base;
    const uint8_t* const* in_ptrs;    // pointer-table form
    uint8_t* const* out_ptrs;
    int64_t in_stride;                // bytes per stripe (strided) / pointers per stripe (table)
    int64_t out_stride;
    int64_t bs;                       // bytes per fragment payload
    uint32_t ntiles;
    uint32_t tiles_per_stripe;
    int ncols;                        // inputs in this launch
    int nrows;                        // outputs in this launch
    int accumulate;                   // 1: out ^= result (later column chunks)
    uint32_t masks[kMaxRows];         // xor kernel: input selection per output
    int64_t in_off[kMaxCols];         // byte offset (strided) / column (table) of input j
    int64_t out_off[kMaxRows];
    uint8_t* copy_base;               // gf16_copy_apply_kernel: input j is also stored at
    int64_t copy_stride;              //   copy_base + s*copy_stride + copy_off[j]
    int64_t copy_off[kMaxCols];
    uint32_t in_records;              // gf16_stream_kernel: bytes addressable from one stripe's
    uint32_t out_records;             //   in_base / out_base (buffer-resource range, < 2^31)
    int32_t in_off32[kMaxCols];       // in_off / out_off as 32-bit buffer offsets
    int32_t out_off32[kMaxRows];
    int limited;                      // 1: input j holds only in_len32[j] valid bytes (the rest
    int32_t in_len32[kMaxCols];       //   of its blocksize reads as zeros), output r / copy j take
    int32_t out_len32[kMaxRows];      //   only out_len32[r] / copy_len32[j] bytes: objects shorter
    int32_t copy_len32[kMaxCols];     //   than the k payloads (encode padding, decode into objects);
    int64_t min_len;                  //   min_len = the smallest of them (tiles past it go byte-exact)
    uint32_t copy_records;            // gf16_stream_kernel copy-through: 0 = off; else range of
    int32_t copy_off32[kMaxCols];     //   copy_base per stripe and 32-bit copy_off (< 0: skip)
    int tile_order;                   // gf16_stream_kernel: 1 = contiguous tile range per workgroup
    int realign_dpp;                  // gf16_realign_kernel: the second aligned chunk of each lane's
                                      //   window from the next lane (DPP), the last lane loads its own
    const int32_t* stripe_list;       // gf16_stream_kernel: logical stripe s is stripe_list[s] of the
                                      //   strided layout (heterogeneous decode groups); null = s
};

// gf16_small_kernel: one pass over fragments at a uniform pitch (input j of stripe s at
// in + s * in_stride + j * in_pitch, output r likewise), for launches of a few chunks.
struct SmallArgs {
    const uint8_t* tables;
    const uint8_t* in;
    uint8_t* out;
    int64_t in_stride, out_stride;
    int64_t in_pitch, out_pitch;
    int64_t bs;
    int64_t cpf;      // G-byte lane groups per fragment (G = 16 or 4 bytes per lane)
    int64_t nchunks;  // cpf * stripes
    int ncols, nrows, accumulate;
    uint32_t masks[kMaxRows];  // xor_small_kernel: inputs of output r
    // gf16_small_kernel CRC (fused payload checksums, one stripe): the CRC32 of every input and output
    // fragment over bs bytes into crc_out[0 .. ncols + nrows) (inputs first); crc_img the fused image
    // (host/crc.hpp build_fused_crc_image, mb 1), crc_part device scratch: word 0 a self-resetting
    // counter (zero before the first launch), partials from word 16; crc_minv / crc_c: SmallCrcConst
    const uint32_t* crc_img;
    uint32_t* crc_out;
    uint32_t* crc_part;
    uint32_t crc_minv[32];
    uint32_t crc_c;
    int crc_dbg;  // development A/B (knob small_crc_dbg): 1 skip the epilogue's lookups, 2 skip the image staging
    // completion flag (ecamd_done_flag_arm): once every output (and checksum) store of the launch is
    // visible system-wide, done_val is stored to *done (pinned host memory) -- the per-call path polls it
    // instead of synchronizing the stream.  Several workgroups: the last one to finish stores it (counter
    // done_ctr, self-resetting, zero before the first launch; with CRC the checksum's last workgroup).
    uint32_t* done;
    uint32_t* done_ctr;
    uint32_t done_val;
};

// The resident small server (small_server_kernel): the per-call path's small launches posted to a
// mailbox in coherent pinned host memory instead of launched -- one per caller thread, kSmallServerWgs
// workgroups polling it until idle_ticks of the 100 MHz constant clock pass without a request.
struct alignas(16) SmallServerSlot {
    SmallArgs args;
};
struct alignas(16) SmallServerBox {
    uint32_t post;        // sequence << 18 | slot generation << 10 | slot << 9 | half << 8 | workgroups, stored last
    uint32_t done_val;    // the request's completion-flag value (read with post, one 8-byte load)
    uint32_t stop;        // host: every workgroup exits at its next poll
    uint32_t variant[2];  // per slot: kSmallServerXor | CRC << 8 | G << 4 | W (gf16_small_body / xor_small_body)
    uint32_t pad[11];
    SmallServerSlot slot[2];  // two argument blocks (an encode and a decode alternating both stay cached)
};
struct SmallServerArgs {
    SmallServerBox* box;
    uint32_t post0;      // the post word already handled: a different one is a request
    uint32_t dup_check;  // relaunched while a request was pending: skip it if its flag is already set
    uint64_t idle_ticks;
};
constexpr int kSmallServerWgs = 16;
constexpr uint32_t kSmallServerXor = 1u << 12;
constexpr uint32_t kSmallServerSlot = 1u << 9;  // post word: argument slot 1 (else 0); bits 10-17 its generation
// post word: the request's LDS (tables, staging, checksum image) fits in kSmallServerLdsHalf bytes, and it runs
// at slot * kSmallServerLdsHalf: an encode and a decode alternating both keep their staged tables
constexpr uint32_t kSmallServerHalf = 1u << 8;
constexpr int kSmallServerLdsHalf = 79 * 1024;
template <uint32_t V>  // V: W | G << 4, or kSmallServerXor (each with and without the fused checksum)
__global__ void small_server_kernel(const SmallServerArgs sa);

// gf16_stream_kernel handles up to kStreamGroups*4 inputs per launch (fully unrolled).
constexpr int kStreamGroups = 5;

struct FillArgs {
    uint8_t* base;
    int64_t stripe_stride;
    int64_t frag_stride;
    int64_t bs;
    int nfrags;
    int nstripes;
    int stripe0;
    uint64_t seed_base;
};

template <int W, bool PTRS, bool NT, bool NIB>
__global__ void gf16_apply_kernel(const ApplyArgs a);
template <int W, int G, bool ST, bool CRC = false>
__global__ void gf16_small_kernel(const SmallArgs a);
// Words of the fused small-launch CRC image for G-byte lanes (host/crc.hpp build_small_crc_image): piece
// tables (byte tables for a piece's dword 0, nibble tables for dwords 1-3), 16 G position maps, 6
// region-shift maps (nibble fields, 128 words each).
constexpr int kSmallCrcPieceWords = 1024 + 3 * 128;
constexpr int small_crc_words(int G) { return kSmallCrcPieceWords + (16 * G + 6) * 128; }
template <bool ST, bool CRC = false>
__global__ void xor_small_kernel(const SmallArgs a);
template <int W>
__global__ void gf16_copy_apply_kernel(const ApplyArgs a);
template <int W, int KG, int CH, bool PF, bool NIB>
__global__ void gf16_stream_kernel(const ApplyArgs a);
template <int W, int KG>
__global__ void gf16_ptrs_stream_kernel(const ApplyArgs a);
template <int KG>
__global__ void gf16_hybrid_kernel(const ApplyArgs a);
template <int W, int KG>
__global__ void gf16_realign_kernel(const ApplyArgs a);
struct FusedCrcArgs;
template <int W, int KG, int MB, bool NIB = false>
__global__ void gf16_frame_crc_kernel(const ApplyArgs a, const FusedCrcArgs c);
template <int W, bool PTRS>
__global__ void xor_apply_kernel(const ApplyArgs a);
template <int KG, bool COPY>
__global__ void xor_stream_kernel(const ApplyArgs a);
__global__ void splitmix_fill_kernel(FillArgs f);
}  // namespace ecamd
