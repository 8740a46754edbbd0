// crc.hpp -- the fragment checksums of the reference as GF(2)-linear state machines, and the
// table images the device CRC kernels (hip/ecamd_frame.hip) consume.
//
// Two machines, both "state' = T[(state ^ byte) & 0xff] ^ shift(state)", init ~0, final ~:
//   * zlib crc32 (system zlib 1.2.11; called at src/erasurecode_postprocessing.c:66-67 and
//     src/erasurecode_helpers.c:485), shift(s) = s >> 8;
//   * liberasurecode_crc32_alt, the legacy checksum (src/utils/chksum/crc32.c:79-91), whose shift
//     sign-extends bit 31 into the top byte.
// Both are linear in (state, message), so with r0(M) = the state after M from state 0:
//   r0(X || Y) = A^|Y| r0(X) ^ r0(Y),   crc(M) = ~(A^|M| ~0 ^ r0(M)),
// where A is the machine's zero-byte step.  Every table below is built by running the machine
// itself, so the device path follows whichever variant is selected without special cases.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace ecamd {

struct CrcMachine {
    bool legacy;
    uint32_t t[256];
    explicit CrcMachine(bool legacy_variant);
    uint32_t step(uint32_t s, uint8_t b) const
    {
        uint32_t sh = s >> 8;
        if (legacy && (s & 0x80000000u)) sh |= 0xff000000u;
        return t[(s ^ b) & 0xffu] ^ sh;
    }
    uint32_t run(uint32_t s, const uint8_t* p, size_t n) const
    {
        while (n--) s = step(s, *p++);
        return s;
    }
    uint32_t crc(const void* p, size_t n) const
    {
        return ~run(~0u, static_cast<const uint8_t*>(p), n);
    }
};

// 32 x 32 matrix over GF(2), stored by columns: M(x) = XOR of col[b] for the set bits b of x.
struct Mat32 {
    uint32_t col[32];
    uint32_t apply(uint32_t x) const
    {
        uint32_t r = 0;
        for (int b = 0; b < 32; b++)
            if (x >> b & 1u) r ^= col[b];
        return r;
    }
};
Mat32 mat_mul(const Mat32& a, const Mat32& b);  // a after b
Mat32 zero_shift(const CrcMachine& m, uint64_t nbytes);  // A^nbytes
Mat32 mat_inverse(const Mat32& a);  // a^-1 (the zero-byte step is invertible: the polynomial has x^0)

// Constants of the small-launch kernel's fused checksum (gf16_small_kernel CRC): it forms r0 of each
// fragment zero-extended by `zext` bytes, S = A^zext r0(M); then r0(M) = minv S with minv = A^-zext, and
// crc(M) = ~(c ^ r0(M)) with c = A^len ~0.  Cached per (machine, len, zext): O(log) matrix products
// once, a lookup afterwards.
// The small-launch kernel's checksum image for G-byte lanes (REGION = 256 * G bytes of a fragment per
// workgroup, NP = REGION / 16 pieces): the piece tables of build_fused_crc_image (mb 1: byte tables for
// dword 0, nibble tables for dwords 1-3; 1408 words), then NP position maps A^(16 (NP - 1 - l)) taking
// piece l's r0 to the end of the region, then 6 maps A^(REGION 2^i) taking a region's r0 past the
// regions after it -- all as 4-bit field tables (128 words each).
std::vector<uint32_t> build_small_crc_image(const CrcMachine& m, int G);

struct SmallCrcConst {
    uint32_t minv[32];
    uint32_t c;
};
SmallCrcConst small_crc_const(bool legacy, uint64_t len, uint64_t zext);

// Field tables of a linear map for B-bit index fields: out[f * 2^B + v] = M(v << (f * B)),
// f = 0 .. 32/B - 1.
void field_tables(const Mat32& M, int B, uint32_t* out);

// Image of one device CRC configuration (layout documented in hip/ecamd_frame.hip):
//   [ piece tables: 128/B tables, r0 of a 16-byte piece holding v in field f of word w
//                   (x4 position sets when pos)                                        ]
//   [ gap tables  : A^(64 lanes * 16 B) (A^4096 when pos) as 32/G field tables         ]
//   [ level tables: A^(16 * 2^t), t = 0..5, for the in-wave butterfly (G-bit fields)     ]
//   [ span tables : A^(J * 1024) as 4 byte tables (finalize kernel)                      ]
//   [ T           : the machine's byte table (finalize: tail bytes and header checksum)  ]
struct CrcImage {
    int B = 8;
    int G = 8;
    int J = 16;
    std::vector<uint32_t> words;
    size_t lds_words = 0;  // prefix staged into LDS by the partial kernel
    size_t span_off = 0;
    size_t t_off = 0;
};
// pos: four position-specific piece-table sets (piece u of a group of 4 pre-shifted by
// A^(1024*(3-u))) and an A^4096 gap map instead of one set and A^1024.
CrcImage build_crc_image(const CrcMachine& m, int B, int J, int G, bool pos = false);

// Image of the fused framed-encode checksum (hip/ecamd_frame_fused.hip): piece tables with byte
// tables for dword 0 and nibble tables for dwords 1-3, then four G = 4 maps: A^tile_bytes (the
// step between a lane's pieces), A^(16*2^t) for t < 6 (in-wave butterfly), A^1024 (across waves).
std::vector<uint32_t> build_fused_crc_image(const CrcMachine& m, uint64_t tile_bytes, int mb = 1);
// The bitsliced crc variant's image: npos position sets of byte piece tables (pieces `step` bytes
// apart, each set shifted to the group's last piece) + gap A^(step*npos) + butterfly levels + A^1024,
// then the lane-shift tables; nib: the piece tables as 16-entry nibble fields (512 words per set);
// mb < 4 (not with nib): byte tables for a piece's first mb dwords, nibble tables for the rest
// (mb * 1024 + (4 - mb) * 128 words per set).
std::vector<uint32_t> build_fused_crc_image_pos(const CrcMachine& m, uint64_t step, int npos, bool nib = false,
                                                int mb = 4);

}  // namespace ecamd
