// tables.hpp -- split multiply tables that the GPU kernels stage into LDS.
//
// c*x over GF(2^16) is linear over GF(2), so c*x = c*(x & 0xff) ^ (c*0x100)*(x >> 8).  For one
// input fragment j and a group of up to W output rows, the LDS image holds
//   T_lo[b] = pack_r( A[r][j] * b )          b = 0..255
//   T_hi[b] = pack_r( A[r][j] * (b << 8) )
// packed as W 16-bit lanes (bits 16r..16r+15) of a W*2-byte entry.  One input word then costs two
// LDS lookups for all W outputs at once (the MI355X hot loop in ecamd_kernels.hip).
#pragma once
#include <cstdint>
#include <vector>

namespace ecamd {

// Bytes per table entry for a row-group width (2 -> 4 B, 4 -> 8 B, 8 -> 16 B).
inline int entry_bytes(int width) { return width * 2; }

// Image for rows [row0, row0+width) and inputs [col0, col0+ncols) of the R x K matrix `coeff`
// (rows beyond R are zero).  Layout: input-major, [T_lo(256) | T_hi(256)] per input.
std::vector<uint8_t> build_split_tables(const std::vector<int>& coeff, int R, int K, int row0,
                                        int width, int col0, int ncols);

}  // namespace ecamd

namespace ecamd {

// Nibble form of the same map: c*x = XOR_q c*(((x >> 4q) & 15) << 4q), q = 0..3, so per input
//   T_q[n] = pack_r( A[r][j] * (n << 4q) )    n = 0..15
// Layout: input-major, [T_0(16) | T_1(16) | T_2(16) | T_3(16)] per input.  A 16-entry table of
// W*2-byte entries spans 16 distinct LDS bank slots (W = 8: exactly one 256-byte bank row), so
// the lookups of a wave never conflict -- four lookups per word instead of two conflicted ones.
std::vector<uint8_t> build_nibble_tables(const std::vector<int>& coeff, int R, int K, int row0,
                                         int width, int col0, int ncols);

}  // namespace ecamd
