// bitslice.hpp -- bitsliced GF(2^16) fragment maps (host side): the XOR network of an R x K
// coefficient matrix and the HIP source of a kernel specialised to it (compiled at run time by
// hip/ecamd_jit.hip).
//
// c*x over GF(2^16) is the 16x16 GF(2) matrix M_c applied to the bits of x (rs_galois_mult is
// carry-less multiplication mod 0x1100b, src/builtin/rs_vand/rs_galois.c:90-100).
// A lane holds 32 words of each fragment; a 16x16 bit transpose inside each 16-bit half of its 16
// dwords turns them into 16 bit planes (plane of bit b in register 15 - b; word w at bit
// (15 - w/2) + 16*(w%2); the transpose is an involution, so the same code maps output planes back
// to words).  Output plane (r, p) is the XOR over inputs j and bits b with M_{A[r][j]}[p][b] = 1 of
// the input planes: VALU XORs only, no table lookups, so the 8-output passes that the LDS tables
// bound (C5: random 16-byte lookups conflict ~2.9-way in the LDS banks) run at VALU rate.  Output
// planes accumulate through three-input XORs (v_bitop3), so a row of n terms costs ceil(n/2) ops;
// per input, up to `cap` temporaries (XORs of 2 or 3 available variables, one op each) are chosen
// by a distance-guided greedy (bitslice.cpp, distance_network) so that the rows become short sums,
// few enough that the network fits the register file at 2 waves per SIMD.
#pragma once
#include <array>
#include <cstdint>
#include <string>
#include <vector>

namespace ecamd {

// The 16 rows of M_c: bit b of row p is set when bit p of c*(1<<b) is.
void gf16_bitmatrix(int c, uint16_t (&rows)[16]);

struct BitsliceNet {
    int R = 0, K = 0;
    // per input j: temporaries (XOR of 2 or 3 variables -- third < 0 for a pair; variables
    // 0..15 are the input planes by bit, 16+ the temps in order) and, per output plane r*16+p,
    // the variables XORed into it
    struct Input {
        std::vector<std::array<int, 3>> temps;
        std::vector<std::vector<int>> rows;
    };
    std::vector<Input> inputs;
    int xor_ops() const;  // VALU ops of the network (temps + 3-input accumulation)
};

// Bumped whenever the network search changes (part of the JIT cache key).
constexpr const char* kBsNetworkVersion = "distance-1";
BitsliceNet bitslice_network(const std::vector<int>& coeff, int R, int K, int cap);

// Evaluate the network on 32 words per input (host check of the construction).
void bitslice_eval(const BitsliceNet& net, const uint16_t* in /* K x 32 */, uint16_t* out /* R x 32 */);

// HIP source of `extern "C" __global__ void ecamd_bs_kernel(ecamd_bs_args)` for the network.
// depth 0: each input's 64 B per lane loaded straight into registers; 2 or 4: through a per-wave
// LDS ring that many inputs deep, filled by LDS-DMA loads (bitslice_depth: the depth used for K).
// Emission choices (A/B experiments through ecamd_jitc's environment; defaults are the product's):
// temporaries computed right before first use (lazy) or all up front; a scheduling barrier after
// each input's network in the LDS-ring form.
struct BitsliceStyle {
    bool lazy_temps = true;
    bool input_barrier = false;
    bool copy_through = false;  // framed paths: every input also stored to its copy slot (BsArgs)
    // framed encode with CRC32 (implies copy_through): the kernel also folds every input and output
    // 16-byte piece into per-lane CRC states (LDS tables, the codec itself needs none) over work
    // units of consecutive tiles and writes r0 of each unit's range (BsArgs crc_*)
    bool crc = false;
    // crc variant: position table sets (1, 2 or 4): a lane's 4 pieces per fragment and tile are
    // folded in groups of crc_pos with per-position tables, one gap step per group
    int crc_pos = 1;
    // crc variant: fold each wave's lane states with lane-shift tables (one map per lane, 32 KiB
    // more LDS) and an XOR reduction instead of the 6-level butterfly; always on for 5-8 outputs
    bool crc_lane = false;
    // crc variant: piece tables of 16-entry nibble fields (2 KiB per position set, conflict-free,
    // 32 lookups per 16-byte piece) instead of 256-entry byte tables (16 KiB, 16 lookups that
    // conflict ~3.5-way in the LDS banks)
    bool crc_nib = false;
    // lanes per workgroup of the plain / copy-through register form: 256 (a tile is 16 KiB of every
    // fragment, a lane's 4 chunks 4 KiB apart) or 64 (one-wave tiles of 4 KiB, chunks 1 KiB apart:
    // the dispatcher then balances 4x finer work units, which interleaved output slots favour)
    int threads = 256;
    // waves per SIMD the plain / copy-through form is built for (its register budget); 0: by R
    // (bitslice_waves_per_simd)
    int waves = 0;
    // the occupancy cap of amdgpu_waves_per_eu (0: = waves, which makes the compiler pad the VGPR
    // count of the kernel descriptor so that exactly `waves` fit, whatever the code uses)
    int waves_max = 0;
    // copy-through forms: input j's bytes start in_shift[j] (0..15) past a 16-byte boundary (object
    // chunks at j*bs when bs % 16 != 0).  Non-zero: each lane loads the ALIGNED chunk under its
    // window, takes the next one from its neighbour lane (DPP wave_shl:1; the wave's last lane loads
    // its own) and realigns in registers (v_alignbyte, compile-time shift), instead of an unaligned
    // 16-byte load.  Empty: every input aligned, or unaligned loads.
    std::vector<int> in_shift;
    // one-wave register form: chunks (0, 2 or 4) of input j + 1 loaded before input j's network, so a
    // wave has the next input's loads in flight while it computes (the compiler otherwise issues each
    // input's loads right before its use and waits for them at once)
    int prefetch = 0;
    // one-wave realigned inputs: the last lane's next chunk for chunks 0-2 is lane 0 of the input's
    // following chunk (1 KiB on), taken by v_readlane instead of a load; only chunk 3's is loaded
    bool realign_lane = false;
    // crc variant: the wave XOR reductions of the lane-shift fold by DPP + v_readlane (wave_xor)
    // instead of a ds_bpermute butterfly, whose 6 LDS instructions per fragment and tile compete with
    // the CRC lookups: C5 framed CRC32 encode 1.380 -> 1.317 ms (profiles/r04_dppred_ab.log);
    // ECAMD_BS_DPPRED=0 in ecamd_jitc's environment restores the butterfly (A/B only)
    bool dpp_reduce = true;
    // crc variant in one-wave 4 KiB tiles (round 5): 0 = off; W > 0 = workgroups of W waves sharing
    // one copy of the tables (crc_pos position sets for pieces 1 KiB apart + the lane-shift tables);
    // the first crc_q workgroups' waves take tiles (b * crc_per + i) * W + wave, i < crc_per, the rest
    // one tile each, each wave on its own (no barrier after the table fill), and write r0 of each
    // fragment's 4 KiB to crc_partial[t * (K + R) + f]
    int crc_wave = 0;
    // one-wave crc form: no scheduling barrier between an input's CRC lookups and its network, so the
    // compiler may interleave the LDS lookups with the network's XORs
    bool crc_mix = false;
    // one-wave crc form: a piece's first crc_mb dwords through byte tables, the rest through
    // conflict-free nibble tables (build_fused_crc_image_pos mb)
    int crc_mb = 4;
    // one-wave crc form with byte tables: dword 3 of each piece looked up in the image in global memory
    // (through the vector L1) instead of LDS -- a second lookup engine for the random-index lookups
    // whose LDS bank conflicts bound the form (round 6 A/B, knob frame_crc_wave_l1)
    bool crc_l1 = false;
};
// LDS words of the CRC image the crc variant reads (host/crc.hpp build_fused_crc_image_pos: byte
// piece tables per position, chain step 4096 B): npos x 4 x 1024 piece words + gap + 6 butterfly
// levels + A^1024
constexpr int bs_crc_words(int npos, bool nib = false) { return npos * (nib ? 512 : 4 * 1024) + 8 * 128; }
constexpr int kBsCrcStep = 4096;  // bytes between a lane's consecutive pieces of one fragment
constexpr int kBsCrcLaneWords = 8 * 16 * 64;  // lane-shift tables after bs_crc_words (fold-each form)
constexpr int kBsCrcWaveStep = 1024;  // one-wave crc form: bytes between a lane's pieces of one fragment
std::string bitslice_source(const BitsliceNet& net, int depth = 0, BitsliceStyle style = {});
int bitslice_depth(int depth, int K);
// Waves per SIMD the kernel of an R-output map is built for: 2 (16 R accumulators + the network
// in <= 256 VGPRs) for 5..8 outputs, 4 (<= 128 VGPRs) for up to 4; the crc variant (up to 4
// outputs) 3 (its K + R CRC states need more than 128).
int bitslice_waves_per_simd(int R, bool crc = false);
// One-wave forms: the kernel's amdgpu_waves_per_eu(wmin, wmax) and whether a scheduling barrier
// closes every input's network.  wmin sets the register budget (512 / wmin VGPRs); wmax caps the
// occupancy (the compiler pads the descriptor's VGPR count so no more waves fit: (2, 2) means 176
// VGPRs, 2 waves per SIMD, whatever the code uses); the barrier keeps the compiler from hoisting the
// next input's loads into the network, which is what holds the extra registers.
struct BsOcc {
    int wmin = 2;
    int wmax = 2;
    bool barrier = false;
    // plain maps in the multi-wave register form only: lanes per workgroup 128 / 512 (8 / 32 KiB tiles)
    // instead of 256 (16 KiB); 0 = 256
    int threads = 0;
};

// A compile request (R, K, cap, depth, coefficients) as the text ecamd_jitc reads, and back.
// in_shift (copy-through only): per-input byte shifts of BitsliceStyle::in_shift; any non-zero makes
// a version-3 request (a line of K shifts after the flags).
std::string bitslice_request(const std::vector<int>& coeff, int R, int K, int cap, int depth, bool copy = false,
                             bool crc = false, int crc_pos = 1, bool crc_lane = false, bool crc_nib = false,
                             bool wave = false, const std::vector<int>* in_shift = nullptr, int prefetch = 0,
                             const BsOcc* occ = nullptr, int crc_wave = 0);
bool bitslice_parse_request(const std::string& text, std::vector<int>& coeff, int& R, int& K, int& cap,
                            int& depth, bool* copy = nullptr, bool* crc = nullptr, int* crc_pos = nullptr,
                            bool* crc_lane = nullptr, bool* crc_nib = nullptr, bool* wave = nullptr,
                            bool* budget2 = nullptr, std::vector<int>* in_shift = nullptr,
                            int* prefetch = nullptr, BsOcc* occ = nullptr, int* crc_wave = nullptr);

// Kernel arguments (layout shared by the generated source and the launcher).
constexpr int kBsTile = 16384;  // bytes of each fragment per workgroup tile (256 lanes x 64 B)
constexpr int kBsTileWave = 4096;  // the same for one-wave workgroups (BitsliceStyle::threads 64)
constexpr int kBsMaxK = 32;
constexpr int kBsMaxR = 8;
struct BsArgs {
    const uint8_t* in_base;
    uint8_t* out_base;
    int64_t in_stride;
    int64_t out_stride;
    const int32_t* stripe_list;  // logical stripe s is stripe_list[s] (null: s)
    uint32_t in_records;
    uint32_t out_records;
    uint32_t ntiles;
    uint32_t tiles_per_stripe;
    int32_t in_off[kBsMaxK];
    int32_t out_off[kBsMaxR];
    // copy-through (framed encode / decode-join, register loads only): input j is also stored at
    // copy_base + s*copy_stride + copy_idx[j]*copy_step (copy_idx 0xff: not copied; packed bytes,
    // not 32-bit offsets, to keep the kernel's scalar registers free); copy_records 0 = off
    uint8_t* copy_base;
    int64_t copy_stride;
    uint32_t copy_records;
    uint32_t copy_step;
    uint8_t copy_idx[kBsMaxK];
    // crc variant: unit u = (stripe u / crc_q, range u % crc_q of crc_per tiles); r0 of the range
    // of fragment f (inputs 0..K-1, then the outputs) lands in crc_partial[(s*crc_nfrag + f)*crc_q + r]
    const uint32_t* crc_img;  // kBsCrcWords
    uint32_t* crc_partial;
    int32_t crc_q;
    int32_t crc_per;
    int32_t crc_nfrag;
};

}  // namespace ecamd
