// bitslice.cpp -- network construction and kernel source for bitsliced GF(2^16) maps
// (bitslice.hpp).  The generated kernel is verified bit-exact against the CPU oracle by
// tests/test_gpu_bitslice.py; the network itself against GF16 products by
// tests/test_bitslice_host.py (ecamd_bitslice_eval).
#include "bitslice.hpp"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <sstream>

#include "gf16.hpp"

namespace ecamd {

void gf16_bitmatrix(int c, uint16_t (&rows)[16])
{
    const GF16& gf = GF16::get();
    for (auto& r : rows) r = 0;
    for (int b = 0; b < 16; b++) {
        const int v = gf.mul(c & 0xffff, 1 << b);
        for (int p = 0; p < 16; p++)
            if ((v >> p) & 1) rows[p] = static_cast<uint16_t>(rows[p] | (1u << b));
    }
}

namespace {

// The network of one input: its R*16 target rows (16-bit masks over the input's planes) built from
// the 16 planes plus up to `cap` temporaries, priced as the kernel runs it -- a row that is the XOR
// of d available variables costs ceil(d/2) three-input XORs into its accumulator, a temporary one
// op (the XOR of 2 or 3 available variables).
//
// Distance-guided greedy in the manner of Boyar and Peralta's circuit heuristic, made exact by the
// small space: dist[v] is the fewest available variables XORing to v, for every v of the 2^16, so
// adding a variable c updates it in one pass (dist'[v] = min(dist[v], dist[v^c] + 1): a minimal
// sum uses c at most once) and the saving of a candidate c is sum over rows t of
// ceil(dist[t]/2) - ceil(min(dist[t], dist[t^c] + 1)/2).  Each step adds the one-op candidate
// (dist 2 or 3) with the largest saving above its own cost; ties go to the smallest mask, so the
// network is a function of the matrix.  Rows are then spelled out along parent links (each v
// remembers the variable its current minimal sum ends with).
void distance_network(const std::vector<uint16_t>& rows, int cap, BitsliceNet::Input& out)
{
    constexpr int N = 1 << 16;
    std::vector<uint8_t> dist(N);
    std::vector<uint8_t> par(N);  // variable id whose removal leaves a minimal sum for v ^ var
    std::vector<uint16_t> var;    // variable id -> mask over the planes
    for (int b = 0; b < 16; b++) var.push_back(static_cast<uint16_t>(1u << b));
    for (int v = 0; v < N; v++) {
        dist[static_cast<size_t>(v)] = static_cast<uint8_t>(__builtin_popcount(static_cast<unsigned>(v)));
        par[static_cast<size_t>(v)] = static_cast<uint8_t>(v ? __builtin_ctz(static_cast<unsigned>(v)) : 0);
    }
    auto spell = [&](uint16_t v) {
        std::vector<int> ids;
        while (v) {
            const int e = par[v];
            ids.push_back(e);
            v = static_cast<uint16_t>(v ^ var[static_cast<size_t>(e)]);
        }
        return ids;
    };
    auto cost = [](int d) { return (d + 1) / 2; };
    std::vector<uint16_t> open;  // rows that a new variable could still make cheaper (dist >= 2)
    out.temps.clear();
    while (static_cast<int>(out.temps.size()) < cap) {
        open.clear();
        for (uint16_t t : rows)
            if (dist[t] >= 2) open.push_back(t);
        if (open.empty()) break;
        int best = 1, bc = -1;  // a temporary costs one op: it must save at least two
        for (int c = 1; c < N; c++) {
            const int dc = dist[static_cast<size_t>(c)];
            if (dc < 2 || dc > 3) continue;
            int g = 0;
            for (uint16_t t : open) {
                const int d = dist[t], d2 = dist[static_cast<size_t>(t ^ c)] + 1;
                if (d2 < d) g += cost(d) - cost(d2);
            }
            if (g > best) {
                best = g;
                bc = c;
            }
        }
        if (bc < 0) break;
        const std::vector<int> def = spell(static_cast<uint16_t>(bc));
        out.temps.push_back({def[0], def[1], def.size() > 2 ? def[2] : -1});
        const int id = static_cast<int>(var.size());
        var.push_back(static_cast<uint16_t>(bc));
        // v ^ bc then v: ascending v would read entries already updated in this pass, so use a copy
        const std::vector<uint8_t> old = dist;
        for (int v = 0; v < N; v++) {
            const int d2 = old[static_cast<size_t>(v ^ bc)] + 1;
            if (d2 < old[static_cast<size_t>(v)]) {
                dist[static_cast<size_t>(v)] = static_cast<uint8_t>(d2);
                par[static_cast<size_t>(v)] = static_cast<uint8_t>(id);
            }
        }
    }
    out.rows.clear();
    for (uint16_t t : rows) out.rows.push_back(spell(t));
}

}  // namespace

BitsliceNet bitslice_network(const std::vector<int>& coeff, int R, int K, int cap)
{
    BitsliceNet net;
    net.R = R;
    net.K = K;
    net.inputs.resize(static_cast<size_t>(K));
    for (int j = 0; j < K; j++) {
        std::vector<uint16_t> rows(static_cast<size_t>(R) * 16);
        for (int r = 0; r < R; r++) {
            uint16_t M[16];
            gf16_bitmatrix(coeff[static_cast<size_t>(r) * K + j], M);
            for (int p = 0; p < 16; p++) rows[static_cast<size_t>(r) * 16 + p] = M[p];
        }
        distance_network(rows, cap, net.inputs[static_cast<size_t>(j)]);
    }
    return net;
}

int BitsliceNet::xor_ops() const
{
    int ops = 0;
    for (const auto& in : inputs) {
        ops += static_cast<int>(in.temps.size());
        for (const auto& r : in.rows) ops += static_cast<int>((r.size() + 1) / 2);
    }
    return ops;
}

void bitslice_eval(const BitsliceNet& net, const uint16_t* in, uint16_t* out)
{
    std::vector<uint32_t> acc(static_cast<size_t>(net.R) * 16, 0u);
    for (int j = 0; j < net.K; j++) {
        const auto& inp = net.inputs[static_cast<size_t>(j)];
        std::vector<uint32_t> val(16, 0u);
        for (int w = 0; w < 32; w++)
            for (int b = 0; b < 16; b++)
                if ((in[j * 32 + w] >> b) & 1) val[static_cast<size_t>(b)] |= 1u << w;
        for (const auto& t : inp.temps)
            val.push_back(val[static_cast<size_t>(t[0])] ^ val[static_cast<size_t>(t[1])] ^
                          (t[2] < 0 ? 0u : val[static_cast<size_t>(t[2])]));
        for (size_t i = 0; i < inp.rows.size(); i++)
            for (int v : inp.rows[i]) acc[i] ^= val[static_cast<size_t>(v)];
    }
    for (int r = 0; r < net.R; r++)
        for (int w = 0; w < 32; w++) {
            uint16_t x = 0;
            for (int p = 0; p < 16; p++)
                if ((acc[static_cast<size_t>(r) * 16 + p] >> w) & 1) x = static_cast<uint16_t>(x | (1u << p));
            out[r * 32 + w] = x;
        }
}

namespace {

const char* kPrelude = R"HIP(
typedef unsigned int u32;
typedef int i32;
typedef long long i64;
typedef unsigned char u8;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
struct ecamd_bs_args {
    const u8* in_base;
    u8* out_base;
    i64 in_stride;
    i64 out_stride;
    const i32* stripe_list;
    u32 in_records;
    u32 out_records;
    u32 ntiles;
    u32 tiles_per_stripe;
    i32 in_off[32];
    i32 out_off[8];
    u8* copy_base;
    i64 copy_stride;
    u32 copy_records;
    u32 copy_step;
    u8 copy_idx[32];
    const u32* crc_img;
    u32* crc_partial;
    i32 crc_q;
    i32 crc_per;
    i32 crc_nfrag;
};
__device__ __forceinline__ u32 x3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ u32 x2(u32 a, u32 b)
{
    u32 r;
    asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ u32 bfi(u32 m, u32 x, u32 y)
{
    u32 r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(x), "v"(y));
    return r;
}
// realigned 16-byte window D bytes into the 32-byte pair (lo, the next aligned chunk): the next
// chunk is the neighbour lane's lo (DPP wave_shl:1); lane 63 has no neighbour and keeps `own`, the
// chunk it loaded itself (bound_ctrl off: an out-of-range source leaves the old value)
// lane 0's 16 bytes in every lane (v_readlane: the last lane's next chunk when it is the next
// 1 KiB chunk's first, one-wave tiles)
__device__ __forceinline__ v4u lane0(v4u x)
{
    return v4u{(u32)__builtin_amdgcn_readlane((int)x[0], 0), (u32)__builtin_amdgcn_readlane((int)x[1], 0),
               (u32)__builtin_amdgcn_readlane((int)x[2], 0), (u32)__builtin_amdgcn_readlane((int)x[3], 0)};
}
template <int D>
__device__ __forceinline__ v4u rlg(v4u lo, v4u own)
{
    u32 w[8] = {lo[0], lo[1], lo[2], lo[3], 0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 4; i++) w[4 + i] = (u32)__builtin_amdgcn_update_dpp((int)own[i], (int)lo[i], 0x130, 0xf, 0xf, false);
    constexpr int dw = D >> 2, by = D & 3;
    if constexpr (by == 0)
        return v4u{w[dw], w[dw + 1], w[dw + 2], w[dw + 3]};
    else
        return v4u{__builtin_amdgcn_alignbyte(w[dw + 1], w[dw], by), __builtin_amdgcn_alignbyte(w[dw + 2], w[dw + 1], by),
                   __builtin_amdgcn_alignbyte(w[dw + 3], w[dw + 2], by), __builtin_amdgcn_alignbyte(w[dw + 4], w[dw + 3], by)};
}
// 16x16 bit transpose inside each 16-bit half of 16 dwords (an involution): bytes by v_perm,
// then 4-, 2- and 1-bit blocks by shift + bit select.
__device__ __forceinline__ void tr16(u32 (&A)[16])
{
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const u32 a = A[k], b = A[k + 8];
        A[k] = __builtin_amdgcn_perm(a, b, 0x07030501u);
        A[k + 8] = __builtin_amdgcn_perm(a, b, 0x06020400u);
    }
#pragma unroll
    for (int j = 4, m = 0x0F0F0F0F; j; j >>= 1, m ^= m << j) {
#pragma unroll
        for (int k = 0; k < 16; k = (k + j + 1) & ~j) {
            const u32 a = A[k], b = A[k + j], mu = (u32)m;
            A[k] = bfi(mu, b >> j, a);
            A[k + j] = bfi(mu, b, a << j);
        }
    }
}
)HIP";

// The crc variant's device helpers -- the same algebra as hip/ecamd_crc_dev.hpp (GF(2)-linear maps
// of the 32-bit CRC state through field tables in LDS), restated for the stand-alone hiprtc source.
const char* kPreludeCrc = R"HIP(
template <int K>
__device__ __forceinline__ u32 bx4(u32 v)  // 4 * byte K of v, one SDWA op
{
    u32 r;
    if constexpr (K == 0)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(v));
    else if constexpr (K == 1)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(v));
    else if constexpr (K == 2)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(v));
    else
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(v));
    return r;
}
__device__ __forceinline__ u32 tab_at(const u32* t, u32 byteoff) { return *(const u32*)((const char*)t + byteoff); }
// nibble fields: table 2b for the low nibble of byte b, 2b+1 for the high one (16 words each)
__device__ __forceinline__ u32 lmap4(const u32* t, u32 x)
{
    const u32 lo = x & 0x0f0f0f0fu, hi = (x >> 4) & 0x0f0f0f0fu;
    const u32 a = x3(tab_at(t, bx4<0>(lo)), tab_at(t + 16, bx4<0>(hi)), tab_at(t + 32, bx4<1>(lo)));
    const u32 b = x3(tab_at(t + 48, bx4<1>(hi)), tab_at(t + 64, bx4<2>(lo)), tab_at(t + 80, bx4<2>(hi)));
    return x3(a, b, tab_at(t + 96, bx4<3>(lo)) ^ tab_at(t + 112, bx4<3>(hi)));
}
// byte fields: table b for byte b (256 words each)
__device__ __forceinline__ u32 lmap8(const u32* t, u32 x)
{
    return x3(tab_at(t, bx4<0>(x)), tab_at(t + 256, bx4<1>(x)), tab_at(t + 512, bx4<2>(x))) ^ tab_at(t + 768, bx4<3>(x));
}
// v through this lane's map A^(16 (63 - lane)): 8 nibble fields, lane-interleaved tables (word
// (t * 16 + n) * 64 + lane: conflict-free), lofs = 4 * lane
__device__ __forceinline__ u32 lane_shift(const u32* t, u32 v, u32 lofs)
{
    const u32 a = x3(tab_at(t, ((v & 15u) << 8) + lofs), tab_at(t + 1024, (((v >> 4) & 15u) << 8) + lofs),
                     tab_at(t + 2048, (((v >> 8) & 15u) << 8) + lofs));
    const u32 b = x3(tab_at(t + 3072, (((v >> 12) & 15u) << 8) + lofs), tab_at(t + 4096, (((v >> 16) & 15u) << 8) + lofs),
                     tab_at(t + 5120, (((v >> 20) & 15u) << 8) + lofs));
    return x3(a, b, tab_at(t + 6144, (((v >> 24) & 15u) << 8) + lofs) ^ tab_at(t + 7168, ((v >> 28) << 8) + lofs));
}
// XOR of v over the wave, in every lane (BitsliceStyle::dpp_reduce): DPP within each row of 16 (quad
// swaps, half-row and row mirrors), then the 4 rows' lane 0 by v_readlane -- no LDS instruction,
// where a ds_bpermute butterfly (__shfl_xor) takes 6 from the LDS the CRC lookups saturate
__device__ __forceinline__ u32 wave_xor(u32 v)
{
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);  // row_half_mirror
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);  // row_mirror
    return (u32)__builtin_amdgcn_readlane((int)v, 0) ^ (u32)__builtin_amdgcn_readlane((int)v, 16) ^
           (u32)__builtin_amdgcn_readlane((int)v, 32) ^ (u32)__builtin_amdgcn_readlane((int)v, 48);
}
// lane F of `held` := lane 0 of v (v_readlane into an SGPR, v_writelane back)
template <int F>
__device__ __forceinline__ u32 put_lane(u32 held, u32 v)
{
    const u32 w = __builtin_amdgcn_readlane(v, 0);
    asm("v_writelane_b32 %0, %1, %2" : "+v"(held) : "s"(w), "i"(F));
    return held;
}
// r0 of a 16-byte piece: dword w through the byte tables at tab + 1024 w
__device__ __forceinline__ u32 piece_r0(const u32* t, u32 a, u32 b, u32 c, u32 d)
{
    return x3(lmap8(t, a), lmap8(t + 1024, b), lmap8(t + 2048, c)) ^ lmap8(t + 3072, d);
}
// byte tables for the first MB dwords (tab + 1024 w), nibble tables for the rest (tab + 1024 MB + 128 (w - MB))
template <int MB>
__device__ __forceinline__ u32 piece_r0m(const u32* t, u32 a, u32 b, u32 c, u32 d)
{
    const u32* n = t + 1024 * MB;
    const u32 ra = lmap8(t, a);
    const u32 rb = MB > 1 ? lmap8(t + 1024, b) : lmap4(n, b);
    const u32 rc = MB > 2 ? lmap8(t + 2048, c) : lmap4(n + 128 * (2 - MB), c);
    const u32 rd = lmap4(n + 128 * (3 - MB), d);
    return x3(ra, rb, rc) ^ rd;
}
// byte tables, dword 3's read from global memory g (the vector L1 as a second lookup engine; same layout)
__device__ __forceinline__ u32 piece_r0g(const u32* t, const u32* g, u32 a, u32 b, u32 c, u32 d)
{
    const u32 rd = lmap8(g + 3072, d);
    return x3(lmap8(t, a), lmap8(t + 1024, b), lmap8(t + 2048, c)) ^ rd;
}
// the same through nibble tables: dword w's 8 fields at tab + 128 w (conflict-free 16-entry tables)
__device__ __forceinline__ u32 piece_r0n(const u32* t, u32 a, u32 b, u32 c, u32 d)
{
    return x3(lmap4(t, a), lmap4(t + 128, b), lmap4(t + 256, c)) ^ lmap4(t + 384, d);
}
)HIP";

}  // namespace

int bitslice_waves_per_simd(int R, bool crc) { return R <= 4 ? (crc ? 3 : 4) : 2; }


int bitslice_depth(int depth, int K)
{
    if (depth < 2) return 0;
    int d = depth >= 4 ? 4 : 2;
    while (d > 2 && d - 1 > K) d /= 2;  // prefetch reaches at most one tile ahead
    return d;
}

std::string bitslice_source(const BitsliceNet& net, int depth, BitsliceStyle style)
{
    const int D = bitslice_depth(depth, net.K);
    std::ostringstream s;
    s << "// generated by liberasurecode_amd bitslice_source: " << net.R << " outputs x " << net.K
      << " inputs, " << net.xor_ops() << " network ops per tile, "
      << (D ? "LDS ring of " + std::to_string(D) + " inputs per wave" : std::string("register loads")) << "\n";
    s << kPrelude;
    if (style.crc) s << kPreludeCrc;
    const int CW = style.crc ? std::clamp(style.crc_wave, 0, 16) : 0;  // one-wave crc form: waves per workgroup
    const int wpe = ((!style.crc || CW) && style.waves >= 1 && style.waves <= 8) ? style.waves
                                                                                : bitslice_waves_per_simd(net.R, style.crc);
    // one-wave tiles: the plain / copy-through register form, and the plain LDS-ring form
    const int T = CW ? 64 * CW
                  : (!style.crc && style.threads == 64) ? 64
                  : (!style.crc && !D && !style.copy_through && (style.threads == 128 || style.threads == 512))
                      ? style.threads
                      : 256;
    const int CS = T * 16;  // bytes between a lane's 4 chunks of one fragment
    const int TILE = T * 64;
    // amdgpu_waves_per_eu(min, max): min sets the register budget (512 / min VGPRs); max is an
    // occupancy CAP -- the compiler raises the kernel descriptor's VGPR count until no more than max
    // waves fit (max 2: 176 VGPRs whatever the code uses).  style.waves_max 0: max = min.
    const int wmax = style.waves_max > 0 ? std::max(style.waves_max, wpe) : wpe;
    // one-wave LDS ring with realigned inputs: the 16-byte window D bytes into the aligned pair (lo, hi)
    // read back from the ring (emitted for that form only)
    bool ring_shift = false;
    if (D && T == 64)
        for (int j = 0; j < net.K && j < static_cast<int>(style.in_shift.size()); j++)
            ring_shift = ring_shift || (style.in_shift[static_cast<size_t>(j)] & 15);
    if (ring_shift)
        s << "template <int D>\n__device__ __forceinline__ v4u rl2(v4u lo, v4u hi)\n{\n"
             "    const u32 w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};\n"
             "    constexpr int dw = D >> 2, by = D & 3;\n"
             "    if constexpr (by == 0)\n        return v4u{w[dw], w[dw + 1], w[dw + 2], w[dw + 3]};\n"
             "    else\n        return v4u{__builtin_amdgcn_alignbyte(w[dw + 1], w[dw], by), "
             "__builtin_amdgcn_alignbyte(w[dw + 2], w[dw + 1], by),\n"
             "                   __builtin_amdgcn_alignbyte(w[dw + 3], w[dw + 2], by), "
             "__builtin_amdgcn_alignbyte(w[dw + 4], w[dw + 3], by)};\n}\n";
    s << "extern \"C\" __global__ void __launch_bounds__(" << T << ") __attribute__((amdgpu_waves_per_eu(" << wpe << ", "
      << wmax << ")))\n"
         "ecamd_bs_kernel(ecamd_bs_args a)\n{\n";
    auto shift_of = [&](int j) {
        return j < static_cast<int>(style.in_shift.size()) ? (style.in_shift[static_cast<size_t>(j)] & 15) : 0;
    };
    bool any_shift = false;
    for (int j = 0; j < net.K; j++) any_shift = any_shift || shift_of(j) != 0;
    if (any_shift && !D) s << "    const bool l63 = (threadIdx.x & 63u) == 63u;\n";
    auto ref = [](int v) {
        char b[24];
        if (v < 16)
            std::snprintf(b, sizeof(b), "P[%d]", 15 - v);
        else
            std::snprintf(b, sizeof(b), "t%d", v);
        return std::string(b);
    };
    // The one-wave LDS-ring form accumulates single terms through an asm XOR too: with plain `^=` the
    // compiler re-associates the sum of a 1-output map over the inputs (a tree over all 20 inputs'
    // planes at K = 20: 256 VGPRs + scratch), which the ring's inline-asm reads leave it free to do.
    const bool opaque_xor = D != 0 && T == 64;
    // the network of input j on P[16] (bit planes), accumulated into acc
    auto network = [&](int j) {
        const auto& in = net.inputs[static_cast<size_t>(j)];
        s << "            tr16(P);\n";
        // each temporary is computed right before its first use, so it lives no longer than needed
        std::vector<char> done(in.temps.size(), 0);
        if (!style.lazy_temps)
            for (size_t i = 0; i < in.temps.size(); i++) {
                const auto& t = in.temps[i];
                done[i] = 1;
                if (t[2] < 0)
                    s << "            const u32 t" << 16 + i << " = " << ref(t[0]) << " ^ " << ref(t[1]) << ";\n";
                else
                    s << "            const u32 t" << 16 + i << " = x3(" << ref(t[0]) << ", " << ref(t[1]) << ", "
                      << ref(t[2]) << ");\n";
            }
        std::function<void(int)> need = [&](int v) {
            if (v < 16 || done[static_cast<size_t>(v - 16)]) return;
            const auto& t = in.temps[static_cast<size_t>(v - 16)];
            for (int u : t)
                if (u >= 0) need(u);
            done[static_cast<size_t>(v - 16)] = 1;
            if (t[2] < 0)
                s << "            const u32 t" << v << " = " << ref(t[0]) << " ^ " << ref(t[1]) << ";\n";
            else
                s << "            const u32 t" << v << " = x3(" << ref(t[0]) << ", " << ref(t[1]) << ", "
                  << ref(t[2]) << ");\n";
        };
        for (size_t i = 0; i < in.rows.size(); i++) {
            const auto& terms = in.rows[i];
            if (terms.empty()) continue;
            for (int v : terms) need(v);
            char dst[32];
            std::snprintf(dst, sizeof(dst), "acc[%zu][%zu]", i / 16, 15 - i % 16);
            size_t q = 0;
            for (; q + 1 < terms.size(); q += 2)
                s << "            " << dst << " = x3(" << dst << ", " << ref(terms[q]) << ", "
                  << ref(terms[q + 1]) << ");\n";
            if (q < terms.size()) {
                if (opaque_xor)  // an asm XOR: the compiler cannot re-associate the sum across inputs
                    s << "            " << dst << " = x2(" << dst << ", " << ref(terms[q]) << ");\n";
                else
                    s << "            " << dst << " ^= " << ref(terms[q]) << ";\n";
            }
        }
    };
    auto acc_init = [&]() {
        s << "        u32 acc[" << net.R << "][16];\n"
          << "#pragma unroll\n        for (int r = 0; r < " << net.R
          << "; r++)\n#pragma unroll\n            for (int p = 0; p < 16; p++) acc[r][p] = 0u;\n";
    };
    auto outputs = [&](const char* rout, const char* off) {
        s << "#pragma unroll\n        for (int r = 0; r < " << net.R
          << "; r++) {\n"
             "            tr16(acc[r]);\n"
             "#pragma unroll\n"
             "            for (int c = 0; c < 4; c++) {\n"
             "                const v4u v = {acc[r][4 * c], acc[r][4 * c + 1], acc[r][4 * c + 2], acc[r][4 * c + 3]};\n"
             "                __builtin_amdgcn_raw_buffer_store_b128(v, "
          << rout << ", a.out_off[r] + " << off
          << " + c * " << CS << ", 0, 2);\n"
             "            }\n"
             "        }\n";
    };
    if (CW) {
        // crc variant in one-wave tiles: every wave of a workgroup streams 4 KiB tiles on its own -- lane
        // l's 4 pieces of a fragment at l*16 + c*1024 -- and the workgroup shares one copy of the tables.
        // Piece c goes through position set c % NP (r0 shifted by A^(1024 (NP - 1 - c % NP)) to the
        // group's last chunk), so a fragment's 4 pieces take 4 / NP - 1 gap steps (A^(1024 NP)); the
        // lane-shift tables move each lane's sum to the tile end, an XOR reduction over the wave gives r0
        // of the fragment's 4 KiB, parked in lane f of `held`, and one store per tile writes the K + R
        // values (crc_partial[t * (K + R) + f]).  The first crc_q workgroups' waves take tiles (b * crc_per
        // + i) * CW + wave, i < crc_per, the later ones one tile each (consecutive waves on neighbouring
        // tiles); no barrier after the table fill.
        const int NS = net.K + net.R;
        const int NP = style.crc_pos >= 4 ? 4 : style.crc_pos >= 2 ? 2 : 1;
        const int MB = std::clamp(style.crc_mb, 1, 4);  // piece dwords on byte tables
        const int PW = MB * 1024 + (4 - MB) * 128;        // piece-table words per position set
        const int maps = NP * PW;                         // gap, levels, A^1024, then the lane tables
        const int words = maps + 8 * 128 + kBsCrcLaneWords;
        constexpr int CS1 = kBsCrcWaveStep;
        const std::string pfn = MB == 4 ? std::string(style.crc_l1 ? "piece_r0g" : "piece_r0")
                                        : "piece_r0m<" + std::to_string(MB) + ">";
        // crc_l1: dword 3's byte tables read from the image in global memory (gimg, same offsets as ctab)
        const std::string gext = MB == 4 && style.crc_l1 ? "gimg + " : "";
        auto crc1 = [&](int f, const char* x) {
            s << "            {\n";
            for (int c0 = 0; c0 < 4; c0 += NP) {
                s << "                " << (c0 ? "cs = lmap4(gap, cs)" : "u32 cs = 0u");
                for (int c = c0; c < c0 + NP; c++)
                    s << " ^ " << pfn << "(ctab + " << (c % NP) * PW << ", "
                      << (gext.empty() ? std::string() : gext + std::to_string((c % NP) * PW) + ", ") << x << c << "[0], "
                      << x << c << "[1], " << x << c << "[2], " << x << c << "[3])";
                s << ";\n";
            }
            s << "                cs = wave_xor(lane_shift(lanes, cs, lofs));\n"
              << "                held = put_lane<" << f << ">(held, cs);\n"
              << "            }\n";
        };
        s << "    __shared__ __attribute__((aligned(16))) u32 ctab[" << words << "];\n"
          << "    for (int i = (int)threadIdx.x * 4; i < " << words << "; i += " << 4 * T
          << ") *(v4u*)(ctab + i) = *(const v4u*)(a.crc_img + i);\n"
             "    __syncthreads();\n"
             "    const u32* gap = ctab + "
          << maps
          << ";\n"
             "    const u32* lanes = ctab + "
          << maps + 8 * 128
          << ";\n"
             "    const u32 lane = threadIdx.x & 63u;\n"
             "    const u32 lofs = lane * 4u;\n"
             "    const u32* gimg = a.crc_img;\n"
             "    const u32 wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
             // the first crc_q workgroups take crc_per tiles per wave, the rest one: long runs (one
             // table fill each) first, single tiles for an even finish
             "    const u32 big = (u32)a.crc_q, per = (u32)a.crc_per;\n"
             "    const u32 nper = blockIdx.x < big ? per : 1u;\n"
             "    const u32 t0 = (blockIdx.x < big ? blockIdx.x * per : big * per + (blockIdx.x - big)) * "
          << CW
          << "u + wv;\n"
             "    for (u32 i = 0; i < nper; i++) {\n"
             "        const u32 t = t0 + i * "
          << CW
          << "u;\n"
             "        if (t >= a.ntiles) break;\n"
             "        const u32 s = t / a.tiles_per_stripe;\n"
             "        const i32 off = (i32)(t - s * a.tiles_per_stripe) * "
          << kBsTileWave
          << " + (i32)lane * 16;\n"
             "        const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.in_base + (i64)s * a.in_stride), 0, (int)a.in_records, 0x00020000);\n"
             "        const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.out_base + (i64)s * a.out_stride), 0, (int)a.out_records, 0x00020000);\n"
             "        const __amdgpu_buffer_rsrc_t rcopy = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.copy_base + (i64)s * a.copy_stride), 0, (int)a.copy_records, 0x00020000);\n";
        for (int j = 0; j < net.K; j++)
            s << "        const i32 cofs" << j << " = a.copy_idx[" << j << "] == 0xff ? (i32)0x80000000u : (i32)(a.copy_idx["
              << j << "] * a.copy_step);\n";
        acc_init();
        s << "        u32 held = 0u;\n";
        // prefetch (style.prefetch 2 / 4): the next unrealigned input's first PFc chunks are loaded with
        // this input's, before its copy stores, CRC lookups and network; 3: all 4 chunks of the input
        // two ahead (PD = 2 register sets)
        const int PD = style.prefetch == 3 ? 2 : 1;
        const int PFc = style.prefetch == 3 ? 4 : (style.prefetch == 2 || style.prefetch == 4) ? style.prefetch : 0;
        auto cpre = [&](int j) { return PFc > 0 && j < net.K && shift_of(j) == 0; };
        auto cload_next = [&](int j) {
            for (int c = 0; c < PFc; c++)
                s << "            xn" << j % PD << "[" << c << "] = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" << j
                  << "] + off + " << c * CS1 << ", 0, 2);\n";
        };
        if (PFc) {
            for (int q = 0; q < PD; q++) s << "        v4u xn" << q << "[" << PFc << "];\n";
            for (int q = 0; q < PD; q++)
                if (cpre(q)) cload_next(q);
        }
        for (int j = 0; j < net.K; j++) {
            s << "        {  // input " << j << "\n            u32 P[16];\n";
            if (const int d = shift_of(j)) {  // aligned chunk + the neighbour's, realigned
                for (int c = 0; c < 4; c++)
                    s << "            const v4u xa" << c << " = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" << j
                      << "] - " << d << " + off + " << c * CS1 << ", 0, 2);\n";
                for (int c = 0; c < 4; c++)
                    s << "            const v4u xh" << c << " = __builtin_amdgcn_raw_buffer_load_b128(rin, l63 ? a.in_off[" << j
                      << "] - " << d << " + off + " << c * CS1 + 16 << " : (i32)0x80000000u, 0, 2);\n";
                for (int c = 0; c < 4; c++)
                    s << "            const v4u xq" << c << " = rlg<" << d << ">(xa" << c << ", xh" << c << ");\n";
            } else {
                for (int c = 0; c < 4; c++) {
                    if (cpre(j) && c < PFc)
                        s << "            const v4u xq" << c << " = xn" << j % PD << "[" << c << "];\n";
                    else
                        s << "            const v4u xq" << c << " = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" << j
                          << "] + off + " << c * CS1 << ", 0, 2);\n";
                }
            }
            if (cpre(j + PD)) cload_next(j + PD);
            // the 4 loads leave together (without the barrier the compiler consumes the first two
            // before issuing the rest, and each wait then also retires the previous copy stores)
            s << "            __builtin_amdgcn_sched_barrier(0);\n";
            for (int c = 0; c < 4; c++)
                s << "            __builtin_amdgcn_raw_buffer_store_b128(xq" << c << ", rcopy, cofs" << j << " + off + "
                  << c * CS1 << ", 0, 2);  // copy-through\n";
            crc1(j, "xq");
            for (int c = 0; c < 4; c++)
                s << "            P[" << 4 * c << "] = xq" << c << "[0]; P[" << 4 * c + 1 << "] = xq" << c << "[1]; P["
                  << 4 * c + 2 << "] = xq" << c << "[2]; P[" << 4 * c + 3 << "] = xq" << c << "[3];\n";
            if (!style.crc_mix) s << "            __builtin_amdgcn_sched_barrier(0);\n";
            network(j);
            if (style.input_barrier) s << "            __builtin_amdgcn_sched_barrier(0);\n";
            s << "        }\n";
        }
        for (int r = 0; r < net.R; r++) {
            s << "        {  // output " << r << "\n            tr16(acc[" << r << "]);\n";
            for (int c = 0; c < 4; c++)
                s << "            const v4u vq" << c << " = {acc[" << r << "][" << 4 * c << "], acc[" << r << "][" << 4 * c + 1
                  << "], acc[" << r << "][" << 4 * c + 2 << "], acc[" << r << "][" << 4 * c + 3 << "]};\n"
                  << "            __builtin_amdgcn_raw_buffer_store_b128(vq" << c << ", rout, a.out_off[" << r << "] + off + "
                  << c * CS1 << ", 0, 2);\n";
            crc1(net.K + r, "vq");
            s << "        }\n";
        }
        s << "        if (lane < " << NS << "u) a.crc_partial[(i64)t * " << NS << " + lane] = held;\n"
             "    }\n"
             "}\n";
        return s.str();
    }
    if (style.crc) {
        // Work unit u = (stripe, range of crc_per consecutive tiles).  Lane l's pieces of one fragment
        // sit at tile*16384 + c*4096 + l*16, c = 0..3: consecutive pieces are 4096 bytes apart across
        // tile boundaries too, so each lane state steps s = A^4096 s ^ r0(piece) (gap map).  At the
        // end of the unit a 6-level shuffle butterfly folds each wave (1 KiB segments of every 4 KiB
        // block), the 4 waves meet in LDS and Horner with A^1024 gives r0 of the range.
        // More than 4 outputs (fold_each): the network leaves no registers for a state per fragment,
        // so a unit is one tile and each fragment's 4 pieces are folded (butterfly, wave value into
        // LDS) right after they are checksummed; only the 4-wave combine waits for the tile's end.
        const bool fold_each = net.R > 4;
        const bool lane_fold = fold_each || style.crc_lane;
        const int NS = net.K + net.R;
        const int NP = style.crc_pos >= 4 ? 4 : style.crc_pos >= 2 ? 2 : 1;
        const int words = bs_crc_words(NP, style.crc_nib);
        const int pw = style.crc_nib ? 512 : 4096;  // piece-table words per position set
        const char* pfn = style.crc_nib ? "piece_r0n" : "piece_r0";
        // the CRC of 4 pieces x0..x3 (4096 bytes apart) of fragment f: NP pieces per gap step, piece c
        // through position set c % NP
        auto crc4 = [&](const std::string& f, const char* x) {
            const std::string sv = fold_each ? std::string("cs") : "st[" + f + "]";
            if (fold_each) s << "            u32 cs;\n";
            for (int c0 = 0; c0 < 4; c0 += NP) {
                if (fold_each && c0 == 0)
                    s << "            cs = 0u";  // a fresh state: no gap step before the first pieces
                else
                    s << "            " << sv << " = lmap4(gap, " << sv << ")";
                for (int c = c0; c < c0 + NP; c++)
                    s << " ^ " << pfn << "(ctab + " << (c % NP) * pw << ", " << x << c << "[0], " << x << c << "[1], "
                      << x << c << "[2], " << x << c << "[3])";
                s << ";\n";
            }
            if (fold_each)  // each lane's state shifted to the segment end, then an XOR reduction
                s << "            cs = lane_shift(lanes, cs, lofs);\n"
                  << (style.dpp_reduce ? "            cs = wave_xor(cs);\n"
                                       : "#pragma unroll\n"
                                         "            for (int l = 0; l < 6; l++) cs ^= __shfl_xor(cs, 1 << l, 64);\n")
                  // lane f of `held` keeps fragment f's wave value: no branch inside the network code
                  << "            held = put_lane<" << f << ">(held, cs);\n";
        };
        const int lds_words = words + (lane_fold ? kBsCrcLaneWords : 0);
        s << "    __shared__ u32 ctab[" << lds_words << "];\n"
          << "    __shared__ u32 xch[4 * " << NS << "];\n"
          << "    for (int i = threadIdx.x; i < " << lds_words << "; i += 256) ctab[i] = a.crc_img[i];\n"
          << "    __syncthreads();\n"
          << "    const u32* gap = ctab + " << NP * pw << ";\n"
             "    const u32* level = gap + 128;\n"
             "    const u32* a1024 = level + 6 * 128;\n"
             "    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;\n";
        if (lane_fold)
            s << "    const u32* lanes = ctab + " << words << ";\n"
                 "    const u32 lofs = (u32)lane * 4u;\n";
        s << "    const u32 units = a.ntiles / a.tiles_per_stripe * (u32)a.crc_q;\n"
             "    for (u32 u = blockIdx.x; u < units; u += gridDim.x) {\n"
             "        const u32 s = u / (u32)a.crc_q;\n"
             "        const u32 rg = u - s * (u32)a.crc_q;\n"
             "        const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.in_base + (i64)s * a.in_stride), 0, (int)a.in_records, 0x00020000);\n"
             "        const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.out_base + (i64)s * a.out_stride), 0, (int)a.out_records, 0x00020000);\n"
             "        const __amdgpu_buffer_rsrc_t rcopy = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.copy_base + (i64)s * a.copy_stride), 0, (int)a.copy_records, 0x00020000);\n";
        for (int j = 0; j < net.K; j++)
            s << "        const i32 cofs" << j << " = a.copy_idx[" << j << "] == 0xff ? (i32)0x80000000u : (i32)(a.copy_idx["
              << j << "] * a.copy_step);\n";
        if (!fold_each)
            s << "        u32 st[" << NS << "];\n"
              << "#pragma unroll\n        for (int f = 0; f < " << NS << "; f++) st[f] = 0u;\n";
        if (fold_each) s << "        u32 held = 0u;\n";
        s << "        for (i32 t = (i32)rg * a.crc_per; t < (i32)(rg + 1) * a.crc_per; t++) {\n"
          << "        const i32 off = t * " << kBsTile << " + (i32)threadIdx.x * 16;\n";
        acc_init();
        // prefetch (style.prefetch): the next unrealigned input's first PFc chunks go out before this
        // input's copy stores (vmcnt retires in issue order: its loads then do not wait for the stores)
        const int PFc = (style.prefetch == 2 || style.prefetch == 4) ? style.prefetch : 0;
        auto cpre = [&](int j) { return PFc > 0 && j < net.K && shift_of(j) == 0; };
        auto cload_next = [&](int j) {
            for (int c = 0; c < PFc; c++)
                s << "            xn[" << c << "] = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" << j << "] + off + "
                  << c * 4096 << ", 0, 2);\n";
        };
        if (PFc) {
            s << "        v4u xn[" << PFc << "];\n";
            if (cpre(0)) cload_next(0);
        }
        for (int j = 0; j < net.K; j++) {
            s << "        {  // input " << j << "\n            u32 P[16];\n";
            if (const int d = shift_of(j)) {  // aligned chunk + the neighbour's, realigned
                for (int c = 0; c < 4; c++)
                    s << "            const v4u xa" << c << " = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" << j
                      << "] - " << d << " + off + " << c * 4096 << ", 0, 2);\n";
                for (int c = 0; c < 4; c++)
                    s << "            const v4u xh" << c << " = __builtin_amdgcn_raw_buffer_load_b128(rin, l63 ? a.in_off[" << j
                      << "] - " << d << " + off + " << c * 4096 + 16 << " : (i32)0x80000000u, 0, 2);\n";
                for (int c = 0; c < 4; c++)
                    s << "            const v4u xq" << c << " = rlg<" << d << ">(xa" << c << ", xh" << c << ");\n";
            } else {
                for (int c = 0; c < 4; c++) {
                    if (cpre(j) && c < PFc)
                        s << "            const v4u xq" << c << " = xn[" << c << "];\n";
                    else
                        s << "            const v4u xq" << c << " = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" << j
                          << "] + off + " << c * 4096 << ", 0, 2);\n";
                }
            }
            if (cpre(j + 1)) cload_next(j + 1);
            for (int c = 0; c < 4; c++)
                s << "            __builtin_amdgcn_raw_buffer_store_b128(xq" << c << ", rcopy, cofs" << j << " + off + "
                  << c * 4096 << ", 0, 2);  // copy-through\n";
            crc4(std::to_string(j), "xq");
            for (int c = 0; c < 4; c++)
                s << "            P[" << 4 * c << "] = xq" << c << "[0]; P[" << 4 * c + 1 << "] = xq" << c << "[1]; P["
                  << 4 * c + 2 << "] = xq" << c << "[2]; P[" << 4 * c + 3 << "] = xq" << c << "[3];\n";
            s << "            __builtin_amdgcn_sched_barrier(0);\n";
            network(j);
            s << "        }\n";
        }
        for (int r = 0; r < net.R; r++) {
            s << "        {  // output " << r << "\n            tr16(acc[" << r << "]);\n";
            for (int c = 0; c < 4; c++)
                s << "            const v4u vq" << c << " = {acc[" << r << "][" << 4 * c << "], acc[" << r << "][" << 4 * c + 1
                  << "], acc[" << r << "][" << 4 * c + 2 << "], acc[" << r << "][" << 4 * c + 3 << "]};\n"
                  << "            __builtin_amdgcn_raw_buffer_store_b128(vq" << c << ", rout, a.out_off[" << r << "] + off + "
                  << c * 4096 << ", 0, 2);\n";
            crc4(std::to_string(net.K + r), "vq");
            s << "        }\n";
        }
        s << "        }\n";  // tiles of the unit (one when fold_each: the host sets crc_per = 1)
        if (fold_each)
            s << "        if (lane < " << NS << ") xch[wave * " << NS << " + lane] = held;\n";
        else if (lane_fold)
            s << "#pragma unroll\n"
                 "        for (int f = 0; f < " << NS << "; f++) {\n"
                 "            u32 x = lane_shift(lanes, st[f], lofs);\n"
              << (style.dpp_reduce ? "            x = wave_xor(x);\n"
                                   : "#pragma unroll\n"
                                     "            for (int l = 0; l < 6; l++) x ^= __shfl_xor(x, 1 << l, 64);\n")
              << "            if (lane == 0) xch[wave * " << NS << " + f] = x;\n"
                 "        }\n";
        else
            s << "#pragma unroll\n"
                 "        for (int f = 0; f < " << NS << "; f++) {\n"
                 "            u32 x = st[f];\n"
                 "#pragma unroll\n"
                 "            for (int l = 0; l < 6; l++) x = lmap4(level + 128 * l, x) ^ __shfl_down(x, 1 << l, 64);\n"
                 "            if (lane == 0) xch[wave * " << NS << " + f] = x;\n"
                 "        }\n";
        s << "        __syncthreads();\n"
             "        if ((int)threadIdx.x < " << NS << ") {\n"
             "            const int f = threadIdx.x;\n"
             "            u32 v = 0u;\n"
             "            for (int w = 0; w < 4; w++) v = lmap4(a1024, v) ^ xch[w * " << NS << " + f];\n"
             "            a.crc_partial[((i64)s * a.crc_nfrag + f) * a.crc_q + rg] = v;\n"
             "        }\n"
             "        __syncthreads();\n"
             "    }\n}\n";
        return s.str();
    }
    if (!D) {
        s << "    for (u32 t = blockIdx.x; t < a.ntiles; t += gridDim.x) {\n"
             "        const u32 sl = t / a.tiles_per_stripe;\n"
             "        const u32 s = a.stripe_list ? (u32)a.stripe_list[sl] : sl;\n"
             "        const i32 off = (i32)(t - sl * a.tiles_per_stripe) * "
          << TILE
          << " + (i32)threadIdx.x * 16;\n"
             "        const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.in_base + (i64)s * a.in_stride), 0, (int)a.in_records, 0x00020000);\n"
             "        const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.out_base + (i64)s * a.out_stride), 0, (int)a.out_records, 0x00020000);\n"
             ;
        if (style.copy_through) {
            // straight-line copy stores (a branch per input breaks the register allocation of the
            // network): a skipped input gets an out-of-range offset, which the buffer unit drops
            s << "        const __amdgpu_buffer_rsrc_t rcopy = __builtin_amdgcn_make_buffer_rsrc(\n"
                 "            (void*)(a.copy_base + (i64)s * a.copy_stride), 0, (int)a.copy_records, 0x00020000);\n";
            for (int j = 0; j < net.K; j++)
                s << "        const i32 cofs" << j << " = a.copy_idx[" << j << "] == 0xff ? (i32)0x80000000u : (i32)(a.copy_idx["
                  << j << "] * a.copy_step);\n";
        }
        acc_init();
        // prefetch (one-wave form): the first PF chunks of input j + 1 are loaded into xn[] before
        // input j's network (not for realigned inputs, which take their loads at their turn)
        const int PF = (T == 64 && (style.prefetch == 2 || style.prefetch == 4)) ? style.prefetch : 0;
        // (realigned inputs: their aligned chunks into xn[], the last lane's next ones into xnh[])
        auto pre = [&](int j) { return PF > 0 && j < net.K; };
        // (style.realign_lane: the last lane's next chunk of chunks 0-2 by v_readlane, T = 64 only)
        const bool rl = style.realign_lane && T == 64;
        auto load_next = [&](int j) {
            const int d = shift_of(j);
            s << "#pragma unroll\n            for (int c = 0; c < " << PF << "; c++) xn[c] = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off["
              << j << "]" << (d ? " - " + std::to_string(d) : std::string()) << " + off + c * " << CS << ", 0, 2);\n";
            if (d && (!rl || PF > 3))
                s << "#pragma unroll\n            for (int c = " << (rl ? 3 : 0) << "; c < " << PF
                  << "; c++) xnh[c] = __builtin_amdgcn_raw_buffer_load_b128(rin, l63 ? a.in_off[" << j << "] - " << d
                  << " + off + c * " << CS << " + 16 : (i32)0x80000000u, 0, 2);\n";
        };
        if (PF) {
            s << "        v4u xn[" << PF << "];\n";
            if (any_shift) s << "        v4u xnh[" << PF << "];\n";
            if (pre(0)) load_next(0);
        }
        // late copy (style.prefetch 1, copy-through, no realigned inputs): input j's copy stores go out
        // AFTER its network and after input j + 1's loads, from the planes transposed back (tr16 is an
        // involution; the network leaves P as it found it), so the next loads never wait for them
        // (vmcnt retires in issue order) and no register outlives the network
        if (style.prefetch == 1 && style.copy_through && !any_shift) {
            auto ld4 = [&](int j) {
                s << "#pragma unroll\n        for (int c = 0; c < 4; c++) xl[c] = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off["
                  << j << "] + off + c * " << CS << ", 0, 2);\n";
            };
            s << "        v4u xl[4];\n";
            ld4(0);
            for (int j = 0; j < net.K; j++) {
                s << "        {  // input " << j << "\n            u32 P[16];\n"
                  << "#pragma unroll\n            for (int c = 0; c < 4; c++) {\n"
                  << "                P[4 * c] = xl[c][0]; P[4 * c + 1] = xl[c][1]; P[4 * c + 2] = xl[c][2]; P[4 * c + 3] = xl[c][3];\n"
                  << "            }\n";
                network(j);
                if (j + 1 < net.K) ld4(j + 1);
                s << "            tr16(P);  // back to the input's own layout\n"
                  << "#pragma unroll\n            for (int c = 0; c < 4; c++) {\n"
                  << "                const v4u x = {P[4 * c], P[4 * c + 1], P[4 * c + 2], P[4 * c + 3]};\n"
                  << "                __builtin_amdgcn_raw_buffer_store_b128(x, rcopy, cofs" << j << " + off + c * " << CS
                  << ", 0, 2);  // copy-through\n"
                  << "            }\n"
                  << "            __builtin_amdgcn_sched_barrier(0);\n"
                  << "        }\n";
            }
            outputs("rout", "off");
            s << "    }\n}\n";
            return s.str();
        }
        for (int j = 0; j < net.K; j++) {
            s << "        {  // input " << j << "\n            u32 P[16];\n";
            const int d = shift_of(j);
            if (d) {  // aligned chunks + the neighbours', realigned (BitsliceStyle::in_shift)
                const std::string la = "__builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" + std::to_string(j) + "] - " +
                                       std::to_string(d) + " + off + c * " + std::to_string(CS) + ", 0, 2)";
                const std::string lh = "__builtin_amdgcn_raw_buffer_load_b128(rin, l63 ? a.in_off[" + std::to_string(j) +
                                       "] - " + std::to_string(d) + " + off + c * " + std::to_string(CS) +
                                       " + 16 : (i32)0x80000000u, 0, 2)";
                const std::string pfs = std::to_string(PF);
                s << "            v4u xa[4], xh[4];\n";
                if (pre(j))
                    s << "#pragma unroll\n            for (int c = 0; c < 4; c++) xa[c] = c < " << pfs << " ? xn[c < " << pfs
                      << " ? c : 0] : " << la << ";\n"
                      << "#pragma unroll\n            for (int c = " << (rl ? 3 : 0) << "; c < 4; c++) xh[c] = c < " << pfs
                      << " ? xnh[c < " << pfs << " ? c : 0] : " << lh << ";\n";
                else
                    s << "#pragma unroll\n            for (int c = 0; c < 4; c++) xa[c] = " << la << ";\n"
                      << "#pragma unroll\n            for (int c = " << (rl ? 3 : 0) << "; c < 4; c++) xh[c] = " << lh << ";\n";
                if (rl) s << "#pragma unroll\n            for (int c = 0; c < 3; c++) xh[c] = lane0(xa[c + 1]);\n";
            }
            const std::string ld = "__builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" + std::to_string(j) +
                                   "] + off + c * " + std::to_string(CS) + ", 0, 2)";
            const std::string cst = "__builtin_amdgcn_raw_buffer_store_b128(x, rcopy, cofs" + std::to_string(j) +
                                    " + off + c * " + std::to_string(CS) + ", 0, 2);  // copy-through\n";
            if (PF && pre(j + 1) && style.copy_through) {
                // the next input's loads go out BEFORE this input's copy stores: vmcnt retires memory
                // operations in issue order, so waiting for those loads then does not wait for the stores
                s << "            v4u xc[4];\n#pragma unroll\n            for (int c = 0; c < 4; c++) {\n"
                  << (d ? "                xc[c] = rlg<" + std::to_string(d) + ">(xa[c], xh[c]);\n"
                        : pre(j) ? "                xc[c] = c < " + std::to_string(PF) + " ? xn[c < " + std::to_string(PF) +
                                       " ? c : 0] : " + ld + ";\n"
                                 : "                xc[c] = " + ld + ";\n")
                  << "                P[4 * c] = xc[c][0]; P[4 * c + 1] = xc[c][1]; P[4 * c + 2] = xc[c][2]; P[4 * c + 3] = xc[c][3];\n"
                  << "            }\n";
                load_next(j + 1);
                s << "#pragma unroll\n            for (int c = 0; c < 4; c++) {\n                const v4u x = xc[c];\n"
                  << "                " << cst << "            }\n";
            } else {
                s << "#pragma unroll\n            for (int c = 0; c < 4; c++) {\n"
                  << (d ? "                const v4u x = rlg<" + std::to_string(d) + ">(xa[c], xh[c]);\n"
                        : pre(j) ? "                const v4u x = c < " + std::to_string(PF) + " ? xn[c < " + std::to_string(PF) +
                                       " ? c : 0] : " + ld + ";\n"
                                 : "                const v4u x = " + ld + ";\n")
                  << "                P[4 * c] = x[0]; P[4 * c + 1] = x[1]; P[4 * c + 2] = x[2]; P[4 * c + 3] = x[3];\n"
                  << (style.copy_through ? "                " + cst : std::string())
                  << "            }\n";
                if (pre(j + 1)) load_next(j + 1);  // the next input's loads go out before this network
            }
            if (style.copy_through || pre(j + 1))
                s << "            __builtin_amdgcn_sched_barrier(0);  // loads / stores leave before the network\n";
            network(j);
            if (style.input_barrier) s << "            __builtin_amdgcn_sched_barrier(0);\n";
            s << "        }\n";
        }
        outputs("rout", "off");
        s << "    }\n}\n";
        return s.str();
    }
    if (T == 64) {
        // One-wave LDS ring: the wave streams the 4 KiB of each input of its tile (4 chunks of 1 KiB, one
        // LDS-DMA load each: lane l's 16 bytes land at slot + c*1024 + l*16) into a ring of D slots,
        // D - 1 inputs ahead of the network, so the next input's loads are in flight while the current
        // network runs -- without the 16 VGPRs per input a register prefetch holds across it.  The
        // code is straight-line per tile, so each wait is exact: before input j's reads, the vector-
        // memory operations issued after its last load may still be outstanding (vmcnt retires in
        // issue order; the previous tile's output stores, issued earlier, are retired by the same
        // wait).  A slot is refilled only after the reads of its previous input returned (lgkmcnt(0)
        // before each network).
        // Copy-through (framed encode / decode-join): each input's 4 chunks are stored to its copy
        // slot from the registers read back.  Realigned inputs (in_shift d != 0): the slot holds the
        // ALIGNED 4 KiB under the tile's windows plus the 16 bytes after it (one more load, by lane 0
        // only -- the other lanes' offsets are out of range and land zeros in the slot's 1 KiB pad);
        // lane l reads the aligned pair at l*16 and l*16 + 16 of each chunk and realigns it (rl2<d>).
        const int SLOT = ring_shift ? 5120 : 4096;
        s << "    __shared__ __attribute__((aligned(16))) u8 ring[" << D << " * " << SLOT << "];\n"
             "    typedef __attribute__((address_space(3))) u8 lds_u8;\n"
             "    const u32 wring = (u32)(unsigned long)(lds_u8*)ring;\n"
             "    const u32 lane = threadIdx.x * 16u;\n"
             "    for (u32 t = blockIdx.x; t < a.ntiles; t += gridDim.x) {\n"
             "        const u32 sl = t / a.tiles_per_stripe;\n"
             "        const u32 s = a.stripe_list ? (u32)a.stripe_list[sl] : sl;\n"
             "        const i32 off = (i32)(t - sl * a.tiles_per_stripe) * "
          << kBsTileWave
          << " + (i32)threadIdx.x * 16;\n"
             "        const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.in_base + (i64)s * a.in_stride), 0, (int)a.in_records, 0x00020000);\n"
             "        const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(\n"
             "            (void*)(a.out_base + (i64)s * a.out_stride), 0, (int)a.out_records, 0x00020000);\n";
        if (style.copy_through) {
            s << "        const __amdgpu_buffer_rsrc_t rcopy = __builtin_amdgcn_make_buffer_rsrc(\n"
                 "            (void*)(a.copy_base + (i64)s * a.copy_stride), 0, (int)a.copy_records, 0x00020000);\n";
            for (int j = 0; j < net.K; j++)
                s << "        const i32 cofs" << j << " = a.copy_idx[" << j << "] == 0xff ? (i32)0x80000000u : (i32)(a.copy_idx["
                  << j << "] * a.copy_step);\n";
        }
        // vector-memory operations of one tile in issue order: the input a load belongs to, -1 a store
        std::vector<int> vmem;
        // (the chunk's byte offset goes into the scalar offset: the instruction's immediate offset
        // would move the LDS destination too)
        auto issue1 = [&](int j) {
            const int d = shift_of(j);
            const std::string base = "a.in_off[" + std::to_string(j) + "]" + (d ? " - " + std::to_string(d) : std::string());
            for (int c = 0; c < 4; c++) {
                s << "        __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (__attribute__((address_space(3))) void*)(unsigned "
                     "long)(wring + "
                  << (j % D) * SLOT + c * 1024 << "u), 16, off, " << base << " + " << c * 1024 << ", 0, 2);\n";
                vmem.push_back(j);
            }
            if (d) {
                s << "        __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (__attribute__((address_space(3))) void*)(unsigned "
                     "long)(wring + "
                  << (j % D) * SLOT + 4096 << "u), 16, threadIdx.x == 0u ? off + " << base
                  << " + 4096 : (i32)0x80000000u, 0, 0, 2);\n";
                vmem.push_back(j);
            }
        };
        auto pending_after = [&](int j) {  // operations issued after input j's last load
            int n = 0;
            for (size_t i = vmem.size(); i-- > 0 && vmem[i] != j;) n++;
            return n;
        };
        acc_init();
        for (int q = 0; q < D - 1 && q < net.K; q++) issue1(q);
        for (int j = 0; j < net.K; j++) {
            const int d = shift_of(j);
            s << "        {  // input " << j << "\n";
            if (j + D - 1 < net.K) issue1(j + D - 1);
            s << "            asm volatile(\"s_waitcnt vmcnt(" << std::min(pending_after(j), 63) << ")\" ::: \"memory\");\n"
              << "            const u32 rd = wring + " << (j % D) * SLOT << "u + lane;\n"
              << "            v4u q0, q1, q2, q3;\n"
              << "            asm volatile(\"ds_read_b128 %0, %1\" : \"=v\"(q0) : \"v\"(rd) : \"memory\");\n"
              << "            asm volatile(\"ds_read_b128 %0, %1 offset:1024\" : \"=v\"(q1) : \"v\"(rd) : \"memory\");\n"
              << "            asm volatile(\"ds_read_b128 %0, %1 offset:2048\" : \"=v\"(q2) : \"v\"(rd) : \"memory\");\n"
              << "            asm volatile(\"ds_read_b128 %0, %1 offset:3072\" : \"=v\"(q3) : \"v\"(rd) : \"memory\");\n";
            if (d)
                s << "            v4u h0, h1, h2, h3;\n"
                  << "            asm volatile(\"ds_read_b128 %0, %1 offset:16\" : \"=v\"(h0) : \"v\"(rd) : \"memory\");\n"
                  << "            asm volatile(\"ds_read_b128 %0, %1 offset:1040\" : \"=v\"(h1) : \"v\"(rd) : \"memory\");\n"
                  << "            asm volatile(\"ds_read_b128 %0, %1 offset:2064\" : \"=v\"(h2) : \"v\"(rd) : \"memory\");\n"
                  << "            asm volatile(\"ds_read_b128 %0, %1 offset:3088\" : \"=v\"(h3) : \"v\"(rd) : \"memory\");\n"
                  << "            asm volatile(\"s_waitcnt lgkmcnt(0)\" : \"+v\"(q0), \"+v\"(q1), \"+v\"(q2), \"+v\"(q3), "
                     "\"+v\"(h0), \"+v\"(h1), \"+v\"(h2), \"+v\"(h3));\n"
                  << "            q0 = rl2<" << d << ">(q0, h0);\n            q1 = rl2<" << d << ">(q1, h1);\n"
                  << "            q2 = rl2<" << d << ">(q2, h2);\n            q3 = rl2<" << d << ">(q3, h3);\n";
            else
                s << "            asm volatile(\"s_waitcnt lgkmcnt(0)\" : \"+v\"(q0), \"+v\"(q1), \"+v\"(q2), \"+v\"(q3));\n";
            if (style.copy_through) {
                for (int c = 0; c < 4; c++) {
                    s << "            __builtin_amdgcn_raw_buffer_store_b128(q" << c << ", rcopy, cofs" << j << " + off + "
                      << c * 1024 << ", 0, 2);  // copy-through\n";
                    vmem.push_back(-1);
                }
            }
            s << "            u32 P[16] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3],\n"
              << "                         q2[0], q2[1], q2[2], q2[3], q3[0], q3[1], q3[2], q3[3]};\n";
            network(j);
            // every network completes before the next input's reads: without it the compiler sinks
            // the networks below later reads and keeps many inputs' planes live (R = 1, K = 20:
            // 256 VGPRs + scratch)
            s << "            __builtin_amdgcn_sched_barrier(0);\n        }\n";
        }
        outputs("rout", "off");
        s << "    }\n"
             "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
             "}\n";
        return s.str();
    }
    // LDS ring: each wave streams its 1 KiB share of the tile's four 4 KiB chunks of every input into
    // a ring of D slots by LDS-DMA loads (no VGPRs), D - 1 inputs ahead of the network -- across the
    // tile boundary too -- and reads its own 64 B per lane back (conflict-free ds_read_b128).  Loads
    // return in order, so waiting until at most 4 (D - 1) vector-memory operations are outstanding
    // retires the input about to be read whatever stores are in flight.  A slot is refilled only
    // after the reads of its previous input have returned.  Past the last tile the prefetches go to a
    // zero-length buffer (no memory traffic, still counted).
    s << "    __shared__ __attribute__((aligned(16))) u8 ring[4 * " << D << " * 4096];\n"
         "    typedef __attribute__((address_space(3))) u8 lds_u8;\n"
         "    const u32 wring = (u32)(unsigned long)(lds_u8*)ring + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * "
      << D * 4096
      << "u;\n"
         "    const u32 lane = (threadIdx.x & 63u) * 16u;\n"
         "    u32 t = blockIdx.x;\n"
         "    if (t >= a.ntiles) return;\n"
         "    u32 sl = t / a.tiles_per_stripe;\n"
         "    u32 s = a.stripe_list ? (u32)a.stripe_list[sl] : sl;\n"
         "    i32 off = (i32)(t - sl * a.tiles_per_stripe) * "
      << kBsTile
      << " + (i32)threadIdx.x * 16;\n"
         "    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(\n"
         "        (void*)(a.in_base + (i64)s * a.in_stride), 0, (int)a.in_records, 0x00020000);\n"
         "    u32 base = 0;\n";
    auto issue = [&](const char* rin, const std::string& voff, const std::string& slot) {
        s << "#pragma unroll\n        for (int c = 0; c < 4; c++)\n"
             "            __builtin_amdgcn_raw_ptr_buffer_load_lds("
          << rin << ", (__attribute__((address_space(3))) void*)(unsigned long)(wring + ((" << slot
          << ") & " << D - 1 << "u) * 4096u + c * 1024u), 16, " << voff << " + c * 4096, 0, 0, 2);\n";
    };
    for (int q = 0; q < D - 1; q++) issue("rin", "a.in_off[" + std::to_string(q) + "] + off", std::to_string(q));
    s << "    for (;;) {\n"
         "        const u32 t2 = t + gridDim.x;\n"
         "        const bool more = t2 < a.ntiles;\n"
         "        const u32 sl2 = more ? t2 / a.tiles_per_stripe : sl;\n"
         "        const u32 s2 = more ? (a.stripe_list ? (u32)a.stripe_list[sl2] : sl2) : s;\n"
         "        const i32 off2 = (i32)(t2 - sl2 * a.tiles_per_stripe) * "
      << kBsTile
      << " + (i32)threadIdx.x * 16;\n"
         "        const __amdgpu_buffer_rsrc_t rin2 = __builtin_amdgcn_make_buffer_rsrc(\n"
         "            (void*)(a.in_base + (i64)s2 * a.in_stride), 0, more ? (int)a.in_records : 0, 0x00020000);\n";
    acc_init();
    for (int j = 0; j < net.K; j++) {
        const int jj = j + D - 1;
        s << "        {  // input " << j << "\n";
        if (jj < net.K)
            issue("rin", "a.in_off[" + std::to_string(jj) + "] + off", "base + " + std::to_string(jj) + "u");
        else
            issue("rin2", "a.in_off[" + std::to_string(jj - net.K) + "] + off2", "base + " + std::to_string(jj) + "u");
        s << "            asm volatile(\"s_waitcnt vmcnt(" << 4 * (D - 1) << ")\" ::: \"memory\");\n"
          << "            const u32 rd = wring + ((base + " << j << "u) & " << D - 1 << "u) * 4096u + lane;\n"
          << "            v4u q0, q1, q2, q3;\n"
          << "            asm volatile(\"ds_read_b128 %0, %1\" : \"=v\"(q0) : \"v\"(rd) : \"memory\");\n"
          << "            asm volatile(\"ds_read_b128 %0, %1 offset:1024\" : \"=v\"(q1) : \"v\"(rd) : \"memory\");\n"
          << "            asm volatile(\"ds_read_b128 %0, %1 offset:2048\" : \"=v\"(q2) : \"v\"(rd) : \"memory\");\n"
          << "            asm volatile(\"ds_read_b128 %0, %1 offset:3072\" : \"=v\"(q3) : \"v\"(rd) : \"memory\");\n"
          << "            asm volatile(\"s_waitcnt lgkmcnt(0)\" : \"+v\"(q0), \"+v\"(q1), \"+v\"(q2), \"+v\"(q3));\n"
          << "            u32 P[16] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3],\n"
          << "                         q2[0], q2[1], q2[2], q2[3], q3[0], q3[1], q3[2], q3[3]};\n";
        network(j);
        // optional scheduling barrier between inputs (style.input_barrier): measured neutral once
        // temporaries are computed lazily (profiles/r02_c5_experiments.log, tools/c5_ab.sh)
        if (style.input_barrier) s << "            __builtin_amdgcn_sched_barrier(0);\n";
        s << "        }\n";
    }
    s << "        const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(\n"
         "            (void*)(a.out_base + (i64)s * a.out_stride), 0, (int)a.out_records, 0x00020000);\n";
    outputs("rout", "off");
    s << "        if (!more) break;\n"
         "        t = t2; sl = sl2; s = s2; off = off2; rin = rin2;\n"
         "        base = (base + "
      << net.K << "u) & " << D - 1
      << "u;\n"
         "    }\n"
         "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // no LDS-DMA outlives the workgroup\n"
         "}\n";
    return s.str();
}

std::string bitslice_request(const std::vector<int>& coeff, int R, int K, int cap, int depth, bool copy,
                             bool crc, int crc_pos, bool crc_lane, bool crc_nib, bool wave,
                             const std::vector<int>* in_shift, int prefetch, const BsOcc* occ, int crc_wave)
{
    std::ostringstream s;
    // flags: bit 0 copy-through, bit 1 crc (which copies too), bits 2-3 log2 of the crc position
    // sets, bit 4 lane-shift fold, bit 5 nibble piece tables, bit 6 one-wave tiles (not with crc),
    // bit 7 the register budget of 2 waves per SIMD (set with bit 6: the compiler then keeps the
    // dense decode networks of <= 4 outputs in ~128 VGPRs without spilling, which a 4-wave budget
    // of exactly 128 does not -- the occupancy follows the registers actually used), bits 8-10 the
    // one-wave form's prefetch chunks (0, 2, 4; BitsliceStyle::prefetch); one-wave forms: bits 11-14
    // BsOcc::wmin, bits 15-18 BsOcc::wmax, bit 19 BsOcc::barrier (bit 7 then unused); plain maps in
    // the multi-wave form, bits 20-21: lanes per workgroup (1 = 128, 2 = 512; 0 = 256); bit 22 the
    // crc variant in one-wave tiles (with the lane fold; bits 11-19 its occupancy as for bit 6), bits
    // 23-26 its waves per workgroup, bit 27 its crc_mix, bits 28-29 its piece dwords on nibble tables,
    // bit 30 a piece's last dword looked up in global memory (with byte tables only)
    const int cw = crc ? std::clamp(crc_wave & 15, 0, 15) : 0;  // (+ 16: crc_mix, + 32 * nibble dwords)
    const int cmix = cw && (crc_wave & 16) ? 1 : 0;
    const int cnib = cw ? (crc_wave >> 5) & 3 : 0;
    const int cl1 = cw && !cnib && (crc_wave & 128) ? 1 : 0;
    if (cw) {  // (the one-wave crc form always folds with the lane tables, on byte piece tables)
        crc_lane = true;
        crc_nib = false;
    }
    const int pcode = crc ? (crc_pos >= 4 ? 2 : crc_pos >= 2 ? 1 : 0) : 0;
    const BsOcc o = occ ? *occ : BsOcc{};
    const int tcode = !wave && !copy && !crc && depth == 0 ? (o.threads == 128 ? 1 : o.threads == 512 ? 2 : 0) : 0;
    wave = wave && !crc;
    // 1: the late copy of the 16 KiB-tile copy-through form
    const int pf = (wave || crc) && (prefetch == 2 || prefetch == 4) ? prefetch
                   : cw && prefetch == 3 ? 3
                   : (copy && !crc && !wave && prefetch == 1) ? 1 : 0;
    bool shifted = false;
    if (in_shift && (copy || crc))
        for (int j = 0; j < K && j < static_cast<int>(in_shift->size()); j++) shifted = shifted || ((*in_shift)[j] & 15);
    if (copy || crc || wave || tcode) {
        s << "ecamd-bitslice-request " << (shifted ? 3 : 2) << "\n" << R << " " << K << " " << cap << " " << depth << " "
          << ((copy || crc ? 1 : 0) | (crc ? 2 : 0) | (pcode << 2) | (crc && crc_lane ? 16 : 0) |
              (crc && crc_nib ? 32 : 0) | (pf << 8) |
              (!wave && !cw ? 0 : (wave ? 64 : 0) | (std::clamp(o.wmin, 1, 8) << 11) |
                                      (std::clamp(o.wmax, o.wmin, 8) << 15) | (o.barrier ? 1 << 19 : 0)) |
              (tcode << 20) | (cw ? (1 << 22) | (cw << 23) | (cmix << 27) | (cnib << 28) | (cl1 << 30) : 0))
          << "\n";
        if (shifted)  // version 3: the per-input byte shifts of the copy-through inputs
            for (int j = 0; j < K; j++)
                s << (j < static_cast<int>(in_shift->size()) ? ((*in_shift)[j] & 15) : 0) << (j + 1 < K ? " " : "\n");
    } else
        s << "ecamd-bitslice-request 1\n" << R << " " << K << " " << cap << " " << depth << "\n";
    for (size_t i = 0; i < coeff.size(); i++) s << coeff[i] << ((i + 1) % static_cast<size_t>(K) ? " " : "\n");
    return s.str();
}

bool bitslice_parse_request(const std::string& text, std::vector<int>& coeff, int& R, int& K, int& cap,
                            int& depth, bool* copy, bool* crc, int* crc_pos, bool* crc_lane, bool* crc_nib,
                            bool* wave, bool* budget2, std::vector<int>* in_shift, int* prefetch, BsOcc* occ,
                            int* crc_wave)
{
    std::istringstream s(text);
    std::string magic;
    int version = 0, cp = 0;
    if (!(s >> magic >> version) || magic != "ecamd-bitslice-request" || version < 1 || version > 3) return false;
    if (!(s >> R >> K >> cap >> depth) || R <= 0 || R > kBsMaxR || K <= 0 || K > kBsMaxK || cap < 0 || cap > 96)
        return false;
    if (version >= 2 && (!(s >> cp) || cp < 0 || (cp & 12) == 12))
        return false;
    const int cw = (cp >> 22) & 1 ? (cp >> 23) & 15 : 0;  // one-wave crc form: waves per workgroup
    if (((cp >> 22) & 1) ? (!cw || (cp & (1 | 2 | 16 | 32)) != (1 | 2 | 16)) : (cp >> 23) != 0)
        return false;
    if (!cw && (cp >> 27)) return false;
    if (((cp >> 30) & 1) && ((cp >> 28) & 3)) return false;  // global-memory lookups: byte tables only
    if (crc_wave) *crc_wave = cw | (((cp >> 27) & 1) << 4) | (((cp >> 28) & 3) << 5) | (((cp >> 30) & 1) << 7);
    const int tcode = (cp >> 20) & 3;  // lanes per workgroup of the multi-wave plain form
    if (tcode == 3 || (tcode && ((cp & (1 | 2 | 64)) || depth != 0))) return false;
    const int wmin = (cp >> 11) & 15, wmax = (cp >> 15) & 15;  // one-wave occupancy (0: bit 7 / by R)
    if (wmin > 8 || wmax > 8 || (wmax && wmax < wmin) ||
        ((wmin || wmax || ((cp >> 19) & 1)) && ((!(cp & 64) && !cw) || (cp & 128))))
        return false;
    if (version >= 2 && depth != 0 && (((cp & ~(128 | (511 << 11))) | 1) != 65 || (depth != 2 && depth != 4) || cw))
        return false;  // crc: register loads; plain / copy-through one-wave tiles: registers or an LDS ring
    if (tcode && cw) return false;
    if (occ) {
        occ->wmin = wmin ? wmin : (cp & 128) ? 2 : 0;
        occ->wmax = wmax ? wmax : occ->wmin;
        occ->barrier = (cp >> 19) & 1;
        occ->threads = tcode == 1 ? 128 : tcode == 2 ? 512 : 0;
    }
    const int pf = (cp >> 8) & 7;
    if ((pf != 0 && pf != 1 && pf != 2 && pf != 4 && !(pf == 3 && cw)) || (pf > 1 && !(cp & 64) && !(cp & 2)) ||
        (pf == 1 && (!(cp & 1) || (cp & 66))))
        return false;  // 2 / 4: one-wave / crc forms; 1 (late copy): the 16 KiB-tile copy-through form
    if (prefetch) *prefetch = pf;
    if (in_shift) in_shift->clear();
    if (version == 3) {  // shifts: copy-through inputs only, at least one non-zero
        if (!(cp & 1)) return false;
        bool any = false;
        for (int j = 0; j < K; j++) {
            int v = 0;
            if (!(s >> v) || v < 0 || v > 15) return false;
            any = any || v;
            if (in_shift) in_shift->push_back(v);
        }
        if (!any) return false;
    }
    if ((cp & 2) && !(cp & 1)) return false;  // crc implies copy
    if ((cp & 192) && (cp & 2)) return false;  // the crc variant keeps 16 KiB tiles and its budget
    if (((cp >> 2) & 15) && !(cp & 2)) return false;  // bits 2-5 describe the crc variant
    if (copy) *copy = (cp & 1) != 0;
    if (crc) *crc = (cp & 2) != 0;
    if (crc_pos) *crc_pos = 1 << ((cp >> 2) & 3);
    if (crc_lane) *crc_lane = (cp & 16) != 0;
    if (crc_nib) *crc_nib = (cp & 32) != 0;
    if (wave) *wave = (cp & 64) != 0;
    if (budget2) *budget2 = (cp & 128) != 0;
    coeff.assign(static_cast<size_t>(R) * K, 0);
    for (int& c : coeff)
        if (!(s >> c) || c < 0 || c > 0xffff) return false;
    return true;
}

}  // namespace ecamd
