// bitslice.cpp -- network construction and kernel source for bitsliced GF(2^16) maps
// (bitslice.hpp).  The generated kernel is verified bit-exact against the CPU oracle by
// tests/test_gpu_bitslice.py; the network itself against GF16 products by
// tests/test_host_planning.py (ecamd_bitslice_eval).
#include "bitslice.hpp"

#include <algorithm>
#include <cstdio>
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

// Greedy common-subexpression elimination priced in three-input XORs (bitslice.hpp): take the
// shared pair or triple with the largest saving (ties: pairs first, then the smallest ids) while it
// saves at least one op and fewer than `cap` temporaries exist.  Deterministic in the matrix.
void share_terms(std::vector<std::vector<int>>& rows, std::vector<std::array<int, 3>>& temps, int cap)
{
    constexpr int V = 64;  // variable ids < 16 + cap <= 64
    std::vector<int> c2(V * V), c3(V * V * V);
    std::vector<int> touched;
    int nvar = 16;
    while (static_cast<int>(temps.size()) < cap && nvar < V) {
        std::fill(c2.begin(), c2.end(), 0);
        for (int t : touched) c3[static_cast<size_t>(t)] = 0;
        touched.clear();
        for (const auto& r : rows) {
            const size_t n = r.size();
            for (size_t i = 0; i < n; i++)
                for (size_t k = i + 1; k < n; k++) {
                    if (n & 1) c2[static_cast<size_t>(r[i]) * V + r[k]]++;
                    for (size_t l = k + 1; l < n; l++) {
                        const int key = (r[i] * V + r[k]) * V + r[l];
                        if (c3[static_cast<size_t>(key)]++ == 0) touched.push_back(key);
                    }
                }
        }
        int best = 1, ba = -1, bb = -1, bc = -1;
        for (int a = 0; a < nvar; a++)
            for (int b = a + 1; b < nvar; b++)
                if (c2[static_cast<size_t>(a) * V + b] > best) {
                    best = c2[static_cast<size_t>(a) * V + b];
                    ba = a, bb = b, bc = -1;
                }
        std::sort(touched.begin(), touched.end());
        for (int key : touched)
            if (c3[static_cast<size_t>(key)] > best) {
                best = c3[static_cast<size_t>(key)];
                ba = key / (V * V), bb = (key / V) % V, bc = key % V;
            }
        if (ba < 0) break;  // nothing saves an op
        temps.push_back({ba, bb, bc});
        for (auto& r : rows) {
            auto has = [&](int v) { return v < 0 || std::find(r.begin(), r.end(), v) != r.end(); };
            if (!has(ba) || !has(bb) || !has(bc)) continue;
            r.erase(std::remove_if(r.begin(), r.end(), [&](int v) { return v == ba || v == bb || v == bc; }),
                    r.end());
            r.push_back(nvar);  // rows stay sorted: new variables are the largest
        }
        nvar++;
    }
}

}  // namespace

BitsliceNet bitslice_network(const std::vector<int>& coeff, int R, int K, int cap)
{
    BitsliceNet net;
    net.R = R;
    net.K = K;
    net.inputs.resize(static_cast<size_t>(K));
    for (int j = 0; j < K; j++) {
        auto& in = net.inputs[static_cast<size_t>(j)];
        in.rows.assign(static_cast<size_t>(R) * 16, {});
        for (int r = 0; r < R; r++) {
            uint16_t M[16];
            gf16_bitmatrix(coeff[static_cast<size_t>(r) * K + j], M);
            for (int p = 0; p < 16; p++)
                for (int b = 0; b < 16; b++)
                    if ((M[p] >> b) & 1) in.rows[static_cast<size_t>(r) * 16 + p].push_back(b);
        }
        share_terms(in.rows, in.temps, cap);
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
};
__device__ __forceinline__ u32 x3(u32 a, u32 b, u32 c)
{
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ u32 bfi(u32 m, u32 x, u32 y)
{
    u32 r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(x), "v"(y));
    return r;
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

}  // namespace

std::string bitslice_source(const BitsliceNet& net)
{
    std::ostringstream s;
    s << "// generated by liberasurecode_amd bitslice_source: " << net.R << " outputs x " << net.K
      << " inputs, " << net.xor_ops() << " network ops per tile\n";
    s << kPrelude;
    s << "extern \"C\" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))\n"
         "ecamd_bs_kernel(ecamd_bs_args a)\n{\n"
         "    for (u32 t = blockIdx.x; t < a.ntiles; t += gridDim.x) {\n"
         "        const u32 sl = t / a.tiles_per_stripe;\n"
         "        const u32 s = a.stripe_list ? (u32)a.stripe_list[sl] : sl;\n"
         "        const i32 off = (i32)(t - sl * a.tiles_per_stripe) * "
      << kBsTile
      << " + (i32)threadIdx.x * 16;\n"
         "        const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(\n"
         "            (void*)(a.in_base + (i64)s * a.in_stride), 0, (int)a.in_records, 0x00020000);\n"
         "        const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(\n"
         "            (void*)(a.out_base + (i64)s * a.out_stride), 0, (int)a.out_records, 0x00020000);\n"
      << "        u32 acc[" << net.R << "][16];\n"
      << "#pragma unroll\n        for (int r = 0; r < " << net.R
      << "; r++)\n#pragma unroll\n            for (int p = 0; p < 16; p++) acc[r][p] = 0u;\n";
    auto ref = [](int v) {
        char b[24];
        if (v < 16)
            std::snprintf(b, sizeof(b), "P[%d]", 15 - v);
        else
            std::snprintf(b, sizeof(b), "t%d", v);
        return std::string(b);
    };
    for (int j = 0; j < net.K; j++) {
        const auto& in = net.inputs[static_cast<size_t>(j)];
        s << "        {  // input " << j << "\n            u32 P[16];\n"
          << "#pragma unroll\n            for (int c = 0; c < 4; c++) {\n"
          << "                const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rin, a.in_off[" << j
          << "] + off + c * 4096, 0, 2);\n"
          << "                P[4 * c] = x[0]; P[4 * c + 1] = x[1]; P[4 * c + 2] = x[2]; P[4 * c + 3] = x[3];\n"
          << "            }\n            tr16(P);\n";
        for (size_t i = 0; i < in.temps.size(); i++) {
            const auto& t = in.temps[i];
            if (t[2] < 0)
                s << "            const u32 t" << 16 + i << " = " << ref(t[0]) << " ^ " << ref(t[1]) << ";\n";
            else
                s << "            const u32 t" << 16 + i << " = x3(" << ref(t[0]) << ", " << ref(t[1]) << ", "
                  << ref(t[2]) << ");\n";
        }
        for (size_t i = 0; i < in.rows.size(); i++) {
            const auto& terms = in.rows[i];
            if (terms.empty()) continue;
            char dst[32];
            std::snprintf(dst, sizeof(dst), "acc[%zu][%zu]", i / 16, 15 - i % 16);
            size_t q = 0;
            for (; q + 1 < terms.size(); q += 2)
                s << "            " << dst << " = x3(" << dst << ", " << ref(terms[q]) << ", "
                  << ref(terms[q + 1]) << ");\n";
            if (q < terms.size()) s << "            " << dst << " ^= " << ref(terms[q]) << ";\n";
        }
        s << "        }\n";
    }
    s << "#pragma unroll\n        for (int r = 0; r < " << net.R
      << "; r++) {\n"
         "            tr16(acc[r]);\n"
         "#pragma unroll\n"
         "            for (int c = 0; c < 4; c++) {\n"
         "                const v4u v = {acc[r][4 * c], acc[r][4 * c + 1], acc[r][4 * c + 2], acc[r][4 * c + 3]};\n"
         "                __builtin_amdgcn_raw_buffer_store_b128(v, rout, a.out_off[r] + off + c * 4096, 0, 2);\n"
         "            }\n"
         "        }\n"
         "    }\n"
         "}\n";
    return s.str();
}

}  // namespace ecamd
