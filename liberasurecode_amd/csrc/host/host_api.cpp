// host_api.cpp -- extern "C" surface of libecamd_host.so (include/ecamd_host.h).
#include "ecamd_host.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bitslice.hpp"
#include "gf16.hpp"
#include "tables.hpp"
#include "xor_plan.hpp"

using namespace ecamd;

namespace {
std::vector<int> minus1_list(const int* missing)
{
    std::vector<int> v;
    if (!missing) return v;
    for (int i = 0; missing[i] > -1; i++) v.push_back(missing[i]);
    return v;
}
}  // namespace

extern "C" {

int ecamd_gf16_mul(int a, int b) { return GF16::get().mul(a & 0xffff, b & 0xffff); }

int ecamd_gf16_inv(int a) { return GF16::get().inv(a & 0xffff); }

int ecamd_rs_generator(int k, int m, int* out)
{
    std::vector<int> g = rs_generator(k, m);
    if (g.empty() || !out) return -1;
    std::memcpy(out, g.data(), g.size() * sizeof(int));
    return 0;
}

int ecamd_gf16_invert(const int* a, int* inv, int n)
{
    if (!a || !inv || n <= 0) return -1;
    std::vector<int> m(a, a + static_cast<size_t>(n) * n), r;
    if (!gf16_invert(m, r, n)) return -1;
    std::memcpy(inv, r.data(), r.size() * sizeof(int));
    return 0;
}

int ecamd_rs_decode_map(const int* G, int k, int m, const int* missing, int rebuild_parity,
                        int* inputs, int* outputs, int* coeff, int* nout)
{
    if (!G || k <= 0 || m < 0) return -1;
    std::vector<int> g(G, G + static_cast<size_t>(k + m) * k);
    FragmentMap fm;
    if (rs_decode_map(g, k, m, minus1_list(missing), rebuild_parity != 0, fm) != 0) return -1;
    std::memcpy(inputs, fm.inputs.data(), fm.inputs.size() * sizeof(int));
    if (!fm.outputs.empty()) {
        std::memcpy(outputs, fm.outputs.data(), fm.outputs.size() * sizeof(int));
        std::memcpy(coeff, fm.coeff.data(), fm.coeff.size() * sizeof(int));
    }
    *nout = static_cast<int>(fm.outputs.size());
    return 0;
}

int ecamd_rs_reconstruct_map(const int* G, int k, int m, const int* missing, int dest, int* inputs,
                             int* ninputs, int* coeff)
{
    if (!G || k <= 0 || m < 0) return -1;
    std::vector<int> g(G, G + static_cast<size_t>(k + m) * k);
    FragmentMap fm;
    if (rs_reconstruct_map(g, k, m, minus1_list(missing), dest, fm) != 0) return -1;
    if (!fm.inputs.empty()) {
        std::memcpy(inputs, fm.inputs.data(), fm.inputs.size() * sizeof(int));
        std::memcpy(coeff, fm.coeff.data(), fm.coeff.size() * sizeof(int));
    }
    *ninputs = static_cast<int>(fm.inputs.size());
    return 0;
}

int ecamd_split_tables(const int* coeff, int R, int K, int row0, int width, int col0, int ncols,
                       uint8_t* out)
{
    if (!coeff || !out || (width != 2 && width != 4 && width != 8)) return -1;
    std::vector<int> c(coeff, coeff + static_cast<size_t>(R) * K);
    std::vector<uint8_t> img = build_split_tables(c, R, K, row0, width, col0, ncols);
    std::memcpy(out, img.data(), img.size());
    return static_cast<int>(img.size());
}

int ecamd_xor_code_tables(int k, int m, int hd, unsigned int* parity_bms, unsigned int* data_bms)
{
    XorCode c;
    if (!xor_code_lookup(k, m, hd, c)) return -1;
    if (parity_bms) std::memcpy(parity_bms, c.parity_bms, sizeof(unsigned int) * m);
    if (data_bms) std::memcpy(data_bms, c.data_bms, sizeof(unsigned int) * k);
    return 0;
}

int ecamd_xor_plan(int op, int k, int m, int hd, const unsigned int* parity_bms,
                   const unsigned int* data_bms, const int* missing, int arg, int* outputs,
                   uint64_t* sources, int* nout)
{
    XorCode c;
    c.k = k;
    c.m = m;
    c.hd = hd;
    c.parity_bms = parity_bms;
    c.data_bms = data_bms;
    if (!parity_bms || !data_bms || k <= 0 || m <= 0 || k + m > 63 || !nout) return -100;
    XorPlan p;
    if (op == 0)
        p = xor_plan_encode(c);
    else if (op == 1)
        p = xor_plan_decode(c, minus1_list(missing), arg);
    else
        p = xor_plan_reconstruct_one(c, minus1_list(missing), arg);
    for (size_t i = 0; i < p.outputs.size(); i++) {
        outputs[i] = p.outputs[i];
        sources[i] = p.sources[i];
    }
    *nout = static_cast<int>(p.outputs.size());
    return p.rc;
}

int ecamd_xor_fragments_needed(int k, int m, int hd, const unsigned int* parity_bms,
                               const unsigned int* data_bms, const int* to_reconstruct,
                               const int* to_exclude, int* needed)
{
    XorCode c;
    c.k = k;
    c.m = m;
    c.hd = hd;
    c.parity_bms = parity_bms;
    c.data_bms = data_bms;
    std::vector<int> out;
    int rc = xor_fragments_needed(c, minus1_list(to_reconstruct), minus1_list(to_exclude), out);
    if (rc >= 0 && needed) std::memcpy(needed, out.data(), out.size() * sizeof(int));
    return rc;
}

int ecamd_fragments_needed_batch(int backend, int k, int m, int hd, const int* recon,
                                 const int* excl, int list_stride, int nstripes, int* needed,
                                 int* rcs)
{
    if (!recon || !excl || !needed || !rcs || list_stride < 1 || nstripes < 0 || k < 1 || m < 0 ||
        k + m > 64)
        return -1;
    unsigned pb[64], db[64];
    if (backend == 3 && ecamd_xor_code_tables(k, m, hd, pb, db) != 0) return -1;
    if (backend != 3 && backend != 6) return -1;
    const int row = k + m + 1;
    for (int s = 0; s < nstripes; s++) {
        const int* r = recon + static_cast<int64_t>(s) * list_stride;
        const int* x = excl + static_cast<int64_t>(s) * list_stride;
        int* out = needed + static_cast<int64_t>(s) * row;
        std::vector<int> rl, xl;
        for (int i = 0; i < list_stride && r[i] >= 0; i++) rl.push_back(r[i]);
        for (int i = 0; i < list_stride && x[i] >= 0; i++) xl.push_back(x[i]);
        rl.push_back(-1);
        xl.push_back(-1);
        if (backend == 3) {
            // xor_hd_fragments_needed (xor_hd_code.c:209-412), exactly as the shim calls it
            std::vector<int> tmp(row, -1);
            rcs[s] = ecamd_xor_fragments_needed(k, m, hd, pb, db, rl.data(), xl.data(), tmp.data());
            std::memcpy(out, tmp.data(), sizeof(int) * row);
            if (rcs[s] >= 0) {
                int n = 0;
                while (n < row && tmp[n] >= 0) n++;
                for (int i = n; i < row; i++) out[i] = -1;
            }
        } else {
            // rs_vand shim (src/backends/rs_vand/liberasurecode_rs_vand.c:119-145): the first k
            // indices neither missing nor excluded.
            std::vector<bool> gone(k + m, false);
            for (int v : xl)
                if (v >= 0 && v < k + m) gone[v] = true;
            for (int v : rl)
                if (v >= 0 && v < k + m) gone[v] = true;
            int j = 0;
            for (int i = 0; i < k + m && j < k; i++)
                if (!gone[i]) out[j++] = i;
            for (int i = j; i < row; i++) out[i] = -1;
            rcs[s] = j == k ? 0 : -1;
        }
    }
    return 0;
}

int ecamd_percall_device_plan(int ndev, const char* spec, int* devs, int max)
{
    if (ndev <= 0 || !devs || max <= 0) return 0;
    std::vector<int> ids;
    std::vector<bool> seen(static_cast<size_t>(ndev), false);
    for (const char* p = spec; p && *p;) {
        char* end = nullptr;
        const long v = std::strtol(p, &end, 10);
        if (end == p) {  // not a number: skip one character (separators, spaces)
            p++;
            continue;
        }
        if (v >= 0 && v < ndev && !seen[static_cast<size_t>(v)]) {
            seen[static_cast<size_t>(v)] = true;
            ids.push_back(static_cast<int>(v));
        }
        p = end;
    }
    if (ids.empty())
        for (int d = 0; d < ndev; d++) ids.push_back(d);
    const int n = std::min(static_cast<int>(ids.size()), max);
    for (int i = 0; i < n; i++) devs[i] = ids[static_cast<size_t>(i)];
    return n;
}

int ecamd_bitslice_eval(const int* coeff, int R, int K, int cap, const uint16_t* in, uint16_t* out,
                        int* ops)
{
    if (!coeff || !in || !out || R <= 0 || R > kBsMaxR || K <= 0 || K > kBsMaxK) return -1;
    std::vector<int> c(coeff, coeff + static_cast<size_t>(R) * K);
    const BitsliceNet net = bitslice_network(c, R, K, cap);
    bitslice_eval(net, in, out);
    if (ops) *ops = net.xor_ops();
    return 0;
}

int64_t ecamd_bitslice_source(const int* coeff, int R, int K, int cap, int depth, char* buf, int64_t size)
{
    if (!coeff || R <= 0 || R > kBsMaxR || K <= 0 || K > kBsMaxK) return -1;
    std::vector<int> c(coeff, coeff + static_cast<size_t>(R) * K);
    const std::string src = bitslice_source(bitslice_network(c, R, K, cap), depth);
    if (buf && size > 0) {
        const size_t n = std::min(static_cast<size_t>(size - 1), src.size());
        std::memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return static_cast<int64_t>(src.size());
}

}  // extern "C"
