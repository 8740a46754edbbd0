// gf16.cpp -- see gf16.hpp for the reference mapping.
#include "gf16.hpp"

#include <algorithm>

namespace ecamd {

GF16::GF16() : log_(65536, 0), exp_(2 * kOrder + 2, 0)
{
    // Powers of the generator 2 (x) in the polynomial basis; rs_galois.c:49-71.
    int v = 1;
    for (int e = 0; e < kOrder; e++) {
        log_[v] = e;
        exp_[e] = v;
        exp_[e + kOrder] = v;
        v <<= 1;
        if (v & 0x10000) v ^= kPoly;
    }
}

const GF16& GF16::get()
{
    static const GF16 field;
    return field;
}

namespace {

// Column elimination helpers over a row-major matrix with `cols` columns.
void scale_column(std::vector<int>& a, int cols, int row0, int nrows, int col, int f)
{
    const GF16& gf = GF16::get();
    for (int r = row0; r < row0 + nrows; r++) a[r * cols + col] = gf.mul(a[r * cols + col], f);
}

void add_scaled_column(std::vector<int>& a, int cols, int nrows, int src, int dst, int f)
{
    const GF16& gf = GF16::get();
    for (int r = 0; r < nrows; r++) a[r * cols + dst] ^= gf.mul(a[r * cols + src], f);
}

int pivot_row(const std::vector<int>& a, int cols, int nrows, int col, int from)
{
    for (int r = from; r < nrows; r++)
        if (a[r * cols + col] != 0) return r;
    return -1;
}

void swap_rows(std::vector<int>& a, int cols, int r1, int r2)
{
    for (int c = 0; c < cols; c++) std::swap(a[r1 * cols + c], a[r2 * cols + c]);
}

}  // namespace

std::vector<int> rs_generator(int k, int m)
{
    const GF16& gf = GF16::get();
    const int n = k + m;
    if (k <= 0 || m < 0 || n > 65536) return {};
    std::vector<int> g(static_cast<size_t>(n) * k, 0);
    g[0] = 1;  // evaluation point 0: row e0
    for (int r = 1; r < n; r++) {
        int p = 1;
        for (int c = 0; c < k; c++) {
            g[r * k + c] = p;
            p = gf.mul(p, r);
        }
    }
    // Reduce the top k x k block to the identity by column operations (the code stays MDS).
    for (int d = 1; d < k; d++) {
        int pr = pivot_row(g, k, n, d, d);
        if (pr < 0) return {};
        if (pr != d) swap_rows(g, k, pr, d);
        if (g[d * k + d] != 1) scale_column(g, k, 0, n, d, gf.inv(g[d * k + d]));
        for (int c = 0; c < k; c++) {
            int v = g[d * k + c];
            if (c != d && v != 0) add_scaled_column(g, k, n, d, c, v);
        }
    }
    // First parity row -> all ones (scales only the parity part of each column).
    for (int c = 0; c < k && m > 0; c++) {
        int v = g[k * k + c];
        if (v != 1) scale_column(g, k, k, m, c, gf.inv(v));
    }
    return g;
}

bool gf16_invert(std::vector<int> a, std::vector<int>& inv, int n)
{
    const GF16& gf = GF16::get();
    inv.assign(static_cast<size_t>(n) * n, 0);
    for (int i = 0; i < n; i++) inv[i * n + i] = 1;
    for (int i = 0; i < n; i++) {
        int pr = pivot_row(a, n, n, i, i);
        if (pr < 0) return false;
        if (pr != i) {
            swap_rows(a, n, pr, i);
            swap_rows(inv, n, pr, i);
        }
        int d = a[i * n + i];
        if (d != 1) {
            int f = gf.inv(d);
            for (int c = 0; c < n; c++) {
                a[i * n + c] = gf.mul(a[i * n + c], f);
                inv[i * n + c] = gf.mul(inv[i * n + c], f);
            }
        }
        for (int r = 0; r < n; r++) {
            int f = a[r * n + i];
            if (r == i || f == 0) continue;
            for (int c = 0; c < n; c++) {
                a[r * n + c] ^= gf.mul(a[i * n + c], f);
                inv[r * n + c] ^= gf.mul(inv[i * n + c], f);
            }
        }
    }
    return true;
}

namespace {

struct Availability {
    std::vector<char> missing;   // per fragment index
    std::vector<int> first_k;    // first k present indices, index order
    int nmissing = 0;            // entries in the -1-terminated list (duplicates counted)
};

bool availability(int k, int m, const std::vector<int>& missing, Availability& av)
{
    const int n = k + m;
    av.missing.assign(n, 0);
    av.nmissing = static_cast<int>(missing.size());
    for (int idx : missing)
        if (idx >= 0 && idx < n) av.missing[idx] = 1;
    if (av.nmissing > m) return false;
    for (int i = 0; i < n && static_cast<int>(av.first_k.size()) < k; i++)
        if (!av.missing[i]) av.first_k.push_back(i);
    return static_cast<int>(av.first_k.size()) == k;
}

// Inverse of the decoding matrix built from the generator rows of `first_k`.
bool decode_inverse(const std::vector<int>& G, int k, const std::vector<int>& first_k,
                    std::vector<int>& inv)
{
    std::vector<int> dec(static_cast<size_t>(k) * k);
    for (int r = 0; r < k; r++)
        std::copy(&G[first_k[r] * k], &G[first_k[r] * k] + k, &dec[r * k]);
    return gf16_invert(dec, inv, k);
}

// Coefficients over first_k that rebuild parity fragment `p` (reconstruct's composite row).
std::vector<int> parity_row(const std::vector<int>& G, int k, const Availability& av,
                            const std::vector<int>& missing, const std::vector<int>& inv, int p)
{
    const GF16& gf = GF16::get();
    std::vector<int> row(k, 0);
    int j = 0;
    for (int d = 0; d < k; d++)
        if (!av.missing[d]) row[j++] = G[p * k + d];
    for (int d : missing) {
        if (d < 0 || d >= k) continue;
        for (int c = 0; c < k; c++) row[c] ^= gf.mul(G[p * k + d], inv[d * k + c]);
    }
    return row;
}

// The reference dot product zeroes its output and then accumulates in input order, so an
// input that IS the output reads the partial sum: out <- (1 + c) * out at that step.  Fold
// that into coefficients over the remaining inputs (bit-exact, per 16-bit word).
void fold_alias(std::vector<int>& inputs, std::vector<int>& row, int out_idx)
{
    auto it = std::find(inputs.begin(), inputs.end(), out_idx);
    if (it == inputs.end()) return;
    const GF16& gf = GF16::get();
    std::vector<int> acc(inputs.size(), 0);
    for (size_t i = 0; i < inputs.size(); i++) {
        if (inputs[i] == out_idx) {
            int f = 1 ^ row[i];
            for (auto& v : acc) v = gf.mul(v, f);
        } else {
            acc[i] ^= row[i];
        }
    }
    size_t pos = static_cast<size_t>(it - inputs.begin());
    acc.erase(acc.begin() + pos);
    inputs.erase(inputs.begin() + pos);
    row = acc;
}

}  // namespace

FragmentMap rs_encode_map(const std::vector<int>& G, int k, int m)
{
    FragmentMap fm;
    for (int j = 0; j < k; j++) fm.inputs.push_back(j);
    for (int p = 0; p < m; p++) {
        fm.outputs.push_back(k + p);
        fm.coeff.insert(fm.coeff.end(), &G[(k + p) * k], &G[(k + p) * k] + k);
    }
    return fm;
}

int rs_decode_map(const std::vector<int>& G, int k, int m, const std::vector<int>& missing,
                  bool rebuild_parity, FragmentMap& out)
{
    Availability av;
    if (!availability(k, m, missing, av)) return -1;
    std::vector<int> inv;
    if (!decode_inverse(G, k, av.first_k, inv)) return -1;
    out = FragmentMap();
    out.inputs = av.first_k;
    for (int d = 0; d < k; d++) {
        if (!av.missing[d]) continue;
        out.outputs.push_back(d);
        out.coeff.insert(out.coeff.end(), &inv[d * k], &inv[d * k] + k);
    }
    if (rebuild_parity) {
        for (int p = k; p < k + m; p++) {
            if (!av.missing[p]) continue;
            std::vector<int> row = parity_row(G, k, av, missing, inv, p);
            out.outputs.push_back(p);
            out.coeff.insert(out.coeff.end(), row.begin(), row.end());
        }
    }
    return 0;
}

int rs_reconstruct_map(const std::vector<int>& G, int k, int m, const std::vector<int>& missing,
                       int dest, FragmentMap& out)
{
    Availability av;
    if (dest < 0 || dest >= k + m) return -1;
    if (!availability(k, m, missing, av)) return -1;
    std::vector<int> inv;
    if (!decode_inverse(G, k, av.first_k, inv)) return -1;
    std::vector<int> row;
    if (dest < k)
        row.assign(&inv[dest * k], &inv[dest * k] + k);
    else
        row = parity_row(G, k, av, missing, inv, dest);
    out = FragmentMap();
    out.inputs = av.first_k;
    fold_alias(out.inputs, row, dest);
    out.outputs.push_back(dest);
    out.coeff = row;
    return 0;
}

}  // namespace ecamd
