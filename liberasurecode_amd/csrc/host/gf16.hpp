// gf16.hpp -- GF(2^16) host arithmetic and Reed-Solomon (systematic Vandermonde) planning.
//
// MI355X design note: all of this runs once per (k,m) or per erasure pattern on the host
// (k <= 255, so at most a 255x255 inversion); the per-byte work runs on the GPU through the
// split-table kernels in ../hip/ecamd_kernels.hip, fed by the tables built in tables.cpp.
//
// Semantics follow the reference built-in codec:
//   field: log/antilog over x^16+x^12+x^3+x+1 ........ src/builtin/rs_vand/rs_galois.c:38-117
//   generator: Vandermonde rows r^c, column-reduced to a systematic form, parity columns
//              normalised so the first parity row is all ones
//                                                      src/builtin/rs_vand/liberasurecode_rs_vand.c:139-289
//   inversion: Gauss-Jordan .......................... liberasurecode_rs_vand.c:293-334
//   decode / reconstruct coefficient rows ............ liberasurecode_rs_vand.c:412-558
#pragma once
#include <cstdint>
#include <vector>

namespace ecamd {

class GF16 {
public:
    static const GF16& get();
    int mul(int a, int b) const
    {
        if (a == 0 || b == 0) return 0;
        return exp_[log_[a] + log_[b]];
    }
    int inv(int a) const { return a == 0 ? -1 : exp_[kOrder - log_[a]]; }
    int log(int a) const { return log_[a]; }
    static constexpr int kPoly = 0x1100b;
    static constexpr int kOrder = 65535;

private:
    GF16();
    std::vector<int> log_;
    std::vector<int> exp_;  // 2*order entries, so log sums need no reduction
};

// (k+m) x k row-major systematic generator; empty on failure.
std::vector<int> rs_generator(int k, int m);

// Inverse of the n x n matrix a; returns false if singular.
bool gf16_invert(std::vector<int> a, std::vector<int>& inv, int n);

// A linear "fragment map": outputs[r] = sum_j coeff[r*K + j] * inputs[j].
struct FragmentMap {
    std::vector<int> inputs;   // fragment indices read (K of them)
    std::vector<int> outputs;  // fragment indices written (R of them)
    std::vector<int> coeff;    // R x K
};

// Decode map (liberasurecode_rs_vand_decode): first k available fragments in index order as
// inputs; every missing data fragment (inverse rows) and, if rebuild_parity, every missing
// parity fragment (generator row composed with the inverse) as outputs, in index order.
// Returns 0, or -1 when more than m fragments are missing.
int rs_decode_map(const std::vector<int>& G, int k, int m, const std::vector<int>& missing,
                  bool rebuild_parity, FragmentMap& out);

// Reconstruct map for one destination (liberasurecode_rs_vand_reconstruct).
int rs_reconstruct_map(const std::vector<int>& G, int k, int m, const std::vector<int>& missing,
                       int dest, FragmentMap& out);

// Encode map: inputs 0..k-1, outputs k..k+m-1, generator parity rows.
FragmentMap rs_encode_map(const std::vector<int>& G, int k, int m);

}  // namespace ecamd
