// rs_vand_abi.cpp -- liberasurecode_rs_vand.so.1 for MI355X (boundary B1, include/liberasurecode_rs_vand.h).
//
// The matrix utilities are host code with the reference's semantics; the three region entry
// points stage the caller's host fragments into HBM, run one GF(2^16) fragment-map launch
// (libecamd) and copy the rebuilt fragments back before returning, as the reference's
// synchronous contract requires (src/erasurecode.c:454-455, 677-678, 898-899 call them under a
// shared read lock from many threads at once).
#include "liberasurecode_rs_vand.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "ecamd.h"
#include "ecamd_host.h"

namespace {

std::mutex g_mu;
int g_refs = 0;

void report(const char* what)
{
    std::fprintf(stderr, "liberasurecode_rs_vand (MI355X): %s: %s\n", what, ecamd_last_error());
}

// out[r] = sum_j coeff[r][j] * in[j] for host buffers, through the GPU (libecamd hostio).
int run_map(const std::vector<int>& coeff, const std::vector<char*>& in,
            const std::vector<char*>& out, int blocksize)
{
    int rc = ecamd_host_map_apply(coeff.data(), static_cast<int>(out.size()),
                                  static_cast<int>(in.size()),
                                  reinterpret_cast<const void* const*>(in.data()),
                                  reinterpret_cast<void* const*>(out.data()), blocksize);
    if (rc) report("region kernel");
    return rc ? -1 : 0;
}

char* frag(char** data, char** parity, int k, int idx) { return idx < k ? data[idx] : parity[idx - k]; }

std::vector<int> g_rows(const int* G, int k, int m)
{
    return std::vector<int>(G, G + static_cast<size_t>(k + m) * k);
}

}  // namespace

extern "C" {

void init_liberasurecode_rs_vand(int k, int m)
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_refs++;
}

void deinit_liberasurecode_rs_vand(void)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_refs > 0) g_refs--;
}

int* make_systematic_matrix(int k, int m)
{
    if (ecamd_init() != 0) {
        report("make_systematic_matrix");
        return nullptr;
    }
    if (k <= 0 || m < 0) return nullptr;
    int* g = static_cast<int*>(std::malloc(sizeof(int) * static_cast<size_t>(k + m) * k));
    if (!g) return nullptr;
    if (ecamd_rs_generator(k, m, g) != 0) {
        std::free(g);
        return nullptr;
    }
    return g;
}

void free_systematic_matrix(int* matrix) { std::free(matrix); }

int is_missing(int* missing_idxs, int index_to_check)
{
    for (int i = 0; missing_idxs[i] > -1; i++)
        if (missing_idxs[i] == index_to_check) return 1;
    return 0;
}

int create_decoding_matrix(int* gen_matrix, int* dec_matrix, int* missing_idxs, int k, int m)
{
    int rows = 0;
    for (int i = 0; i < k + m && rows < k; i++) {
        if (is_missing(missing_idxs, i)) continue;
        std::memcpy(&dec_matrix[rows * k], &gen_matrix[i * k], sizeof(int) * k);
        rows++;
    }
    return rows == k;
}

int gaussj_inversion(int* matrix, int* inverse, int n)
{
    if (ecamd_gf16_invert(matrix, inverse, n) != 0) return -1;
    // The reference eliminates in place, leaving the identity behind in `matrix`.
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) matrix[r * n + c] = (r == c);
    return 0;
}

int is_identity_matrix(int* matrix, int n)
{
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++)
            if (matrix[r * n + c] != (r == c ? 1 : 0)) return 0;
    return 1;
}

void print_matrix(int* matrix, int rows, int cols)
{
    std::printf("\n");
    for (int r = 0; r < rows; r++) {
        for (int c = 0; c < cols; c++) std::printf("%d ", matrix[r * cols + c]);
        std::printf("\n");
    }
    std::printf("\n");
}

void square_matrix_multiply(int* m1, int* m2, int* prod, int n)
{
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) {
            int acc = 0;
            for (int t = 0; t < n; t++) acc ^= ecamd_gf16_mul(m1[r * n + t], m2[t * n + c]);
            prod[r * n + c] = acc;
        }
}

int liberasurecode_rs_vand_encode(int* generator_matrix, char** data, char** parity, int k, int m,
                                  int blocksize)
{
    if (!generator_matrix || k <= 0 || m <= 0) return 0;
    std::vector<int> coeff(generator_matrix + static_cast<size_t>(k) * k,
                           generator_matrix + static_cast<size_t>(k + m) * k);
    std::vector<char*> in(data, data + k), out(parity, parity + m);
    return run_map(coeff, in, out, blocksize);
}

int liberasurecode_rs_vand_decode(int* generator_matrix, char** data, char** parity, int k, int m,
                                  int* missing, int blocksize, int rebuild_parity)
{
    std::vector<int> inputs(k), outputs(k + m), coeff(static_cast<size_t>(k + m) * k);
    int nout = 0;
    if (ecamd_rs_decode_map(g_rows(generator_matrix, k, m).data(), k, m, missing, rebuild_parity,
                            inputs.data(), outputs.data(), coeff.data(), &nout) != 0)
        return -1;
    std::vector<char*> in, out;
    for (int i : inputs) in.push_back(frag(data, parity, k, i));
    for (int r = 0; r < nout; r++) out.push_back(frag(data, parity, k, outputs[r]));
    coeff.resize(static_cast<size_t>(nout) * k);
    return run_map(coeff, in, out, blocksize);
}

int liberasurecode_rs_vand_reconstruct(int* generator_matrix, char** data, char** parity, int k,
                                       int m, int* missing, int destination_idx, int blocksize)
{
    std::vector<int> inputs(k), coeff(k);
    int nin = 0;
    if (ecamd_rs_reconstruct_map(g_rows(generator_matrix, k, m).data(), k, m, missing,
                                 destination_idx, inputs.data(), &nin, coeff.data()) != 0)
        return -1;
    std::vector<char*> in;
    for (int j = 0; j < nin; j++) in.push_back(frag(data, parity, k, inputs[j]));
    coeff.resize(nin);
    std::vector<char*> out = {frag(data, parity, k, destination_idx)};
    return run_map(coeff, in, out, blocksize);
}

}  // extern "C"
