// xorcode_abi.cpp -- libXorcode.so.1 for MI355X (boundary B1', include/xor_code.h).
//
// Each operation is planned on the host by replaying the reference's control flow symbolically
// (host/xor_plan.cpp: which buffers end up holding the XOR of which originals), then executed
// for the caller's host buffers by one GPU XOR launch per chunk (libecamd hostio).
#include "xor_code.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "ecamd.h"
#include "ecamd_host.h"

namespace {

void report(const char* what)
{
    std::fprintf(stderr, "libXorcode (MI355X): %s: %s\n", what, ecamd_last_error());
}

std::vector<int> list(const int* l)
{
    std::vector<int> v;
    if (l)
        for (int i = 0; l[i] > -1; i++) v.push_back(l[i]);
    v.push_back(-1);
    return v;
}

// Plan op (0 encode, 1 decode, 2 reconstruct) and run it on the GPU; returns the reference rc.
int run(xor_code_t* c, int op, char** data, char** parity, const int* missing, int arg,
        int blocksize)
{
    const int n = c->k + c->m;
    std::vector<int> outs(n);
    std::vector<uint64_t> srcs(n);
    int nout = 0;
    std::vector<int> miss = list(missing);
    int rc = ecamd_xor_plan(op, c->k, c->m, c->hd, c->parity_bms, c->data_bms, miss.data(), arg,
                            outs.data(), srcs.data(), &nout);
    if (rc == -100) return -1;
    if (nout == 0 || blocksize <= 0) return rc;
    std::vector<void*> bufs(n);
    for (int i = 0; i < c->k; i++) bufs[i] = data[i];
    for (int i = 0; i < c->m; i++) bufs[c->k + i] = parity[i];
    std::vector<void*> out(nout);
    for (int r = 0; r < nout; r++) out[r] = bufs[outs[r]];
    if (ecamd_host_xor_apply(srcs.data(), nout, n, bufs.data(), out.data(), blocksize) != 0) {
        report("xor kernel");
        return -1;
    }
    return rc;
}

}  // namespace

extern "C" {

void xor_code_encode(xor_code_t* code_desc, char** data, char** parity, int blocksize)
{
    run(code_desc, 0, data, parity, nullptr, 0, blocksize);
}

int xor_hd_decode(xor_code_t* code_desc, char** data, char** parity, int* missing_idxs,
                  int blocksize, int decode_parity)
{
    return run(code_desc, 1, data, parity, missing_idxs, decode_parity, blocksize);
}

int xor_reconstruct_one(xor_code_t* code_desc, char** data, char** parity, int* missing_idxs,
                        int index_to_reconstruct, int blocksize)
{
    return run(code_desc, 2, data, parity, missing_idxs, index_to_reconstruct, blocksize);
}

int xor_hd_fragments_needed(xor_code_t* code_desc, int* fragments_to_reconstruct,
                            int* fragments_to_exclude, int* fragments_needed)
{
    return ecamd_xor_fragments_needed(code_desc->k, code_desc->m, code_desc->hd,
                                      code_desc->parity_bms, code_desc->data_bms,
                                      fragments_to_reconstruct, fragments_to_exclude,
                                      fragments_needed);
}

xor_code_t* init_xor_hd_code(int k, int m, int hd)
{
    // Bitmap tables live as long as the library, like the reference's static arrays
    // (callers free() only the descriptor, src/backends/xor/flat_xor_hd.c:186-193).
    static std::mutex mu;
    static std::map<std::tuple<int, int, int>, std::pair<std::vector<unsigned int>,
                                                         std::vector<unsigned int>>> tables;
    std::vector<unsigned int> pb(m > 0 ? m : 1), db(k > 0 ? k : 1);
    if (k <= 0 || m <= 0 || ecamd_xor_code_tables(k, m, hd, pb.data(), db.data()) != 0)
        return nullptr;
    if (ecamd_init() != 0) {
        report("init_xor_hd_code");
        return nullptr;
    }
    auto* c = static_cast<xor_code_t*>(std::malloc(sizeof(xor_code_t)));
    if (!c) return nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto& t = tables[std::make_tuple(k, m, hd)];  // map nodes never move
        if (t.first.empty()) t = std::make_pair(pb, db);
        c->parity_bms = t.first.data();
        c->data_bms = t.second.data();
    }
    c->k = k;
    c->m = m;
    c->hd = hd;
    c->decode = xor_hd_decode;
    c->encode = xor_code_encode;
    c->fragments_needed = xor_hd_fragments_needed;
    return c;
}

}  // extern "C"
