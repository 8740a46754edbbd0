// xor_plan.hpp -- flat-XOR HD codes: code tables and exact decode planning.
//
// The reference decodes by a sequence of buffer copies and XORs whose choice depends on the
// erasure pattern (src/builtin/xor_codes/xor_hd_code.c:418-662, xor_code.c:193-314).  Here that
// control flow is replayed SYMBOLICALLY: every buffer carries the set (bitmask) of the ORIGINAL
// k+m buffer contents it is the XOR of.  The result is, for each buffer the reference would
// modify, the exact set of original buffers whose XOR it ends up holding -- which one GPU launch
// (xor_apply_kernel) then computes for any number of stripes.  Bit-exact with the reference for
// any input, consistent or not, including its partial writes before a failure return.
#pragma once
#include <cstdint>
#include <vector>

namespace ecamd {

struct XorCode {
    int k = 0, m = 0, hd = 0;
    const unsigned int* parity_bms = nullptr;  // m entries: data bits in each parity
    const unsigned int* data_bms = nullptr;    // k entries: parity bits covering each data
};

// The reference's hand-made / "goldilocks" tables (include/xor_codes/xor_hd_code_defs.h:29-173);
// false if (k, m, hd) is not one of the supported codes (xor_hd_code.c:664-708).
bool xor_code_lookup(int k, int m, int hd, XorCode& out);

// Result of a planned operation: final content of each modified buffer.
struct XorPlan {
    int rc = 0;                       // the reference's return code
    std::vector<int> outputs;         // buffer indices (0..k-1 data, k.. parity) modified
    std::vector<uint64_t> sources;    // per output: bitmask over ORIGINAL buffers to XOR
};

// xor_code_encode: parity[j] ^= data[i] for i in parity_bms[j] (accumulates).
XorPlan xor_plan_encode(const XorCode& c);
// xor_hd_decode(..., missing, decode_parity).
XorPlan xor_plan_decode(const XorCode& c, const std::vector<int>& missing, int decode_parity);
// xor_reconstruct_one(..., missing, index).
XorPlan xor_plan_reconstruct_one(const XorCode& c, const std::vector<int>& missing, int index);

// xor_hd_fragments_needed: fills `needed` (ends with -1); returns the reference's rc.
int xor_fragments_needed(const XorCode& c, const std::vector<int>& to_reconstruct,
                         const std::vector<int>& to_exclude, std::vector<int>& needed);

}  // namespace ecamd
