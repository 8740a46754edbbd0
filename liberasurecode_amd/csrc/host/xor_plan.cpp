// xor_plan.cpp -- see xor_plan.hpp.  Every function below restates the control flow of the
// reference function named in its comment; buffer operations act on symbolic masks.
#include "xor_plan.hpp"

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>

namespace ecamd {

namespace {

// Parity bitmaps per (k, m, hd), include/xor_codes/xor_hd_code_defs.h:29-173 (code definitions).
struct CodeDef {
    int k, m, hd;
    std::vector<unsigned int> parity;
};

const std::vector<CodeDef>& code_defs()
{
    static const std::vector<CodeDef> defs = {
        {12, 6, 4, {1649, 3235, 2375, 718, 1436, 2872}},
        {10, 5, 3, {163, 300, 337, 582, 664}},
        {3, 3, 3, {5, 6, 3}},
        {6, 6, 3, {3, 48, 36, 24, 9, 6}},
        {7, 6, 3, {67, 112, 36, 24, 9, 6}},
        {8, 6, 3, {67, 112, 164, 152, 9, 6}},
        {9, 6, 3, {67, 112, 164, 152, 265, 262}},
        {10, 6, 3, {579, 112, 676, 152, 265, 262}},
        {11, 6, 3, {579, 1136, 676, 152, 1289, 262}},
        {12, 6, 3, {579, 1136, 676, 2200, 1289, 2310}},
        {13, 6, 3, {4675, 1136, 676, 6296, 1289, 2310}},
        {14, 6, 3, {4675, 9328, 676, 6296, 1289, 10502}},
        {15, 6, 3, {4675, 9328, 17060, 6296, 17673, 10502}},
        {6, 6, 4, {7, 56, 56, 11, 21, 38}},
        {7, 6, 4, {71, 120, 120, 11, 21, 38}},
        {8, 6, 4, {71, 120, 120, 139, 149, 166}},
        {9, 6, 4, {327, 376, 120, 395, 149, 166}},
        {10, 6, 4, {327, 376, 632, 395, 661, 678}},
        {11, 6, 4, {1351, 1400, 632, 395, 1685, 678}},
        {13, 6, 4, {5447, 5496, 2680, 2443, 1685, 6822}},
        {14, 6, 4, {5447, 5496, 10872, 10635, 9877, 6822}},
        {15, 6, 4, {21831, 5496, 27256, 27019, 9877, 6822}},
        {16, 6, 4, {21831, 38264, 27256, 27019, 42645, 39590}},
        {17, 6, 4, {87367, 38264, 92792, 27019, 108181, 39590}},
        {18, 6, 4, {87367, 169336, 92792, 158091, 108181, 170662}},
        {19, 6, 4, {349511, 169336, 354936, 158091, 108181, 432806}},
        {20, 6, 4, {349511, 693624, 354936, 682379, 632469, 432806}},
        {5, 5, 3, {3, 12, 17, 6, 24}},
        {6, 5, 3, {35, 44, 17, 6, 24}},
        {7, 5, 3, {35, 44, 81, 70, 24}},
        {8, 5, 3, {163, 44, 81, 70, 152}},
        {9, 5, 3, {163, 300, 337, 70, 152}},
        {5, 5, 4, {7, 25, 14, 19, 28}},
        {6, 5, 4, {39, 57, 46, 19, 28}},
        {7, 5, 4, {103, 57, 46, 83, 92}},
        {8, 5, 4, {103, 185, 174, 211, 92}},
        {9, 5, 4, {359, 441, 174, 211, 348}},
        {10, 5, 4, {359, 441, 686, 723, 860}},
    };
    return defs;
}

// data_bms[i] = set of parities covering data i (the transpose of the parity bitmaps; the
// reference lists them explicitly, tests check equality).
struct Tables {
    std::vector<unsigned int> parity, data;
};

const Tables* tables_for(int k, int m, int hd)
{
    static std::mutex mu;
    static std::map<std::tuple<int, int, int>, Tables> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(k, m, hd);
    auto it = cache.find(key);
    if (it != cache.end()) return &it->second;
    for (const auto& d : code_defs()) {
        if (d.k != k || d.m != m || d.hd != hd) continue;
        Tables t;
        t.parity = d.parity;
        t.data.assign(k, 0u);
        for (int j = 0; j < m; j++)
            for (int i = 0; i < k; i++)
                if ((t.parity[j] >> i) & 1u) t.data[i] |= 1u << j;
        return &cache.emplace(key, t).first->second;
    }
    return nullptr;
}

bool in_parity(int data_idx, unsigned int parity_bm) { return (parity_bm >> data_idx) & 1u; }
bool parity_has(int parity_rel, unsigned int data_bm) { return (data_bm >> parity_rel) & 1u; }

// A -1 terminated list as the reference keeps it (a fixed array; entries after the first -1
// are never read).
using List = std::vector<int>;

List terminated(const std::vector<int>& v)
{
    List l(v);
    l.push_back(-1);
    return l;
}

enum Pattern { GE_HD, P0D0P, P1D0P, P2D0P, P3D0P, P1D1P, P1D2P, P2D1P, P0D1P, P0D2P, P0D3P };

// get_failure_pattern, xor_code.c:74-128
Pattern failure_pattern(const XorCode& c, const List& missing)
{
    int nfail = 0;
    Pattern p = P0D0P;
    for (int i = 0; missing[i] > -1; i++) {
        nfail++;
        if (nfail >= c.hd) p = GE_HD;
        const bool d = missing[i] < c.k;
        switch (p) {
        case P0D0P: p = d ? P1D0P : P0D1P; break;
        case P1D0P: p = d ? P2D0P : P1D1P; break;
        case P2D0P: p = d ? P3D0P : P2D1P; break;
        case P3D0P: p = GE_HD; break;
        case P1D1P: p = d ? P2D1P : P1D2P; break;
        case P1D2P: p = GE_HD; break;
        case P2D1P: p = GE_HD; break;
        case P0D1P: p = d ? P1D1P : P0D2P; break;
        case P0D2P: p = d ? P1D2P : P0D3P; break;
        case P0D3P: p = GE_HD; break;
        default: break;
        }
        if (p == GE_HD) break;
    }
    return p;
}

List missing_data(const XorCode& c, const List& missing)  // get_missing_data, xor_code.c:224-239
{
    List out;
    for (int i = 0; missing[i] > -1; i++)
        if (missing[i] < c.k) out.push_back(missing[i]);
    out.push_back(-1);
    return out;
}

List missing_parity(const XorCode& c, const List& missing)  // get_missing_parity, :207-222
{
    List out;
    for (int i = 0; missing[i] > -1; i++)
        if (missing[i] >= c.k) out.push_back(missing[i]);
    out.push_back(-1);
    return out;
}

// num_missing_data_in_parity, xor_code.c:316-335 (parity_idx absolute)
int missing_data_in_parity(const XorCode& c, int parity_idx, const List* md)
{
    if (!md) return 0;
    int n = 0;
    const int rel = parity_idx - c.k;
    for (int i = 0; (*md)[i] > -1; i++)
        if (parity_has(rel, c.data_bms[(*md)[i]])) n++;
    return n;
}

// index_of_connected_parity, xor_code.c:337-371 (returns an absolute index or -1)
int connected_parity(const XorCode& c, int data_index, const List* mp, const List* md)
{
    for (int i = 0; i < c.m; i++) {
        if (missing_data_in_parity(c, i + c.k, md) > 1) continue;
        if (!in_parity(data_index, c.parity_bms[i])) continue;
        if (!mp) return i + c.k;
        bool gone = false;
        for (int j = 0; (*mp)[j] > -1; j++)
            if ((*mp)[j] == c.k + i) {
                gone = true;
                break;
            }
        if (!gone) return i + c.k;
    }
    return -1;
}

// remove_from_missing_list, xor_code.c:373-395 (element is always present when called)
void remove_from_list(int element, List& l)
{
    int elem_idx = -1, n = 0;
    for (n = 0; n < static_cast<int>(l.size()) && l[n] > -1; n++) {  // visits every entry
        if (l[n] == element) {
            elem_idx = n;
            l[n] = -1;
        }
    }
    for (int i = elem_idx; i >= 0 && i < n - 1; i++) std::swap(l[i], l[i + 1]);
}

// ---- symbolic buffers --------------------------------------------------------------------

struct Sym {
    const XorCode& c;
    std::vector<uint64_t> mask;  // k + m buffers + 1 scratch (P^Q)
    std::vector<char> touched;
    explicit Sym(const XorCode& code) : c(code), mask(code.k + code.m + 1, 0), touched(mask.size(), 0)
    {
        for (int i = 0; i < c.k + c.m; i++) mask[i] = 1ull << i;
    }
    int data(int i) const { return i; }
    int parity(int rel) const { return c.k + rel; }
    int scratch() const { return c.k + c.m; }
    void copy(int dst, int src) { mask[dst] = mask[src]; touched[dst] = 1; }
    void xor_into(int src, int dst) { mask[dst] ^= mask[src]; touched[dst] = 1; }
    void zero(int dst) { mask[dst] = 0; touched[dst] = 1; }
    XorPlan finish(int rc) const
    {
        XorPlan p;
        p.rc = rc;
        for (int i = 0; i < c.k + c.m; i++)
            if (touched[i]) {
                p.outputs.push_back(i);
                p.sources.push_back(mask[i]);
            }
        return p;
    }
};

// decode_one_data, xor_hd_code.c:418-439
int decode_one(Sym& b, const List& md, const List* mp)
{
    const XorCode& c = b.c;
    int di = md[0];
    int pi = connected_parity(c, di, mp, &md);
    if (pi < 0) return -2;  // the reference would index parity[-1 - k] here (never reached)
    b.copy(b.data(di), b.parity(pi - c.k));
    for (int i = 0; i < c.k; i++)
        if (i != di && in_parity(i, c.parity_bms[pi - c.k])) b.xor_into(b.data(i), b.data(di));
    return 0;
}

// decode_two_data, xor_hd_code.c:441-478
int decode_two(Sym& b, List& md, const List* mp)
{
    const XorCode& c = b.c;
    int di = md[0];
    int pi = connected_parity(c, di, mp, &md);
    if (pi < 0) {
        di = md[1];
        pi = connected_parity(c, di, mp, &md);
        if (pi < 0) return -2;
        md[1] = -1;
    } else {
        md[0] = md[1];
        md[1] = -1;
    }
    b.copy(b.data(di), b.parity(pi - c.k));
    for (int i = 0; i < c.k; i++)
        if (i != di && in_parity(i, c.parity_bms[pi - c.k])) b.xor_into(b.data(i), b.data(di));
    decode_one(b, md, mp);
    return 0;
}

// decode_three_data, xor_hd_code.c:480-572
int decode_three(Sym& b, List& md, const List* mp)
{
    const XorCode& c = b.c;
    int pi = -1, di = -1;
    unsigned int pbm = ~0u;
    int src = -1;
    for (int i = 0; md[i] > -1; i++) {
        pi = connected_parity(c, md[i], mp, &md);
        if (pi > -1) {
            di = md[i];
            src = b.parity(pi - c.k);
            pbm = c.parity_bms[pi - c.k];
            break;
        }
    }
    if (pi < 0) {
        int c2 = -1, c3 = -1;
        for (int i = 0; i < c.m; i++) {
            int n = missing_data_in_parity(c, c.k + i, &md);
            if (n == 2 && c2 < 0)
                c2 = i;
            else if (n == 3 && c3 < 0)
                c3 = i;
        }
        if (c2 < 0 || c3 < 0) return -2;
        pbm = c.parity_bms[c2] ^ c.parity_bms[c3];
        b.copy(b.scratch(), b.parity(c2));
        b.xor_into(b.parity(c3), b.scratch());
        di = -1;
        for (int i = 0; md[i] > -1; i++)
            if (in_parity(md[i], pbm)) {
                di = md[i];
                break;
            }
        if (di < 0) return -2;
        src = b.scratch();
    }
    b.copy(b.data(di), src);
    for (int i = 0; i < c.k; i++)
        if (i != di && in_parity(i, pbm)) b.xor_into(b.data(i), b.data(di));
    remove_from_list(di, md);
    return decode_two(b, md, mp);
}

// selective_encode, xor_code.c:193-207
void selective_encode(Sym& b, const List& mp)
{
    const XorCode& c = b.c;
    for (int i = 0; i < c.k; i++)
        for (int j = 0; mp[j] > -1; j++) {
            int rel = mp[j] - c.k;
            if (in_parity(i, c.parity_bms[rel])) b.xor_into(b.data(i), b.parity(rel));
        }
}

// xor_hd_decode, xor_hd_code.c:574-662
int decode(Sym& b, const List& missing, int decode_parity)
{
    const XorCode& c = b.c;
    int ret = 0;
    Pattern p = failure_pattern(c, missing);
    List md = missing_data(c, missing), mp = missing_parity(c, missing);
    switch (p) {
    case P0D0P: break;
    case P1D0P: decode_one(b, md, nullptr); break;
    case P2D0P: ret = decode_two(b, md, nullptr); break;
    case P3D0P: ret = decode_three(b, md, nullptr); break;
    case P1D1P:
    case P1D2P:
        decode_one(b, md, &mp);
        if (decode_parity) selective_encode(b, mp);
        break;
    case P2D1P:
        ret = decode_two(b, md, &mp);
        if (decode_parity) selective_encode(b, mp);
        break;
    case P0D1P:
    case P0D2P:
    case P0D3P:
        if (decode_parity) selective_encode(b, mp);
        break;
    default: ret = -1; break;
    }
    return ret;
}

// ---- fragments_needed (pure index logic) ---------------------------------------------------

// fragments_needed_one_data, xor_hd_code.c:33-53
int fn_one(const XorCode& c, const List& md, const List* mp, unsigned& dbm, unsigned& pbm)
{
    int di = md[0];
    int pi = connected_parity(c, di, mp, &md);
    if (pi < 0) return -1;
    dbm |= c.parity_bms[pi - c.k];
    pbm |= 1u << (pi - c.k);
    dbm &= ~(1u << di);
    return 0;
}

// fragments_needed_two_data, xor_hd_code.c:55-88
int fn_two(const XorCode& c, List& md, const List* mp, unsigned& dbm, unsigned& pbm)
{
    int di = md[0];
    int pi = connected_parity(c, di, mp, &md);
    if (pi < 0) {
        di = md[1];
        pi = connected_parity(c, di, mp, &md);
        if (pi < 0) return -1;
        md[1] = -1;
    } else {
        md[0] = md[1];
        md[1] = -1;
    }
    dbm |= c.parity_bms[pi - c.k];
    pbm |= 1u << (pi - c.k);
    int ret = fn_one(c, md, mp, dbm, pbm);
    dbm &= ~(1u << di);
    return ret;
}

// fragments_needed_three_data, xor_hd_code.c:90-168.  The reference shifts by the RELATIVE
// parity index minus k (`1 << (contains_2d - k)`), a negative count; x86 `shl` masks the count
// to 5 bits, which is what the reference build computes and what is reproduced here.
int fn_three(const XorCode& c, List& md, const List* mp, unsigned& dbm, unsigned& pbm)
{
    int pi = -1, di = -1, c2 = -1, c3 = -1;
    unsigned tmp = ~0u;
    for (int i = 0; md[i] > -1; i++) {
        pi = connected_parity(c, md[i], mp, &md);
        if (pi > -1) {
            di = md[i];
            tmp = c.parity_bms[pi - c.k];
            break;
        }
    }
    if (pi < 0) {
        for (int i = 0; i < c.m; i++) {
            int n = missing_data_in_parity(c, c.k + i, &md);
            if (n == 2 && c2 < 0)
                c2 = i;
            else if (n == 3 && c3 < 0)
                c3 = i;
        }
        if (c2 < 0 || c3 < 0) return -1;
        tmp = c.parity_bms[c2] ^ c.parity_bms[c3];
        di = -1;
        for (int i = 0; md[i] > -1; i++)
            if (in_parity(md[i], tmp)) {
                di = md[i];
                break;
            }
        if (di < 0) return -1;
    }
    remove_from_list(di, md);
    if (pi > -1) {
        pbm |= 1u << (pi - c.k);
        dbm |= c.parity_bms[pi - c.k];
    } else {
        pbm |= 1u << ((c2 - c.k) & 31);
        pbm |= 1u << ((c3 - c.k) & 31);
        dbm |= tmp;
    }
    int ret = fn_two(c, md, mp, dbm, pbm);
    dbm &= ~(1u << di);
    return ret;
}

}  // namespace

bool xor_code_lookup(int k, int m, int hd, XorCode& out)
{
    // validity exactly as init_xor_hd_code, xor_hd_code.c:664-693
    bool ok = false;
    if (hd == 3)
        ok = (m == 6 && k >= 6 && k <= 15) || (m == 5 && k >= 5 && k <= 10) || (m == 3 && k == 3);
    if (hd == 4) ok = (m == 6 && k >= 6 && k <= 20) || (m == 5 && k >= 5 && k <= 10);
    if (!ok) return false;
    const Tables* t = tables_for(k, m, hd);
    if (!t) return false;
    out.k = k;
    out.m = m;
    out.hd = hd;
    out.parity_bms = t->parity.data();
    out.data_bms = t->data.data();
    return true;
}

XorPlan xor_plan_encode(const XorCode& c)
{
    Sym b(c);
    for (int i = 0; i < c.k; i++)  // xor_code_encode, xor_code.c:180-191
        for (int j = 0; j < c.m; j++)
            if (in_parity(i, c.parity_bms[j])) b.xor_into(b.data(i), b.parity(j));
    return b.finish(0);
}

XorPlan xor_plan_decode(const XorCode& c, const std::vector<int>& missing, int decode_parity)
{
    Sym b(c);
    int rc = decode(b, terminated(missing), decode_parity);
    return b.finish(rc);
}

XorPlan xor_plan_reconstruct_one(const XorCode& c, const std::vector<int>& missing, int index)
{
    // xor_reconstruct_one, xor_code.c:248-314
    Sym b(c);
    const List miss = terminated(missing);
    List md = missing_data(c, miss), mp = missing_parity(c, miss);
    int ret;
    if (index < c.k) {
        int cp = connected_parity(c, index, &mp, &md);
        if (cp >= 0) {
            int rel = cp - c.k;
            b.copy(b.data(index), b.parity(rel));
            for (int i = 0; i < c.k; i++)
                if (in_parity(i, c.parity_bms[rel]) && i != index) b.xor_into(b.data(i), b.data(index));
            ret = 0;
        } else {
            ret = decode(b, miss, 1);
        }
    } else {
        if (missing_data_in_parity(c, index, &md) == 0) {
            int rel = index - c.k;
            b.zero(b.parity(rel));
            for (int i = 0; i < c.k; i++)
                if (in_parity(i, c.parity_bms[rel])) b.xor_into(b.data(i), b.parity(rel));
            ret = 0;
        } else {
            ret = decode(b, miss, 1);
        }
    }
    return b.finish(ret);
}

int xor_fragments_needed(const XorCode& c, const std::vector<int>& to_reconstruct,
                         const std::vector<int>& to_exclude, std::vector<int>& needed)
{
    // xor_hd_fragments_needed, xor_hd_code.c:209-412
    const List rec = terminated(to_reconstruct), exc = terminated(to_exclude);
    Pattern p = failure_pattern(c, rec);
    unsigned dbm = 0, pbm = 0;
    int ret = -1;
    if (p == P1D0P) {  // fragments_needed_one_data_local, :170-191
        List md = missing_data(c, exc), mp = missing_parity(c, exc);
        int pi = connected_parity(c, rec[0], &mp, &md);
        if (pi >= 0) {
            dbm |= c.parity_bms[pi - c.k];
            pbm |= 1u << (pi - c.k);
            dbm &= ~(1u << rec[0]);
            ret = 0;
        }
    }
    if (ret == -1) {
        List all;
        for (int i = 0; rec[i] > -1; i++) all.push_back(rec[i]);
        for (int i = 0; exc[i] > -1; i++) all.push_back(exc[i]);
        all.push_back(-1);
        p = failure_pattern(c, all);
        List md = missing_data(c, all), mp = missing_parity(c, all);
        unsigned mdbm = 0;
        for (int i = 0; md[i] > -1; i++) mdbm |= 1u << md[i];
        switch (p) {
        case P0D0P: break;
        case P1D0P: ret = fn_one(c, md, nullptr, dbm, pbm); break;
        case P2D0P: ret = fn_two(c, md, nullptr, dbm, pbm); break;
        case P3D0P: ret = fn_three(c, md, nullptr, dbm, pbm); break;
        case P1D1P:
        case P1D2P:
        case P2D1P:
            ret = (p == P2D1P) ? fn_two(c, md, &mp, dbm, pbm) : fn_one(c, md, &mp, dbm, pbm);
            for (int i = 0; mp[i] > -1; i++) {
                dbm |= c.parity_bms[mp[i] - c.k];
                dbm &= ~mdbm;
            }
            break;
        case P0D1P:
        case P0D2P:
        case P0D3P:
            for (int i = 0; mp[i] > -1; i++) dbm |= c.parity_bms[mp[i] - c.k];
            ret = 0;
            break;
        default: ret = -1; break;
        }
    }
    needed.clear();
    if (ret >= 0) {
        for (int i = 0; dbm; i++, dbm >>= 1)
            if (dbm & 1u) needed.push_back(i);
        for (int i = 0; pbm; i++, pbm >>= 1)
            if (pbm & 1u) needed.push_back(i + c.k);
        needed.push_back(-1);
    }
    return ret;
}

}  // namespace ecamd
