// crc.cpp -- checksum machines and device table images (see crc.hpp).
#include "crc.hpp"

#include <algorithm>
#include <cstddef>
#include <map>
#include <mutex>
#include <tuple>

#include <cstring>

namespace ecamd {

CrcMachine::CrcMachine(bool legacy_variant) : legacy(legacy_variant)
{
    // The reflected CRC-32 byte table (polynomial 0xEDB88320) shared by both variants.
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        t[n] = c;
    }
}

Mat32 mat_mul(const Mat32& a, const Mat32& b)
{
    Mat32 r;
    for (int i = 0; i < 32; i++) r.col[i] = a.apply(b.col[i]);
    return r;
}

Mat32 zero_shift(const CrcMachine& m, uint64_t nbytes)
{
    Mat32 step, acc;
    for (int b = 0; b < 32; b++) {
        step.col[b] = m.step(1u << b, 0);
        acc.col[b] = 1u << b;
    }
    while (nbytes) {
        if (nbytes & 1u) acc = mat_mul(step, acc);
        step = mat_mul(step, step);
        nbytes >>= 1;
    }
    return acc;
}

Mat32 mat_inverse(const Mat32& a)
{
    // Gauss-Jordan over GF(2) on rows: row i of a (bit i of every column) beside row i of I
    uint32_t row[32], inv[32];
    for (int i = 0; i < 32; i++) {
        row[i] = 0;
        for (int b = 0; b < 32; b++) row[i] |= ((a.col[b] >> i) & 1u) << b;
        inv[i] = 1u << i;
    }
    for (int c = 0; c < 32; c++) {
        int p = c;
        while (p < 32 && !((row[p] >> c) & 1u)) p++;
        if (p == 32) return Mat32{};  // singular (never for a CRC zero-byte step)
        std::swap(row[p], row[c]);
        std::swap(inv[p], inv[c]);
        for (int r = 0; r < 32; r++)
            if (r != c && ((row[r] >> c) & 1u)) {
                row[r] ^= row[c];
                inv[r] ^= inv[c];
            }
    }
    Mat32 out;
    for (int b = 0; b < 32; b++) {
        out.col[b] = 0;
        for (int i = 0; i < 32; i++) out.col[b] |= ((inv[i] >> b) & 1u) << i;
    }
    return out;
}

std::vector<uint32_t> build_small_crc_image(const CrcMachine& m, int G)
{
    const int region = 256 * G, np = region / 16;
    const CrcImage pieces = build_crc_image(m, 5, 4, 4, false);  // byte tables for dword 0, nibbles after
    const size_t pw = 4 * 256 + 3 * 8 * 16;
    std::vector<uint32_t> w(pw + static_cast<size_t>(np + 6) * 128, 0);
    std::copy(pieces.words.begin(), pieces.words.begin() + static_cast<std::ptrdiff_t>(pw), w.begin());
    for (int l = 0; l < np; l++)
        field_tables(zero_shift(m, 16ull * static_cast<uint64_t>(np - 1 - l)), 4, w.data() + pw + 128 * l);
    for (int i = 0; i < 6; i++)
        field_tables(zero_shift(m, static_cast<uint64_t>(region) << i), 4, w.data() + pw + 128 * (np + i));
    return w;
}

SmallCrcConst small_crc_const(bool legacy, uint64_t len, uint64_t zext)
{
    static std::mutex mu;
    static auto& cache = *new std::map<std::tuple<bool, uint64_t, uint64_t>, SmallCrcConst>();
    static const CrcMachine machines[2] = {CrcMachine(false), CrcMachine(true)};
    const auto key = std::make_tuple(legacy, len, zext);
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    const CrcMachine& m = machines[legacy ? 1 : 0];
    SmallCrcConst k{};
    const Mat32 inv = mat_inverse(zero_shift(m, zext));
    std::copy(inv.col, inv.col + 32, k.minv);
    k.c = zero_shift(m, len).apply(~0u);
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() > 65536) cache.clear();
    return cache.emplace(key, k).first->second;
}

void field_tables(const Mat32& M, int B, uint32_t* out)
{
    const int E = 1 << B;
    for (int f = 0; f < 32 / B; f++)
        for (int v = 0; v < E; v++) out[f * E + v] = M.apply(static_cast<uint32_t>(v) << (f * B));
}

CrcImage build_crc_image(const CrcMachine& m, int B, int J, int G, bool pos)
{
    CrcImage img;
    img.B = B;
    img.G = G;
    img.J = J;
    // B = 8: byte tables for all 4 dwords of a piece; 4: nibble tables; 5..7: byte tables for the
    // first B - 4 dwords, nibble tables for the rest (crc_partial_kernel<MB = B-4 or 4 or 0, G>).
    const int mb = B == 8 ? 4 : B - 4;
    size_t pw = 0;
    for (int word = 0; word < 4; word++) pw += word < mb ? 4 * 256 : 8 * 16;
    const size_t piece = pos ? 4 * pw : pw;
    const size_t fields = static_cast<size_t>(32 / G) << G;  // one gap / level map
    img.lds_words = piece + fields * 7;
    img.span_off = img.lds_words;
    img.t_off = img.span_off + 4 * 256;
    img.words.assign(img.t_off + 256, 0);
    uint32_t* w = img.words.data();
    // piece tables: word w of the 16-byte piece = v << (f * b), the rest zero; r0 by running it
    // (then shifted to the group's last piece for position set u when pos).
    for (int u = 0; u < (pos ? 4 : 1); u++) {
        const Mat32 sh = zero_shift(m, pos ? 1024ull * (3 - u) : 0);
        size_t off = u * pw;
        for (int word = 0; word < 4; word++) {
            const int b = word < mb ? 8 : 4, E = 1 << b, NF = 32 / b;
            for (int f = 0; f < NF; f++)
                for (int v = 0; v < E; v++) {
                    uint8_t bytes[16] = {0};
                    const uint32_t x = static_cast<uint32_t>(v) << (f * b);
                    for (int q = 0; q < 4; q++) bytes[4 * word + q] = static_cast<uint8_t>(x >> (8 * q));
                    w[off + static_cast<size_t>(f) * E + v] = sh.apply(m.run(0, bytes, 16));
                }
            off += static_cast<size_t>(NF) * E;
        }
    }
    field_tables(zero_shift(m, pos ? 4 * 1024 : 64 * 16), G, w + piece);
    for (int t = 0; t < 6; t++) field_tables(zero_shift(m, 16ull << t), G, w + piece + fields * (1 + t));
    field_tables(zero_shift(m, static_cast<uint64_t>(J) * 1024), 8, w + img.span_off);
    std::memcpy(w + img.t_off, m.t, sizeof(m.t));
    return img;
}

std::vector<uint32_t> build_fused_crc_image_pos(const CrcMachine& m, uint64_t step, int npos, bool nib, int mb)
{
    // npos sets of all-byte (or all-nibble, or byte for the first mb dwords) piece tables, set u
    // shifted to the group's last piece (A^(step*(npos-1-u)) folded in), then the gap map
    // A^(step*npos) and the 6 butterfly levels and A^1024 of build_fused_crc_image, then the
    // lane-shift tables
    mb = nib ? 0 : std::clamp(mb, 0, 4);
    const CrcImage pieces = build_crc_image(m, mb == 4 ? 8 : 4 + mb, 4, 4, false);
    const size_t pw = static_cast<size_t>(mb) * 4 * 256 + static_cast<size_t>(4 - mb) * 8 * 16;
    std::vector<uint32_t> w(static_cast<size_t>(npos) * pw + 8 * 128, 0);
    for (int u = 0; u < npos; u++) {
        const Mat32 sh = zero_shift(m, step * static_cast<uint64_t>(npos - 1 - u));
        for (size_t i = 0; i < pw; i++) w[u * pw + i] = sh.apply(pieces.words[i]);
    }
    uint32_t* maps = w.data() + static_cast<size_t>(npos) * pw;
    field_tables(zero_shift(m, step * static_cast<uint64_t>(npos)), 4, maps);
    for (int t = 0; t < 6; t++) field_tables(zero_shift(m, 16ull << t), 4, maps + 128 * (1 + t));
    field_tables(zero_shift(m, 1024), 4, maps + 128 * 7);
    // lane-shift tables (the fold-each kernel of maps of 5-8 outputs): lane l's map A^(16 (63 - l))
    // as 8 nibble tables, word ((t * 16 + n) * 64 + l), so the 32 lanes of a bank group read 32
    // distinct banks
    w.resize(w.size() + 8 * 16 * 64, 0);
    uint32_t* lanes = w.data() + static_cast<size_t>(npos) * pw + 8 * 128;
    uint32_t tab[128];
    for (int l = 0; l < 64; l++) {
        field_tables(zero_shift(m, 16ull * static_cast<uint64_t>(63 - l)), 4, tab);
        for (int i = 0; i < 128; i++) lanes[static_cast<size_t>(i) * 64 + l] = tab[i];
    }
    return w;
}

std::vector<uint32_t> build_fused_crc_image(const CrcMachine& m, uint64_t tile_bytes, int mb)
{
    // piece tables first: byte tables for the first mb dwords (B = 4 + mb; 8 = all four)
    const CrcImage pieces = build_crc_image(m, mb == 4 ? 8 : 4 + mb, 4, 4, false);
    size_t pw = static_cast<size_t>(mb) * 4 * 256 + static_cast<size_t>(4 - mb) * 8 * 16;
    std::vector<uint32_t> w(pw + 8 * 128, 0);
    std::copy(pieces.words.begin(), pieces.words.begin() + static_cast<std::ptrdiff_t>(pw), w.begin());
    field_tables(zero_shift(m, tile_bytes), 4, w.data() + pw);
    for (int t = 0; t < 6; t++) field_tables(zero_shift(m, 16ull << t), 4, w.data() + pw + 128 * (1 + t));
    field_tables(zero_shift(m, 1024), 4, w.data() + pw + 128 * 7);
    return w;
}

}  // namespace ecamd
