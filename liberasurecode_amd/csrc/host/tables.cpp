#include "tables.hpp"

#include <cstring>

#include "gf16.hpp"

namespace ecamd {

std::vector<uint8_t> build_split_tables(const std::vector<int>& coeff, int R, int K, int row0,
                                        int width, int col0, int ncols)
{
    const GF16& gf = GF16::get();
    const int eb = entry_bytes(width);
    std::vector<uint8_t> img(static_cast<size_t>(ncols) * 512 * eb, 0);
    for (int jj = 0; jj < ncols; jj++) {
        const int j = col0 + jj;
        uint8_t* lo = img.data() + static_cast<size_t>(jj) * 512 * eb;
        uint8_t* hi = lo + 256 * eb;
        for (int w = 0; w < width; w++) {
            const int r = row0 + w;
            if (r >= R) break;
            const int c = coeff[static_cast<size_t>(r) * K + j];
            const int c_hi = gf.mul(c, 0x100);
            for (int b = 0; b < 256; b++) {
                uint16_t vlo = static_cast<uint16_t>(gf.mul(c, b));
                uint16_t vhi = static_cast<uint16_t>(gf.mul(c_hi, b));
                std::memcpy(lo + b * eb + 2 * w, &vlo, 2);  // little-endian 16-bit lanes
                std::memcpy(hi + b * eb + 2 * w, &vhi, 2);
            }
        }
    }
    return img;
}

}  // namespace ecamd

namespace ecamd {

std::vector<uint8_t> build_nibble_tables(const std::vector<int>& coeff, int R, int K, int row0,
                                         int width, int col0, int ncols)
{
    const GF16& gf = GF16::get();
    const int eb = entry_bytes(width);
    std::vector<uint8_t> img(static_cast<size_t>(ncols) * 64 * eb, 0);
    for (int jj = 0; jj < ncols; jj++) {
        const int j = col0 + jj;
        uint8_t* base = img.data() + static_cast<size_t>(jj) * 64 * eb;
        for (int w = 0; w < width; w++) {
            const int r = row0 + w;
            if (r >= R) break;
            const int c = coeff[static_cast<size_t>(r) * K + j];
            for (int q = 0; q < 4; q++)
                for (int n = 0; n < 16; n++) {
                    const uint16_t v = static_cast<uint16_t>(gf.mul(c, n << (4 * q)));
                    std::memcpy(base + (q * 16 + n) * eb + 2 * w, &v, 2);
                }
        }
    }
    return img;
}

}  // namespace ecamd
