// ecamd_crc_dev.hpp -- device side of the CRC32 table maps (host/crc.hpp has the algebra): a
// GF(2)-linear map of a 32-bit state applied through B-bit field tables in LDS, and the r0 of a
// 16-byte piece.  Shared by the CRC kernels (ecamd_frame.hip) and the fused framed encode
// (ecamd_frame_fused.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ecamd_isa.hpp"

namespace ecamd {
namespace crcdev {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 4 * byte K of v in one VALU op (ecamd_isa.hpp).
template <int K>
__device__ __forceinline__ uint32_t byte_x4(uint32_t v)
{
    return byte_shl<K, 2>(v);
}

template <int B>
__device__ __forceinline__ uint32_t lmap(const uint32_t* tab, uint32_t x)
{
    constexpr int E = 1 << B;
    const char* t = reinterpret_cast<const char*>(tab);
    auto at = [&](int f, uint32_t off) { return *reinterpret_cast<const uint32_t*>(t + f * E * 4 + off); };
    if constexpr (B == 4) {
        // Spread the nibbles into bytes once (3 ops for 8 fields); every lookup address is then
        // one SDWA byte-select shift (the compiler re-fuses a plain shift+mask, hence the asm).
        const uint32_t lo = x & 0x0f0f0f0fu, hi = (x >> 4) & 0x0f0f0f0fu;
        const uint32_t a = xor3(at(0, byte_x4<0>(lo)), at(1, byte_x4<0>(hi)), at(2, byte_x4<1>(lo)));
        const uint32_t b = xor3(at(3, byte_x4<1>(hi)), at(4, byte_x4<2>(lo)), at(5, byte_x4<2>(hi)));
        return xor3(a, b, at(6, byte_x4<3>(lo)) ^ at(7, byte_x4<3>(hi)));
    } else {
        static_assert(B == 8, "byte or nibble tables");
        return xor3(at(0, byte_x4<0>(x)), at(1, byte_x4<1>(x)), at(2, byte_x4<2>(x))) ^ at(3, byte_x4<3>(x));
    }
}

// Piece tables of dword w: byte tables (4 x 256 words) for the first MB dwords, nibble tables
// (8 x 16 words) for the rest -- MB trades LDS bank conflicts (byte tables) against VALU work
// (nibble tables: twice the lookups, conflict-free).
constexpr int piece_off(int MB, int w) { return (w < MB ? w : MB) * 1024 + (w < MB ? 0 : w - MB) * 128; }
constexpr int piece_words(int MB) { return piece_off(MB, 4); }

template <int MB, typename V>
__device__ __forceinline__ uint32_t piece_r0(const uint32_t* tab, V v)
{
    auto map = [&](auto W, uint32_t x) {
        constexpr int w = decltype(W)::value;
        if constexpr (w < MB)
            return lmap<8>(tab + piece_off(MB, w), x);
        else
            return lmap<4>(tab + piece_off(MB, w), x);
    };
    return xor3(map(std::integral_constant<int, 0>{}, v.x), map(std::integral_constant<int, 1>{}, v.y),
                map(std::integral_constant<int, 2>{}, v.z)) ^
           map(std::integral_constant<int, 3>{}, v.w);
}


}  // namespace crcdev
}  // namespace ecamd
