// ecamd_isa.hpp -- two gfx950 VALU idioms the compiler does not pick on its own for the table
// lookups of the GF(2^16) and CRC kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ecamd {

// a ^ b ^ c in one VALU op (v_bitop3_b32 with truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// a ^ (b & c) in one VALU op (v_bitop3_b32, truth table 0x78): masked accumulate.
__device__ __forceinline__ uint32_t xor_and(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x78" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

// (byte K of v) << S in one VALU op: v_lshlrev_b32 with an SDWA byte-select source.  Given a
// shift-and-mask instead, the compiler re-fuses it into two ops.
template <int K, int S>
__device__ __forceinline__ uint32_t byte_shl(uint32_t v)
{
    static_assert(K >= 0 && K < 4 && S >= 0 && S < 32, "byte select");
    uint32_t r;
    if constexpr (K == 0)
        asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
            : "=v"(r) : "v"(v), "i"(S));
    else if constexpr (K == 1)
        asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
            : "=v"(r) : "v"(v), "i"(S));
    else if constexpr (K == 2)
        asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
            : "=v"(r) : "v"(v), "i"(S));
    else
        asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
            : "=v"(r) : "v"(v), "i"(S));
    return r;
}

}  // namespace ecamd
