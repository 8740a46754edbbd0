// ecamd_apply.hpp -- device helpers of the gf16 kernels (16-byte streaming loads / stores, byte-exact
// fragment tails, LDS table entries, the split-table multiply-accumulate and one tile of the
// generic apply), shared by ecamd_kernels.hip and the gf16_stream_kernel instantiation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ecamd_isa.hpp"
#include "ecamd_kernels.hpp"

namespace ecamd {

namespace {

__device__ __forceinline__ uint4 load16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 stream_load16(const uint8_t* p)
{
    if constexpr (NT) {
        u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *reinterpret_cast<const uint4*>(p);
    }
}

template <bool NT>
__device__ __forceinline__ void stream_store16(uint8_t* p, uint4 v)
{
    if constexpr (NT) {
        u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
    } else {
        *reinterpret_cast<uint4*>(p) = v;
    }
}

// Partial 16-byte chunk at the end of a fragment: bytes [0, rem) of p, zero filled (rem >= 16:
// one 16-byte load).
__device__ __forceinline__ uint4 load_tail(const uint8_t* p, int rem)
{
    if (rem >= 16) return *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; i++) {
        uint32_t b = (i < rem) ? static_cast<uint32_t>(p[i]) : 0u;
        w[i >> 2] |= b << (8 * (i & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_tail(uint8_t* p, uint4 v, int rem)
{
    if (rem >= 16) {
        *reinterpret_cast<uint4*>(p) = v;
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; i++)
        if (i < rem) p[i] = static_cast<uint8_t>(w[i >> 2] >> (8 * (i & 3)));
}

template <bool PTRS>
__device__ __forceinline__ const uint8_t* in_frag(const ApplyArgs& a, uint32_t s, int j)
{
    if constexpr (PTRS)
        return a.in_ptrs[static_cast<int64_t>(s) * a.in_stride + a.in_off[j]];
    else
        return a.in_base + static_cast<int64_t>(s) * a.in_stride + a.in_off[j];
}

template <bool PTRS>
__device__ __forceinline__ uint8_t* out_frag(const ApplyArgs& a, uint32_t s, int r)
{
    if constexpr (PTRS)
        return a.out_ptrs[static_cast<int64_t>(s) * a.out_stride + a.out_off[r]];
    else
        return a.out_base + static_cast<int64_t>(s) * a.out_stride + a.out_off[r];
}

// One LDS table entry of D dwords (D = W/2): ds_read_b32 / b64 / b128.
template <int D>
__device__ __forceinline__ void lds_entry(const uint8_t* p, uint32_t (&e)[D])
{
    if constexpr (D == 1) {
        e[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (D == 2) {
        uint2 v = *reinterpret_cast<const uint2*>(p);
        e[0] = v.x;
        e[1] = v.y;
    } else {
        uint4 v = *reinterpret_cast<const uint4*>(p);
        e[0] = v.x;
        e[1] = v.y;
        e[2] = v.z;
        e[3] = v.w;
    }
}

// acc[w] ^= T_lo[j][lo(x_w)] ^ T_hi[j][hi(x_w)] for the 8 words of one 16-byte chunk.
template <int W>
__device__ __forceinline__ void mac_chunk(const uint8_t* tl, uint4 x, uint32_t (&acc)[8][W / 2])
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    const uint8_t* th = tl + 256 * EB;
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const uint32_t v = xs[w >> 1] >> ((w & 1) * 16);
        uint32_t e0[D], e1[D];
        lds_entry<D>(tl + (v & 0xffu) * EB, e0);
        lds_entry<D>(th + ((v >> 8) & 0xffu) * EB, e1);
#pragma unroll
        for (int d = 0; d < D; d++) acc[w][d] = xor3(acc[w][d], e0[d], e1[d]);
    }
}

constexpr int log2i(int v) { return v <= 1 ? 0 : 1 + log2i(v / 2); }

// Nibble tables (host/tables.hpp build_nibble_tables): four conflict-free lookups per word.  The
// nibbles of a data dword are spread into bytes once; each table offset is then one SDWA shift.
template <int W, int H>
__device__ __forceinline__ void mac_word_nib(const uint8_t* t, uint32_t lo, uint32_t hi,
                                             uint32_t (&acc)[W / 2])
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    constexpr int S = log2i(EB);
    uint32_t e0[D], e1[D], e2[D], e3[D];
    lds_entry<D>(t + 0 * 16 * EB + byte_shl<2 * H, S>(lo), e0);      // bits 0-3 of the word
    lds_entry<D>(t + 1 * 16 * EB + byte_shl<2 * H, S>(hi), e1);      // bits 4-7
    lds_entry<D>(t + 2 * 16 * EB + byte_shl<2 * H + 1, S>(lo), e2);  // bits 8-11
    lds_entry<D>(t + 3 * 16 * EB + byte_shl<2 * H + 1, S>(hi), e3);  // bits 12-15
#pragma unroll
    for (int d = 0; d < D; d++) acc[d] = xor3(xor3(acc[d], e0[d], e1[d]), e2[d], e3[d]);
}

template <int W>
__device__ __forceinline__ void mac_chunk_nib(const uint8_t* t, uint4 x, uint32_t (&acc)[8][W / 2])
{
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo = xs[i] & 0x0f0f0f0fu, hi = (xs[i] >> 4) & 0x0f0f0f0fu;
        mac_word_nib<W, 0>(t, lo, hi, acc[2 * i]);
        mac_word_nib<W, 1>(t, lo, hi, acc[2 * i + 1]);
    }
}

template <int W, bool PTRS, bool NT, bool NIB, bool COPY, bool TAIL>
__device__ __forceinline__ void apply_tile(const ApplyArgs& a, const uint8_t* lds, uint32_t s,
                                           int64_t off, int rem)
{
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    const int K = a.ncols;
    uint32_t acc[8][D];
#pragma unroll
    for (int w = 0; w < 8; w++)
#pragma unroll
        for (int d = 0; d < D; d++) acc[w][d] = 0u;

    auto fetch = [&](int j) -> uint4 {
        const uint8_t* p = in_frag<PTRS>(a, s, j) + off;
        if (a.limited) {  // padded objects: bytes past in_len32[j] read as zeros
            const int64_t lim = a.in_len32[j] - off < rem ? a.in_len32[j] - off : rem;
            if (lim >= 16) return stream_load16<NT>(p);
            return lim > 0 ? load_tail(p, static_cast<int>(lim)) : make_uint4(0, 0, 0, 0);
        }
        return TAIL ? load_tail(p, rem) : stream_load16<NT>(p);
    };
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int i = 0; i < 4; i++) cur[i] = (i < K) ? fetch(i) : make_uint4(0, 0, 0, 0);
    for (int j0 = 0; j0 < K; j0 += 4) {
#pragma unroll
        for (int i = 0; i < 4; i++)
            nxt[i] = (j0 + 4 + i < K) ? fetch(j0 + 4 + i) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (j0 + i < K) {
                if constexpr (COPY) {  // copy-through: the input also lands in its own slot
                    if (a.copy_off[j0 + i] >= 0) {  // wave-uniform
                        uint8_t* c = a.copy_base + static_cast<int64_t>(s) * a.copy_stride +
                                     a.copy_off[j0 + i] + off;
                        const int64_t lim = a.limited && a.copy_len32[j0 + i] - off < rem
                                                ? a.copy_len32[j0 + i] - off : rem;
                        if (lim >= 16 && !TAIL)
                            stream_store16<NT>(c, cur[i]);
                        else if (lim > 0)
                            store_tail(c, cur[i], static_cast<int>(lim < 16 ? lim : 16));
                    }
                }
                if constexpr (NIB)
                    mac_chunk_nib<W>(lds + static_cast<size_t>(j0 + i) * 64 * EB, cur[i], acc);
                else
                    mac_chunk<W>(lds + static_cast<size_t>(j0 + i) * 512 * EB, cur[i], acc);
            }
#pragma unroll
        for (int i = 0; i < 4; i++) cur[i] = nxt[i];
    }

#pragma unroll
    for (int r = 0; r < W; r++) {
        if (r >= a.nrows) break;
        uint32_t o[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const uint32_t A = acc[2 * d][r >> 1], B = acc[2 * d + 1][r >> 1];
            o[d] = (r & 1) ? ((A >> 16) | (B & 0xffff0000u)) : ((A & 0xffffu) | (B << 16));
        }
        uint4 v = make_uint4(o[0], o[1], o[2], o[3]);
        uint8_t* q = out_frag<PTRS>(a, s, r) + off;
        // limited outputs (decode straight into objects shorter than k*bs): nothing past out_len32
        const int64_t lim = a.limited && a.out_len32[r] - off < rem ? a.out_len32[r] - off : rem;
        if (lim <= 0) continue;
        if (a.accumulate) {
            uint4 prev = (TAIL || lim < 16) ? load_tail(q, static_cast<int>(lim < 16 ? lim : 16)) : load16(q);
            v.x ^= prev.x;
            v.y ^= prev.y;
            v.z ^= prev.z;
            v.w ^= prev.w;
        }
        if (TAIL || lim < 16)
            store_tail(q, v, static_cast<int>(lim < 16 ? lim : 16));
        else
            stream_store16<NT>(q, v);
    }
}

}  // namespace

}  // namespace ecamd
