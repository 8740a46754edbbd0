// ecamd_kernels.hip -- gfx950 (MI355X / CDNA4) kernels for the erasure-code hot path.
//
// gf16_apply_kernel: out[r] = sum_j A[r][j] * in[j] over GF(2^16) on little-endian 16-bit words,
// for many independent stripes in one launch.  This is the GPU form of the reference's
// region_dot_product / region_multiply / region_xor (src/builtin/rs_vand/liberasurecode_rs_vand.c:
// 336-397), which encode, decode and reconstruct all reduce to (:399-558).
//
//   * HBM: every lane moves 16 B per fragment per tile (global_load_dwordx4), a wave covers a
//     contiguous 1 KiB of each fragment; inputs are read once and all outputs written once per
//     tile, so algorithmic traffic = (K + R) * blocksize per stripe.
//   * LDS: multiply-by-constant is GF(2)-linear, so c*x = T_lo[x & 0xff] ^ T_hi[x >> 8].  The
//     tables of one input pack all W outputs of the row group into one W*2-byte entry, so one
//     16-bit input word costs two ds_read_b{32,64,128} for every output at once (W = 2, 4, 8).
//     The whole image (K * 512 * 2W bytes) is staged into LDS once per workgroup; workgroups are
//     persistent and grid-stride over tiles, so the staging cost is amortised.
//   * Inputs are fetched one group of 4 fragments ahead of the lookups (software pipeline) so
//     each wave keeps >= 4 KiB of loads in flight while its LDS lookups run.
//
// xor_apply_kernel: out[r] = XOR of the inputs selected by mask[r] (flat-XOR HD codes,
// src/builtin/xor_codes/xor_code.c:141-207); pure streaming.
//
// splitmix_fill_kernel: synthetic fragment bytes (bench / tests), same stream as tests/ecdata.py.
//
// The device helpers live in ecamd_apply.hpp; gf16_stream_kernel -- the form every strided launch
// that fits it takes (buffer loads, unrolled inputs) -- in ecamd_stream.hpp, instantiated per
// output width in ecamd_stream_w{2,4,8}.hip.  gf16_apply_kernel below remains for pointer-table
// launches, more than 20 inputs per pass, offsets beyond 2 GiB and the nibble / ablation sweeps.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ecamd_crc_dev.hpp"
#include "ecamd_isa.hpp"
#include "ecamd_kernels.hpp"

#include "ecamd_apply.hpp"

namespace ecamd {


template <int W, bool PTRS, bool NT, bool NIB, bool COPY>
__device__ __forceinline__ void gf16_apply_body(const ApplyArgs& a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int EB = 2 * W;
    const int tbytes = a.ncols * (NIB ? 64 : 512) * EB;
    for (int o = threadIdx.x * 16; o < tbytes; o += blockDim.x * 16)
        *reinterpret_cast<uint4*>(lds + o) = *reinterpret_cast<const uint4*>(a.tables + o);
    __syncthreads();

    const int64_t span = static_cast<int64_t>(blockDim.x) * 16;
    for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const uint32_t s = t / a.tiles_per_stripe;
        const int64_t off = static_cast<int64_t>(t - s * a.tiles_per_stripe) * span +
                            static_cast<int64_t>(threadIdx.x) * 16;
        const int64_t rem = a.bs - off;
        if (rem <= 0) continue;
        if (rem >= 16)
            apply_tile<W, PTRS, NT, NIB, COPY, false>(a, lds, s, off, 16);
        else
            apply_tile<W, PTRS, NT, NIB, COPY, true>(a, lds, s, off, static_cast<int>(rem));
    }
}

template <int W, bool PTRS, bool NT, bool NIB>
__global__ void __launch_bounds__(NIB ? 512 : 1024) gf16_apply_kernel(const ApplyArgs a)
{
    gf16_apply_body<W, PTRS, NT, NIB, false>(a);
}

// Framed encode (hip/ecamd_frame_api.hip): the k data inputs are read straight from the object
// and copied into their fragment payloads by the same launch that computes the parity.
template <int W>
__global__ void __launch_bounds__(1024) gf16_copy_apply_kernel(const ApplyArgs a)
{
    gf16_apply_body<W, false, true, false, true>(a);
}
template __global__ void gf16_copy_apply_kernel<2>(const ApplyArgs);
template __global__ void gf16_copy_apply_kernel<4>(const ApplyArgs);
template __global__ void gf16_copy_apply_kernel<8>(const ApplyArgs);


// Staged inputs of a small launch (one stripe): the K fragments' bytes [c0 * G, c0 * G + region) into
// stg + j * region as 16-byte pieces, up to 8 loads per thread in flight before the first LDS store (from
// pinned host memory each load is a PCIe round trip).  The range ends at the last input's last 16-byte
// granule (the buffer unit checks whole dwords; a granule never crosses a page).  ZERO: the whole region,
// zeros past bs (a checksum's zero extension); else only up to bs (bytes past bs staged, never read).
template <bool ZERO>
__device__ __forceinline__ void small_stage_inputs(uint8_t* stg, const SmallArgs& a, int K, int64_t base, int region)
{
    const int64_t left = a.bs - base;
    const int nseg = static_cast<int>(((left < region ? left : region) + 15) / 16);
    // (uniform by construction; readfirstlane says so to the compiler when the argument block is in LDS --
    // the resident server -- so the loads below need no per-lane resource loop)
    const uint64_t ip = reinterpret_cast<uint64_t>(a.in);
    const uint64_t ipu = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(ip))) |
                         (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(ip >> 32)))) << 32);
    const auto rin = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(ipu), 0,
        __builtin_amdgcn_readfirstlane(static_cast<int>((K - 1) * a.in_pitch + ((a.bs + 15) & ~int64_t(15)))),
        0x00020000);
    const int nq = ZERO ? region / 16 : nseg;
    const int total = K * nq;
    for (int i0 = static_cast<int>(threadIdx.x); i0 < total; i0 += 8 * static_cast<int>(blockDim.x)) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int idx = i0 + u * static_cast<int>(blockDim.x);
            const int j = idx / nq, q = idx - j * nq;
            v[u] = u32x4{0u, 0u, 0u, 0u};
            if (idx < total && q < nseg)
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, static_cast<int>(j * a.in_pitch + base + q * 16), 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int idx = i0 + u * static_cast<int>(blockDim.x);
            if (idx >= total) break;
            const int j = idx / nq, q = idx - j * nq;
            if constexpr (ZERO) {
                const int64_t keep = left - q * 16;  // bytes of this piece inside the fragment
                if (keep < 16) {
#pragma unroll
                    for (int d = 0; d < 4; d++) {
                        const int64_t kd = keep - 4 * d;
                        const uint32_t m = kd >= 4 ? 0xffffffffu : kd <= 0 ? 0u : (1u << (8 * kd)) - 1u;
                        v[u][d] &= m;
                    }
                }
            }
            *reinterpret_cast<u32x4*>(stg + j * region + q * 16) = v[u];
        }
    }
}

// The completion flag of a small launch (SmallArgs::done), after every output store of every workgroup
// is visible system-wide: one workgroup stores it, several count first (done_ctr, self-resetting).
// (bid / nblk: this workgroup's index and the launch's workgroups -- blockIdx / gridDim, or a request of
// the resident small server, small_server_kernel)
__device__ __forceinline__ void small_done(const SmallArgs& a, int bid, int nblk)
{
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned n = static_cast<unsigned>(nblk);
        const bool last = n == 1 || atomicInc(reinterpret_cast<unsigned*>(a.done_ctr), n - 1) == n - 1;
        if (last) {
            __threadfence_system();
            __hip_atomic_store(a.done, a.done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The fused checksum epilogue of a small launch (gf16_small_kernel / xor_small_kernel CRC): the K inputs
// and nrows outputs of this workgroup's region are in LDS at stg + f * REGION (zeros past bs), the image
// of build_small_crc_image at cimg.  r0(X||Y) = A^|Y| r0(X) ^ r0(Y), so r0 of a region is the XOR over
// its 16-byte pieces l of A^(16 (NP - 1 - l)) r0(piece l): lane l looks up r0 of its piece and its
// position map (two rounds of independent LDS lookups), the wave XOR-reduces, and each wave works on up
// to 4 fragments at once.  A workgroup's region r0 goes past the regions after it with the binary maps
// A^(REGION 2^i); the last workgroup to finish (a self-resetting counter) XORs them: S = r0 of the fragment
// zero-extended to gridDim * REGION bytes, then r0 = A^-zext S and crc = ~(A^len ~0 ^ r0) with host
// constants (crc_minv, crc_c).  With several workgroups it also stores the completion flag and returns
// true (the caller stores it otherwise).
// SRV: the resident server's form (small_server_kernel: the argument block in LDS, not in kernel arguments)
// -- the final maps' 32 words are read in a rolled loop, which keeps the compiler from holding them (and
// the rest of the block) in registers across the epilogue.
template <int REGION, bool SRV = false>
__device__ __forceinline__ bool small_crc_epilogue(const SmallArgs& a, const uint8_t* stg, const uint32_t* cimg, int K, int bid,
                                   int nblk)
{
    using namespace crcdev;
    constexpr int NP = REGION / 16;  // 16-byte pieces of a region: 32 or 64
    const uint32_t* const pos = cimg + kSmallCrcPieceWords;  // A^(16 (NP - 1 - l)), l < NP
    const uint32_t* const wgs = pos + NP * 128;             // A^(REGION 2^i), i < 6
    const int lane = static_cast<int>(threadIdx.x) & 63, wave = static_cast<int>(threadIdx.x) >> 6;
    const int nw = static_cast<int>(blockDim.x) >> 6;
    const int nfr = K + a.nrows;
    const int nwg = nblk;
    const int after = nwg - 1 - bid;  // regions after this workgroup's
    __syncthreads();  // every lane's outputs are in LDS
    auto finish = [&](int f, uint32_t S) {  // S = r0 of fragment f zero-extended: the CRC
        uint32_t r0 = 0;
        if constexpr (SRV) {
#pragma unroll 1
            for (int b = 0; b < 32; b++)
                if ((S >> b) & 1u) r0 ^= a.crc_minv[b];
        } else {
#pragma unroll
            for (int b = 0; b < 32; b++)
                if ((S >> b) & 1u) r0 ^= a.crc_minv[b];
        }
        a.crc_out[f] = ~(a.crc_c ^ r0);
    };
    for (int f0 = wave; f0 < nfr; f0 += 4 * nw) {
        uint32_t s[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {  // up to 4 fragments per wave at once: independent lookups
            const int f = f0 + i * nw;
            s[i] = 0;
            if (f < nfr && lane < NP && !(a.crc_dbg & 1)) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(stg + f * REGION + lane * 16);
                s[i] = lmap<4>(pos + lane * 128, piece_r0<1>(cimg, v));
            }
        }
#pragma unroll
        for (int t = 0; t < 6; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) s[i] ^= __shfl_xor(s[i], 1 << t);
        // every lane now holds the 4 totals: lane i finishes fragment f0 + i * nw, in parallel
        if (lane < 4) {
            const int f = f0 + lane * nw;
            uint32_t x = lane == 0 ? s[0] : lane == 1 ? s[1] : lane == 2 ? s[2] : s[3];
            if (f < nfr) {
                if (nwg == 1) {
                    finish(f, x);
                } else {
#pragma unroll
                    for (int b = 0; b < 6; b++)
                        if ((after >> b) & 1) x = lmap<4>(wgs + 128 * b, x);
                    __hip_atomic_store(a.crc_part + 16 + f * nwg + bid, x, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    if (nwg > 1) {
        __shared__ int last;
        // this workgroup's partials (and, with a completion flag, its output stores, system-wide)
        // before its count
        if (a.done)
            __threadfence_system();
        else
            __threadfence();
        __syncthreads();
        if (threadIdx.x == 0)
            last = atomicInc(reinterpret_cast<unsigned*>(a.crc_part), static_cast<unsigned>(nwg - 1)) ==
                   static_cast<unsigned>(nwg - 1);  // wraps to 0: ready for the next launch
        __syncthreads();
        if (last) {
            __threadfence();
            for (int f = static_cast<int>(threadIdx.x); f < nfr; f += static_cast<int>(blockDim.x)) {
                uint32_t S = 0;
                for (int w = 0; w < nwg; w++)
                    S ^= __hip_atomic_load(a.crc_part + 16 + f * nwg + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                finish(f, S);
            }
            if (a.done) {  // every workgroup's stores are visible: the checksums, then the flag
                __threadfence_system();
                __syncthreads();
                if (threadIdx.x == 0)
                    __hip_atomic_store(a.done, a.done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        return true;
    }
    return false;
}

// gf16_small_kernel<W>: launches of a few thousand 16-byte chunks (per-call objects of a few KiB:
// one stripe, fragments at a uniform pitch).  Same split tables and chunk arithmetic as
// apply_tile; what differs is the argument block.  ApplyArgs carries ~1.7 KB of per-fragment
// arrays, read inside apply_tile's rolled loops with a scalar-load round trip each -- at one tile
// those dependent kernel-argument fetches are most of the launch (kernel arguments in host memory,
// HIP_FORCE_DEV_KERNARG=0: 9.7 -> 19.3 us; tools/small_kernel_probe.py).  SmallArgs is ~100 bytes
// fetched up front, and every fragment address is base + j * pitch in registers.
//
// ST (staged inputs): the workgroup first copies its share of every input -- 256 * G bytes of each
// fragment, one stripe -- into LDS with 16-byte buffer loads, all issued before one wait, and the lanes
// read their G bytes from there.  Meant for inputs in pinned HOST memory (the per-call path with no H2D
// DMA, ECAMD_PERCALL_ZEROCOPY_MODE bit 0): there each load instruction is a PCIe round trip, and
// K dependent 2-4-byte loads per lane cost far more than one burst of wide ones.
//
// CRC (with ST, G = 2 or 4, one pass, one stripe): the payload CRC32 of every input and output fragment
// in the same launch -- the per-call CHKSUM_CRC32 encode's checksums without the two launches of
// ecamd_crc32.  The outputs join the staged inputs in LDS.  r0(X||Y) = A^|Y| r0(X) ^
// r0(Y), so r0 of a region is the XOR over its 16-byte pieces l of A^(16 (NP - 1 - l)) r0(piece l):
// lane l looks up r0 of its piece and its position map (two rounds of independent LDS lookups), the
// wave XOR-reduces, and each wave works on up to 4 fragments at once.  A workgroup's region r0 goes
// past the regions after it with the binary maps A^(REGION 2^i); the last workgroup to finish (a
// self-resetting counter) XORs them: S = r0 of the fragment zero-extended to gridDim * REGION bytes,
// then r0 = A^-zext S and crc = ~(A^len ~0 ^ r0) with host constants (crc_minv, crc_c).  Bytes past
// bs are zero in LDS.
// resident (the server, a request with the previous one's arguments): the tables and checksum image this
// workgroup staged for it are still in LDS
template <int W, int G, bool ST, bool CRC, bool SRV = false>
__device__ __forceinline__ void gf16_small_body(const SmallArgs& a, uint8_t* lds, int bid, int nblk,
                                                bool resident = false)
{
    static_assert(!CRC || (ST && (G == 2 || G == 4)), "fused CRC: staged inputs, 2- or 4-byte lanes");
    constexpr int D = W / 2;
    constexpr int EB = 2 * W;
    constexpr int TB = 512 * EB;  // table bytes per input
    constexpr int NW = G / 2;                // 16-bit words per lane
    constexpr int ND = G >= 4 ? G / 4 : 1;  // dwords per lane (G = 2: the low half of one)
    const int K = a.ncols;
    const int64_t step = static_cast<int64_t>(nblk) * blockDim.x;
    int64_t c = static_cast<int64_t>(bid) * blockDim.x + threadIdx.x;
    auto load = [](const uint8_t* p, int rem, uint32_t (&x)[ND]) {
        if constexpr (G == 16) {
            const uint4 v = load_tail(p, rem);
            x[0] = v.x;
            x[1] = v.y;
            x[2] = v.z;
            x[3] = v.w;
        } else if (rem >= G) {
            x[0] = G == 4 ? *reinterpret_cast<const uint32_t*>(p) : *reinterpret_cast<const uint16_t*>(p);
        } else {
            x[0] = 0u;
            for (int i = 0; i < rem; i++) x[0] |= static_cast<uint32_t>(p[i]) << (8 * i);
        }
    };
    // the first lane-group's first four inputs are in flight while the tables stage
    uint32_t cur[4][ND], nxt[4][ND];
    constexpr int REGION = 256 * G;  // ST: bytes of each input this workgroup stages
    uint8_t* const stg = lds + K * TB;
    const int64_t c0 = static_cast<int64_t>(bid) * blockDim.x;
    auto fetch4 = [&](int64_t cc, int j0, uint32_t (&x)[4][ND]) {
        const int64_t s = cc / a.cpf;
        const int64_t off = (cc - s * a.cpf) * G;
        const int rem = a.bs - off < G ? static_cast<int>(a.bs - off) : G;
        if constexpr (ST) {  // one stripe, one chunk per lane: this lane's bytes of the staged region
            const uint8_t* in = stg + (cc - c0) * G;
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (j0 + i < K) load(in + (j0 + i) * REGION, rem, x[i]);
        } else {
            const uint8_t* in = a.in + s * a.in_stride + off;
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (j0 + i < K) load(in + (j0 + i) * a.in_pitch, rem, x[i]);
        }
    };
    if constexpr (ST) {
        small_stage_inputs<CRC>(stg, a, K, c0 * G, REGION);
    } else if (c < a.nchunks) {
        fetch4(c, 0, cur);
    }
    // tables (and the CRC image) into LDS, 8 loads per thread in flight
    auto stage = [&](uint8_t* dst, const uint8_t* src, int bytes) {
        const int step = static_cast<int>(blockDim.x) * 16;
        for (int o0 = static_cast<int>(threadIdx.x) * 16; o0 < bytes; o0 += 8 * step) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (o0 + u * step < bytes) v[u] = load16(src + o0 + u * step);
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (o0 + u * step < bytes) *reinterpret_cast<uint4*>(dst + o0 + u * step) = v[u];
        }
    };
    if (!resident) stage(lds, a.tables, K * TB);
    // CRC: the checksum image after the staged inputs and outputs
    uint32_t* const cimg = reinterpret_cast<uint32_t*>(stg + (K + a.nrows) * REGION);
    if constexpr (CRC)
        if (!(a.crc_dbg & 2) && !resident)
            stage(reinterpret_cast<uint8_t*>(cimg), reinterpret_cast<const uint8_t*>(a.crc_img), small_crc_words(G) * 4);
    __syncthreads();
    if constexpr (ST)
        if (c < a.nchunks) fetch4(c, 0, cur);
    if constexpr (CRC)  // a lane past the last chunk: its slot of every output region holds zeros
        if (c >= a.nchunks)
            for (int r = 0; r < a.nrows; r++) {
                uint8_t* q = stg + (K + r) * REGION + (c - c0) * G;
                if constexpr (G == 4)
                    *reinterpret_cast<uint32_t*>(q) = 0u;
                else
                    *reinterpret_cast<uint16_t*>(q) = 0;
            }

    for (; c < a.nchunks; c += step) {
        uint32_t acc[NW][D];
#pragma unroll
        for (int w = 0; w < NW; w++)
#pragma unroll
            for (int d = 0; d < D; d++) acc[w][d] = 0u;
        for (int j0 = 0; j0 < K; j0 += 4) {
            if (j0 + 4 < K) fetch4(c, j0 + 4, nxt);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (j0 + i >= K) break;
                const uint8_t* tl = lds + static_cast<size_t>(j0 + i) * TB;
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    const uint32_t v = cur[i][w >> 1] >> ((w & 1) * 16);
                    uint32_t e0[D], e1[D];
                    lds_entry<D>(tl + (v & 0xffu) * EB, e0);
                    lds_entry<D>(tl + 256 * EB + ((v >> 8) & 0xffu) * EB, e1);
#pragma unroll
                    for (int d = 0; d < D; d++) acc[w][d] = xor3(acc[w][d], e0[d], e1[d]);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int d = 0; d < ND; d++) cur[i][d] = nxt[i][d];
        }
        const int64_t s = c / a.cpf;
        const int64_t off = (c - s * a.cpf) * G;
        const int rem = a.bs - off < G ? static_cast<int>(a.bs - off) : G;
        uint8_t* out = a.out + s * a.out_stride + off;
#pragma unroll
        for (int r = 0; r < W; r++) {
            if (r >= a.nrows) break;
            uint32_t o[ND];
            if constexpr (G == 2) {
                o[0] = (r & 1) ? (acc[0][r >> 1] >> 16) : (acc[0][r >> 1] & 0xffffu);
            } else {
#pragma unroll
                for (int d = 0; d < ND; d++) {
                    const uint32_t A = acc[2 * d][r >> 1], B = acc[2 * d + 1][r >> 1];
                    o[d] = (r & 1) ? ((A >> 16) | (B & 0xffff0000u)) : ((A & 0xffffu) | (B << 16));
                }
            }
            if constexpr (CRC) {  // the output's bytes (zeros past bs) beside the staged inputs
                const uint32_t m = rem >= G ? (G == 4 ? 0xffffffffu : 0xffffu) : (1u << (8 * rem)) - 1u;
                uint8_t* l = stg + (K + r) * REGION + (c - c0) * G;
                if constexpr (G == 4)
                    *reinterpret_cast<uint32_t*>(l) = o[0] & m;
                else
                    *reinterpret_cast<uint16_t*>(l) = static_cast<uint16_t>(o[0] & m);
            }
            uint8_t* q = out + r * a.out_pitch;
            if (a.accumulate) {
                uint32_t prev[ND];
                load(q, rem, prev);
#pragma unroll
                for (int d = 0; d < ND; d++) o[d] ^= prev[d];
            }
            if constexpr (G == 16) {
                store_tail(q, make_uint4(o[0], o[1], o[2], o[3]), rem);
            } else if (rem >= G) {
                if constexpr (G == 4)
                    *reinterpret_cast<uint32_t*>(q) = o[0];
                else
                    *reinterpret_cast<uint16_t*>(q) = static_cast<uint16_t>(o[0]);
            } else {
                for (int i = 0; i < rem; i++) q[i] = static_cast<uint8_t>(o[0] >> (8 * i));
            }
        }
        if (c + step < a.nchunks) fetch4(c + step, 0, cur);
    }
    if constexpr (CRC)
        if (small_crc_epilogue<REGION, SRV>(a, stg, cimg, K, bid, nblk)) return;
    if (a.done) small_done(a, bid, nblk);  // one workgroup, or no checksum: the flag after every output store
}
template <int W, int G, bool ST, bool CRC>
__global__ void __launch_bounds__(256) gf16_small_kernel(const SmallArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    gf16_small_body<W, G, ST, CRC>(a, lds, static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x));
}
#define ECAMD_SMALL(G, ST)                                                 \
    template __global__ void gf16_small_kernel<2, G, ST>(const SmallArgs); \
    template __global__ void gf16_small_kernel<4, G, ST>(const SmallArgs); \
    template __global__ void gf16_small_kernel<8, G, ST>(const SmallArgs);
ECAMD_SMALL(16, false) ECAMD_SMALL(4, false) ECAMD_SMALL(2, false)
ECAMD_SMALL(16, true) ECAMD_SMALL(4, true) ECAMD_SMALL(2, true)
#undef ECAMD_SMALL
#define ECAMD_SMALL_CRC(G)                                                       \
    template __global__ void gf16_small_kernel<2, G, true, true>(const SmallArgs); \
    template __global__ void gf16_small_kernel<4, G, true, true>(const SmallArgs); \
    template __global__ void gf16_small_kernel<8, G, true, true>(const SmallArgs);
ECAMD_SMALL_CRC(4) ECAMD_SMALL_CRC(2)
#undef ECAMD_SMALL_CRC

#define ECAMD_INST(W, P, N, B) \
    template __global__ void gf16_apply_kernel<W, P, N, B>(const ApplyArgs);
#define ECAMD_INST2(P, N, B) ECAMD_INST(2, P, N, B) ECAMD_INST(4, P, N, B) ECAMD_INST(8, P, N, B)
ECAMD_INST2(false, false, false) ECAMD_INST2(true, false, false)
ECAMD_INST2(false, true, false) ECAMD_INST2(true, true, false)
ECAMD_INST2(false, true, true) ECAMD_INST2(true, true, true)
#undef ECAMD_INST2
#undef ECAMD_INST

// ---------------------------------------------------------------- flat XOR ----

template <int W, bool PTRS, bool TAIL>
__device__ __forceinline__ void xor_tile(const ApplyArgs& a, uint32_t s, int64_t off, int rem)
{
    const int K = a.ncols;
    uint4 acc[W];
#pragma unroll
    for (int r = 0; r < W; r++) acc[r] = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < K; j++) {
        const uint8_t* p = in_frag<PTRS>(a, s, j) + off;
        const uint4 x = TAIL ? load_tail(p, rem) : load16(p);
#pragma unroll
        for (int r = 0; r < W; r++) {
            const uint32_t m = 0u - ((a.masks[r] >> j) & 1u);  // wave-uniform select
            acc[r].x ^= x.x & m;
            acc[r].y ^= x.y & m;
            acc[r].z ^= x.z & m;
            acc[r].w ^= x.w & m;
        }
    }
#pragma unroll
    for (int r = 0; r < W; r++) {
        if (r >= a.nrows) break;
        uint8_t* q = out_frag<PTRS>(a, s, r) + off;
        uint4 v = acc[r];
        if (a.accumulate) {
            uint4 prev = TAIL ? load_tail(q, rem) : load16(q);
            v.x ^= prev.x;
            v.y ^= prev.y;
            v.z ^= prev.z;
            v.w ^= prev.w;
        }
        if (TAIL)
            store_tail(q, v, rem);
        else
            *reinterpret_cast<uint4*>(q) = v;
    }
}

// xor_small_kernel: flat XOR launches of a few chunks (per-call objects), 4-byte lanes, on the
// compact SmallArgs (see gf16_small_kernel); the masks are scalars read once.  ST: the workgroup's 1 KiB of
// every input staged into LDS first (small_stage_inputs; one stripe, one chunk per lane), as the RS kernel
// does for inputs in pinned host memory; the completion flag (SmallArgs::done) after the outputs.
// CRC (with ST): the fused checksums of every input and output (small_crc_epilogue), as gf16_small_kernel.
template <bool ST, bool CRC, bool SRV = false>
__device__ __forceinline__ void xor_small_body(const SmallArgs& a, uint8_t* lds, int bid, int nblk,
                                               bool resident = false)
{
    static_assert(!CRC || ST, "fused CRC: staged inputs");
    constexpr int REGION = 256 * 4;
    const int K = a.ncols;
    const int64_t step = static_cast<int64_t>(nblk) * blockDim.x;
    const int64_t c0 = static_cast<int64_t>(bid) * blockDim.x;
    uint32_t* const cimg = reinterpret_cast<uint32_t*>(lds + (K + a.nrows) * REGION);
    if constexpr (ST) {
        small_stage_inputs<CRC>(lds, a, K, c0 * 4, REGION);
        if constexpr (CRC) {
            const int bytes = resident ? 0 : small_crc_words(4) * 4, stp = static_cast<int>(blockDim.x) * 16;
            for (int o = static_cast<int>(threadIdx.x) * 16; o < bytes; o += stp)
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(cimg) + o) =
                    load16(reinterpret_cast<const uint8_t*>(a.crc_img) + o);
            const int64_t c = c0 + threadIdx.x;  // a lane past the last chunk: zeros in its output slots
            if (c >= a.nchunks)
                for (int r = 0; r < a.nrows; r++)
                    *reinterpret_cast<uint32_t*>(lds + (K + r) * REGION + threadIdx.x * 4) = 0u;
        }
        __syncthreads();
    }
    for (int64_t c = c0 + threadIdx.x; c < a.nchunks; c += step) {
        const int64_t s = c / a.cpf;
        const int64_t off = (c - s * a.cpf) * 4;
        const int rem = a.bs - off < 4 ? static_cast<int>(a.bs - off) : 4;
        auto load = [rem](const uint8_t* p) -> uint32_t {
            if (rem >= 4) return *reinterpret_cast<const uint32_t*>(p);
            uint32_t x = 0u;
            for (int i = 0; i < rem; i++) x |= static_cast<uint32_t>(p[i]) << (8 * i);
            return x;
        };
        const uint8_t* in = ST ? lds + (c - c0) * 4 : a.in + s * a.in_stride + off;
        const int64_t ipitch = ST ? REGION : a.in_pitch;
        uint32_t acc[kMaxRows];
#pragma unroll
        for (int r = 0; r < kMaxRows; r++) acc[r] = 0u;
        uint32_t cur[4], nxt[4];
#pragma unroll
        for (int i = 0; i < 4; i++) cur[i] = i < K ? load(in + i * ipitch) : 0u;
        for (int j0 = 0; j0 < K; j0 += 4) {
#pragma unroll
            for (int i = 0; i < 4; i++) nxt[i] = j0 + 4 + i < K ? load(in + (j0 + 4 + i) * ipitch) : 0u;
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int r = 0; r < kMaxRows; r++)
                    acc[r] ^= cur[i] & (0u - ((a.masks[r] >> ((j0 + i) & 31)) & 1u));
#pragma unroll
            for (int i = 0; i < 4; i++) cur[i] = nxt[i];
        }
        uint8_t* out = a.out + s * a.out_stride + off;
#pragma unroll
        for (int r = 0; r < kMaxRows; r++) {
            if (r >= a.nrows) break;
            uint8_t* q = out + r * a.out_pitch;
            uint32_t v = acc[r];
            if (a.accumulate) v ^= load(q);
            if constexpr (CRC)  // the output's bytes (zeros past bs) beside the staged inputs
                *reinterpret_cast<uint32_t*>(lds + (K + r) * REGION + (c - c0) * 4) =
                    v & (rem >= 4 ? 0xffffffffu : (1u << (8 * rem)) - 1u);
            if (rem >= 4) {
                *reinterpret_cast<uint32_t*>(q) = v;
            } else {
                for (int i = 0; i < rem; i++) q[i] = static_cast<uint8_t>(v >> (8 * i));
            }
        }
    }
    if constexpr (CRC)
        if (small_crc_epilogue<REGION, SRV>(a, lds, cimg, K, bid, nblk)) return;
    if (a.done) small_done(a, bid, nblk);
}
template <bool ST, bool CRC>
__global__ void __launch_bounds__(256) xor_small_kernel(const SmallArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    xor_small_body<ST, CRC>(a, lds, static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x));
}
template __global__ void xor_small_kernel<false, false>(const SmallArgs);
template __global__ void xor_small_kernel<true, false>(const SmallArgs);
template __global__ void xor_small_kernel<true, true>(const SmallArgs);

// small_server_kernel: the resident form of the per-call small launches.  Lane 0 of each
// workgroup polls the mailbox (system-scope acquire loads of the host-written post word, s_sleep between
// them); a new post names its sequence and workgroup count, and workgroups below that count read the
// argument block and variant (one word per lane, into LDS) and run the same body a launch would, with
// (blockIdx, post's count) for (blockIdx, gridDim) -- the completion flag, checksums and counters as in
// a launch.  The others only note the post.  Every workgroup exits on stop, or idle_ticks after its last
// post: the grid always drains on its own.  The host writes a request only after the previous one's
// flag, so no participating workgroup can see its arguments change under it.
template <uint32_t V>
__global__ void __launch_bounds__(256) small_server_kernel(const SmallServerArgs sa)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int kArgWords = static_cast<int>(sizeof(SmallServerSlot) / 4);
    __shared__ __attribute__((aligned(16))) uint32_t argw[2][kArgWords];
    __shared__ uint32_t varw[2];
    __shared__ uint32_t cmd[3];  // post word, go, the request's flag value
    uint32_t last = sa.post0;
    bool check = sa.dup_check != 0;
    int have[2] = {-1, -1};  // the generation of slot i's block argw[i] holds (-1: none)
    // per slot: the generation whose tables (and checksum image) this workgroup's LDS holds where that slot's
    // requests run (-1: none), and whether they run at 0 over more than half the LDS (not kSmallServerHalf)
    int tab[2] = {-1, -1};
    bool whole[2] = {false, false};
    const int bid = static_cast<int>(blockIdx.x);
    for (;;) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint64_t pv = last;
            uint32_t go = 0;
            for (;;) {  // the post word and the flag value in one 8-byte load
                pv = __hip_atomic_load(reinterpret_cast<uint64_t*>(&sa.box->post), __ATOMIC_ACQUIRE,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                if (static_cast<uint32_t>(pv) != last) {
                    go = 1;
                    break;
                }
                if (__hip_atomic_load(&sa.box->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > sa.idle_ticks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            cmd[0] = static_cast<uint32_t>(pv);
            cmd[1] = go;
            cmd[2] = static_cast<uint32_t>(pv >> 32);
        }
        __syncthreads();
        const uint32_t p = cmd[0];
        if (!cmd[1]) return;
        last = p;
        const int nblk = static_cast<int>(p & 0xffu);
        const int sl = (p & kSmallServerSlot) ? 1 : 0;
        const int gen = static_cast<int>((p >> 10) & 0xffu);
        // the host rewrites a slot only with a new generation: a workgroup holding that generation's block
        // reuses its copy (the flag value aside), and its staged tables when they are that block's -- whatever
        // posts it may have missed while it polled
        const bool reuse = have[sl] == gen;
        const bool half = (p & kSmallServerHalf) != 0;
        const bool resident = reuse && tab[sl] == gen;
        uint8_t* const base = half ? lds + sl * kSmallServerLdsHalf : lds;
        if (bid < nblk) {
            if (!reuse) {
                // the argument block in 16-byte pieces, one per lane, system-coherent (sc0 | sc1): one PCIe round trip
                static_assert(offsetof(SmallServerBox, slot) % 16 == 0 && sizeof(SmallServerSlot) % 16 == 0, "box layout");
                const auto rbox = __builtin_amdgcn_make_buffer_rsrc(
                    sa.box, 0, static_cast<int>(sizeof(SmallServerBox)), 0x00020000);
                if (threadIdx.x < sizeof(SmallServerSlot) / 16)
                    *reinterpret_cast<u32x4*>(argw[sl] + 4 * threadIdx.x) = __builtin_amdgcn_raw_buffer_load_b128(
                        rbox, static_cast<int>(offsetof(SmallServerBox, slot) + sl * sizeof(SmallServerSlot) + 16 * threadIdx.x),
                        0, 17);
                if (threadIdx.x == 0)
                    varw[sl] = __hip_atomic_load(&sa.box->variant[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            __syncthreads();
            if (threadIdx.x == 0) argw[sl][offsetof(SmallArgs, done_val) / 4] = cmd[2];
            __syncthreads();
            const SmallArgs& a = *reinterpret_cast<const SmallArgs*>(argw[sl]);
            bool skip = false;
            if (check && a.done)  // a relaunch: the previous server may have finished this request
                skip = __hip_atomic_load(a.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == a.done_val;
            if (!skip) {  // the checksum form or not: this kernel's (W, G) or XOR in either (V: its key)
                constexpr int W = V & 15, G = (V >> 4) & 15;
                const bool crc = (varw[sl] & 256u) != 0;
                if constexpr ((V & kSmallServerXor) != 0) {
                    if (crc)
                        xor_small_body<true, true, true>(a, base, bid, nblk, resident);
                    else
                        xor_small_body<true, false, true>(a, base, bid, nblk, resident);
                } else {
                    if (crc)
                        gf16_small_body<W, G, true, true, true>(a, base, bid, nblk, resident);
                    else
                        gf16_small_body<W, G, true, false, true>(a, base, bid, nblk, resident);
                }
                // a half request overlaps the other slot's tables only when those run at 0 over more than half;
                // a whole one may overlap them wherever they are
                if (!half || whole[sl ^ 1]) tab[sl ^ 1] = -1;
                tab[sl] = gen;
                whole[sl] = !half;
            }
            have[sl] = gen;
        } else if (!reuse) {
            // a rewrite of slot sl this workgroup sits out: its copy is stale from here on (the 8-bit
            // generation would otherwise match again after 256 rewrites it did not take part in)
            have[sl] = -1;
        }
        check = false;
        __syncthreads();  // argw, cmd and the LDS are reused by the next request
    }
}
template __global__ void small_server_kernel<2 | (2 << 4)>(const SmallServerArgs);
template __global__ void small_server_kernel<4 | (2 << 4)>(const SmallServerArgs);
template __global__ void small_server_kernel<8 | (2 << 4)>(const SmallServerArgs);
template __global__ void small_server_kernel<2 | (4 << 4)>(const SmallServerArgs);
template __global__ void small_server_kernel<4 | (4 << 4)>(const SmallServerArgs);
template __global__ void small_server_kernel<8 | (4 << 4)>(const SmallServerArgs);
template __global__ void small_server_kernel<kSmallServerXor>(const SmallServerArgs);

template <int W, bool PTRS>
__global__ void __launch_bounds__(256) xor_apply_kernel(const ApplyArgs a)
{
    const int64_t span = static_cast<int64_t>(blockDim.x) * 16;
    for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const uint32_t s = t / a.tiles_per_stripe;
        const int64_t off = static_cast<int64_t>(t - s * a.tiles_per_stripe) * span +
                            static_cast<int64_t>(threadIdx.x) * 16;
        const int64_t rem = a.bs - off;
        if (rem <= 0) continue;
        if (rem >= 16)
            xor_tile<W, PTRS, false>(a, s, off, 16);
        else
            xor_tile<W, PTRS, true>(a, s, off, static_cast<int>(rem));
    }
}

template __global__ void xor_apply_kernel<8, false>(const ApplyArgs);
template __global__ void xor_apply_kernel<8, true>(const ApplyArgs);

// xor_stream_kernel<KG>: the strided flat-XOR apply for up to 4*KG inputs in the form of
// gf16_stream_kernel (ecamd_stream.hpp): buffer loads on one resource per stripe, the loads of a
// group of 4 inputs unconditional (out-of-range offsets read zeros, no traffic), inputs unrolled.
// Output r accumulates input j under the wave-uniform mask bit j of masks[r]: one v_bitop3 per
// dword (acc ^ (x & m)), no branches.  COPY (framed flat-XOR encode, round 4): every input is also
// stored at copy_base + s*copy_stride + copy_off32[j] as it is loaded (object chunk -> data payload;
// the caller runs whole tiles only).
template <int KG, bool COPY>
__global__ void __launch_bounds__(256) xor_stream_kernel(const ApplyArgs a)
{
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const int cstride = static_cast<int>(blockDim.x) * 16;
    for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const uint32_t sl = t / a.tiles_per_stripe;
        const int64_t toff = static_cast<int64_t>(t - sl * a.tiles_per_stripe) * cstride;
        const uint32_t s = a.stripe_list ? static_cast<uint32_t>(a.stripe_list[sl]) : sl;
        const int64_t o64 = toff + static_cast<int64_t>(threadIdx.x) * 16;
        if (toff + cstride > a.bs) {  // last, partial tile of each fragment
            const int64_t rem = a.bs - o64;
            if (rem >= 16)
                xor_tile<8, false, false>(a, s, o64, 16);
            else if (rem > 0)
                xor_tile<8, false, true>(a, s, o64, static_cast<int>(rem));
            continue;
        }
        const int off = static_cast<int>(o64);
        const auto rin = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.in_base) + static_cast<int64_t>(s) * a.in_stride, 0,
            static_cast<int>(a.in_records), 0x00020000);
        const auto rout = __builtin_amdgcn_make_buffer_rsrc(
            a.out_base + static_cast<int64_t>(s) * a.out_stride, 0, static_cast<int>(a.out_records),
            0x00020000);
        v4 acc[8];
#pragma unroll
        for (int r = 0; r < 8; r++) acc[r] = v4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int g = 0; g < KG; g++) {
            v4 x[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int j = 4 * g + i;
                const int o = (j < a.ncols) ? a.in_off32[j] + off : static_cast<int>(0x80000000u);
                x[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, o, 0, 2);
            }
            if constexpr (COPY) {
                const auto rcopy = __builtin_amdgcn_make_buffer_rsrc(
                    a.copy_base + static_cast<int64_t>(s) * a.copy_stride, 0, static_cast<int>(a.copy_records), 0x00020000);
#pragma unroll
                for (int i = 0; i < 4; i++) {  // skipped inputs: an out-of-range offset, dropped
                    const int j = 4 * g + i;
                    const int o = (j < a.ncols && a.copy_off32[j] >= 0) ? a.copy_off32[j] + off
                                                                         : static_cast<int>(0x80000000u);
                    __builtin_amdgcn_raw_buffer_store_b128(x[i], rcopy, o, 0, 2);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int j = 4 * g + i;
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    if (r >= a.nrows) break;
                    const uint32_t msk = 0u - ((a.masks[r] >> j) & 1u);  // wave-uniform
#pragma unroll
                    for (int d = 0; d < 4; d++) acc[r][d] = xor_and(acc[r][d], x[i][d], msk);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 8; r++) {
            if (r >= a.nrows) break;
            const int o = a.out_off32[r] + off;
            v4 v = acc[r];
            if (a.accumulate) v ^= __builtin_amdgcn_raw_buffer_load_b128(rout, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(v, rout, o, 0, 2);
        }
    }
}

template __global__ void xor_stream_kernel<1, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<2, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<3, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<4, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<8, false>(const ApplyArgs);
template __global__ void xor_stream_kernel<1, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<2, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<3, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<4, true>(const ApplyArgs);
template __global__ void xor_stream_kernel<8, true>(const ApplyArgs);

// ---------------------------------------------------------------- synthetic data ----

__global__ void __launch_bounds__(256) splitmix_fill_kernel(FillArgs f)
{
    const int64_t words = (f.bs + 7) / 8;
    const int64_t total = words * f.nfrags * static_cast<int64_t>(f.nstripes);
    for (int64_t g = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; g < total;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = g % words;
        const int64_t fs = g / words;
        const int frag = static_cast<int>(fs % f.nfrags);
        const int64_t s = fs / f.nfrags;
        const uint64_t seed = f.seed_base ^ (static_cast<uint64_t>(s + f.stripe0) << 8) ^
                              static_cast<uint64_t>(frag);
        uint64_t z = seed + static_cast<uint64_t>(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        uint8_t* p = f.base + s * f.stripe_stride + frag * f.frag_stride + i * 8;
        const int64_t left = f.bs - i * 8;
        if (left >= 8) {
            *reinterpret_cast<uint64_t*>(p) = z;
        } else {
            for (int b = 0; b < left; b++) p[b] = static_cast<uint8_t>(z >> (8 * b));
        }
    }
}

}  // namespace ecamd
