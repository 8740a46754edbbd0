// ecamd_frame_api.hip -- C ABI of the device-resident framed path (include/ecamd.h, "framing"):
// whole liberasurecode_encode / _decode / _reconstruct_fragment equivalents over S stripes whose
// objects and fragments live in HBM, byte-identical to the reference's wire format.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "../host/crc.hpp"
#include "ecamd.h"
#include "ecamd_frame.hpp"
#include "ecamd_host.h"
#include "ecamd_internal.hpp"
#include "ecamd_kernels.hpp"

using namespace ecamd;

namespace {

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return dev_fail(ECAMD_EHIP, "%s: %s", #expr, hipGetErrorString(e_));           \
    } while (0)

constexpr int kBackendXor = 3;   // EC_BACKEND_FLAT_XOR_HD
constexpr int kBackendRs = 6;    // EC_BACKEND_LIBERASURECODE_RS_VAND
constexpr uint32_t kLibecVersion = (1u << 16) | (8u << 8);  // LIBERASURECODE_VERSION 1.8.0
constexpr uint32_t kBackendVersion = 1u << 16;              // ec_backend_version 1.0.0

// LIBERASURECODE_WRITE_LEGACY_CRC, read per call as the reference does
// (src/erasurecode_postprocessing.c:59-60, src/erasurecode_helpers.c:479-480).
bool legacy_crc()
{
    const char* f = std::getenv("LIBERASURECODE_WRITE_LEGACY_CRC");
    return f && !(f[0] == '\0' || (f[0] == '0' && f[1] == '\0'));
}

struct DevImage {
    uint32_t* d = nullptr;
    CrcImage img;
};

std::mutex g_mu;
std::map<std::tuple<int, int, int, int, int, int>, std::unique_ptr<DevImage>> g_images;  // dev, legacy, B, J, G, pos

int image(int dev, bool legacy, int B, int J, int G, bool pos, const DevImage** out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_tuple(dev, legacy ? 1 : 0, B, J, G, pos ? 1 : 0);
    auto it = g_images.find(key);
    if (it == g_images.end()) {
        auto di = std::make_unique<DevImage>();
        di->img = build_crc_image(CrcMachine(legacy), B, J, G, pos);
        const size_t bytes = di->img.words.size() * sizeof(uint32_t);
        HIP_TRY(hipMalloc(&di->d, bytes));
        HIP_TRY(hipMemcpy(di->d, di->img.words.data(), bytes, hipMemcpyHostToDevice));
        it = g_images.emplace(key, std::move(di)).first;
    }
    *out = it->second.get();
    return 0;
}

// Knob frame_copy_per_cu: resident workgroups per CU of the streaming split / join kernels (a dynamic
// LDS share of 160 KiB / N; 0 = none).
size_t copy_lds()
{
    const int n = dev_tune("frame_copy_per_cu");
    return n > 0 ? (size_t(163840) / static_cast<size_t>(n)) & ~size_t(511) : 0;
}

// Per-(device, stream) scratch for span partials (the stream's context, ecamd_internal.hpp).
int scratch(int dev, void* stream, size_t words, uint32_t** out, int slot = 0)
{
    return stream_scratch(dev, stream, slot, words, out);
}

// Knob frame_tail_fork: 2 forks every padded framed encode's tail; 1 (default) only the encodes
// without checksum whose payloads' rest is 1-4 KiB (its codec then one LDS-table launch; the headers
// go to the side stream too): Swift segments RS 1.316 -> 1.225 ms, flat XOR 1.339 -> 1.312, 4 MiB
// objects 1.276 -> 1.260.  A rest that takes a bitsliced tile too (C3 + 10 B: 1.184 -> 1.232) and the
// CRC32 encodes (LDS-bound side work beside an LDS-bound launch) measured slower
// (profiles/r04_tail_fork_ab1.log .. _ab3.log).
bool fork_tail(int64_t rest, bool crc)
{
    const int knob = dev_tune("frame_tail_fork");
    return rest > 0 && (knob == 2 || (knob == 1 && !crc && rest >= 1024 && rest < 4096));
}

struct Code {
    int backend, k, m, hd, w;
};

int check_code(const Code& c)
{
    if (c.backend == kBackendRs) {
        if (c.k < 1 || c.m < 1 || c.k + c.m > 32)
            return dev_fail(ECAMD_EINVAL, "rs_vand: need k >= 1, m >= 1, k + m <= 32");
    } else if (c.backend == kBackendXor) {
        unsigned pb[32], db[32];
        if (c.k < 1 || c.m < 1 || c.k > 32 || c.m > 32 ||
            ecamd_xor_code_tables(c.k, c.m, c.hd, pb, db) != 0)
            return dev_fail(ECAMD_EINVAL, "flat_xor_hd: (k=%d, m=%d, hd=%d) is not a supported code",
                            c.k, c.m, c.hd);
    } else {
        return dev_fail(ECAMD_EINVAL, "backend %d has no device path (3 flat_xor_hd, 6 rs_vand)",
                        c.backend);
    }
    return 0;
}

Code make_code(int backend, int k, int m, int hd)
{
    return Code{backend, k, m, hd, backend == kBackendXor ? 32 : 16};
}

// get_aligned_data_size (src/erasurecode_helpers.c:186-208) / k, in int as the reference.
int64_t blocksize_of(const Code& c, uint64_t size)
{
    const int64_t a = static_cast<int64_t>(c.k) * (c.w / 8);
    const int64_t aligned = ((static_cast<int64_t>(size) + a - 1) / a) * a;
    return aligned / c.k;
}

bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int check_frames(const void* frags, int64_t stripe_stride, int64_t frag_stride, int64_t bs,
                 int nfrag, int nstripes)
{
    if (!frags || nstripes < 0) return dev_fail(ECAMD_EINVAL, "null fragments or nstripes < 0");
    if (!a16(frags) || stripe_stride % 16 || frag_stride % 16)
        return dev_fail(ECAMD_EINVAL, "fragment base and strides must be 16-byte aligned");
    if (frag_stride < kHeaderBytes + ((bs + 15) & ~int64_t(15)))
        return dev_fail(ECAMD_EINVAL, "frag_stride %lld < 80 + blocksize rounded to 16 (%lld)",
                        (long long)frag_stride, (long long)(kHeaderBytes + ((bs + 15) & ~int64_t(15))));
    return 0;
}

// CRC32 of nfrag payloads per stripe (fragment f at base + s*ss + f*fs, payload at +payload_off)
// and, if h.write, the headers.  crc_out may be null.
int run_crc(int dev, bool legacy, bool with_crc, const uint8_t* base, int64_t ss, int64_t fs,
            int64_t payload_off, int nfrag, int64_t len, int nstripes, uint32_t* crc_out,
            const HeaderArgs& h, void* stream)
{
    const int64_t items = static_cast<int64_t>(nfrag) * nstripes;
    if (items == 0) return 0;
    const int B = dev_tune("crc_bits");  // 4 .. 8 (host/crc.cpp build_crc_image)
    const int G = B != 4 ? 8 : (dev_tune("crc_gap_bits") == 4 ? 4 : 8);
    const bool pos = dev_tune("crc_pos") != 0 && G == 8;
    const int64_t body = len & ~int64_t(15);
    const int jmax = dev_tune("crc_span_kib") > 0 ? dev_tune("crc_span_kib") : 16;  // KiB per span
    int J = static_cast<int>(std::min<int64_t>(jmax, std::max<int64_t>(4, ((body / 1024 + 3) / 4) * 4)));
    const DevImage* di = nullptr;
    int rc = image(dev, legacy, B, J, G, pos, &di);
    if (rc) return rc;
    CrcArgs a{};
    a.base = base;
    a.stripe_stride = ss;
    a.frag_stride = fs;
    a.payload_off = payload_off;
    a.len = len;
    a.body = body;
    a.items = items;
    a.nfrag = nfrag;
    a.J = J;
    a.legacy = legacy ? 1 : 0;
    a.span_off = static_cast<uint32_t>(di->img.span_off);
    a.t_off = static_cast<uint32_t>(di->img.t_off);
    a.nspans = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint32_t* partial = nullptr;
    if (with_crc) {
        const int64_t span = static_cast<int64_t>(J) * 1024;
        a.nspans = static_cast<int>(std::max<int64_t>(1, (body + span - 1) / span));
        a.c0 = zero_shift(CrcMachine(legacy), static_cast<uint64_t>(len)).apply(~0u);
        const int64_t waves = items * a.nspans;
        rc = scratch(dev, stream, static_cast<size_t>(waves), &partial);
        if (rc) return rc;
        int wpc = dev_tune("crc_wgs");
        // Measured on MI355X (C3 payloads, 3.5 GiB): B=8 at 2 workgroups/CU 6.35 TB/s, 3: 5.94,
        // 4 (LDS-capped to 3): 5.95; B=4 at 4: 5.36 ("Framing"); the default B=5 with
        // position tables at 8 (twice the resident grid): 0.703 -> 0.724 of 8 TB/s against 4
        // (tools/crc_grid_sweep.py, profiles/r03_crc_grid_sweep.log)
        if (wpc <= 0) wpc = B == 8 ? 2 : 8;
        const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(
                                                      static_cast<int64_t>(dev_cu_count(dev)) * wpc,
                                                      (waves + 7) / 8));
        const dim3 gd(static_cast<unsigned>(grid)), bd(512);
        // template: number of byte-table dwords per piece, gap field bits, position tables
#define ECAMD_CRC_LAUNCH(MB, GG, P) \
    hipLaunchKernelGGL((crc_partial_kernel<MB, GG, P>), gd, bd, 0, st, a, di->d, partial)
        if (pos) {
            switch (B) {
            case 8: ECAMD_CRC_LAUNCH(4, 8, true); break;
            case 7: ECAMD_CRC_LAUNCH(3, 8, true); break;
            case 6: ECAMD_CRC_LAUNCH(2, 8, true); break;
            case 5: ECAMD_CRC_LAUNCH(1, 8, true); break;
            default: ECAMD_CRC_LAUNCH(0, 8, true); break;
            }
        } else {
            switch (B) {
            case 8: ECAMD_CRC_LAUNCH(4, 8, false); break;
            case 7: ECAMD_CRC_LAUNCH(3, 8, false); break;
            case 6: ECAMD_CRC_LAUNCH(2, 8, false); break;
            case 5: ECAMD_CRC_LAUNCH(1, 8, false); break;
            default:
                if (G == 8)
                    ECAMD_CRC_LAUNCH(0, 8, false);
                else
                    ECAMD_CRC_LAUNCH(0, 4, false);
            }
        }
#undef ECAMD_CRC_LAUNCH
        HIP_TRY(hipGetLastError());
    }
    if (with_crc || h.write) {
        hipLaunchKernelGGL(crc_finalize_kernel, dim3(static_cast<unsigned>((items + 127) / 128)),
                           dim3(128), 0, st, a, di->d, partial, crc_out, h);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

HeaderArgs header_args(const Code& c, int checksum, int64_t bs, uint64_t obj_size, int idx0)
{
    HeaderArgs h{};
    h.write = 1;
    h.idx0 = idx0;
    h.size = static_cast<uint32_t>(bs);
    h.backend_meta_size = 0;  // get_backend_metadata_size is 0 for both backends
    h.orig_data_size = obj_size;
    h.backend_version = kBackendVersion;
    h.libec_version = kLibecVersion;
    h.chksum_type = static_cast<uint8_t>(checksum);
    h.backend_id = static_cast<uint8_t>(c.backend);
    return h;
}

int grid_for(int dev, int64_t work)
{
    return static_cast<int>(std::max<int64_t>(
        1, std::min<int64_t>((work + 255) / 256, static_cast<int64_t>(dev_cu_count(dev)) * 16)));
}

// The streaming split / join kernels address a stripe's payloads and an object with 32-bit
// buffer offsets.
bool copy_fits32(int k, int64_t frag_stride, int64_t bs, int64_t obj_size)
{
    const int64_t lim = (int64_t{1} << 31) - 4096;
    return k > 0 && bs > 0 && obj_size < lim && bs + 16 < lim &&
           (k - 1) * frag_stride + kHeaderBytes + bs + 16 < lim && k * bs < lim;
}

// Lanes and chunks per lane of the split / join stream tiles (knobs frame_copy_threads 64 / 128 /
// 256, frame_copy_u 1 / 4).  By default one chunk per lane: one-wave 1 KiB tiles when the payloads
// are 16-byte multiples, 4-wave 4 KiB tiles when they are not (the realigning path).  Systematic
// join, ~2.5 GiB of objects: 1 MiB payloads 0.757 -> 0.830 of 8 TB/s, 4 MiB 0.761 -> 0.825, 16 KiB
// 0.62 -> 0.77 against the round's first 16 KiB tiles; Swift's 1 MiB segments (bs = 104858) 0.648
// -> 0.705 (tools/copy_shape_ab.py, profiles/r03_copy_shape_ab1.log, _ab2.log).
struct CopyShape {
    int threads = 256, u = 1;
};
CopyShape copy_shape(int64_t bs)
{
    CopyShape c;
    c.threads = bs % 16 == 0 ? 64 : 256;
    const int t = dev_tune("frame_copy_threads"), u = dev_tune("frame_copy_u");
    if (t == 64 || t == 128 || t == 256) c.threads = t;
    if (u == 1 || u == 4) c.u = u;
    return c;
}

// Tiles of u x threads chunks per (stripe, data fragment); 8 resident 256-thread workgroups per CU
// (grid-stride), or one workgroup per tile (knob frame_copy_grid).
int copy_grid(int dev, int64_t chunks_per_frag, int k, int nstripes, const CopyShape& cs)
{
    const int64_t per = static_cast<int64_t>(cs.threads) * cs.u;
    const int64_t tiles = (chunks_per_frag + per - 1) / per * k * static_cast<int64_t>(nstripes);
    const int64_t cap = dev_tune("frame_copy_grid") ? (int64_t{1} << 30) : static_cast<int64_t>(dev_cu_count(dev)) * 8;
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(tiles, cap)));
}

// XOR plan of a reference operation applied in place on the payloads of every stripe.
int xor_plan_apply(const Code& c, int op, const int* missing, int arg, uint8_t* payload0,
                   int64_t ss, int64_t fs, int64_t bs, int nstripes, void* stream,
                   const int32_t* d_list = nullptr)
{
    unsigned pb[32], db[32];
    ecamd_xor_code_tables(c.k, c.m, c.hd, pb, db);
    std::vector<int> outs(c.k + c.m);
    std::vector<uint64_t> srcs(c.k + c.m);
    int n = 0;
    const int prc = ecamd_xor_plan(op, c.k, c.m, c.hd, pb, db, missing, arg, outs.data(),
                                   srcs.data(), &n);
    if (prc < 0)
        return dev_fail(ECAMD_EINVAL, "flat_xor_hd: erasure pattern not recoverable (rc %d)", prc);
    if (n == 0) return 0;
    // The frontend hands the codec zero-filled buffers for missing fragments
    // (src/erasurecode_preprocessing.c:141-147, 180-186) and the XOR code accumulates into them,
    // so whatever the missing slots hold here counts as zero.
    uint64_t lost = 0;
    for (int i = 0; missing[i] >= 0; i++) lost |= uint64_t(1) << missing[i];
    uint64_t used = 0;
    for (int i = 0; i < n; i++) {
        srcs[i] &= ~lost;
        used |= srcs[i];
    }
    std::vector<int> col(64, -1);
    std::vector<int64_t> in_off, out_off;
    for (int b = 0; b < c.k + c.m; b++)
        if (used >> b & 1u) {
            col[b] = static_cast<int>(in_off.size());
            in_off.push_back(b * fs);
        }
    if (in_off.empty()) in_off.push_back(0);  // every output is all-zero: one unused input
    std::vector<uint32_t> masks;
    for (int i = 0; i < n; i++) {
        uint32_t mk = 0;
        for (int b = 0; b < c.k + c.m; b++)
            if (srcs[i] >> b & 1u) mk |= 1u << col[b];
        masks.push_back(mk);
        out_off.push_back(outs[i] * fs);
    }
    if (d_list)
        return xor_apply_list(masks.data(), n, static_cast<int>(in_off.size()), payload0, ss, in_off.data(),
                              out_off.data(), bs, nstripes, d_list, stream);
    return ecamd_xor_apply_strided(masks.data(), n, static_cast<int>(in_off.size()), payload0, ss,
                                   in_off.data(), payload0, ss, out_off.data(), bs, nstripes, stream);
}

// Strided flat_xor_hd batches (fragment f of stripe s at base + s*ss + f*fs, bs bytes).
int xor_batch_check(const Code& c, const void* base, int64_t ss, int64_t fs, int64_t bs, int nstripes)
{
    int rc = check_code(c);
    if (rc) return rc;
    if (!base || nstripes < 0 || bs < 0) return dev_fail(ECAMD_EINVAL, "null base or negative sizes");
    if (!a16(base) || ss % 16 || fs % 16) return dev_fail(ECAMD_EINVAL, "fragment addresses must be 16-byte aligned");
    if (fs < bs) return dev_fail(ECAMD_EINVAL, "frag_stride < blocksize");
    return 0;
}

// ---- fused CHKSUM_CRC32 framed encode (hip/ecamd_frame_fused.hip) ----

std::map<std::pair<int, int>, uint32_t*> g_fused_images;  // (dev, legacy + 2 * mb) -> device image

int fused_image(int dev, bool legacy, int mb, const uint32_t** out, int tile = 8192, int npos = 0,
                bool nib = false)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_pair(dev, (legacy ? 1 : 0) + 2 * mb + 16 * npos + 128 * (nib ? 1 : 0) + 256 * tile);
    auto it = g_fused_images.find(key);
    if (it == g_fused_images.end()) {
        // npos > 0: the bitsliced crc variant's image (position sets of byte or nibble tables, step = tile)
        const std::vector<uint32_t> w =
            npos ? build_fused_crc_image_pos(CrcMachine(legacy), static_cast<uint64_t>(tile), npos, nib, mb)
                 : build_fused_crc_image(CrcMachine(legacy), static_cast<uint64_t>(tile), mb);
        uint32_t* d = nullptr;
        HIP_TRY(hipMalloc(&d, w.size() * sizeof(uint32_t)));
        HIP_TRY(hipMemcpy(d, w.data(), w.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        it = g_fused_images.emplace(key, d).first;
    }
    *out = it->second;
    return 0;
}

// The object-filling rs_vand encode with CRC32 checksums as ONE codec launch that also folds the
// payload checksums (q ranges per payload), then crc_finalize_kernel over the ranges and the
// headers.  ECAMD_EINVAL (nothing launched) when the shape does not fit: the caller runs the
// copy-through encode + separate CRC pass instead.
// Ranges per payload for the fused CRC kernels: enough work units (stripes x ranges) to fill the
// chip, each a long sequential run of whole tiles.
// q divides `tiles`: the smallest divisor that gives per_cu units per CU, else one tile per unit (odd
// tile counts -- C3 objects 10 bytes long have 63 whole tiles per payload -- once took q = 1, one
// unit per stripe: 0.51 of 8 TB/s instead of 0.6x).
int fused_ranges(int dev, int64_t tiles, int nstripes, int default_per_cu)
{
    const int64_t per_cu = dev_tune("frame_crc_units") > 0 ? dev_tune("frame_crc_units") : default_per_cu;
    const int64_t want = per_cu * dev_cu_count(dev);
    for (int64_t q = 1; q < tiles; q++)
        if (tiles % q == 0 && static_cast<int64_t>(nstripes) * q >= want) return static_cast<int>(q);
    return static_cast<int>(std::max<int64_t>(1, tiles));
}

// crc_finalize_kernel over the q ranges of every payload of the batch and the 80-byte headers.
// cover < bs: the ranges span the payloads' first `cover` bytes and tail_crc[item] holds the CRC32
// of the rest (bs - cover bytes), folded in after them.
int finalize_ranges(int dev, const Code& c, bool legacy, uint64_t obj_size, uint8_t* frags, int64_t ss,
                    int64_t fs, int64_t bs, int nstripes, const uint32_t* partial, int q, void* stream,
                    int64_t cover = -1, const uint32_t* tail_crc = nullptr)
{
    const int nf = c.k + c.m;
    if (cover < 0) cover = bs;
    const int J = static_cast<int>(cover / q / 1024);  // KiB per range
    const DevImage* di = nullptr;
    int rc = image(dev, legacy, 5, J, 8, false, &di);
    if (rc) return rc;
    CrcArgs a{};
    if (cover < bs) {
        if (!tail_crc) return dev_fail(ECAMD_EINVAL, "finalize: ranges end before the payload, no tail CRC");
        // A^tail as its 32 columns in the kernel arguments (no per-length device table to cache)
        const Mat32 sh = zero_shift(CrcMachine(legacy), static_cast<uint64_t>(bs - cover));
        for (int b = 0; b < 32; b++) a.tail_cols[b] = sh.col[b];
        a.tail_crc = tail_crc;
        a.tail_c0 = sh.apply(~0u);
    }
    a.base = frags;
    a.stripe_stride = ss;
    a.frag_stride = fs;
    a.payload_off = kHeaderBytes;
    a.len = cover;  // (no byte steps: the ranges end exactly at `cover`)
    a.body = cover;
    a.items = static_cast<int64_t>(nstripes) * nf;
    a.nfrag = nf;
    a.nspans = q;
    a.J = J;
    a.legacy = legacy ? 1 : 0;
    a.c0 = zero_shift(CrcMachine(legacy), static_cast<uint64_t>(bs)).apply(~0u);
    a.span_off = static_cast<uint32_t>(di->img.span_off);
    a.t_off = static_cast<uint32_t>(di->img.t_off);
    hipLaunchKernelGGL(crc_finalize_kernel, dim3(static_cast<unsigned>((a.items + 127) / 128)), dim3(128), 0,
                       static_cast<hipStream_t>(stream), a, di->d, partial, nullptr,
                       header_args(c, kChksumCrc32, bs, obj_size, 0));
    HIP_TRY(hipGetLastError());
    return 0;
}

// The crc variant in one-wave 4 KiB tiles (knob frame_crc_wave = its waves per workgroup, 4 by default;
// maps of up to 8 outputs): its per-tile partials go to scratch slot 3, crc_combine_kernel folds them into q
// ranges of g tiles per payload (g the largest divisor of the tile count up to 16) in `partial`, and
// finalize_ranges takes those.  crc_wave_form: the crc_pos flags of the form (0: not this form).
int crc_wave_form(const Code& c, int64_t cover)
{
    int cw = dev_tune("frame_crc_wave");
    if (cw <= 0 || cover <= 0 || cover % 4096) return 0;
    if (c.m > 4) cw = std::min(cw, 8);  // (5-8 outputs: built for 2 waves per SIMD)
    const int nibw = 4 - std::clamp(dev_tune("frame_crc_wave_mb"), 1, 4);  // piece dwords on nibble tables
    return dev_tune("frame_crc_wave_pos") | 8 | 32 | (cw << 6) | (dev_tune("frame_crc_wave_mix") ? 1024 : 0) |
           (nibw << 11) | (nibw == 0 && dev_tune("frame_crc_wave_l1") ? 8192 : 0);
}
int crc_wave_mb(int wf) { return 4 - ((wf >> 11) & 3); }  // byte-table dwords per piece of the form wf
int crc_wave_groups(int64_t tps)
{
    int g = 1;
    for (int d = 2; d <= 16; d++)
        if (tps % d == 0) g = d;
    return g;
}
int crc_wave_combine(int dev, bool legacy, const uint32_t* tiles, int64_t items, int nf, int64_t tps, int g,
                     uint32_t* partial, void* stream)
{
    const DevImage* di = nullptr;
    int rc = image(dev, legacy, 5, 4, 8, false, &di);  // span tables: A^4096
    if (rc) return rc;
    const int64_t n = items * (tps / g);
    hipLaunchKernelGGL(crc_combine_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), tiles, partial, di->d + di->img.span_off, items, nf,
                       static_cast<int>(tps), g);
    HIP_TRY(hipGetLastError());
    return 0;
}

// The same framed encode on the bitsliced kernel's crc variant (no codec tables: the LDS serves
// only the CRC lookups) for maps of up to 4 outputs over whole 16 KiB tiles.  ECAMD_EINVAL when it
// does not apply or its kernel is still compiling (knob bitslice 1): the caller runs the LDS-table
// fused kernel instead.
int encode_crc_bitsliced(int dev, const Code& c, bool legacy, const void* obj, int64_t obj_stride,
                         uint64_t obj_size, uint8_t* frags, int64_t ss, int64_t fs, int64_t bs,
                         int nstripes, void* stream)
{
    if (dev_tune("frame_crc_bs") == 0 || c.m > 8 || nstripes <= 0) return ECAMD_EINVAL;
    if (const int wf = crc_wave_form(c, bs)) {
        const int nf = c.k + c.m;
        const int64_t tps = bs / 4096;
        const int g = crc_wave_groups(tps);
        uint32_t *tiles = nullptr, *partial = nullptr;
        int rc = scratch(dev, stream, static_cast<size_t>(nstripes) * static_cast<size_t>(tps) * nf, &tiles, 3);
        if (rc || (rc = scratch(dev, stream, static_cast<size_t>(nstripes) * nf * static_cast<size_t>(tps / g),
                                &partial)))
            return rc;
        const uint32_t* img = nullptr;
        if ((rc = fused_image(dev, legacy, crc_wave_mb(wf), &img, 1024, wf & 7, false))) return rc;
        if ((rc = rs_encode_copy_crc_bs(c.k, c.m, obj, obj_stride, frags + kHeaderBytes, ss, fs, bs, nstripes, img,
                                        tiles, 0, stream, wf)))
            return rc == ECAMD_EINVAL && dev_tune("frame_crc_wave_strict")
                       ? dev_fail(ECAMD_EHIP, "framed encode: the one-wave crc form declined")
                       : rc;
        if ((rc = crc_wave_combine(dev, legacy, tiles, static_cast<int64_t>(nstripes) * nf, nf, tps, g, partial,
                                   stream)))
            return rc;
        return finalize_ranges(dev, c, legacy, obj_size, frags, ss, fs, bs, nstripes, partial,
                               static_cast<int>(tps / g), stream);
    }
    if (bs % 16384) return ECAMD_EINVAL;
    // one 16 KiB tile per work unit at C3 (64 units per CU, one per workgroup): the dispatcher
    // balances them (32 / 16 per CU measured 3 / 6% slower, profiles/r03_fused_sweep_pos.log);
    // maps of 5-8 outputs fold every tile on its own (one range per tile)
    const int q = c.m > 4 ? static_cast<int>(bs / 16384) : fused_ranges(dev, bs / 16384, nstripes, 64);
    uint32_t* partial = nullptr;
    int rc = scratch(dev, stream, static_cast<size_t>(nstripes) * (c.k + c.m) * q, &partial);
    if (rc) return rc;
    const uint32_t* img = nullptr;
    // maps of 5-8 outputs always fold with the lane-shift tables (bitslice.cpp fold_each)
    const bool lane = c.m > 4 || dev_tune("frame_crc_lane") != 0;
    int npos = dev_tune("frame_crc_pos");
    if (npos <= 0) npos = lane && c.m <= 4 ? 1 : 2;
    const bool nib = dev_tune("frame_crc_bs_nib") > 0;
    if ((rc = fused_image(dev, legacy, 4, &img, 4096, npos, nib))) return rc;
    rc = rs_encode_copy_crc_bs(c.k, c.m, obj, obj_stride, frags + kHeaderBytes, ss, fs, bs, nstripes, img,
                               partial, q, stream, npos | (lane ? 8 : 0) | (nib ? 16 : 0));
    if (rc) return rc;
    return finalize_ranges(dev, c, legacy, obj_size, frags, ss, fs, bs, nstripes, partial, q, stream);
}

// prepare_fragments_for_encode for payload bytes [from, bs) only (from a multiple of 16; 0 = all):
// the streaming split kernel (callers check copy_fits32).
int split_range(int dev, int k, const void* obj, int64_t obj_stride, uint64_t obj_size, uint8_t* frags, int64_t ss,
                int64_t fs, int64_t bs, int nstripes, int64_t from, void* stream)
{
    const int64_t r16 = (bs + 15) & ~int64_t(15);
    SplitArgs sa{static_cast<const uint8_t*>(obj), obj_stride, static_cast<int64_t>(obj_size), frags, ss, fs, bs,
                 k, nstripes, 0, from};
    const CopyShape cs = copy_shape(bs);
    const dim3 grid(copy_grid(dev, (r16 - from) / 16, k, nstripes, cs)), block(cs.threads);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const bool dpp = dev_tune("frame_copy_dpp") != 0;
    if (cs.u == 1)
        hipLaunchKernelGGL((dpp ? frame_split_stream_kernel<1, true> : frame_split_stream_kernel<1, false>), grid, block,
                           copy_lds(), st, sa);
    else
        hipLaunchKernelGGL((dpp ? frame_split_stream_kernel<4, true> : frame_split_stream_kernel<4, false>), grid, block,
                           copy_lds(), st, sa);
    HIP_TRY(hipGetLastError());
    return 0;
}

// The rest [from, bs) of every payload of an RS copy-through encode whose first `from` bytes are
// done (bytes [0, from) of the data payloads written): a streaming split copies the object chunks'
// rest into the data payloads (zero padded past the object's end and through the 16-byte slack),
// then the plain encode runs over the payloads' last n whole 4 KiB tiles [r16 - 4096 n, r16), r16 =
// bs rounded up to 16 -- overlapping [0, from) where it recomputes the same parity bytes -- on the
// bitsliced one-wave kernel the C3 encode uses.  The LDS-table copy-through launch it replaces spent
// most of its time staging 40 KiB of tables per workgroup for ~2.5-6.5 KiB of work per stripe
// (profiles/r04_swift_prof_*: 0.10-0.17 ms of a 1.3-1.5 ms encode).  ECAMD_EINVAL, nothing
// launched, when it does not apply (payloads shorter than the tiles, 32-bit offsets, knob
// frame_tail_bs 0).  Whole 4 KiB tiles every object chunk still holds past `from` (the 16 KiB-tile
// crc variant leaves one on Swift's segments) go first through the copy-through launch of exactly
// that range, so the split and the re-encoded tiles shrink to the last partial tile (knob
// frame_tail_tiles, default on).
int encode_tail(int dev, const Code& c, const void* obj, int64_t obj_stride, uint64_t obj_size, uint8_t* frags,
                int64_t ss, int64_t fs, int64_t bs, int nstripes, int64_t from, void* stream)
{
    constexpr int64_t kTile = 4096;
    if (dev_tune("frame_tail_bs") == 0 || from <= 0 || from % 16 || from >= bs ||
        !copy_fits32(c.k, fs, bs, static_cast<int64_t>(obj_size)) || dev_tune("frame_copy_stream") == 0)
        return ECAMD_EINVAL;
    const int64_t last = static_cast<int64_t>(obj_size) - (c.k - 1) * bs;
    const int64_t c4 = last > 0 ? std::min(bs, last) / kTile * kTile : 0;  // whole 4 KiB tiles of every chunk
    const int64_t r16 = (bs + 15) & ~int64_t(15);
    const int64_t mid = dev_tune("frame_tail_tiles") != 0 && c4 > from && c4 < bs ? c4 : from;
    const int64_t n = (r16 - mid + kTile - 1) / kTile;
    const int64_t t0 = r16 - n * kTile;
    if (t0 < 0) return ECAMD_EINVAL;
    int rc;
    if (mid > from && (rc = rs_encode_copy(c.k, c.m, obj, obj_stride, frags + kHeaderBytes, ss, fs, bs, nstripes,
                                           stream, static_cast<int64_t>(obj_size), from, mid)))
        return rc == ECAMD_EINVAL ? dev_fail(ECAMD_EHIP, "framed encode: tail tiles failed") : rc;
    from = mid;
    rc = split_range(dev, c.k, obj, obj_stride, obj_size, frags, ss, fs, bs, nstripes, from, stream);
    if (rc) return rc;
    rc = ecamd_rs_encode(c.k, c.m, frags + kHeaderBytes + t0, ss, fs, n * kTile, nstripes, stream);
    return rc == ECAMD_EINVAL ? dev_fail(ECAMD_EHIP, "framed encode: tail encode failed") : rc;
}

// Objects that do not fill k payloads of whole 16 KiB tiles (Swift's 1 MiB segments: bs = 104858,
// object chunks at unaligned offsets j*bs, the last one 4 bytes short): the bitsliced crc variant
// over the tiles every payload holds in full ([0, cover), cover = the last chunk's whole tiles),
// then the copy-through codec over [cover, bs) of every payload, the CRC32 of those tails on their
// own (run_crc), and the finalize folding each tail into its payload's ranges:
// r0(X || Y) = A^|Y| r0(X) ^ r0(Y).  ECAMD_EINVAL, nothing launched, when it does not apply or the
// bitsliced kernel is still compiling: the caller runs the copy-through encode + CRC pass.
int encode_crc_cover(int dev, const Code& c, bool legacy, const void* obj, int64_t obj_stride,
                     uint64_t obj_size, uint8_t* frags, int64_t ss, int64_t fs, int64_t bs, int nstripes,
                     void* stream)
{
    const bool xorc = c.backend == kBackendXor;
    if (dev_tune("frame_crc_cover") == 0 || dev_tune("frame_crc_bs") == 0 || dev_tune("frame_crc_fused") == 0 ||
        c.m > 8 || bs % 2 || nstripes <= 0 || (xorc && !copy_fits32(c.k, fs, bs, static_cast<int64_t>(obj_size))))
        return ECAMD_EINVAL;
    const int64_t last = static_cast<int64_t>(obj_size) - (c.k - 1) * bs;  // bytes of the last data chunk
    // the one-wave crc form covers whole 4 KiB tiles, the 16 KiB-tile crc variant whole 16 KiB tiles
    const int wf = last > 0 ? crc_wave_form(c, std::min(bs, last) / 4096 * 4096) : 0;
    const int64_t kTile = wf ? 4096 : 16384;
    const int64_t cover = last > 0 ? std::min(bs, last) / kTile * kTile : 0;
    if (last <= 0 || cover < kTile) return ECAMD_EINVAL;
    const int64_t tail = bs - cover;
    const int nf = c.k + c.m;
    const int64_t tps = cover / kTile;
    const int g = wf ? crc_wave_groups(tps) : 1;
    const int q = wf ? static_cast<int>(tps / g)
                     : c.m > 4 ? static_cast<int>(tps) : fused_ranges(dev, tps, nstripes, 64);
    uint32_t *partial = nullptr, *tail_crc = nullptr, *tiles = nullptr;
    int rc = scratch(dev, stream, static_cast<size_t>(nstripes) * nf * q, &partial, 1);
    if (rc) return rc;
    if (tail && (rc = scratch(dev, stream, static_cast<size_t>(nstripes) * nf, &tail_crc, 2))) return rc;
    if (wf && (rc = scratch(dev, stream, static_cast<size_t>(nstripes) * static_cast<size_t>(tps) * nf, &tiles, 3)))
        return rc;
    const uint32_t* img = nullptr;
    const bool lane = c.m > 4 || dev_tune("frame_crc_lane") != 0;
    int npos = dev_tune("frame_crc_pos");
    if (npos <= 0) npos = lane && c.m <= 4 ? 1 : 2;
    const bool nib = dev_tune("frame_crc_bs_nib") > 0;
    if ((rc = wf ? fused_image(dev, legacy, crc_wave_mb(wf), &img, 1024, wf & 7, false)
                 : fused_image(dev, legacy, 4, &img, 4096, npos, nib)))
        return rc;
    unsigned pb[32], db[32];
    if (xorc) ecamd_xor_code_tables(c.k, c.m, c.hd, pb, db);
    const int pos = wf ? wf : npos | (lane ? 8 : 0) | (nib ? 16 : 0);
    uint32_t* out = wf ? tiles : partial;  // (one-wave form: per-tile partials, combined below)
    auto whole = [&] {  // the whole tiles [0, cover): codec + copy + CRC partials in one launch
        const int r = xorc ? xor_encode_copy_crc_bs(pb, c.k, c.m, obj, obj_stride, frags + kHeaderBytes, ss, fs, bs,
                                                    nstripes, img, out, q, stream, pos, cover)
                           : rs_encode_copy_crc_bs(c.k, c.m, obj, obj_stride, frags + kHeaderBytes, ss, fs, bs, nstripes,
                                                   img, out, q, stream, pos, cover);
        return r == ECAMD_EINVAL && wf && dev_tune("frame_crc_wave_strict")
                   ? dev_fail(ECAMD_EHIP, "framed encode: the one-wave crc form declined")
                   : r;
    };
    // the payloads' rest [cover, bs): codec, then the CRC32 of that range on its own; `exact`: no byte
    // below cover is touched (the side stream runs it beside whole())
    auto rest = [&](void* st, bool exact) {
        int r;
        if (xorc) {  // the data payloads' rest by the split, then the XOR of that range
            r = split_range(dev, c.k, obj, obj_stride, obj_size, frags, ss, fs, bs, nstripes, cover, st);
            if (r == 0) {
                std::vector<int64_t> in_off(c.k), out_off(c.m);
                for (int j = 0; j < c.k; j++) in_off[j] = j * fs;
                for (int o = 0; o < c.m; o++) out_off[o] = (c.k + o) * fs;
                uint8_t* pc = frags + kHeaderBytes + cover;
                r = ecamd_xor_apply_strided(pb, c.m, c.k, pc, ss, in_off.data(), pc, ss, out_off.data(), bs - cover,
                                            nstripes, st);
            }
        } else {
            // encode_tail re-encodes whole 4 KiB tiles reaching below cover from the payloads: only
            // after whole() on the same stream
            r = exact ? ECAMD_EINVAL : encode_tail(dev, c, obj, obj_stride, obj_size, frags, ss, fs, bs, nstripes, cover, st);
            if (r == ECAMD_EINVAL)
                r = rs_encode_copy(c.k, c.m, obj, obj_stride, frags + kHeaderBytes, ss, fs, bs, nstripes, st,
                                   static_cast<int64_t>(obj_size), cover);
        }
        if (r) return r == ECAMD_EINVAL ? dev_fail(ECAMD_EHIP, "framed encode: tail codec failed") : r;
        HeaderArgs none{};
        if ((r = run_crc(dev, legacy, true, frags, ss, fs, kHeaderBytes + cover, nf, tail, nstripes, tail_crc, none,
                         st)))
            return r == ECAMD_EINVAL ? dev_fail(ECAMD_EHIP, "framed encode: tail CRC failed") : r;
        return 0;
    };
    if (fork_tail(tail, true)) {
        void* side = nullptr;
        if ((rc = side_fork(dev, stream, &side))) return rc;
        rc = rest(side, true);
        // whole() may decline (ECAMD_EINVAL: the kernel is still compiling): the caller's fallback then
        // rewrites every payload after the tails (joined first), byte-identically
        if (rc == 0) rc = whole();
        const int rj = side_join(dev, stream);
        if (rc || rj) return rc ? rc : rj;
    } else {
        if ((rc = whole())) return rc;
        // from here on a failure is an error, not a fallback: part of the payloads is written
        if (tail && (rc = rest(stream, false))) return rc;
    }
    if (wf && (rc = crc_wave_combine(dev, legacy, tiles, static_cast<int64_t>(nstripes) * nf, nf, tps, g, partial,
                                     stream)))
        return rc;
    return finalize_ranges(dev, c, legacy, obj_size, frags, ss, fs, bs, nstripes, partial, q, stream, cover,
                           tail_crc);
}

int encode_crc_fused(int dev, const Code& c, bool legacy, const void* obj, int64_t obj_stride,
                     uint64_t obj_size, uint8_t* frags, int64_t ss, int64_t fs, int64_t bs,
                     int nstripes, void* stream)
{
    if (dev_tune("frame_crc_fused") == 0 || bs % 8192 || nstripes <= 0) return ECAMD_EINVAL;
    int rc = encode_crc_bitsliced(dev, c, legacy, obj, obj_stride, obj_size, frags, ss, fs, bs, nstripes, stream);
    if (rc != ECAMD_EINVAL) return rc;
    const int q = fused_ranges(dev, bs / 8192, nstripes, 4);
    const int nf = c.k + c.m;
    uint32_t* partial = nullptr;
    rc = scratch(dev, stream, static_cast<size_t>(nstripes) * nf * q, &partial);
    if (rc) return rc;
    const uint32_t* img = nullptr;
    // all-byte piece tables (16 KiB) measured 4% faster than byte + nibble (MB = 1, 5.5 KiB) in the
    // fused kernel, where the LDS also serves the codec; MB = 1 when the larger image does not fit
    // codec on nibble tables (knob frame_crc_nib): conflict-free lookups and an image 1/8 the size
    const bool nib = dev_tune("frame_crc_nib") != 0;
    int mb = dev_tune("frame_crc_mb") == 1 ? 1 : 4;
    if (mb == 4 && fused_crc_lds(c.k, c.m, 4, nib) > static_cast<size_t>(kLdsBytes)) mb = 1;
    if ((rc = fused_image(dev, legacy, mb, &img))) return rc;
    rc = rs_encode_copy_crc(c.k, c.m, obj, obj_stride, frags + kHeaderBytes, ss, fs, bs, nstripes, img,
                            partial, q, stream, mb, nib);
    if (rc) return rc;
    return finalize_ranges(dev, c, legacy, obj_size, frags, ss, fs, bs, nstripes, partial, q, stream);
}

}  // namespace

extern "C" {

// Build time (no GPU): the CRC32 framed encode's bitsliced kernel for a code, into the library's jit/
// directory (prebuild.py) -- the kernel does not depend on the object size (object chunks at offsets
// that are not multiples of 16 take unaligned loads), so one per code serves whole objects and Swift's
// segments alike.  1 present, 0 not a bitsliced form under the current knobs, < 0 failed.
int ecamd_frame_prebuild(int backend, int k, int m, int hd, const char* arch, const char* dir)
{
    const Code c = make_code(backend, k, m, hd);
    const int rc = check_code(c);
    if (rc) return rc;
    if (!arch || !dir) return dev_fail(ECAMD_EINVAL, "null arch / dir");
    const int wf = crc_wave_form(c, 4096);
    if (!wf || c.m > 8) return 0;
    unsigned pb[32], db[32];
    if (c.backend == kBackendXor) ecamd_xor_code_tables(c.k, c.m, c.hd, pb, db);
    const int r = crc_encode_prebuild(c.k, c.m, c.backend == kBackendXor ? pb : nullptr, wf, arch, dir);
    return r < 0 ? dev_fail(ECAMD_EHIP, "framed CRC32 prebuild failed (%d)", r) : r;
}

int ecamd_frame_geometry(int backend, int k, int m, int hd, uint64_t obj_size, int64_t* blocksize,
                         int64_t* fragment_len)
{
    const Code c = make_code(backend, k, m, hd);
    int rc = check_code(c);
    if (rc) return rc;
    if (obj_size > 0x7fffffffull) return dev_fail(ECAMD_EINVAL, "object larger than INT_MAX");
    const int64_t bs = blocksize_of(c, obj_size);
    if (blocksize) *blocksize = bs;
    if (fragment_len) *fragment_len = kHeaderBytes + bs;
    return 0;
}

int ecamd_frame_encode(int backend, int k, int m, int hd, int checksum, const void* d_obj,
                       int64_t obj_stride, uint64_t obj_size, void* d_frags, int64_t stripe_stride,
                       int64_t frag_stride, int nstripes, void* stream)
{
    int dev = 0;
    int rc = dev_ensure(&dev);
    if (rc) return rc;
    const StreamUse use(dev, stream);  // its stream context outlives this call
    const Code c = make_code(backend, k, m, hd);
    if ((rc = check_code(c))) return rc;
    if (obj_size > 0x7fffffffull) return dev_fail(ECAMD_EINVAL, "object larger than INT_MAX");
    const int64_t bs = blocksize_of(c, obj_size);
    if ((rc = check_frames(d_frags, stripe_stride, frag_stride, bs, k + m, nstripes))) return rc;
    if (nstripes == 0) return 0;
    if (!d_obj && obj_size) return dev_fail(ECAMD_EINVAL, "null object buffer");
    auto* frags = static_cast<uint8_t*>(d_frags);
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint8_t* p0 = frags + kHeaderBytes;
    const bool aligned = a16(d_obj) && obj_stride % 16 == 0 && bs % 16 == 0;
    if (backend == kBackendRs && aligned && static_cast<int64_t>(obj_size) == k * bs &&
        dev_tune("frame_unfused") == 0) {
        // The object fills the k payloads exactly (no padding): one launch reads it, copies the
        // data into the payloads and writes the parity (10 MiB read + 14 MiB written per C3
        // stripe instead of a separate split pass) -- with CRC32 checksums, the same launch also
        // folds the payload checksums (no re-read of the 14 MiB).
        if (checksum == kChksumCrc32) {
            rc = encode_crc_fused(dev, c, legacy_crc(), d_obj, obj_stride, obj_size, frags, stripe_stride,
                                  frag_stride, bs, nstripes, stream);
            if (rc != ECAMD_EINVAL) return rc;
            rc = encode_crc_cover(dev, c, legacy_crc(), d_obj, obj_stride, obj_size, frags, stripe_stride,
                                  frag_stride, bs, nstripes, stream);
            if (rc != ECAMD_EINVAL) return rc;
        }
        rc = rs_encode_copy(k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, nstripes,
                            stream);
        if (rc) return rc;
        return run_crc(dev, legacy_crc(), checksum == kChksumCrc32, frags, stripe_stride,
                       frag_stride, kHeaderBytes, k + m, bs, nstripes, nullptr,
                       header_args(c, checksum, bs, obj_size, 0), stream);
    }
    if (backend == kBackendRs && a16(d_obj) && obj_stride % 16 == 0 && dev_tune("frame_unfused") == 0 &&
        dev_tune("frame_copy_padded") != 0) {
        // Objects that do not fill the payloads exactly (any size: Swift's 1 MiB segments give
        // bs = 104858): the same copy-through launch reads each chunk j*bs of the object with
        // unaligned loads and reads zeros past the object's end, so no split pass either; with
        // CRC32 checksums the whole tiles also fold them in the same launch (encode_crc_cover).
        if (checksum == kChksumCrc32) {
            rc = encode_crc_cover(dev, c, legacy_crc(), d_obj, obj_stride, obj_size, frags, stripe_stride,
                                  frag_stride, bs, nstripes, stream);
            if (rc != ECAMD_EINVAL) return rc;
        }
        // the whole 4 KiB tiles every payload holds on the copy-through launch; the rest by the
        // copy-through codec of exactly [cover, bs) on the side stream beside it (knob
        // frame_tail_fork), or after it by encode_tail (split + plain encode of the payloads' last tiles)
        const int64_t last = static_cast<int64_t>(obj_size) - (k - 1) * bs;
        const int64_t cover = last > 0 ? std::min(bs, last) / 4096 * 4096 : 0;
        rc = ECAMD_EINVAL;
        if (cover > 0 && fork_tail(bs - cover, checksum == kChksumCrc32)) {
            // the rest [cover, bs) on the side stream, from the objects (exact range), beside the whole tiles
            void* side = nullptr;
            if ((rc = side_fork(dev, stream, &side))) return rc;
            rc = rs_encode_copy(k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, nstripes, side,
                                static_cast<int64_t>(obj_size), cover);
            const bool heads = checksum != kChksumCrc32;  // no checksum: the headers read no payload byte
            if (rc == 0 && heads)
                rc = run_crc(dev, legacy_crc(), false, frags, stripe_stride, frag_stride, kHeaderBytes, k + m, bs,
                             nstripes, nullptr, header_args(c, checksum, bs, obj_size, 0), side);
            if (rc == 0)
                rc = rs_encode_copy(k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, nstripes, stream,
                                    static_cast<int64_t>(obj_size), 0, cover);
            const int rj = side_join(dev, stream);
            if (rc || rj || heads) return rc ? rc : rj;
        } else if (cover > 0 && cover < bs && dev_tune("frame_tail_bs") != 0) {
            if ((rc = rs_encode_copy(k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, nstripes, stream,
                                     static_cast<int64_t>(obj_size), 0, cover)))
                return rc;
            rc = encode_tail(dev, c, d_obj, obj_stride, obj_size, frags, stripe_stride, frag_stride, bs, nstripes,
                             cover, stream);
            if (rc == ECAMD_EINVAL)
                rc = rs_encode_copy(k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, nstripes, stream,
                                    static_cast<int64_t>(obj_size), cover);
        } else {
            rc = rs_encode_copy(k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, nstripes,
                                stream, static_cast<int64_t>(obj_size));
        }
        if (rc) return rc;
        return run_crc(dev, legacy_crc(), checksum == kChksumCrc32, frags, stripe_stride,
                       frag_stride, kHeaderBytes, k + m, bs, nstripes, nullptr,
                       header_args(c, checksum, bs, obj_size, 0), stream);
    }
    if (backend == kBackendXor && a16(d_obj) && obj_stride % 16 == 0 && dev_tune("frame_unfused") == 0 &&
        dev_tune("frame_xor_copy") != 0 && dev_tune("frame_copy_stream") != 0 &&
        copy_fits32(k, frag_stride, bs, static_cast<int64_t>(obj_size))) {
        // flat XOR, copy-through (round 4): the whole 4 KiB tiles every object chunk holds in one
        // launch that reads the chunks, writes the data payloads and the parity; the payloads' rest by
        // the streaming split + the XOR of that range; then the CRC pass and headers.  Against split +
        // XOR it moves 26 instead of 36 payload-sized units of HBM traffic per stripe at (10,6).
        if (checksum == kChksumCrc32) {  // the checksums folded into the codec launch, as for RS
            rc = encode_crc_cover(dev, c, legacy_crc(), d_obj, obj_stride, obj_size, frags, stripe_stride,
                                  frag_stride, bs, nstripes, stream);
            if (rc != ECAMD_EINVAL) return rc;
        }
        const int64_t last = static_cast<int64_t>(obj_size) - (k - 1) * bs;
        const int64_t cover = last > 0 ? std::min(bs, last) / 4096 * 4096 : 0;
        unsigned pb[32], db[32];
        ecamd_xor_code_tables(k, m, hd, pb, db);
        // the payloads' rest [cover, bs): split, then the XOR of that range (bytes disjoint from the
        // copy-through launch: on the side stream beside it, knob frame_tail_fork)
        auto rest = [&](void* st2) {
            int r = split_range(dev, k, d_obj, obj_stride, obj_size, frags, stripe_stride, frag_stride, bs, nstripes,
                                cover, st2);
            if (r == 0) {
                std::vector<int64_t> in_off(k), out_off(m);
                for (int j = 0; j < k; j++) in_off[j] = j * frag_stride;
                for (int o = 0; o < m; o++) out_off[o] = (k + o) * frag_stride;
                r = ecamd_xor_apply_strided(pb, m, k, p0 + cover, stripe_stride, in_off.data(), p0 + cover,
                                            stripe_stride, out_off.data(), bs - cover, nstripes, st2);
            }
            return r == ECAMD_EINVAL ? dev_fail(ECAMD_EHIP, "framed xor encode: tail failed") : r;
        };
        if (cover > 0 && fork_tail(bs - cover, checksum == kChksumCrc32)) {
            void* side = nullptr;
            if ((rc = side_fork(dev, stream, &side))) return rc;
            rc = rest(side);
            const bool heads = checksum != kChksumCrc32;  // no checksum: the headers read no payload byte
            if (rc == 0 && heads)
                rc = run_crc(dev, legacy_crc(), false, frags, stripe_stride, frag_stride, kHeaderBytes, k + m, bs,
                             nstripes, nullptr, header_args(c, checksum, bs, obj_size, 0), side);
            if (rc == 0)  // ECAMD_EINVAL (declined): the split path below rewrites everything after the join
                rc = xor_encode_copy(pb, k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, cover, nstripes,
                                     stream);
            const int rj = side_join(dev, stream);
            if (rj) return rj;
            if (rc == 0 && heads) return 0;
        } else {
            rc = cover > 0 ? xor_encode_copy(pb, k, m, d_obj, obj_stride, p0, stripe_stride, frag_stride, bs, cover,
                                             nstripes, stream)
                           : ECAMD_EINVAL;
            // from here on a failure is an error: part of the payloads is written
            if (rc == 0 && cover < bs && (rc = rest(stream))) return rc;
        }
        if (rc == 0)
            return run_crc(dev, legacy_crc(), checksum == kChksumCrc32, frags, stripe_stride, frag_stride,
                           kHeaderBytes, k + m, bs, nstripes, nullptr, header_args(c, checksum, bs, obj_size, 0),
                           stream);
        if (rc != ECAMD_EINVAL) return rc;
    }
    SplitArgs sa{static_cast<const uint8_t*>(d_obj), obj_stride, static_cast<int64_t>(obj_size),
                 frags, stripe_stride, frag_stride, bs, k, nstripes, aligned ? 1 : 0};
    if (copy_fits32(k, frag_stride, bs, static_cast<int64_t>(obj_size)) && dev_tune("frame_copy_stream") != 0) {
        const CopyShape cs = copy_shape(bs);
        const dim3 grid(copy_grid(dev, (bs + 15) / 16, k, nstripes, cs)), block(cs.threads);
        const bool dpp = dev_tune("frame_copy_dpp") != 0;
        if (cs.u == 1)
            hipLaunchKernelGGL((dpp ? frame_split_stream_kernel<1, true> : frame_split_stream_kernel<1, false>), grid,
                               block, copy_lds(), st, sa);
        else
            hipLaunchKernelGGL((dpp ? frame_split_stream_kernel<4, true> : frame_split_stream_kernel<4, false>), grid,
                               block, copy_lds(), st, sa);
    } else
        hipLaunchKernelGGL(frame_split_kernel, dim3(grid_for(dev, ((bs + 15) / 16) * k * nstripes)),
                           dim3(256), 0, st, sa);
    HIP_TRY(hipGetLastError());
    if (backend == kBackendRs) {
        rc = ecamd_rs_encode(k, m, p0, stripe_stride, frag_stride, bs, nstripes, stream);
    } else {
        // xor_code_encode accumulates into zeroed parity (src/builtin/xor_codes/xor_code.c:180-191):
        // parity j = XOR of the data fragments in parity_bms[j].
        unsigned pb[32], db[32];
        ecamd_xor_code_tables(k, m, hd, pb, db);
        std::vector<int64_t> in_off(k), out_off(m);
        for (int j = 0; j < k; j++) in_off[j] = j * frag_stride;
        for (int r = 0; r < m; r++) out_off[r] = (k + r) * frag_stride;
        rc = ecamd_xor_apply_strided(pb, m, k, p0, stripe_stride, in_off.data(), p0, stripe_stride,
                                     out_off.data(), bs, nstripes, stream);
    }
    if (rc) return rc;
    const bool legacy = legacy_crc();
    return run_crc(dev, legacy, checksum == kChksumCrc32, frags, stripe_stride, frag_stride,
                   kHeaderBytes, k + m, bs, nstripes, nullptr, header_args(c, checksum, bs, obj_size, 0),
                   stream);
}

int ecamd_frame_decode(int backend, int k, int m, int hd, const int* missing, void* d_frags,
                       int64_t stripe_stride, int64_t frag_stride, int nstripes, void* d_obj,
                       int64_t obj_stride, uint64_t obj_size, void* stream)
{
    int dev = 0;
    int rc = dev_ensure(&dev);
    if (rc) return rc;
    const StreamUse use(dev, stream);  // its stream context outlives this call
    const Code c = make_code(backend, k, m, hd);
    if ((rc = check_code(c))) return rc;
    if (!missing) return dev_fail(ECAMD_EINVAL, "null missing list");
    const int64_t bs = blocksize_of(c, obj_size);
    if ((rc = check_frames(d_frags, stripe_stride, frag_stride, bs, k + m, nstripes))) return rc;
    if (nstripes == 0) return 0;
    int nmiss = 0, data_missing = 0;
    for (; missing[nmiss] >= 0; nmiss++) {
        if (missing[nmiss] >= k + m) return dev_fail(ECAMD_EINVAL, "missing index out of range");
        data_missing += missing[nmiss] < k;
    }
    if (nmiss > m) return dev_fail(ECAMD_EINVAL, "%d fragments missing, at most m = %d", nmiss, m);
    auto* frags = static_cast<uint8_t*>(d_frags);
    uint8_t* p0 = frags + kHeaderBytes;
    if (data_missing && backend == kBackendRs && d_obj && a16(d_obj) && obj_stride % 16 == 0 &&
        dev_tune("frame_unfused") == 0 &&
        (static_cast<int64_t>(obj_size) == k * bs || dev_tune("frame_copy_padded") != 0)) {
        // One launch: the lost data are computed straight into the objects and the surviving data
        // payloads are copied there as they stream through (no separate join pass); objects of
        // any size (unaligned chunk offsets j*bs, nothing written past an object's end).
        return rs_decode_join(k, m, missing, p0, stripe_stride, frag_stride, d_obj, obj_stride, bs,
                              nstripes, stream, static_cast<int64_t>(obj_size));
    }
    if (data_missing && backend == kBackendXor && d_obj && a16(d_obj) && obj_stride % 16 == 0 &&
        dev_tune("frame_unfused") == 0 && dev_tune("frame_xor_copy") != 0 &&
        (static_cast<int64_t>(obj_size) == k * bs || dev_tune("frame_copy_padded") != 0)) {
        // flat XOR, as the RS decode-join: the plan is one 0 / 1 matrix over the surviving fragments
        // (lost ones count as zero, as in xor_plan_apply), so the lost data go straight into the
        // objects and the surviving data payloads are copied there by the same launch
        unsigned pb[32], db[32];
        ecamd_xor_code_tables(k, m, hd, pb, db);
        std::vector<int> outs(k + m);
        std::vector<uint64_t> srcs(k + m);
        int n = 0;
        if (ecamd_xor_plan(1, k, m, hd, pb, db, missing, 0, outs.data(), srcs.data(), &n) < 0)
            return dev_fail(ECAMD_EINVAL, "flat_xor_hd: erasure pattern not recoverable");
        uint64_t lost = 0;
        for (int i = 0; missing[i] >= 0; i++) lost |= uint64_t(1) << missing[i];
        std::vector<int> douts, inputs, coeff;
        std::vector<uint64_t> dsrc;
        uint64_t need = 0, got = 0;
        for (int i = 0; i < n; i++)
            if (outs[i] < k) {
                douts.push_back(outs[i]);
                dsrc.push_back(srcs[i] & ~lost);
                need |= srcs[i] & ~lost;
                got |= uint64_t(1) << outs[i];
            }
        if (got == (lost & ((uint64_t(1) << k) - 1))) {  // every lost data fragment has its row
            for (int f = 0; f < k + m; f++)
                if (!(lost >> f & 1) && (f < k || (need >> f & 1))) inputs.push_back(f);
            for (uint64_t sm : dsrc)
                for (int f : inputs) coeff.push_back(static_cast<int>(sm >> f & 1));
            return xor_decode_join(k, inputs, douts, coeff, p0, stripe_stride, frag_stride, d_obj, obj_stride, bs,
                                   nstripes, stream, static_cast<int64_t>(obj_size));
        }
    }
    if (data_missing) {  // the systematic fast path (src/erasurecode.c:597-607) skips this
        if (backend == kBackendRs)
            rc = ecamd_rs_decode(k, m, missing, 0, p0, stripe_stride, frag_stride, bs, nstripes, stream);
        else
            rc = xor_plan_apply(c, 1, missing, 0, p0, stripe_stride, frag_stride, bs, nstripes, stream);
        if (rc) return rc;
    }
    if (obj_size == 0) return 0;
    if (!d_obj) return dev_fail(ECAMD_EINVAL, "null object buffer");
    JoinArgs ja{frags, stripe_stride, frag_stride, bs, static_cast<uint8_t*>(d_obj), obj_stride,
                static_cast<int64_t>(obj_size), nstripes,
                (a16(d_obj) && obj_stride % 16 == 0 && bs % 16 == 0) ? 1 : 0};
    if (copy_fits32(k, frag_stride, bs, static_cast<int64_t>(obj_size)) && bs >= 32 &&
        dev_tune("frame_copy_stream") != 0) {
        const CopyShape cs = copy_shape(bs);
        const int ja_knob = dev_tune("frame_join_align");
        const int align = (ja_knob == 1 || (ja_knob == 2 && bs % 16)) && a16(d_obj) && obj_stride % 16 == 0 ? 1 : 0;
        const int64_t span = static_cast<int64_t>(cs.threads) * cs.u;
        const dim3 grid(copy_grid(dev, bs / 16 + 2 + (align ? span - 1 : 0), k, nstripes, cs)), block(cs.threads);
        const bool dpp = dev_tune("frame_copy_dpp") != 0;
        if (cs.u == 1)
            hipLaunchKernelGGL((dpp ? frame_join_stream_kernel<1, true> : frame_join_stream_kernel<1, false>), grid,
                               block, copy_lds(), static_cast<hipStream_t>(stream), ja, k, align);
        else
            hipLaunchKernelGGL((dpp ? frame_join_stream_kernel<4, true> : frame_join_stream_kernel<4, false>), grid,
                               block, copy_lds(), static_cast<hipStream_t>(stream), ja, k, align);
    } else
        hipLaunchKernelGGL(frame_join_kernel,
                           dim3(grid_for(dev, ((static_cast<int64_t>(obj_size) + 15) / 16) * nstripes)),
                           dim3(256), 0, static_cast<hipStream_t>(stream), ja);
    HIP_TRY(hipGetLastError());
    return 0;
}

int ecamd_frame_reconstruct(int backend, int k, int m, int hd, int checksum, const int* missing,
                            int dest, void* d_frags, int64_t stripe_stride, int64_t frag_stride,
                            uint64_t obj_size, int nstripes, void* stream)
{
    int dev = 0;
    int rc = dev_ensure(&dev);
    if (rc) return rc;
    const StreamUse use(dev, stream);  // its stream context outlives this call
    const Code c = make_code(backend, k, m, hd);
    if ((rc = check_code(c))) return rc;
    if (!missing || dest < 0 || dest >= k + m) return dev_fail(ECAMD_EINVAL, "bad missing / dest");
    const int64_t bs = blocksize_of(c, obj_size);
    if ((rc = check_frames(d_frags, stripe_stride, frag_stride, bs, k + m, nstripes))) return rc;
    if (nstripes == 0) return 0;
    int nmiss = 0;
    while (missing[nmiss] >= 0) nmiss++;
    if (nmiss > m) return dev_fail(ECAMD_EINVAL, "%d fragments missing, at most m = %d", nmiss, m);
    auto* frags = static_cast<uint8_t*>(d_frags);
    uint8_t* p0 = frags + kHeaderBytes;
    if (backend == kBackendRs)
        rc = ecamd_rs_reconstruct(k, m, missing, dest, p0, stripe_stride, frag_stride, bs, nstripes,
                                  stream);
    else
        rc = xor_plan_apply(c, 2, missing, dest, p0, stripe_stride, frag_stride, bs, nstripes, stream);
    if (rc) return rc;
    // liberasurecode_reconstruct_fragment stamps the rebuilt fragment with its checksum
    // (src/erasurecode.c:907-915 -> add_fragment_metadata).
    return run_crc(dev, legacy_crc(), checksum == kChksumCrc32, frags + dest * frag_stride,
                   stripe_stride, frag_stride, kHeaderBytes, 1, bs, nstripes, nullptr,
                   header_args(c, checksum, bs, obj_size, dest), stream);
}

int ecamd_frame_verify(int nfrag, int64_t blocksize, int legacy, const void* d_frags,
                       int64_t stripe_stride, int64_t frag_stride, int nstripes,
                       uint32_t* d_status, uint32_t* d_crc, void* stream)
{
    int dev = 0;
    int rc = dev_ensure(&dev);
    if (rc) return rc;
    const StreamUse use(dev, stream);  // its stream context outlives this call
    if (nfrag < 1 || nfrag > 64 || blocksize < 0 || !d_status)
        return dev_fail(ECAMD_EINVAL, "bad nfrag / blocksize / status");
    if ((rc = check_frames(d_frags, stripe_stride, frag_stride, blocksize, nfrag, nstripes))) return rc;
    if (nstripes == 0) return 0;
    const int64_t items = static_cast<int64_t>(nfrag) * nstripes;
    uint32_t* crc = d_crc;
    std::unique_ptr<void, int (*)(void*)> tmp(nullptr, [](void* p) { return static_cast<int>(hipFree(p)); });
    if (!crc) {
        void* t = nullptr;
        HIP_TRY(hipMalloc(&t, items * sizeof(uint32_t)));
        tmp.reset(t);
        crc = static_cast<uint32_t*>(t);
    }
    const auto* frags = static_cast<const uint8_t*>(d_frags);
    HeaderArgs none{};
    rc = run_crc(dev, legacy != 0, true, frags, stripe_stride, frag_stride, kHeaderBytes, nfrag,
                 blocksize, nstripes, crc, none, stream);
    if (rc) return rc;
    const DevImage *iz = nullptr, *il = nullptr;
    if ((rc = image(dev, false, 8, 4, 8, false, &iz)) || (rc = image(dev, true, 8, 4, 8, false, &il))) return rc;
    CrcArgs a{};
    a.base = frags;
    a.stripe_stride = stripe_stride;
    a.frag_stride = frag_stride;
    a.items = items;
    a.nfrag = nfrag;
    a.t_off = static_cast<uint32_t>(iz->img.t_off);
    hipLaunchKernelGGL(frame_verify_kernel, dim3(static_cast<unsigned>((items + 127) / 128)), dim3(128),
                       0, static_cast<hipStream_t>(stream), a, iz->d, il->d, crc, blocksize, d_status);
    HIP_TRY(hipGetLastError());
    if (tmp) HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return 0;
}

int ecamd_crc32(int legacy, const void* d_base, int64_t stripe_stride, int64_t frag_stride,
                int nfrag, int64_t len, int nstripes, uint32_t* d_crc, void* stream)
{
    int dev = 0;
    int rc = dev_ensure(&dev);
    if (rc) return rc;
    const StreamUse use(dev, stream);  // its stream context outlives this call
    if (!d_base || !d_crc || nfrag < 1 || len < 0 || nstripes < 0)
        return dev_fail(ECAMD_EINVAL, "bad crc32 arguments");
    if (!a16(d_base) || stripe_stride % 16 || frag_stride % 16)
        return dev_fail(ECAMD_EINVAL, "crc32: base and strides must be 16-byte aligned");
    HeaderArgs none{};
    return run_crc(dev, legacy != 0, true, static_cast<const uint8_t*>(d_base), stripe_stride,
                   frag_stride, 0, nfrag, len, nstripes, d_crc, none, stream);
}

// ---- flat_xor_hd on strided batches (no framing): encode / decode / reconstruct in place ----

int ecamd_xor_encode(int k, int m, int hd, void* base, int64_t stripe_stride, int64_t frag_stride,
                     int64_t blocksize, int nstripes, void* stream)
{
    int rc = dev_ensure(nullptr);
    if (rc) return rc;
    const Code c = make_code(kBackendXor, k, m, hd);
    if ((rc = xor_batch_check(c, base, stripe_stride, frag_stride, blocksize, nstripes))) return rc;
    if (nstripes == 0 || blocksize == 0) return 0;
    // xor_code_encode (src/builtin/xor_codes/xor_code.c:180-191) accumulates into the zeroed
    // parity the frontend allocates: parity j = XOR of the data fragments in parity_bms[j], which
    // is written here (overwriting whatever the parity slots held)
    unsigned pb[32], db[32];
    ecamd_xor_code_tables(k, m, hd, pb, db);
    std::vector<int64_t> in_off(k), out_off(m);
    for (int j = 0; j < k; j++) in_off[j] = j * frag_stride;
    for (int r = 0; r < m; r++) out_off[r] = (k + r) * frag_stride;
    return ecamd_xor_apply_strided(pb, m, k, base, stripe_stride, in_off.data(), base, stripe_stride,
                                   out_off.data(), blocksize, nstripes, stream);
}

int ecamd_xor_decode(int k, int m, int hd, const int* missing, int decode_parity, void* base,
                     int64_t stripe_stride, int64_t frag_stride, int64_t blocksize, int nstripes,
                     void* stream)
{
    int rc = dev_ensure(nullptr);
    if (rc) return rc;
    const Code c = make_code(kBackendXor, k, m, hd);
    if ((rc = xor_batch_check(c, base, stripe_stride, frag_stride, blocksize, nstripes))) return rc;
    if (!missing) return dev_fail(ECAMD_EINVAL, "null missing list");
    for (int i = 0; missing[i] >= 0; i++)
        if (missing[i] >= k + m) return dev_fail(ECAMD_EINVAL, "missing index %d out of range", missing[i]);
    if (nstripes == 0 || blocksize == 0) return 0;
    return xor_plan_apply(c, 1, missing, decode_parity ? 1 : 0, static_cast<uint8_t*>(base), stripe_stride,
                          frag_stride, blocksize, nstripes, stream);
}

int ecamd_xor_reconstruct(int k, int m, int hd, const int* missing, int dest, void* base,
                          int64_t stripe_stride, int64_t frag_stride, int64_t blocksize, int nstripes,
                          void* stream)
{
    int rc = dev_ensure(nullptr);
    if (rc) return rc;
    const Code c = make_code(kBackendXor, k, m, hd);
    if ((rc = xor_batch_check(c, base, stripe_stride, frag_stride, blocksize, nstripes))) return rc;
    if (!missing || dest < 0 || dest >= k + m) return dev_fail(ECAMD_EINVAL, "bad missing list / destination");
    for (int i = 0; missing[i] >= 0; i++)
        if (missing[i] >= k + m) return dev_fail(ECAMD_EINVAL, "missing index %d out of range", missing[i]);
    if (nstripes == 0 || blocksize == 0) return 0;
    return xor_plan_apply(c, 2, missing, dest, static_cast<uint8_t*>(base), stripe_stride, frag_stride,
                          blocksize, nstripes, stream);
}

int ecamd_xor_decode_multi(int k, int m, int hd, const int* missing, int missing_stride, int decode_parity,
                           void* base, int64_t stripe_stride, int64_t frag_stride, int64_t blocksize,
                           int nstripes, void* stream)
{
    int dev = 0;
    int rc = dev_ensure(&dev);
    if (rc) return rc;
    const Code c = make_code(kBackendXor, k, m, hd);
    if ((rc = xor_batch_check(c, base, stripe_stride, frag_stride, blocksize, nstripes))) return rc;
    if (!missing || missing_stride < 1) return dev_fail(ECAMD_EINVAL, "bad missing lists");
    if (nstripes == 0 || blocksize == 0) return 0;
    if ((k + m - 1) * frag_stride + blocksize >= (int64_t(1) << 31))
        return dev_fail(ECAMD_EINVAL, "stripes wider than 2 GiB");
    // Group stripes by their erasure list as given: xor_hd_decode's control flow (which equation
    // rebuilds what) follows the list, so stripes share a launch only with identical lists.
    std::map<std::vector<int>, std::vector<int32_t>> groups;
    for (int s = 0; s < nstripes; s++) {
        const int* row = missing + static_cast<int64_t>(s) * missing_stride;
        std::vector<int> pat;
        for (int i = 0; i < missing_stride && row[i] >= 0; i++) {
            if (row[i] >= k + m) return dev_fail(ECAMD_EINVAL, "stripe %d: missing index %d", s, row[i]);
            pat.push_back(row[i]);
        }
        groups[pat].push_back(s);
    }
    std::vector<int32_t> list;
    list.reserve(nstripes);
    for (const auto& g : groups) list.insert(list.end(), g.second.begin(), g.second.end());
    StagedUpload up;
    if ((rc = up.begin(dev, stream, list.data(), list.size() * sizeof(int32_t)))) return rc;
    const auto* d_list = static_cast<const int32_t*>(up.dev);
    size_t at = 0;
    for (const auto& g : groups) {
        const int G = static_cast<int>(g.second.size());
        const int32_t* sl = d_list + at;
        at += static_cast<size_t>(G);
        if (g.first.empty()) continue;
        std::vector<int> pat(g.first);
        pat.push_back(-1);
        rc = xor_plan_apply(c, 1, pat.data(), decode_parity ? 1 : 0, static_cast<uint8_t*>(base), stripe_stride,
                            frag_stride, blocksize, G, stream, sl);
        if (rc) break;
    }
    const int rc2 = up.end(stream);
    return rc ? rc : rc2;
}

}  // extern "C"
