/*
 * ecamd_probe.h -- libecamd_probe.so: MI355X measurement probes (NOT the codec product).
 *
 * HBM ceilings and lookup-engine rates that DESIGN.md judges the codec kernels against; bench.py
 * uses ecamd_probe_bw for its live copy-peak denominator, tools/ for sweeps.  Pointers are device
 * pointers, `stream` a hipStream_t; every call returns 0 or a negative code
 * (ecamd_probe_last_error() gives the reason).
 */
#ifndef ECAMD_PROBE_H
#define ECAMD_PROBE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char *ecamd_probe_last_error(void);

/* ---- non-temporal 16 B/lane streaming copy (HBM ceiling probe) ---- */
int ecamd_probe_stream_copy(void *d_dst, const void *d_src, int64_t bytes, void *stream);
/* kind 0 copy / 1 read-only / 2 write-only over `bytes`, unroll in {1,4,8} 16-B loads per lane in
 * flight, grid = CUs x wgs_per_cu workgroups of 256 lanes (bandwidth ceilings for DESIGN.md). */
/* Copy of `bytes` (a multiple of threads*16) with one workgroup of `threads` (64 / 128 / 256) lanes per
 * tile of threads*16 bytes, 16 B per lane, non-temporal, in dispatcher order: with one-wave 1 KiB
 * tiles the fastest HBM copy measured here. */
int ecamd_probe_copy_tiles(int threads, void *d_dst, const void *d_src, int64_t bytes, void *stream);
int ecamd_probe_bw(int kind, int unroll, int wgs_per_cu, void *d_dst, const void *d_src,
                         int64_t bytes, void *stream);
/* Codec-shaped streaming probe: K fragment reads and R fragment writes per tile over nstripes
 * stripes of (K+R) fragments of blocksize bytes at d_base (stripe stride (K+R)*blocksize), the tile
 * order of gf16_apply_kernel, no table work.  lp / sp: buffer-load / store cache policy (gfx950
 * cpol: 1 sc0, 2 nt, 16 sc1; pairs listed in ECAMD_MIX_POLICIES), ch: 16-B chunks per lane (1, 2).
 * blocksize must be a multiple of threads*16*ch; stripe stride < 2 GiB. */
int ecamd_probe_mix(int lp, int sp, int ch, int threads, int wgs_per_cu, void *d_base,
                          int64_t blocksize, int K, int R, int nstripes, void *stream);
/* Lookup-engine probe: random 16-byte lookups into four 4 KiB tables (d_table, 16 KiB) from LDS
 * (mode 0), from global memory through the vector L1 (1) or half each (2); grid = CUs x wgs_per_cu
 * workgroups of 256 lanes, iters x 4 lookups per lane. */
int ecamd_probe_lookup(int mode, int wgs_per_cu, int iters, const void *d_table, void *stream);
/* One workgroup of 256 threads: mode 0 a single store, 1 / 2 first stage `bytes` of d_src into LDS
 * (one / eight 16-byte loads in flight per thread), 3 / 4 1024 / 4096 straight-line VALU steps
 * (a long kernel body).  Kernel-trace durations give a small launch's fixed costs. */
int ecamd_probe_launch(int mode, const void *d_src, int bytes, void *stream);
/* The same with the tile order (0 grid-stride, 1 a contiguous tile range per workgroup, 2 grid-stride
 * with each tile's fragment order rotated by the tile index) and the
 * chunk layout (wave_contig 1: a wave's ch chunks are 1 KiB apart, contiguous) as parameters. */
int ecamd_probe_mix2(int lp, int sp, int ch, int threads, int wgs_per_cu, int order,
                           int wave_contig, void *d_base, int64_t blocksize, int K, int R,
                           int nstripes, void *stream);
/* The same with an explicit slot per logical fragment: frag[i] (i < K) is read, frag[K + r] is
 * written (a permutation of 0..K+R-1; NULL = identity). */
int ecamd_probe_mix3(int lp, int sp, int ch, int threads, int wgs_per_cu, int order, int wave_contig,
                     void *base, int64_t bs, int K, int R, int nstripes, const int *frag, void *stream);
/* The same with the codec's launch shapes: wgs_per_cu <= 0 gives one workgroup per tile (the
 * dispatcher hands tiles out, as ecamd_bs_kernel's bs_grid form), and cap_per_cu > 0 limits the
 * resident workgroups per CU with a dynamic LDS share of 160 KiB / cap (the codec's per-CU caps). */
/* Mailbox round trip (round 6): one wave polls a word in coherent pinned host memory for requests
 * 1..n posted by this thread, optionally reads `payload` bytes of the mailbox, and acks each; the host
 * times post -> ack.  out_us: mean, min, median, 90th percentile (first request excluded), in us.  The
 * wave exits after n requests, on stop, or after idle_us with no request. */
int ecamd_probe_mailbox(int n, int payload, int idle_us, double *out_us);

int ecamd_probe_mix4(int lp, int sp, int ch, int threads, int wgs_per_cu, int cap_per_cu, int wave_contig,
                     void *base, int64_t bs, int K, int R, int nstripes, const int *frag, void *stream);

/* VALU / LDS issue-cost probe: grid = CUs x wgs_per_cu workgroups of 256 lanes, each lane `iters`
 * rounds of 8 independent instructions of form op (0 v_xor_b32, 1 v_bitop3_b32, 2 SDWA byte-select
 * shift, 3 v_bfe_u32, 4 v_and_b32, 5 v_perm_b32, 6 v_lshl_or_b32, 7 conflict-free ds_read_b128 +
 * wait). */
int ecamd_probe_valu(int op, int wgs_per_cu, int iters, void *stream);
/* Unaligned-copy probe: `bytes` (a multiple of 4096) copied in one-workgroup 4 KiB tiles with one side
 * displaced by `shift` (0..15) bytes; mode 0 aligned, 1 unaligned 16-byte loads, 2 two aligned loads
 * realigned, 3 one aligned load + the next lane's (DPP), 4 dword-aligned 16-byte load + one dword,
 * 5 unaligned 16-byte stores.  Buffers need bytes + 32 of room. */
int ecamd_probe_unaligned(int mode, int shift, void *d_dst, const void *d_src, int64_t bytes, void *stream);
#ifdef __cplusplus
}
#endif
#endif
