/*
 * ecamd_host.h -- host-side planning for the MI355X erasure-code backend (libecamd_host.so).
 *
 * Pure host C ABI (no HIP types): GF(2^16) arithmetic, the reference generator matrix, and the
 * "fragment maps" (which fragments to read, which to write, with which coefficients) that the
 * device kernels apply.  Each entry point restates a piece of the reference's built-in
 * liberasurecode_rs_vand codec:
 *
 *   ecamd_gf16_mul / ecamd_gf16_inv   rs_galois_mult / rs_galois_inverse
 *                                     (src/builtin/rs_vand/rs_galois.c:90-117)
 *   ecamd_rs_generator                make_systematic_matrix (liberasurecode_rs_vand.c:240-289)
 *   ecamd_gf16_invert                 gaussj_inversion (liberasurecode_rs_vand.c:293-334)
 *   ecamd_rs_decode_map               coefficient rows of liberasurecode_rs_vand_decode
 *                                     (liberasurecode_rs_vand.c:426-481); missing parity is
 *                                     expressed directly over the first k available fragments
 *   ecamd_rs_reconstruct_map          coefficient row of liberasurecode_rs_vand_reconstruct
 *                                     (liberasurecode_rs_vand.c:483-558)
 */
#ifndef ECAMD_HOST_H
#define ECAMD_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int ecamd_gf16_mul(int a, int b);
int ecamd_gf16_inv(int a);

/* (k+m) x k row-major systematic generator into out; 0 on success. */
int ecamd_rs_generator(int k, int m, int *out);

/* Inverse of the n x n matrix a into inv; 0 on success, -1 if singular. */
int ecamd_gf16_invert(const int *a, int *inv, int n);

/* Decode map for a -1 terminated missing list.  inputs[k] receives the first k available
 * fragment indices; outputs[*nout] the rebuilt fragment indices (missing data, then missing
 * parity if rebuild_parity); coeff[*nout * k] the rows.  Returns -1 if more than m are missing. */
int ecamd_rs_decode_map(const int *G, int k, int m, const int *missing, int rebuild_parity,
                        int *inputs, int *outputs, int *coeff, int *nout);

/* Reconstruct map for one destination: inputs[*ninputs] and coeff[*ninputs]. */
int ecamd_rs_reconstruct_map(const int *G, int k, int m, const int *missing, int dest, int *inputs,
                             int *ninputs, int *coeff);

/* LDS split-table image for rows [row0,row0+width) x inputs [col0,col0+ncols) of the R x K
 * matrix coeff; width in {2,4,8}.  Returns the byte count written (ncols*512*width*2). */
int ecamd_split_tables(const int *coeff, int R, int K, int row0, int width, int col0, int ncols,
                       uint8_t *out);

/* ---- flat-XOR HD codes (src/builtin/xor_codes/) ---- */

/* Parity / data bitmaps of a supported (k, m, hd) code (include/xor_codes/xor_hd_code_defs.h);
 * -1 if the code is not one init_xor_hd_code accepts (xor_hd_code.c:664-693). */
int ecamd_xor_code_tables(int k, int m, int hd, unsigned int *parity_bms, unsigned int *data_bms);

/* Exact plan of a reference operation on k+m buffers: op 0 = xor_code_encode, 1 = xor_hd_decode
 * (arg = decode_parity), 2 = xor_reconstruct_one (arg = index).  outputs[*nout] are the buffers
 * the reference modifies, sources[i] the bitmask of ORIGINAL buffers whose XOR output i ends up
 * holding.  Returns the reference's return code (-100 for bad arguments). */
int ecamd_xor_plan(int op, int k, int m, int hd, const unsigned int *parity_bms,
                   const unsigned int *data_bms, const int *missing, int arg, int *outputs,
                   uint64_t *sources, int *nout);

/* xor_hd_fragments_needed (xor_hd_code.c:209-412); needed ends with -1. */
int ecamd_xor_fragments_needed(int k, int m, int hd, const unsigned int *parity_bms,
                               const unsigned int *data_bms, const int *to_reconstruct,
                               const int *to_exclude, int *needed);

/* Batched planning: liberasurecode_fragments_needed for nstripes stripes at once.
 * Stripe s: to_reconstruct at recon + s*list_stride, to_exclude at excl + s*list_stride (each
 * -1 terminated within list_stride entries); its needed list (-1 terminated, padded with -1) at
 * needed + s*(k+m+1) and its return code at rcs[s].  backend 6 (rs_vand): the first k indices
 * neither missing nor excluded (src/backends/rs_vand/liberasurecode_rs_vand.c:119-145), rc -1 if
 * fewer remain; backend 3 (flat_xor_hd): xor_hd_fragments_needed.  Returns -1 on bad arguments. */
int ecamd_fragments_needed_batch(int backend, int k, int m, int hd, const int *recon,
                                 const int *excl, int list_stride, int nstripes, int *needed,
                                 int *rcs);

/* Devices the per-call path (ecamd_host_map_apply / ecamd_host_xor_apply) spreads calls over:
 * every one of ndev visible devices, or the comma-separated subset named by spec (the
 * ECAMD_PERCALL_DEVICES environment variable; NULL or "" = all; out-of-range or repeated ids are
 * dropped, and a spec naming none of them means all).  Writes up to max ids to devs, returns the
 * count.  Call n of a process goes to devs[n % count].  One process per GPU names its device
 * ("3": liberasurecode_amd/shard.py does so for its ranks); the spec "current" (not parsed here)
 * makes the per-call path use the device current on the thread of its first call, resolved once. */
int ecamd_percall_device_plan(int ndev, const char *spec, int *devs, int max);

/* Host copies of one per-call request (host/copy_pool.cpp): dst[i] <- src[i], len[i] bytes, i < n,
 * regions not overlapping.  Batches of 1 MiB or more are split into 256 KiB pieces shared by the
 * caller and ECAMD_COPY_THREADS helper threads (default 4, 0 = off; one request uses them at a
 * time, a caller that finds them busy copies alone).  Complete on return; 0, or ECAMD_EINVAL
 * (-22) for null arrays.  Used by the per-call staging (pack / unpack) and by liberasurecode.so.1
 * for its object <-> fragment copies. */
int ecamd_host_copy(int n, void *const *dst, const void *const *src, const int64_t *len);
/* The same with a second destination per copy: dst[i] <- src[i] and, when dst2 and dst2[i] are
 * not null, dst2[i] <- src[i], reading the source from DRAM once (each 256 KiB piece is copied to
 * dst2 and then from there, cache-resident, to dst).  Used by the per-call staging pack when the
 * frontend hands it an input tee (ecamd_percall_tee_arm, ecamd.h). */
int ecamd_host_copy2(int n, void *const *dst, void *const *dst2, const void *const *src,
                     const int64_t *len);

/* Bitsliced GF(2^16) maps (host/bitslice.hpp): the XOR network built for an R x K matrix
 * (R <= 8, K <= 32, at most `cap` shared temporaries per input) evaluated on 32 words per input
 * (in: K x 32, out: R x 32; *ops = VALU ops of the network per tile), and the HIP source of the
 * kernel specialised to it, inputs loaded into registers (depth 0) or through a per-wave LDS ring
 * of 2 or 4 inputs (returns the source length; writes up to size-1 bytes + NUL). */
int ecamd_bitslice_eval(const int *coeff, int R, int K, int cap, const uint16_t *in, uint16_t *out,
                        int *ops);
int64_t ecamd_bitslice_source(const int *coeff, int R, int K, int cap, int depth, char *buf,
                              int64_t size);

#ifdef __cplusplus
}
#endif
#endif
