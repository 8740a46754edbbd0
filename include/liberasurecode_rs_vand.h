/*
 * liberasurecode_rs_vand.h -- drop-in codec library ABI (boundary B1), MI355X implementation.
 *
 * Built as liberasurecode_rs_vand.so.1, the soname the reference frontend dlopen()s
 * (src/backends/rs_vand/liberasurecode_rs_vand.c:43, src/erasurecode.c:136-142), exporting exactly
 * the 13 symbols of the reference's liberasurecode_rs_vand.sym:1-13 with the prototypes of
 * include/rs_vand/liberasurecode_rs_vand.h:27-44.  The reference shim dlsym()s seven of them
 * (src/backends/rs_vand/liberasurecode_rs_vand.c:187-233, typedefs :49-57); its unit test links
 * the rest (test/builtin/rs_vand/liberasurecode_rs_vand_test.c).
 *
 * Contract kept from the reference:
 *   - buffers are caller-owned host memory, `blocksize` bytes each, processed as little-endian
 *     16-bit GF(2^16) words (poly 0x1100b);
 *   - encode overwrites parity; decode rewrites every missing fragment (parity too when
 *     rebuild_parity) from the first k available in index order; reconstruct rewrites one
 *     destination; results are complete when the call returns;
 *   - decode / reconstruct return -1 when more than m fragments are missing, else 0;
 *   - make_systematic_matrix returns malloc()ed memory (callers may free() it directly);
 *   - encode / decode / reconstruct may run concurrently from many threads on one matrix.
 * Difference: the region arithmetic runs on the GPU.  With no HIP device, make_systematic_matrix
 * prints the reason to stderr and returns NULL (so the frontend's instance_create fails with
 * -EBACKENDINITERR) and encode/decode/reconstruct return -1; there is no CPU fallback.
 */
#ifndef LIBERASURECODE_RS_VAND_AMD_H
#define LIBERASURECODE_RS_VAND_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

/* reference: include/rs_vand/liberasurecode_rs_vand.h:27-44 */
void free_systematic_matrix(int *matrix);                              /* rs_vand.c:291 */
int *make_systematic_matrix(int k, int m);                             /* rs_vand.c:240-289 */
int is_missing(int *missing_idxs, int index_to_check);                 /* rs_vand.c:108-118 */
int gaussj_inversion(int *matrix, int *inverse, int n);                /* rs_vand.c:293-334 */
void init_liberasurecode_rs_vand(int k, int m);                        /* rs_vand.c:135 */
void deinit_liberasurecode_rs_vand(void);                              /* rs_vand.c:137 */
void print_matrix(int *matrix, int rows, int cols);                    /* rs_vand.c:44-56 */
void square_matrix_multiply(int *m1, int *m2, int *prod, int n);       /* rs_vand.c:58-71 */
int create_decoding_matrix(int *gen_matrix, int *dec_matrix, int *missing_idxs, int k,
                           int m);                                      /* rs_vand.c:120-133 */
int is_identity_matrix(int *matrix, int n);                            /* rs_vand.c:73-92 */
int liberasurecode_rs_vand_encode(int *generator_matrix, char **data, char **parity, int k, int m,
                                  int blocksize);                       /* rs_vand.c:399-410 */
int liberasurecode_rs_vand_decode(int *generator_matrix, char **data, char **parity, int k, int m,
                                  int *missing, int blocksize,
                                  int rebuild_parity);                  /* rs_vand.c:426-481 */
int liberasurecode_rs_vand_reconstruct(int *generator_matrix, char **data, char **parity, int k,
                                       int m, int *missing, int destination_idx,
                                       int blocksize);                  /* rs_vand.c:483-558 */

#ifdef __cplusplus
}
#endif
#endif
