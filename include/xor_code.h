/*
 * xor_code.h -- drop-in flat-XOR HD codec library ABI (boundary B1'), MI355X implementation.
 *
 * Built as libXorcode.so.1, the library liberasurecode.so links (src/Makefile.am:37-41) and the
 * flat_xor_hd backend calls (src/backends/xor/flat_xor_hd.c:65-184), exporting the 5 symbols of
 * the reference's libXorcode.sym:1-5.  xor_code_t has the layout of the reference's
 * include/xor_codes/xor_code.h:54-65; its function pointers point into this library.
 *
 * Semantics kept bit-for-bit (including for inconsistent fragments, and the reference's partial
 * writes before a failure return): xor_code_encode XOR-accumulates into the parity buffers;
 * xor_hd_decode / xor_reconstruct_one pick exactly the reference's parity equations
 * (src/builtin/xor_codes/xor_hd_code.c:418-662, xor_code.c:248-314).  The byte work runs on the
 * GPU; with no HIP device init_xor_hd_code prints the reason and returns NULL (instance_create
 * then fails with -EBACKENDINITERR) -- there is no CPU fallback.
 */
#ifndef XOR_CODE_AMD_H
#define XOR_CODE_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define MAX_DATA 32
#define MAX_PARITY MAX_DATA

typedef struct xor_code_s {
    int k;
    int m;
    int hd;
    unsigned int *parity_bms;
    unsigned int *data_bms;
    int (*decode)(struct xor_code_s *code_desc, char **data, char **parity, int *missing_idxs,
                  int blocksize, int decode_parity);
    void (*encode)(struct xor_code_s *code_desc, char **data, char **parity, int blocksize);
    int (*fragments_needed)(struct xor_code_s *code_desc, int *missing_idxs,
                            int *fragments_to_exclude, int *fragments_needed);
} xor_code_t;

/* reference prototypes: include/xor_codes/xor_code.h:67-105 */
xor_code_t *init_xor_hd_code(int k, int m, int hd);                          /* xor_hd_code.c:664 */
void xor_code_encode(xor_code_t *code_desc, char **data, char **parity,
                     int blocksize);                                          /* xor_code.c:180 */
int xor_hd_decode(xor_code_t *code_desc, char **data, char **parity, int *missing_idxs,
                  int blocksize, int decode_parity);                         /* xor_hd_code.c:574 */
int xor_hd_fragments_needed(xor_code_t *code_desc, int *fragments_to_reconstruct,
                            int *fragments_to_exclude,
                            int *fragments_needed);                          /* xor_hd_code.c:209 */
int xor_reconstruct_one(xor_code_t *code_desc, char **data, char **parity, int *missing_idxs,
                        int index_to_reconstruct, int blocksize);            /* xor_code.c:248 */

#ifdef __cplusplus
}
#endif
#endif
