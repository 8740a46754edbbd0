/*
 * erasurecode.h -- liberasurecode frontend C API (boundary B2), MI355X build.
 *
 * liberasurecode.so.1 from this repo exports the 28 symbols of the reference's
 * liberasurecode.sym:1-28 with the reference signatures (include/erasurecode/erasurecode.h:
 * 109-376) and the same on-wire fragment format (80-byte packed header, :254-324), so PyECLib /
 * Swift style callers switch by library path alone.  Backends driven: EC_BACKEND_FLAT_XOR_HD
 * (libXorcode.so.1) and EC_BACKEND_LIBERASURECODE_RS_VAND (liberasurecode_rs_vand.so.1), both
 * the GPU drop-ins of this repo; every other backend id reports "not available", as the
 * reference does when its external library is absent.
 */
#ifndef ERASURECODE_AMD_H
#define ERASURECODE_AMD_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EC_MAX_FRAGMENTS 256

#define _VERSION(x, y, z) (((x) << 16) | ((y) << 8) | (z))
#define LIBERASURECODE_VERSION _VERSION(1, 8, 0) /* the reference release this API mirrors */

/* Build-time suffix of every backend library name the frontend dlopen()s, e.g. "-amd" gives
 * "liberasurecode_rs_vand-amd.so.1" (include/erasurecode/erasurecode_version.h:35-37 and each
 * backend's SO_NAME, e.g. src/backends/rs_vand/liberasurecode_rs_vand.c:43).  Set with
 * `make SO_SUFFIX=...`; the codec libraries of this build carry it in their sonames too. */
#ifndef LIBERASURECODE_SO_SUFFIX
#define LIBERASURECODE_SO_SUFFIX ""
#endif

typedef enum {
    EC_BACKEND_NULL = 0,
    EC_BACKEND_JERASURE_RS_VAND = 1,
    EC_BACKEND_JERASURE_RS_CAUCHY = 2,
    EC_BACKEND_FLAT_XOR_HD = 3,
    EC_BACKEND_ISA_L_RS_VAND = 4,
    EC_BACKEND_SHSS = 5,
    EC_BACKEND_LIBERASURECODE_RS_VAND = 6,
    EC_BACKEND_ISA_L_RS_CAUCHY = 7,
    EC_BACKEND_LIBPHAZR = 8,
    EC_BACKEND_ISA_L_RS_VAND_INV = 9,
    EC_BACKEND_ISA_L_RS_LRC = 10,
    EC_BACKENDS_MAX,
} ec_backend_id_t;

typedef enum { CHKSUM_NONE = 1, CHKSUM_CRC32 = 2, CHKSUM_MD5 = 3, CHKSUM_TYPES_MAX } ec_checksum_type_t;

struct ec_args {
    int k, m, w, hd;
    union {
        struct { uint64_t arg1; } null_args;
        struct { int l; } lrc_args;
        struct { uint64_t x, y, z, a; } reserved;
    } priv_args1;
    void *priv_args2;
    ec_checksum_type_t ct;
};

#define LIBERASURECODE_MAX_CHECKSUM_LEN 8
#define LIBERASURECODE_FRAG_HEADER_MAGIC 0xb0c5ecc

typedef struct __attribute__((__packed__)) fragment_metadata {
    uint32_t idx;
    uint32_t size;
    uint32_t frag_backend_metadata_size;
    uint64_t orig_data_size;
    uint8_t chksum_type;
    uint32_t chksum[LIBERASURECODE_MAX_CHECKSUM_LEN];
    uint8_t chksum_mismatch;
    uint8_t backend_id;
    uint32_t backend_version;
} fragment_metadata_t; /* 59 bytes */

typedef struct __attribute__((__packed__)) fragment_header_s {
    fragment_metadata_t meta;
    uint32_t magic;
    uint32_t libec_version;
    uint32_t metadata_chksum;
    uint8_t aligned_padding[9];
} fragment_header_t; /* 80 bytes; the payload follows */

typedef enum {
    EBACKENDNOTSUPP = 200,
    EECMETHODNOTIMPL = 201,
    EBACKENDINITERR = 202,
    EBACKENDINUSE = 203,
    EBACKENDNOTAVAIL = 204,
    EBADCHKSUM = 205,
    EINVALIDPARAMS = 206,
    EBADHEADER = 207,
    EINSUFFFRAGS = 208,
} LIBERASURECODE_ERROR_CODES;

typedef struct ec_backend *ec_backend_t; /* layout: erasurecode_backend.h */

/* ---- the 28 exported symbols (reference liberasurecode.sym:1-28) ---- */
int liberasurecode_backend_available(const ec_backend_id_t backend_id);
int liberasurecode_instance_create(const ec_backend_id_t id, struct ec_args *args);
int liberasurecode_instance_destroy(int desc);
int liberasurecode_encode(int desc, const char *orig_data, uint64_t orig_data_size,
                          char ***encoded_data, char ***encoded_parity, uint64_t *fragment_len);
int liberasurecode_encode_cleanup(int desc, char **encoded_data, char **encoded_parity);
int liberasurecode_decode(int desc, char **available_fragments, int num_fragments,
                          uint64_t fragment_len, int force_metadata_checks, char **out_data,
                          uint64_t *out_data_len);
int liberasurecode_decode_cleanup(int desc, char *data);
int liberasurecode_reconstruct_fragment(int desc, char **available_fragments, int num_fragments,
                                        uint64_t fragment_len, int destination_idx,
                                        char *out_fragment);
int liberasurecode_fragments_needed(int desc, int *fragments_to_reconstruct,
                                    int *fragments_to_exclude, int *fragments_needed);
int liberasurecode_get_fragment_metadata(char *fragment, fragment_metadata_t *fragment_metadata);
int is_invalid_fragment(int desc, char *fragment);
int is_invalid_fragment_header(fragment_header_t *header);
int liberasurecode_verify_stripe_metadata(int desc, char **fragments, int num_fragments);
int liberasurecode_verify_fragment_metadata(ec_backend_t be, fragment_metadata_t *md);
int liberasurecode_get_aligned_data_size(int desc, uint64_t data_len);
int liberasurecode_get_minimum_encode_size(int desc);
int liberasurecode_get_fragment_size(int desc, int data_len);
uint32_t liberasurecode_get_version(void);
ec_backend_t liberasurecode_backend_instance_get_by_desc(int desc);
int liberasurecode_crc32_alt(int crc, const void *buf, size_t size);
void liberasurecode_init(void);
void liberasurecode_exit(void);
/* fragment helpers the reference also exports (src/erasurecode_helpers.c,
 * src/erasurecode_preprocessing.c) */
void *alloc_and_set_buffer(int size, int value);
char *get_data_ptr_from_fragment(char *buf);
int get_libec_version(char *buf, uint32_t *ver);
int get_backend_id(char *buf, ec_backend_id_t *id);
int get_backend_version(char *buf, uint32_t *version);
int get_fragment_partition(int k, int m, char **fragments, int num_fragments, char **data,
                           char **parity, int *missing);

#ifdef __cplusplus
}
#endif
#endif
