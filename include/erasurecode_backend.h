/*
 * erasurecode_backend.h -- backend plugin surface of the B2 frontend.
 *
 * Layout-compatible with the reference's include/erasurecode/erasurecode_backend.h:76-142, so
 * callers that reach into an instance (the reference's own tests swap common.ops->encode and
 * read common.id / common.ec_backend_version, test/liberasurecode_test.c:713-718, 1531, 2210)
 * keep working.  The frontend always dispatches through common.ops.
 */
#ifndef ERASURECODE_BACKEND_AMD_H
#define ERASURECODE_BACKEND_AMD_H

#include "erasurecode.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MAX_PRIV_ARGS 4
struct ec_backend_args {
    struct ec_args uargs;
    void *pargs[MAX_PRIV_ARGS];
};

struct ec_backend_op_stubs {
    void *(*init)(struct ec_backend_args *args, void *sohandle);
    int (*exit)(void *desc);
    bool is_systematic;
    int (*encode)(void *desc, char **data, char **parity, int blocksize);
    int (*decode)(void *desc, char **data, char **parity, int *missing_idxs, int blocksize);
    int (*fragments_needed)(void *desc, int *missing_idxs, int *fragments_to_exclude,
                            int *fragments_needed);
    int (*reconstruct)(void *desc, char **data, char **parity, int *missing_idxs,
                       int destination_idx, int blocksize);
    int (*element_size)(void *desc);
    bool (*is_compatible_with)(uint32_t version);
    size_t (*get_backend_metadata_size)(void *desc, int blocksize);
    size_t (*get_encode_offset)(void *desc, int metadata_size);
    int (*check_reconstruct_fragments)(void *desc, int *missing_idxs, int destination_idx);
};

struct ec_backend_desc {
    void *backend_desc;
    void *backend_sohandle;
};

#define MAX_LEN 64
struct ec_backend_common {
    ec_backend_id_t id;
    char name[MAX_LEN];
    const char *soname;
    char soversion[MAX_LEN];
    struct ec_backend_op_stubs *ops;
    uint32_t ec_backend_version;
};

struct ec_backend {
    struct ec_backend_common common;
    struct ec_backend_args args;
    int idesc;
    struct ec_backend_desc desc;
    struct { struct ec_backend *sle_next; } link;
};

#ifdef __cplusplus
}
#endif
#endif
