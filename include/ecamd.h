/*
 * ecamd.h -- MI355X device-resident erasure-code engine (libecamd.so), C ABI.
 *
 * This is the batched extension the reference does not have ("B2 ... A batched,
 * device-pointer extension API is new"): S independent stripes whose fragments already live in
 * HBM are encoded / decoded / reconstructed by one kernel launch.  The per-call drop-in ABIs of
 * the reference (liberasurecode_rs_vand.h, xor_code.h, erasurecode.h) are layered on top of it.
 *
 * All pointers named d_* are device pointers; `stream` is a hipStream_t (NULL = default stream).
 * Calls are asynchronous on `stream` unless stated.  Every entry point returns 0 on success and a
 * negative value on failure (ecamd_last_error() gives the reason).  There is no CPU fallback: with
 * no HIP device every call fails with ECAMD_ENODEV.
 *
 * Fragment layout ("strided"): fragment f of stripe s starts at
 *     base + s * stripe_stride + f * frag_stride
 * so both [S][k+m][F] (frag_stride = F, stripe_stride = (k+m)*F) and fragment-major
 * [k+m][S][F] layouts are expressible.  base, strides and offsets must be 16-byte aligned;
 * blocksize (bytes per fragment payload) may be any value >= 1.
 */
#ifndef ECAMD_H
#define ECAMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ECAMD_ENODEV (-19)
#define ECAMD_EINVAL (-22)
#define ECAMD_ENOMEM (-12)
#define ECAMD_EHIP (-5)

/* 0 if a HIP device is usable, ECAMD_ENODEV otherwise. */
int ecamd_init(void);
int ecamd_device_count(void);
/* The calling thread's current HIP device (every call below works on it). */
int ecamd_get_device(int *dev);
int ecamd_set_device(int dev);
const char *ecamd_last_error(void);
/* Launch-geometry knobs for sweeps ("threads", "wgs_per_cu", "nt", "grid_mult", "tiles_per_slot",
 * "xor_tiles_per_slot", "bs_tiles_per_slot", "scatter_lanes", ...; every setting produces
 * bit-identical results, only the launch shape changes); 0 restores the default (for
 * xor_ / bs_tiles_per_slot 0 means one launch per pass, a negative value the default).  Safe to
 * call while other threads launch: each launch reads each knob once. */
int ecamd_tune(const char *key, int value);

/* Bitsliced 8-output passes (hip/ecamd_jit.hip): 1 if run-time compilation (hiprtc) is usable;
 * ecamd_bitslice_wait() blocks until every kernel compile started so far has finished and returns
 * how many failed (their maps keep using the LDS-table kernels); ecamd_bitslice_entries() is the
 * number of matrices held (bounded by the "bitslice_entries" knob, least recently used evicted and
 * their modules unloaded once no launch can still use them). */
int ecamd_bitslice_available(void);
int ecamd_bitslice_wait(void);
int ecamd_bitslice_entries(void);
/* Bitsliced kernel launches this process has enqueued (tests pin which kernel ran). */
long long ecamd_bitslice_launches(void);

/* Which kernel an rs_vand operation's passes run on this process's current device, for fragments
 * of `blocksize` bytes: encode (missing NULL), decode of the -1 terminated `missing` (dest < 0;
 * rebuild_parity as ecamd_rs_decode) or single-destination reconstruct of `dest`.  Returns
 * ECAMD_FORM_TABLES (the LDS-table kernels serve it by shape or knob), ECAMD_FORM_BITSLICED (its
 * bitsliced kernel is loaded: shipped with the library, cached, or compiled), ECAMD_FORM_COMPILING
 * (being compiled; the LDS tables serve it meanwhile) or ECAMD_FORM_UNAVAILABLE (it would take the
 * bitsliced kernel but none can be had -- no shipped code object and no ecamd_jitc / libhiprtc, or
 * the compile failed: the LDS tables serve it, byte-identically); < 0 on error.  Asking starts the
 * compile of a map not seen before (knob "bitslice" 2: waits for it), as its first launch would. */
#define ECAMD_FORM_TABLES 0
#define ECAMD_FORM_BITSLICED 1
#define ECAMD_FORM_COMPILING 2
#define ECAMD_FORM_UNAVAILABLE 3
int ecamd_rs_kernel_form(int k, int m, const int *missing, int dest, int rebuild_parity, int64_t blocksize);

/* Build time, no GPU needed: compile the bitsliced kernels of one rs_vand operation (arguments as
 * ecamd_rs_kernel_form) for target `arch` ("gfx950") into `dir` -- the library's jit/ directory,
 * which the run time searches before the per-user cache -- under the names the run time looks up
 * with the current knobs.  Returns the number of code objects present (0: the operation takes no
 * bitsliced kernel), < 0 on error (ecamd_jitc missing or failed). */
int ecamd_bitslice_prebuild(int k, int m, const int *missing, int dest, int rebuild_parity, const char *arch,
                            const char *dir);
/* The same for the CHKSUM_CRC32 framed encode (ecamd_frame_encode) of a code (backend 6 rs_vand or 3
 * flat_xor_hd): its bitsliced codec-and-checksum kernel, one per code whatever the object size.
 * Returns 1 when present, 0 when that encode takes no bitsliced kernel, < 0 on error. */
int ecamd_frame_prebuild(int backend, int k, int m, int hd, const char *arch, const char *dir);

/* ---- GF(2^16) fragment maps: outputs[r] = sum_j coeff[r*K+j] * inputs[j] (16-bit LE words) ---- */
typedef struct ecamd_map ecamd_map;

/* Prepare the R x K coefficient matrix for the current device (split tables in HBM). */
int ecamd_map_create(const int *coeff, int R, int K, ecamd_map **out);
void ecamd_map_destroy(ecamd_map *map);

/* Input j of stripe s at in_base + s*in_stripe_stride + in_off[j] (K host-side offsets), output r
 * at out_base + s*out_stripe_stride + out_off[r] (R offsets). */
int ecamd_map_apply_strided(const ecamd_map *map, const void *in_base, int64_t in_stripe_stride,
                            const int64_t *in_off, void *out_base, int64_t out_stripe_stride,
                            const int64_t *out_off, int64_t blocksize, int nstripes, void *stream);
/* ecamd_map_apply_strided for ONE stripe, plus the CRC32 of every input and output fragment over its
 * `blocksize` bytes -- zlib's crc32, or the legacy liberasurecode_crc32_alt when legacy != 0 -- written
 * to crc_out[0 .. K + R) (inputs first; device or pinned host memory), all in ONE launch of the
 * small-launch kernel.  Returns 0 when done, 1 when the shape does not fuse (nothing launched: more
 * than 4096 16-byte chunks per fragment, several passes, tables and staged fragments over the LDS, ...;
 * the caller runs ecamd_map_apply_strided and ecamd_crc32), < 0 on error.  The per-call CHKSUM_CRC32
 * encode's checksums (src/erasurecode_postprocessing.c:37-69) without two more launches. */
int ecamd_map_apply_strided_crc(const ecamd_map *map, const void *in_base, const int64_t *in_off, void *out_base,
                                const int64_t *out_off, int64_t blocksize, int legacy, uint32_t *crc_out,
                                void *stream);
/* The same for a flat-XOR map (masks as ecamd_xor_apply_strided, at most 8 outputs): one launch of the
 * small-launch XOR kernel with the checksums folded in; 0 done, 1 not fused (nothing launched), < 0 error. */
int ecamd_xor_apply_strided_crc(const uint32_t *masks, int R, int K, const void *in_base, const int64_t *in_off,
                                void *out_base, const int64_t *out_off, int64_t blocksize, int legacy,
                                uint32_t *crc_out, void *stream);
/* Launches of ecamd_map_apply_strided_crc / ecamd_xor_apply_strided_crc that fused the checksums (tests
 * pin which path ran). */
long long ecamd_small_crc_launches(void);
/* Completion flag of the calling thread's next operation (the per-call path, host/hostio.cpp): when the
 * small-launch kernel that ends it runs (gf16_small_kernel), it stores `value` to *flag -- pinned host
 * memory -- after every output and checksum store of the operation is visible system-wide, so the host
 * can poll the flag instead of synchronizing the stream.  ecamd_done_flag_taken() says whether the
 * operation took it (1), posted it to the resident small server (2: wait with ecamd_small_server_wait,
 * not on the stream, which it never touched) or not (0: other kernels; synchronize as usual) and disarms. */
void ecamd_done_flag_arm(uint32_t *flag, uint32_t value);
int ecamd_done_flag_taken(void);
/* The same, and the operation may be posted to the calling thread's resident small server (small_server_kernel,
 * DESIGN.md §6) instead of launched when it is ONE small launch with staged inputs: mode 1 any such launch,
 * 2 only one with the checksums fused (a separate checksum pass would follow on the stream); 0 as
 * ecamd_done_flag_arm.  The caller guarantees nothing it enqueued earlier on the stream is still pending. */
void ecamd_done_flag_arm_server(uint32_t *flag, uint32_t value, int mode);
/* Waits for a served operation's flag; relaunches the server if it exited before the request (its idle
 * time).  0, or < 0 after 10 s or a HIP error. */
int ecamd_small_server_wait(const uint32_t *flag, uint32_t value);
/* Operations posted to small servers, and server kernels launched (first use, after idle exits, variant
 * switches, relaunches in ecamd_small_server_wait), in this process (tests pin which path ran). */
long long ecamd_small_server_posts(void);
long long ecamd_small_server_launches(void);
/* Posts that wrote a new argument block into one of the server's two slots (the others reused a cached one). */
long long ecamd_small_server_rewrites(void);

/* Pointer tables in device memory: input j of stripe s is d_in_ptrs[s*in_row + in_col[j]],
 * output r is d_out_ptrs[s*out_row + out_col[r]] (in_col / out_col are host arrays). */
int ecamd_map_apply_ptrs(const ecamd_map *map, const void *const *d_in_ptrs, int in_row,
                         const int *in_col, void *const *d_out_ptrs, int out_row,
                         const int *out_col, int64_t blocksize, int nstripes, void *stream);

/* ---- GF(2) (flat XOR) fragment maps: outputs[r] = XOR of inputs j with bit j of mask[r] ---- */
int ecamd_xor_apply_strided(const uint32_t *masks, int R, int K, const void *in_base,
                            int64_t in_stripe_stride, const int64_t *in_off, void *out_base,
                            int64_t out_stripe_stride, const int64_t *out_off, int64_t blocksize,
                            int nstripes, void *stream);
int ecamd_xor_apply_ptrs(const uint32_t *masks, int R, int K, const void *const *d_in_ptrs,
                         int in_row, const int *in_col, void *const *d_out_ptrs, int out_row,
                         const int *out_col, int64_t blocksize, int nstripes, void *stream);

/* ---- liberasurecode_rs_vand on strided batches (maps cached per (k, m, pattern)) ---- */
/* Encode: parity fragments k..k+m-1 from data 0..k-1. */
int ecamd_rs_encode(int k, int m, void *base, int64_t stripe_stride, int64_t frag_stride,
                    int64_t blocksize, int nstripes, void *stream);
/* Decode: rebuild every fragment in the -1 terminated `missing` list in place (data, and parity
 * if rebuild_parity) from the first k available, as liberasurecode_rs_vand_decode does. */
int ecamd_rs_decode(int k, int m, const int *missing, int rebuild_parity, void *base,
                    int64_t stripe_stride, int64_t frag_stride, int64_t blocksize, int nstripes,
                    void *stream);
/* Heterogeneous batch decode: stripe s has its own -1 terminated erasure list at
 * missing + s*missing_stride (at most missing_stride entries).  Stripes are grouped by erasure
 * set; each group is one launch over a device stripe list (a pointer table when k > 20 or a
 * stripe spans 2 GiB), so a batch of stripes that lost different fragments costs one launch per
 * distinct pattern, not per stripe. */
int ecamd_rs_decode_multi(int k, int m, const int *missing, int missing_stride,
                          int rebuild_parity, void *base, int64_t stripe_stride,
                          int64_t frag_stride, int64_t blocksize, int nstripes, void *stream);
/* Fragment placement across GPUs: fragment f of every stripe (frag_len bytes at
 * d_src + s*stripe_stride + f*frag_stride on the current device) goes to d_dst[f] +
 * s*dst_stride[f] on device dst_dev[f]: one strided DMA per fragment, over xGMI when dst_dev[f]
 * is a peer (peer access is enabled on first use).  Copies to different peers run at once on
 * per-destination copy lanes forked from and joined back into `stream`; every destination is
 * checked before anything is queued.  Asynchronous on `stream`. */
int ecamd_scatter_fragments(const void *d_src, int64_t stripe_stride, int64_t frag_stride,
                            int64_t frag_len, int nfrags, int nstripes, const int *dst_dev,
                            void *const *d_dst, const int64_t *dst_stride, void *stream);
/* The rs_* calls above cache one prepared map (device coefficient tables) per (device, k, m,
 * erasure pattern, destination), least recently used first out once the tables exceed `limit`
 * bytes: entries and bytes currently held. */
int ecamd_map_cache_stats(int64_t *entries, int64_t *bytes, int64_t *limit);
/* Reconstruct one destination, as liberasurecode_rs_vand_reconstruct does. */
int ecamd_rs_reconstruct(int k, int m, const int *missing, int dest, void *base,
                         int64_t stripe_stride, int64_t frag_stride, int64_t blocksize,
                         int nstripes, void *stream);

/* ---- flat_xor_hd on strided batches: the reference's xor_code_encode,
 * xor_hd_decode (decode_parity as its argument) and xor_reconstruct_one
 * (src/builtin/xor_codes/xor_code.c:180-314, xor_hd_code.c:574-662) replayed exactly per erasure
 * list, missing slots read as zero (the frontend's zero-filled buffers); (k, m, hd) one of the
 * codes init_xor_hd_code accepts.  encode overwrites the parity slots (the reference accumulates
 * into the zeroed parity the frontend allocates: the same bytes).  decode_multi groups stripes by
 * identical erasure lists and runs one stripe-list launch per group.  ECAMD_EINVAL for patterns
 * the code cannot recover. */
int ecamd_xor_encode(int k, int m, int hd, void *base, int64_t stripe_stride, int64_t frag_stride,
                     int64_t blocksize, int nstripes, void *stream);
int ecamd_xor_decode(int k, int m, int hd, const int *missing, int decode_parity, void *base,
                     int64_t stripe_stride, int64_t frag_stride, int64_t blocksize, int nstripes,
                     void *stream);
int ecamd_xor_reconstruct(int k, int m, int hd, const int *missing, int dest, void *base,
                          int64_t stripe_stride, int64_t frag_stride, int64_t blocksize, int nstripes,
                          void *stream);
int ecamd_xor_decode_multi(int k, int m, int hd, const int *missing, int missing_stride,
                           int decode_parity, void *base, int64_t stripe_stride, int64_t frag_stride,
                           int64_t blocksize, int nstripes, void *stream);

/* ---- synchronous host-buffer execution (used by the per-call drop-in ABIs) ----
 * Pooled pinned staging + two streams, chunked so host copies overlap PCIe and the kernel.
 * Calls are spread round-robin over the visible devices (or ECAMD_PERCALL_DEVICES, see
 * ecamd_percall_device_plan in ecamd_host.h), each with its own staging pool; the caller's
 * current device is restored on return.
 * ecamd_host_map_apply: out[r] = sum_j coeff[r*K+j] * in[j] over GF(2^16).
 * ecamd_host_xor_apply: out[r] = XOR of bufs[b] for bits b of sources[r] (nbuf <= 64, at most 32
 * distinct buffers referenced); outputs may alias bufs, every output sees the original inputs. */
int ecamd_host_map_apply(const int *coeff, int R, int K, const void *const *in, void *const *out,
                         int64_t blocksize);
int ecamd_host_xor_apply(const uint64_t *sources, int R, int nbuf, const void *const *bufs,
                         void *const *out, int64_t blocksize);

/* Per-call checksum handoff (used by liberasurecode.so.1 around encode / reconstruct): while armed
 * on the calling thread, the two calls above also compute the CRC32 (zlib, or the legacy
 * liberasurecode_crc32_alt when legacy != 0) of every input and output fragment on the GPU while
 * the bytes are resident; lookup returns 0 and the CRC for a (pointer, length) seen since arm. */
int ecamd_percall_crc_arm(int legacy);
int ecamd_percall_crc_lookup(const void *ptr, int64_t len, uint32_t *crc);
void ecamd_percall_crc_disarm(void);
/* Per-call execution status: the first failure (staging allocation, copy, launch) of the two
 * synchronous calls above on the calling thread since ecamd_percall_reset(), 0 if none.  The
 * reference codec cannot fail mid-call and its shims discard the codec's return code
 * (src/backends/rs_vand/liberasurecode_rs_vand.c:86-90); liberasurecode.so.1 reads this around
 * each codec call and fails the call (-EIO) instead of stamping unwritten fragments. */
void ecamd_percall_reset(void);
int ecamd_percall_status(void);
/* Per-call input tees (used by liberasurecode.so.1 around encode and decode): while armed on the
 * calling thread, the synchronous calls above pack input `key[i]` -- when it is one of their input
 * pointers -- by reading bytes [0, len[i]) from src[i] (the rest from key[i]) and writing them to
 * dst2[i] as well, so a host copy the frontend would make anyway (object -> data payloads on
 * encode, surviving data payloads -> decoded object on decode) rides on the staging pack instead of
 * reading its source a second time.  disarm writes into done[i] (may be NULL) how many of the
 * len[i] bytes were delivered to dst2[i] -- all of them or none -- and forgets the tees; the
 * caller copies whatever was not delivered.  n <= 64.  0, or ECAMD_EINVAL. */
int ecamd_percall_tee_arm(int n, const void *const *key, const void *const *src, void *const *dst2,
                          const int64_t *len);
void ecamd_percall_tee_disarm(int64_t *done);
/* Fault injection for tests: site "staging" makes the next `count` staging acquisitions of the
 * synchronous host-buffer calls fail with ECAMD_ENOMEM (0 disarms). */
int ecamd_fault_inject(const char *site, int count);

/* ---- on-device framing: the wire format of liberasurecode_encode, in HBM ----
 * backend 6 = liberasurecode_rs_vand, 3 = flat_xor_hd (hd used only there); checksum is the
 * ec_checksum_type_t of the instance (1 none, 2 CRC32; anything else is stored, not computed, as the
 * reference does).  Object s lives at d_obj + s*obj_stride (obj_size bytes, all stripes the same
 * size); fragment f of stripe s at d_frags + s*stripe_stride + f*frag_stride: the 80-byte
 * fragment_header_t followed by the payload.  frag_stride >= 80 + blocksize rounded up to 16, all
 * fragment addresses 16-byte aligned.  For full HBM rate put every payload on a 128-byte line:
 * frag_stride a multiple of 128 and d_frags = (128-aligned buffer) + 48, so each header sits at
 * offset 48 of its slot (packed fragments run 13-19% slower; DESIGN.md §4 "Payload alignment").
 * LIBERASURECODE_WRITE_LEGACY_CRC selects the legacy checksum exactly as in the reference.
 * Asynchronous on `stream`. */

/* blocksize = get_aligned_data_size(obj_size) / k; fragment_len = 80 + blocksize. */
int ecamd_frame_geometry(int backend, int k, int m, int hd, uint64_t obj_size, int64_t *blocksize,
                         int64_t *fragment_len);
/* liberasurecode_encode (src/erasurecode.c:383-477) for nstripes objects at once: split + pad,
 * parity, payload CRC32 and headers; fragments byte-identical to the reference's. */
int ecamd_frame_encode(int backend, int k, int m, int hd, int checksum, const void *d_obj,
                       int64_t obj_stride, uint64_t obj_size, void *d_frags, int64_t stripe_stride,
                       int64_t frag_stride, int nstripes, void *stream);
/* liberasurecode_decode (src/erasurecode.c:523-734) with fragments already in their index slots:
 * write the objects, rebuilding the missing (-1 terminated) data.  Surviving fragments are not
 * modified; the slots of missing ones may be overwritten (with their rebuilt payload). */
int ecamd_frame_decode(int backend, int k, int m, int hd, const int *missing, void *d_frags,
                       int64_t stripe_stride, int64_t frag_stride, int nstripes, void *d_obj,
                       int64_t obj_stride, uint64_t obj_size, void *stream);
/* liberasurecode_reconstruct_fragment (src/erasurecode.c:748-949): rebuild fragment `dest` of
 * every stripe in its slot, header and checksum included. */
int ecamd_frame_reconstruct(int backend, int k, int m, int hd, int checksum, const int *missing,
                            int dest, void *d_frags, int64_t stripe_stride, int64_t frag_stride,
                            uint64_t obj_size, int nstripes, void *stream);
/* Header / checksum audit of nfrag fragments per stripe: d_status[s*nfrag+f] bit 0 bad magic, 1 bad
 * metadata checksum (neither zlib nor legacy), 2 idx != f, 3 size != blocksize, 4 payload CRC32
 * mismatch (when the header says CRC32; `legacy` picks the machine).  d_crc (optional) receives the
 * computed payload CRCs. */
int ecamd_frame_verify(int nfrag, int64_t blocksize, int legacy, const void *d_frags,
                       int64_t stripe_stride, int64_t frag_stride, int nstripes, uint32_t *d_status,
                       uint32_t *d_crc, void *stream);
/* zlib crc32(0, buf, len) (legacy = 0) or liberasurecode_crc32_alt(0, buf, len) (legacy = 1) of
 * every buffer d_base + s*stripe_stride + f*frag_stride, f < nfrag: d_crc[s*nfrag + f]. */
int ecamd_crc32(int legacy, const void *d_base, int64_t stripe_stride, int64_t frag_stride,
                int nfrag, int64_t len, int nstripes, uint32_t *d_crc, void *stream);

/* ---- synthetic data: splitmix64 stream per fragment, seed = seed_base ^ (s<<8) ^ f ---- */
int ecamd_fill_splitmix(void *base, int64_t stripe_stride, int64_t frag_stride, int nfrags,
                        int64_t blocksize, int nstripes, int stripe0, uint64_t seed_base,
                        void *stream);

/* ---- device memory helpers for C / ctypes callers ---- */
int ecamd_malloc(void **d_ptr, int64_t bytes);
/* Device memory the host may also write directly (the same address, through the PCIe BAR), uncached on the
 * GPU side; ECAMD_EINVAL where the platform does not map device memory for the host.  The per-call path
 * packs small calls' inputs there instead of staging them through a DMA. */
int ecamd_malloc_host_writable(void **d_ptr, int64_t bytes);
int ecamd_free(void *d_ptr);
int ecamd_memcpy_h2d(void *d_dst, const void *h_src, int64_t bytes);
int ecamd_memcpy_d2h(void *h_dst, const void *d_src, int64_t bytes);
int ecamd_memset(void *d_ptr, int value, int64_t bytes); /* synchronous: complete on return */
/* kind: 0 host->device, 1 device->host, 2 device->device; asynchronous on stream */
int ecamd_memcpy_async(void *dst, const void *src, int64_t bytes, int kind, void *stream);
int ecamd_host_alloc(void **h_ptr, int64_t bytes); /* pinned host memory */
int ecamd_host_free(void *h_ptr);
int ecamd_synchronize(void);
int ecamd_stream_create(void **stream);
/* Also releases the library's per-stream context of that stream (side stream, scratch). */
int ecamd_stream_destroy(void *stream);
/* hipStreamDestroy on the library's own HIP runtime WITHOUT releasing its context -- what a caller that
 * destroys a stream behind the library's back does (tests: the contexts stay bounded anyway). */
int ecamd_stream_destroy_unmanaged(void *stream);
int ecamd_stream_synchronize(void *stream);
/* 0 when all work on stream is complete, 1 while some is pending, ECAMD_EHIP on error. */
int ecamd_stream_query(void *stream);
/* Per-(device, stream) contexts the framed calls hold (side stream + events + CRC scratch): bounded --
 * released by ecamd_stream_destroy, and idle ones of other streams past a cap of 16 (diagnostics). */
int ecamd_stream_contexts(void);
/* HIP events for timing work on a stream (elapsed_ms waits for `stop`). */
int ecamd_event_create(void **ev);
int ecamd_event_destroy(void *ev);
int ecamd_event_record(void *ev, void *stream);
int ecamd_event_elapsed_ms(void *start, void *stop, float *ms);

#ifdef __cplusplus
}
#endif
#endif
