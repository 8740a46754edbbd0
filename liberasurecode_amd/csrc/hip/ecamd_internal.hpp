// ecamd_internal.hpp -- helpers ecamd_device.hip shares with the other launch files.
#pragma once
#include <vector>
#include <stddef.h>
#include <stdint.h>

#include <mutex>

namespace ecamd {

// Asynchronous upload of a small host table (stripe list, pointer table) on `stream` through a
// ring of pinned slots per (device, stream); call end() after enqueuing the launches that read
// `dev` (ecamd_device.hip).
struct StagedSlot;
struct StagedRing;
struct StagedUpload {
    void* dev = nullptr;
    int begin(int device, void* stream, const void* src, size_t bytes);
    int end(void* stream);  // records the slot's event behind the launches and releases it
    ~StagedUpload() { end(stream_); }

private:
    StagedRing* ring_ = nullptr;
    StagedSlot* slot_ = nullptr;
    void* stream_ = nullptr;
};

// Strided flat-XOR apply (ecamd_xor_apply_strided) over the stripes listed in the device array
// d_list (logical stripe i is stripe d_list[i] of the layout); ECAMD_EINVAL when the stream
// kernel cannot take the shape.
int xor_apply_list(const uint32_t* masks, int R, int K, void* base, int64_t stripe_stride,
                   const int64_t* in_off, const int64_t* out_off, int64_t blocksize, int nstripes,
                   const int32_t* d_list, void* stream);

int dev_ensure(int* dev_out);                       // 0, or ECAMD_ENODEV / ECAMD_EHIP
int dev_cu_count(int dev);
int dev_fail(int code, const char* fmt, ...);       // sets ecamd_last_error(), returns code
int dev_tune(const char* key);                      // current value of an ecamd_tune() knob

// rs_vand encode whose k data inputs are read from objects (input j of stripe s at
// obj + s*obj_stride + j*bs) and copied into payload j while the parity is computed
// (payload f of stripe s at payload0 + s*stripe_stride + f*frag_stride).  Objects of obj_size
// bytes (< 0: k*bs) are zero-padded past their end (prepare_fragments_for_encode).  16-byte aligned
// object base / stride and payloads; bs even (the object side may be read unaligned).  from > 0 (a
// multiple of 16): only bytes [from, bs) of every payload (the rest of a partly fused encode); to > 0:
// only bytes [from, to).
// Side stream of (dev, stream) for work beside the caller's launches (knob frame_tail_fork):
// side_fork orders it after everything issued to `stream` so far, side_join orders `stream` after
// everything issued to the side stream since.
// The side stream and the scratch slots live in a per-(dev, stream) context (ecamd_device.hip),
// bounded: ecamd_stream_destroy releases a stream's, and idle ones are released past a small cap.
int side_fork(int dev, void* stream, void** side);
int side_join(int dev, void* stream);
// Device scratch of `words` 32-bit words in slot 0..kStreamScratchSlots-1 of (dev, stream); calls
// on one stream are ordered, so reuse is safe (slot 1 holds values that must outlive a CRC pass on
// the same stream, whose partials use slot 0).
// Slot 4: the small-launch fused CRC's counter and partials (ecamd_map_apply_strided_crc).  A slot is
// zeroed when it is (re)allocated.
constexpr int kStreamScratchSlots = 5;
constexpr int kSmallCrcScratchSlot = 4;
int stream_scratch(int dev, void* stream, int slot, size_t words, uint32_t** out);
// A framed call in progress on (dev, stream): its context is not released until the call has
// returned and its work on the stream has completed.
int stream_use_begin(int dev, void* stream);
void stream_use_end(int dev, void* stream);
struct StreamUse {
    int dev;
    void* stream;
    StreamUse(int d, void* s) : dev(d), stream(s) { (void)stream_use_begin(d, s); }
    ~StreamUse() { stream_use_end(dev, stream); }
    StreamUse(const StreamUse&) = delete;
    StreamUse& operator=(const StreamUse&) = delete;
};
void stream_forget(void* stream);
int stream_contexts();

int rs_encode_copy(int k, int m, const void* obj, int64_t obj_stride, void* payload0,
                   int64_t stripe_stride, int64_t frag_stride, int64_t bs, int nstripes,
                   void* stream, int64_t obj_size = -1, int64_t from = 0, int64_t to = -1);

// Framed flat-XOR decode with data lost, straight into the objects: data output r (outputs[r] < k) =
// XOR of the inputs (fragment indices) whose coeff[r*K + col] is 1; every data input is copied into
// its object chunk by the same launch (the RS decode-join with a 0 / 1 matrix).
int xor_decode_join(int k, const std::vector<int>& inputs, const std::vector<int>& outputs,
                    const std::vector<int>& coeff, const void* payload0, int64_t stripe_stride, int64_t frag_stride,
                    void* obj, int64_t obj_stride, int64_t bs, int nstripes, void* stream, int64_t obj_size);

// The same crc variant for a flat-XOR code (parity r = XOR of the data chunks in masks[r], run as a
// 0 / 1 coefficient matrix through the bitsliced generator).
int xor_encode_copy_crc_bs(const uint32_t* masks, int k, int m, const void* obj, int64_t obj_stride, void* payload0,
                           int64_t stripe_stride, int64_t frag_stride, int64_t bs, int nstripes,
                           const uint32_t* d_img, uint32_t* d_partial, int q, void* stream, int crc_pos = 1,
                           int64_t cover = -1);

// Framed flat-XOR encode, copy-through: bytes [0, cover) of every payload (cover a multiple of 4096,
// every object chunk at least that long) from objects of obj_stride bytes whose chunk j starts at j*bs
// (unaligned loads when bs % 16 != 0): the data payloads are written as the chunks stream through the
// XOR kernel, parity r = XOR of the chunks in masks[r].  ECAMD_EINVAL, nothing launched, when it
// does not apply.
int xor_encode_copy(const uint32_t* masks, int k, int m, const void* obj, int64_t obj_stride, void* payload0,
                    int64_t stripe_stride, int64_t frag_stride, int64_t bs, int64_t cover, int nstripes, void* stream);

// rs_vand decode straight into objects: the missing data fragments (at least one, -1 terminated
// `missing`) are computed into their object positions (j*bs) and the available data inputs are
// copied there by the same launch (fragments_to_string without a separate join pass).
// Objects of obj_size bytes (< 0: k*bs): nothing is written past an object's end.
int rs_decode_join(int k, int m, const int* missing, const void* payload0, int64_t stripe_stride,
                   int64_t frag_stride, void* obj, int64_t obj_stride, int64_t bs, int nstripes,
                   void* stream, int64_t obj_size = -1);

// rs_encode_copy with the payload CRC32s folded into the same launch (ecamd_frame_fused.hip):
// d_img = build_fused_crc_image(machine, 8192) in device memory; r0 of range r (q ranges of
// bs/q bytes) of payload f of stripe s -> d_partial[(s*(k+m) + f)*q + r].  ECAMD_EINVAL, with
// nothing launched, when the shape does not fit (bs % 8192, q must divide bs/8192, one map pass).
int rs_encode_copy_crc(int k, int m, const void* obj, int64_t obj_stride, void* payload0,
                       int64_t stripe_stride, int64_t frag_stride, int64_t bs, int nstripes,
                       const uint32_t* d_img, uint32_t* d_partial, int q, void* stream, int mb = 1,
                       bool nib = false);
size_t fused_crc_lds(int k, int m, int mb, bool nib = false);  // LDS bytes of the fused framed encode
// The same on the bitsliced kernel's crc variant (up to 4 outputs, 16 KiB tiles, q ranges of
// 16 KiB tiles per payload; d_img: the CRC image built for a 4096-byte chain step).  ECAMD_EINVAL,
// nothing launched, when it does not apply or the kernel is not compiled yet.
int rs_encode_copy_crc_bs(int k, int m, const void* obj, int64_t obj_stride, void* payload0,
                          int64_t stripe_stride, int64_t frag_stride, int64_t bs, int nstripes,
                          const uint32_t* d_img, uint32_t* d_partial, int q, void* stream, int crc_pos = 1,
                          int64_t cover = -1);  // cover: the first `cover` bytes of each payload only
// Build time (no GPU): the code object the CRC32 framed encode's crc variant (crc_pos flags as
// rs_encode_copy_crc_bs takes them) will ask for, for the rs_vand code (k, m) (masks null) or the
// flat-XOR code with parity masks `masks`, into `dir` (ecamd_frame_prebuild).  1: present, 0: this
// form takes no bitsliced kernel, < 0: failed.
int crc_encode_prebuild(int k, int m, const uint32_t* masks, int crc_pos, const char* arch, const char* dir);
// fused image words with byte tables for the first mb dwords of a piece, nibble tables after
constexpr int crc_fused_words(int mb = 1) { return mb * 1024 + (4 - mb) * 128 + 8 * 128; }

}  // namespace ecamd
