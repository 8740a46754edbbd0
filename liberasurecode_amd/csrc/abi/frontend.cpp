// frontend.cpp -- liberasurecode.so.1 (boundary B2): the liberasurecode C API over the MI355X
// codec libraries of this repo.
//
// Restates the reference frontend (src/erasurecode.c, erasurecode_helpers.c,
// erasurecode_preprocessing.c, erasurecode_postprocessing.c): instance registry under one
// reader/writer lock, 80-byte fragment framing with zlib CRC-32 (and the legacy sign-extending
// variant), the systematic decode fast path, and the two built-in backend shims:
//   flat_xor_hd             -> libXorcode.so.1            (src/backends/xor/flat_xor_hd.c)
//   liberasurecode_rs_vand  -> liberasurecode_rs_vand.so.1 (src/backends/rs_vand/liberasurecode_rs_vand.c)
// Both libraries are the GPU drop-ins built next to this one (RUNPATH $ORIGIN), so every region
// operation of encode / decode / reconstruct runs on the GPU.
#include <dlfcn.h>
#include <pthread.h>
#include <syslog.h>
#include <zlib.h>

#include <algorithm>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <unordered_map>
#include <vector>

#include "erasurecode.h"
#include "erasurecode_backend.h"
#include "xor_code.h"

#define LOGE(...) syslog(LOG_ERR, __VA_ARGS__)
#define LOGW(...) syslog(LOG_WARNING, __VA_ARGS__)

namespace {

constexpr size_t kHdr = sizeof(fragment_header_t);
static_assert(sizeof(fragment_metadata_t) == 59, "packed metadata");
static_assert(sizeof(fragment_header_t) == 80, "packed header");

uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

fragment_header_t* hdr(char* buf) { return reinterpret_cast<fragment_header_t*>(buf); }
bool has_magic(char* buf) { return hdr(buf)->magic == LIBERASURECODE_FRAG_HEADER_MAGIC; }

bool env_legacy_crc()
{
    const char* f = getenv("LIBERASURECODE_WRITE_LEGACY_CRC");
    return f && !(f[0] == '\0' || (f[0] == '0' && f[1] == '\0'));
}

uint32_t zcrc(const void* p, size_t n)
{
    return static_cast<uint32_t>(crc32(0, static_cast<const Bytef*>(p), static_cast<uInt>(n)));
}

// ---------------------------------------------------------------- fragment buffers ----

// Recycled large buffers.  Fragments and decoded objects are allocated here and come back through
// liberasurecode_encode_cleanup / _decode_cleanup (and the frontend's own temporaries): a buffer
// of 64 KiB or more is kept (up to ECAMD_FRONTEND_POOL_MIB in total, default 256, 0 = off) and
// handed out again to a request of between half its size and its size, so the next call writes
// into pages that are already mapped instead of faulting fresh ones in (a copy into fresh pages
// runs at ~40% of a copy into mapped ones).  Every buffer is an ordinary posix_memalign block: a
// caller that free()s one directly just returns it to libc (the reference's own tests do,
// test/liberasurecode_test.c:1110); the address's record is refreshed by every later allocation.
class BufferPool {
public:
    void* get(size_t n)
    {
        if (n >= kMin && limit() > 0) {
            std::lock_guard<std::mutex> lk(mu_);
            size_t best = free_.size();
            for (size_t i = 0; i < free_.size(); i++)
                if (free_[i].cap >= n && free_[i].cap / 2 <= n &&
                    (best == free_.size() || free_[i].cap < free_[best].cap))
                    best = i;
            if (best < free_.size()) {
                void* p = free_[best].ptr;
                held_ -= free_[best].cap;
                free_[best] = free_.back();
                free_.pop_back();
                return p;
            }
        }
        void* p = nullptr;
        if (posix_memalign(&p, 16, n ? n : 1) != 0) return nullptr;
        // Every fresh block refreshes its address's record: a pooled block the caller free()d
        // directly may come back from libc at the same address for a smaller request, and must
        // then never be recycled as the large block it once was.
        if (limit() > 0) {
            std::lock_guard<std::mutex> lk(mu_);
            if (n >= kMin) {
                if (caps_.size() > 65536) caps_.clear();  // callers free()d many directly: forget them
                caps_[p] = n;
            } else if (!caps_.empty()) {
                caps_.erase(p);
            }
        }
        return p;
    }
    void put(void* p)
    {
        if (!p) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = caps_.find(p);
            if (it != caps_.end()) {
                const size_t cap = it->second;
                if (held_ + cap <= limit() && free_.size() < 256) {
                    free_.push_back({p, cap});
                    held_ += cap;
                    return;
                }
                caps_.erase(it);
            }
        }
        std::free(p);
    }

private:
    static constexpr size_t kMin = 64 << 10;
    static size_t limit()
    {
        static const size_t bytes = [] {
            const char* s = getenv("ECAMD_FRONTEND_POOL_MIB");
            const long v = s && *s ? std::atol(s) : 256;
            return v > 0 ? static_cast<size_t>(v) << 20 : size_t(0);
        }();
        return bytes;
    }
    struct Free {
        void* ptr;
        size_t cap;
    };
    std::mutex mu_;
    std::vector<Free> free_;
    std::unordered_map<void*, size_t> caps_;  // every pooled-size block handed out, by address
    size_t held_ = 0;
};

BufferPool& pool()
{
    static BufferPool* p = new BufferPool();  // outlives every caller's static destructors
    return *p;
}

void* buf_alloc(size_t n) { return pool().get(n); }
void buf_free(void* p) { pool().put(p); }

// 16-byte aligned, zeroed (get_aligned_buffer16, erasurecode_helpers.c:61-76)
void* aligned_zero(size_t n)
{
    void* p = buf_alloc(n);
    if (!p) return nullptr;
    std::memset(p, 0, n);
    return p;
}

// header + payload, zeroed, magic set (alloc_fragment_buffer, :124-138).  zero_payload = false
// zeroes the header only: for buffers whose payload the codec overwrites in full.
char* new_fragment(int payload, bool zero_payload = true)
{
    const size_t n = static_cast<size_t>(payload) + kHdr;
    char* f = nullptr;
    if (zero_payload) {
        f = static_cast<char*>(aligned_zero(n));
    } else if ((f = static_cast<char*>(buf_alloc(n)))) {
        std::memset(f, 0, kHdr);
    }
    if (f) hdr(f)->magic = LIBERASURECODE_FRAG_HEADER_MAGIC;
    return f;
}

// ECAMD_FRONTEND_ZERO_ALL=1 zeroes every buffer in full as the reference does, for A/B runs of
// the host passes skipped below (tools/e2e_bench.py); the bytes returned are the same either way.
bool zero_all()
{
    static const bool on = [] {
        const char* f = getenv("ECAMD_FRONTEND_ZERO_ALL");
        return f && f[0] == '1';
    }();
    return on;
}

// Zero [0, n) of p except [lo, hi), the part the caller fills next.
void zero_outside(char* p, size_t n, size_t lo, size_t hi)
{
    if (lo > 0) std::memset(p, 0, lo);
    if (hi < n) std::memset(p + hi, 0, n - hi);
}

int frag_idx(char* f) { return has_magic(f) ? static_cast<int>(hdr(f)->meta.idx) : -1; }
int frag_size(char* f) { return has_magic(f) ? static_cast<int>(hdr(f)->meta.size) : -1; }
int frag_orig_size(char* f) { return has_magic(f) ? static_cast<int>(hdr(f)->meta.orig_data_size) : -1; }
char* payload(char* f) { return f + kHdr; }

// ---------------------------------------------------------------- registry ----

pthread_rwlock_t g_lock = PTHREAD_RWLOCK_INITIALIZER;
ec_backend* g_instances = nullptr;  // singly linked through link.sle_next
int g_next_desc = 0;

struct ReadLock {
    int rc;
    ReadLock() : rc(pthread_rwlock_rdlock(&g_lock)) {}
    ~ReadLock()
    {
        if (rc == 0) pthread_rwlock_unlock(&g_lock);
    }
};

ec_backend* find(int desc)
{
    for (ec_backend* b = g_instances; b; b = b->link.sle_next)
        if (b->idesc == desc) return b;
    return nullptr;
}

int new_desc()
{
    for (;;) {
        if (++g_next_desc <= 0) g_next_desc = 1;
        if (!find(g_next_desc)) return g_next_desc;
    }
}

size_t zero_metadata(void*, int) { return 0; }
size_t zero_offset(void*, int) { return 0; }

// ------------------------------------------------ codec hooks of this repo's libraries ----

// Resolved with dlsym through the codec library's dependencies (libecamd.so, include/ecamd.h);
// a foreign codec library (e.g. the reference's own) has none of them and gets the reference
// behaviour: host zlib checksums, codec return codes discarded as the reference shims do.
struct CodecHooks {
    int (*crc_arm)(int) = nullptr;                               // ecamd_percall_crc_*
    int (*crc_lookup)(const void*, int64_t, uint32_t*) = nullptr;
    void (*crc_disarm)(void) = nullptr;
    void (*exec_reset)(void) = nullptr;                          // ecamd_percall_reset / _status
    int (*exec_status)(void) = nullptr;
    int (*copy)(int, void* const*, const void* const*, const int64_t*) = nullptr;  // ecamd_host_copy
    int (*tee_arm)(int, const void* const*, const void* const*, void* const*, const int64_t*) = nullptr;
    void (*tee_disarm)(int64_t*) = nullptr;  // ecamd_percall_tee_*
    bool crc() const { return crc_arm && crc_lookup && crc_disarm; }
    bool tee() const { return tee_arm && tee_disarm; }
    bool ours() const { return exec_reset && exec_status; }
};

CodecHooks resolve_hooks(void* so)
{
    CodecHooks h;
    if (!so) return h;
    h.crc_arm = reinterpret_cast<int (*)(int)>(dlsym(so, "ecamd_percall_crc_arm"));
    h.crc_lookup = reinterpret_cast<int (*)(const void*, int64_t, uint32_t*)>(
        dlsym(so, "ecamd_percall_crc_lookup"));
    h.crc_disarm = reinterpret_cast<void (*)(void)>(dlsym(so, "ecamd_percall_crc_disarm"));
    h.exec_reset = reinterpret_cast<void (*)(void)>(dlsym(so, "ecamd_percall_reset"));
    h.exec_status = reinterpret_cast<int (*)(void)>(dlsym(so, "ecamd_percall_status"));
    h.copy = reinterpret_cast<int (*)(int, void* const*, const void* const*, const int64_t*)>(
        dlsym(so, "ecamd_host_copy"));
    h.tee_arm = reinterpret_cast<int (*)(int, const void* const*, const void* const*, void* const*,
                                         const int64_t*)>(dlsym(so, "ecamd_percall_tee_arm"));
    h.tee_disarm = reinterpret_cast<void (*)(int64_t*)>(dlsym(so, "ecamd_percall_tee_disarm"));
    dlerror();
    return h;
}

// Every backend_desc this frontend creates starts with its hooks, resolved once at init and
// living exactly as long as the instance (no shared cache to reallocate or go stale on dlclose).
struct ShimBase {
    CodecHooks hooks;
};

const CodecHooks& hooks_of(ec_backend* be) { return static_cast<ShimBase*>(be->desc.backend_desc)->hooks; }

// Brackets one codec call: true when this repo's codec failed to EXECUTE it (staging, copy,
// launch).  The reference shims discard codec return codes (flat_xor_hd.c:65-72,
// liberasurecode_rs_vand.c:86-90) because a CPU codec cannot fail mid-call; a GPU codec can, and
// a failed call must not come back as success with unwritten fragments.
struct ExecCheck {
    const CodecHooks& h;
    explicit ExecCheck(const CodecHooks& hooks) : h(hooks)
    {
        if (h.ours()) h.exec_reset();
    }
    bool failed() const { return h.ours() && h.exec_status() != 0; }
};

// ------------------------------------------------ flat_xor_hd shim (flat_xor_hd.c:65-226) ----

struct XorDesc : ShimBase {
    xor_code_t* code = nullptr;
};

int fx_encode(void* d, char** data, char** parity, int bs)
{
    auto* x = static_cast<XorDesc*>(d);
    ExecCheck ex(x->hooks);
    x->code->encode(x->code, data, parity, bs);
    return ex.failed() ? -EIO : 0;
}

int fx_decode(void* d, char** data, char** parity, int* missing, int bs)
{
    auto* x = static_cast<XorDesc*>(d);
    ExecCheck ex(x->hooks);
    const int rc = x->code->decode(x->code, data, parity, missing, bs, 1);
    return ex.failed() ? -EIO : rc;
}

int fx_reconstruct(void* d, char** data, char** parity, int* missing, int dest, int bs)
{
    auto* x = static_cast<XorDesc*>(d);
    ExecCheck ex(x->hooks);
    const int rc = xor_reconstruct_one(x->code, data, parity, missing, dest, bs);
    return ex.failed() ? -EIO : rc;
}

int fx_needed(void* d, int* missing, int* exclude, int* needed)
{
    xor_code_t* c = static_cast<XorDesc*>(d)->code;
    c->fragments_needed(c, missing, exclude, needed);
    return 0;  // the reference shim ignores the library's return code
}

int fx_check_reconstruct(void* d, int* missing, int)
{
    const xor_code_t* c = static_cast<XorDesc*>(d)->code;
    bool seen[EC_MAX_FRAGMENTS] = {};
    for (int i = 0; missing[i] >= 0; i++)
        if (missing[i] < EC_MAX_FRAGMENTS) seen[missing[i]] = true;
    int avail = c->k + c->m;
    for (bool s : seen) avail -= s ? 1 : 0;
    const int k = c->k, m = c->m;
    if (c->hd == 3) {
        if (avail < 2) return -EINSUFFFRAGS;
        if (m == 5 && ((k == 8 || k == 9) && avail < 3)) return -EINSUFFFRAGS;
        if (m == 5 && k == 10 && avail < 4) return -EINSUFFFRAGS;
        if (m == 6 && k >= 9 && k <= 11 && avail < 3) return -EINSUFFFRAGS;
        if (m == 6 && k >= 12 && k <= 14 && avail < 4) return -EINSUFFFRAGS;
        if (m == 6 && k == 15 && avail < 5) return -EINSUFFFRAGS;
    } else {
        if (avail < 3) return -EINSUFFFRAGS;
        if (m == 5 && (k == 7 || k == 8) && avail < 4) return -EINSUFFFRAGS;
        if (m == 5 && k + m - avail > 9) return -EINSUFFFRAGS;
        if (m == 6 && avail < (k + m) / 2 - 3) return -EINSUFFFRAGS;
    }
    return 0;
}

int fx_element_size(void*) { return 32; }

void* fx_init(ec_backend_args* args, void* so)
{
    args->uargs.w = 32;
    xor_code_t* c = init_xor_hd_code(args->uargs.k, args->uargs.m, args->uargs.hd);
    if (!c) return nullptr;
    auto* d = new (std::nothrow) XorDesc();
    if (!d) {
        std::free(c);
        return nullptr;
    }
    d->hooks = resolve_hooks(so);
    d->code = c;
    return d;
}

int fx_exit(void* d)
{
    auto* x = static_cast<XorDesc*>(d);
    std::free(x->code);
    delete x;
    return 0;
}

bool fx_compatible(uint32_t v) { return v == _VERSION(1, 0, 0); }

ec_backend_op_stubs g_xor_ops = {fx_init, fx_exit, true, fx_encode, fx_decode, fx_needed,
                                 fx_reconstruct, fx_element_size, fx_compatible, zero_metadata,
                                 zero_offset, fx_check_reconstruct};

// ---------------------------------- liberasurecode_rs_vand shim (rs_vand.c:82-311) ----

struct RsDesc : ShimBase {
    void (*init)(int, int) = nullptr;
    void (*deinit)(void) = nullptr;
    void (*free_matrix)(int*) = nullptr;
    int* (*make_matrix)(int, int) = nullptr;
    int (*encode)(int*, char**, char**, int, int, int) = nullptr;
    int (*decode)(int*, char**, char**, int, int, int*, int, int) = nullptr;
    int (*reconstruct)(int*, char**, char**, int, int, int*, int, int) = nullptr;
    int* matrix = nullptr;
    int k = 0, m = 0, w = 0;
};

// The codec refused the call (more than m missing, e.g. k fragments with duplicate indices):
// liberasurecode_rs_vand.c:444-447 / 502-505 return -1 before writing anything, so the missing
// slots keep the zeros the reference frontend allocated them with.  This frontend skips that
// zeroing in front of its own codec (prepare_decode, realign = false), so it zeroes them here.
void zero_missing(char** data, char** parity, int k, const int* missing, int bs)
{
    for (int i = 0; missing[i] >= 0; i++)
        std::memset(missing[i] < k ? data[missing[i]] : parity[missing[i] - k], 0,
                    static_cast<size_t>(bs));
}

int rs_encode(void* d, char** data, char** parity, int bs)
{
    auto* r = static_cast<RsDesc*>(d);
    ExecCheck ex(r->hooks);
    r->encode(r->matrix, data, parity, r->k, r->m, bs);
    return ex.failed() ? -EIO : 0;  // otherwise the reference shim discards the codec's rc
}

int rs_decode(void* d, char** data, char** parity, int* missing, int bs)
{
    auto* r = static_cast<RsDesc*>(d);
    ExecCheck ex(r->hooks);
    const int rc = r->decode(r->matrix, data, parity, r->k, r->m, missing, bs, 1);
    if (ex.failed()) return -EIO;
    if (rc != 0) zero_missing(data, parity, r->k, missing, bs);
    return 0;
}

int rs_reconstruct(void* d, char** data, char** parity, int* missing, int dest, int bs)
{
    auto* r = static_cast<RsDesc*>(d);
    ExecCheck ex(r->hooks);
    const int rc = r->reconstruct(r->matrix, data, parity, r->k, r->m, missing, dest, bs);
    if (ex.failed()) return -EIO;
    if (rc != 0) zero_missing(data, parity, r->k, missing, bs);
    return 0;
}

int rs_needed(void* d, int* missing, int* exclude, int* needed)
{
    auto* r = static_cast<RsDesc*>(d);
    bool gone[EC_MAX_FRAGMENTS] = {};
    for (int i = 0; exclude[i] >= 0; i++)
        if (exclude[i] < EC_MAX_FRAGMENTS) gone[exclude[i]] = true;
    for (int i = 0; missing[i] >= 0; i++)
        if (missing[i] < EC_MAX_FRAGMENTS) gone[missing[i]] = true;
    int j = 0;
    for (int i = 0; i < r->k + r->m; i++) {
        if (!gone[i]) needed[j++] = i;
        if (j == r->k) {
            needed[j] = -1;
            return 0;
        }
    }
    return -1;
}

int rs_element_size(void* d) { return static_cast<RsDesc*>(d)->w; }

template <typename F>
bool bind(void* so, const char* name, F& fn)
{
    fn = reinterpret_cast<F>(dlsym(so, name));
    return fn != nullptr;
}

void* rs_init(ec_backend_args* args, void* so)
{
    auto* r = new (std::nothrow) RsDesc();
    if (!r) return nullptr;
    r->hooks = resolve_hooks(so);
    r->k = args->uargs.k;
    r->m = args->uargs.m;
    args->uargs.w = r->w = 16;
    bool ok = r->k + r->m <= 65536 && bind(so, "init_liberasurecode_rs_vand", r->init) &&
              bind(so, "deinit_liberasurecode_rs_vand", r->deinit) &&
              bind(so, "make_systematic_matrix", r->make_matrix) &&
              bind(so, "free_systematic_matrix", r->free_matrix) &&
              bind(so, "liberasurecode_rs_vand_encode", r->encode) &&
              bind(so, "liberasurecode_rs_vand_decode", r->decode) &&
              bind(so, "liberasurecode_rs_vand_reconstruct", r->reconstruct);
    if (ok) {
        r->init(r->k, r->m);
        r->matrix = r->make_matrix(r->k, r->m);
        ok = r->matrix != nullptr;
    }
    if (!ok) {
        delete r;
        return nullptr;
    }
    return r;
}

int rs_exit(void* d)
{
    auto* r = static_cast<RsDesc*>(d);
    r->free_matrix(r->matrix);
    r->deinit();
    delete r;
    return 0;
}

bool rs_compatible(uint32_t v) { return v == _VERSION(1, 0, 0); }

ec_backend_op_stubs g_rs_ops = {rs_init, rs_exit, true, rs_encode, rs_decode, rs_needed,
                                rs_reconstruct, rs_element_size, rs_compatible, zero_metadata,
                                zero_offset, nullptr};

// ------------------------------------------------------------ backend table (:58-71) ----

struct TableEntry {
    ec_backend_id_t id;
    const char* name;
    const char* soname;
    ec_backend_op_stubs* ops;  // nullptr: no shim in this build (reported as not available)
};

#define SONAME(base, ver) base LIBERASURECODE_SO_SUFFIX ver
const TableEntry kBackends[EC_BACKENDS_MAX] = {
    {EC_BACKEND_NULL, "null", SONAME("libnullcode", ".so.1"), nullptr},
    {EC_BACKEND_JERASURE_RS_VAND, "jerasure_rs_vand", SONAME("libJerasure", ".so.2"), nullptr},
    {EC_BACKEND_JERASURE_RS_CAUCHY, "jerasure_rs_cauchy", SONAME("libJerasure", ".so.2"), nullptr},
    {EC_BACKEND_FLAT_XOR_HD, "flat_xor_hd", SONAME("libXorcode", ".so.1"), &g_xor_ops},
    {EC_BACKEND_ISA_L_RS_VAND, "isa_l_rs_vand", SONAME("libisal", ".so.2"), nullptr},
    {EC_BACKEND_SHSS, "shss", SONAME("libshss", ".so.1"), nullptr},
    {EC_BACKEND_LIBERASURECODE_RS_VAND, "liberasurecode_rs_vand",
     SONAME("liberasurecode_rs_vand", ".so.1"), &g_rs_ops},
    {EC_BACKEND_ISA_L_RS_CAUCHY, "isa_l_rs_cauchy", SONAME("libisal", ".so.2"), nullptr},
    {EC_BACKEND_LIBPHAZR, "libphazr", SONAME("libphazr", ".so.1"), nullptr},
    {EC_BACKEND_ISA_L_RS_VAND_INV, "isa_l_rs_vand_inv", SONAME("libisal", ".so.2"), nullptr},
    {EC_BACKEND_ISA_L_RS_LRC, "isa_l_rs_lrc", SONAME("libisal", ".so.2"), nullptr},
};
#undef SONAME

void fill_common(ec_backend_common& c, const TableEntry& e)
{
    std::memset(&c, 0, sizeof(c));
    c.id = e.id;
    std::snprintf(c.name, sizeof(c.name), "%s", e.name);
    c.soname = e.soname;
    std::snprintf(c.soversion, sizeof(c.soversion), "1.0");
    c.ops = e.ops;
    c.ec_backend_version = _VERSION(1, 0, 0);
}

void* open_backend(const TableEntry& e)
{
    if (!e.ops) return nullptr;
    return dlopen(e.soname, RTLD_LAZY | RTLD_LOCAL);
}

// ------------------------------------------------------------ framing ----

// get_aligned_data_size (erasurecode_helpers.c:186-208): round up to k * w/8, in int.
int aligned_size(ec_backend* be, int data_len)
{
    const int a = be->args.uargs.k * (be->args.uargs.w / 8);
    return ((data_len + a - 1) / a) * a;
}

// GPU checksum handoff (include/ecamd.h ecamd_percall_crc_*), armed for one encode / reconstruct
// call when the instance stores CRC32 checksums: the codec call then checksums the fragments on
// the GPU while they are resident.  With a foreign codec library zlib runs here.
thread_local const CodecHooks* t_hooks = nullptr;

struct CrcArm {
    const CodecHooks* h = nullptr;
    CrcArm(ec_backend* be, bool want)
    {
        if (want && hooks_of(be).crc()) {
            h = &hooks_of(be);  // lives in the instance, which the read lock keeps alive
            h->crc_arm(env_legacy_crc() ? 1 : 0);
            t_hooks = h;
        }
    }
    ~CrcArm()
    {
        if (h) {
            h->crc_disarm();
            t_hooks = nullptr;
        }
    }
};

void write_checksum(char* f, ec_checksum_type_t ct, int bs)
{
    fragment_header_t* h = hdr(f);
    h->meta.chksum_type = static_cast<uint8_t>(ct);
    h->meta.chksum_mismatch = 0;
    if (ct != CHKSUM_CRC32) return;
    uint32_t c = 0;
    if (t_hooks && t_hooks->crc_lookup(payload(f), bs, &c) == 0)
        h->meta.chksum[0] = c;
    else
        h->meta.chksum[0] = env_legacy_crc()
                                ? static_cast<uint32_t>(liberasurecode_crc32_alt(0, payload(f), bs))
                                : zcrc(payload(f), static_cast<size_t>(bs));
}

// add_fragment_metadata (erasurecode_postprocessing.c:37-69)
void stamp(ec_backend* be, char* f, int idx, uint64_t orig, int bs, ec_checksum_type_t ct,
           bool with_payload_crc)
{
    if (!has_magic(f)) return;
    fragment_header_t* h = hdr(f);
    h->libec_version = LIBERASURECODE_VERSION;
    h->meta.idx = static_cast<uint32_t>(idx);
    h->meta.orig_data_size = orig;
    h->meta.size = static_cast<uint32_t>(bs);
    h->meta.backend_id = static_cast<uint8_t>(be->common.id);
    h->meta.backend_version = be->common.ec_backend_version;
    h->meta.frag_backend_metadata_size =
        static_cast<uint32_t>(be->common.ops->get_backend_metadata_size(be->desc.backend_desc, bs));
    if (with_payload_crc) write_checksum(f, ct, bs);
    h->metadata_chksum = env_legacy_crc() ? static_cast<uint32_t>(liberasurecode_crc32_alt(
                                                0, &h->meta, sizeof(fragment_metadata_t)))
                                          : zcrc(&h->meta, sizeof(fragment_metadata_t));
}

// A batch of host copies: through this repo's helper threads when the codec library offers them
// (ecamd_host_copy, include/ecamd_host.h), else one memcpy after the other.
struct CopyBatch {
    std::vector<void*> dst;
    std::vector<const void*> src;
    std::vector<int64_t> len;
    void add(void* d, const void* s, int64_t n)
    {
        if (n <= 0) return;
        dst.push_back(d);
        src.push_back(s);
        len.push_back(n);
    }
    void run(const CodecHooks* h)
    {
        const int n = static_cast<int>(dst.size());
        if (h && h->copy && h->copy(n, dst.data(), src.data(), len.data()) == 0) return;
        for (int i = 0; i < n; i++) std::memcpy(dst[i], src[i], static_cast<size_t>(len[i]));
    }
};

// These copies ride on this repo's codec's staging pack (ecamd_percall_tee_arm, include/ecamd.h):
// the codec, packing input key[i], reads it from the copy's source and writes the copy's
// destination too, so the source leaves DRAM once.  Armed only when every key is a codec input of
// the coming call; whatever the codec did not deliver (it refused, or failed) is copied here after.
struct TeeCopies {
    const CodecHooks& h;
    CopyBatch cb;
    std::vector<const void*> key;
    bool armed = false;
    explicit TeeCopies(const CodecHooks& hooks) : h(hooks) {}
    void add(const void* k, void* d, const void* sr, int64_t n)
    {
        if (n <= 0) return;
        key.push_back(k);
        cb.add(d, sr, n);
    }
    void start(bool use_tee)  // before the codec call
    {
        armed = use_tee && h.tee() && !key.empty() && key.size() <= 64 &&
                h.tee_arm(static_cast<int>(key.size()), key.data(), cb.src.data(), cb.dst.data(), cb.len.data()) == 0;
        if (!armed) cb.run(&h);  // no tees: the copies now, as without them
    }
    void finish()  // after the codec call
    {
        if (!armed) return;
        std::vector<int64_t> done(key.size(), 0);
        h.tee_disarm(done.data());
        armed = false;
        CopyBatch rest;
        for (size_t i = 0; i < key.size(); i++)
            if (done[i] < cb.len[i]) rest.add(cb.dst[i], cb.src[i], cb.len[i]);
        rest.run(&h);
    }
    ~TeeCopies()
    {
        if (armed) h.tee_disarm(nullptr);
    }
};

// fragments_to_string (erasurecode_preprocessing.c:269-370): concatenate data payloads.
int assemble(int k, char** frags, int n, char** out, uint64_t* out_len, const CodecHooks* h)
{
    *out = nullptr;
    if (n < k) return -1;
    std::vector<char*> data(k, nullptr);
    int orig = -1, have = 0;
    for (int i = 0; i < n; i++) {
        int idx = frag_idx(frags[i]), sz = frag_size(frags[i]);
        if (idx < 0 || sz < 0) {
            LOGE("Invalid fragment header information!");
            return -EBADHEADER;
        }
        if (orig < 0) {
            orig = frag_orig_size(frags[i]);
        } else if (frag_orig_size(frags[i]) != orig) {
            LOGE("Inconsistent orig_data_size in fragment header!");
            return -EBADHEADER;
        }
        if (idx < k && !data[idx]) {
            data[idx] = frags[i];
            have++;
        }
    }
    if (have != k) return -1;
    // get_aligned_buffer16 zeroes the whole object before the payloads are copied over it; only
    // what the payloads do not cover (short fragments) is zeroed here, the result is the same
    const size_t len = static_cast<size_t>(orig > 0 ? orig : 0);
    char* s = nullptr;
    if (zero_all()) {
        s = static_cast<char*>(aligned_zero(len));
    } else {
        s = static_cast<char*>(buf_alloc(len));
    }
    if (!s) return -ENOMEM;
    *out_len = static_cast<uint64_t>(orig);
    int off = 0, left = orig;
    CopyBatch cb;
    for (int i = 0; i < k && left > 0; i++) {
        int take = std::min(frag_size(data[i]), left);
        if (take <= 0) continue;  // a corrupt (negative or zero) size copies nothing
        cb.add(s + off, payload(data[i]), take);
        left -= take;
        off += take;
    }
    cb.run(h);
    if (left > 0) std::memset(s + off, 0, static_cast<size_t>(left));
    *out = s;
    return 0;
}

// prepare_fragments_for_decode (erasurecode_preprocessing.c:117-217)
// realign = false keeps unaligned caller fragments in place: this repo's codec stages every
// fragment through its own pinned slabs, so 16-byte alignment buys nothing there, and
// liberasurecode_rs_vand writes only the missing slots (which are always fresh buffers).
int prepare_decode(int k, int m, char** data, char** parity, const int* missing, int* orig,
                   int* bs, uint64_t frag_len, std::vector<char*>& owned, bool realign = true)
{
    bool gone[EC_MAX_FRAGMENTS] = {};
    for (int i = 0; missing[i] >= 0; i++) gone[missing[i]] = true;
    int o = -1, p = -1;
    auto fix = [&](char*& slot, int idx) -> int {
        if (!slot) {
            // this repo's RS codec (realign == false) writes every missing slot it is asked
            // for in full and never reads the others, so they need no zeroing pass
            slot = new_fragment(static_cast<int>(frag_len - kHdr), realign);
            if (!slot) return -ENOMEM;
            owned.push_back(slot);
        } else if (realign && (reinterpret_cast<uintptr_t>(slot) & 15u)) {
            char* t = new_fragment(static_cast<int>(frag_len - kHdr));
            if (!t) return -ENOMEM;
            std::memcpy(t, slot, frag_len);
            slot = t;
            owned.push_back(t);
        }
        if (!gone[idx] && o < 0) {
            o = frag_orig_size(slot);
            if (o < 0) return -EBADHEADER;
            p = frag_size(slot);
            if (p < 0) return -EBADHEADER;
        }
        return 0;
    };
    for (int i = 0; i < k; i++)
        if (int rc = fix(data[i], i)) return rc;
    for (int i = 0; i < m; i++)
        if (int rc = fix(parity[i], k + i)) return rc;
    *orig = o;
    *bs = p;
    return 0;
}

// ECAMD_FRONTEND_TEE=0 turns the staging-pack tees off (TeeCopies; A/B runs, tools/percall_ab.py).
bool tee_on()
{
    static const bool on = [] {
        const char* f = getenv("ECAMD_FRONTEND_TEE");
        return !(f && f[0] == '0');
    }();
    return on;
}

// ECAMD_FRONTEND_DECODE_DIRECT=0 turns decode_direct off (A/B runs, tools/percall_ab.py).
bool decode_direct_on()
{
    static const bool on = [] {
        const char* f = getenv("ECAMD_FRONTEND_DECODE_DIRECT");
        return !(f && f[0] == '0');
    }();
    return on;
}

// liberasurecode_decode straight into the object, in front of this repo's rs_vand codec only: the
// rebuilt data payloads are written by the codec (its staging unpack) at their places in the
// decoded object, and only the surviving data payloads are copied there.  The reference allocates a
// fragment per missing index, rebuilds the missing parity too (the shim's rebuild_parity = 1,
// src/backends/rs_vand/liberasurecode_rs_vand.c:100-101, discarded by a decode) and concatenates
// every data payload afterwards (fragments_to_string, erasurecode_preprocessing.c:269-370): two
// host passes over the rebuilt bytes and a device pass over unneeded parity.  Same bytes out, same
// error codes.  Returns 1 (nothing done) when the surviving data fragments disagree on size or
// orig_data_size -- the general path then handles them exactly as the reference does.
int decode_direct(ec_backend* be, char** data, char** parity, int* missing, char** out,
                  uint64_t* out_len)
{
    auto* r = static_cast<RsDesc*>(be->desc.backend_desc);
    const int k = r->k, m = r->m;
    bool gone[EC_MAX_FRAGMENTS] = {};
    for (int i = 0; missing[i] >= 0; i++) gone[missing[i]] = true;
    int orig = -1, bs = -1;
    for (int i = 0; i < k + m && orig < 0; i++) {  // prepare_decode's first surviving fragment
        char* f = i < k ? data[i] : parity[i - k];
        if (gone[i] || !f) continue;
        orig = frag_orig_size(f);
        if (orig < 0) return -EBADHEADER;
        bs = frag_size(f);
        if (bs < 0) return -EBADHEADER;
    }
    if (orig < 0) return 1;
    for (int i = 0; i < k; i++)
        if (!gone[i] && data[i] && (frag_size(data[i]) != bs || frag_orig_size(data[i]) != orig)) return 1;
    const int64_t span = static_cast<int64_t>(k) * bs;
    const size_t cap = static_cast<size_t>(std::max<int64_t>(orig, span));
    char* obj = static_cast<char*>(buf_alloc(cap ? cap : 1));
    if (!obj) return -ENOMEM;
    std::vector<char*> dp(k), pp(m, nullptr);  // missing parity: not rebuilt, never touched
    for (int i = 0; i < k; i++) dp[i] = gone[i] ? obj + static_cast<int64_t>(i) * bs : payload(data[i]);
    for (int i = 0; i < m; i++)
        if (!gone[k + i]) pp[i] = payload(parity[i]);
    // surviving data payloads -> object: on the codec's staging pack (they are all among its first
    // k inputs), else after the call
    TeeCopies cb(r->hooks);
    for (int i = 0; i < k; i++) {
        const int64_t off = static_cast<int64_t>(i) * bs;
        const int64_t take = std::min<int64_t>(bs, orig - off);
        if (take > 0 && !gone[i]) cb.add(payload(data[i]), obj + off, payload(data[i]), take);
    }
    cb.start(tee_on());
    int rc = 0;
    {
        ExecCheck ex(r->hooks);
        rc = r->decode(r->matrix, dp.data(), pp.data(), k, m, missing, bs, 0);
        if (ex.failed()) {
            buf_free(obj);
            LOGE("Encountered error in backend decode function!");
            return -EIO;
        }
    }
    cb.finish();
    for (int i = 0; i < k && rc != 0; i++) {  // the codec refused (more than m missing): the zeroed
        const int64_t off = static_cast<int64_t>(i) * bs;  // slots of the reference
        const int64_t take = std::min<int64_t>(bs, orig - off);
        if (take <= 0) break;
        if (gone[i]) std::memset(obj + off, 0, static_cast<size_t>(take));
    }
    if (orig > span) std::memset(obj + span, 0, static_cast<size_t>(orig - span));
    *out = obj;
    *out_len = static_cast<uint64_t>(orig);
    return 0;
}

// is_invalid_fragment_metadata (erasurecode.c:1156-1187), caller holds the read lock
int check_metadata(int desc, fragment_metadata_t* md)
{
    ec_backend* be = find(desc);
    if (!be) {
        LOGE("Unable to verify fragment metadata: invalid backend id %d.", desc);
        return -EINVALIDPARAMS;
    }
    if (liberasurecode_verify_fragment_metadata(be, md) != 0) return -EBADHEADER;
    if (!be->common.ops->is_compatible_with(md->backend_version)) return -EBADHEADER;
    if (md->chksum_mismatch == 1) return -EBADCHKSUM;
    return 0;
}

// is_invalid_fragment (erasurecode.c:1189-1222), caller holds the read lock
int invalid_fragment(int desc, char* f)
{
    if (!find(desc) || !f) return 1;
    uint32_t ver = 0;
    if (get_libec_version(f, &ver) != 0 || ver > LIBERASURECODE_VERSION) return 1;
    fragment_metadata_t md;
    if (liberasurecode_get_fragment_metadata(f, &md) != 0) return 1;
    return check_metadata(desc, &md) != 0 ? 1 : 0;
}

void free_owned(std::vector<char*>& owned)
{
    for (char* p : owned) buf_free(p);
    owned.clear();
}

}  // namespace

extern "C" {

__attribute__((constructor)) void liberasurecode_init(void)
{
    openlog("liberasurecode", LOG_PID | LOG_CONS, LOG_USER);
}

__attribute__((destructor)) void liberasurecode_exit(void) { closelog(); }

int liberasurecode_crc32_alt(int crc, const void* buf, size_t size)
{
    // The legacy checksum of bug 1666320 (src/utils/chksum/crc32.c:79-91): reflected CRC-32
    // whose 8-bit shift sign-extends from bit 23.
    struct Table {
        uint32_t t[256];
        Table()
        {
            for (uint32_t n = 0; n < 256; n++) {
                uint32_t c = n;
                for (int b = 0; b < 8; b++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
                t[n] = c;
            }
        }
    };
    static const Table table;  // thread-safe one-time initialisation
    const uint32_t* tab = table.t;
    const signed char* p = static_cast<const signed char*>(buf);
    int32_t c = crc ^ ~0;
    while (size--) {
        int32_t shifted = ((((c >> 8) & 0x00FFFFFF) ^ 0x00800000) - 0x00800000);
        c = static_cast<int32_t>(tab[(c ^ *p++) & 0xFF]) ^ shifted;
    }
    return c ^ ~0;
}

void* alloc_and_set_buffer(int size, int value)
{
    void* b = std::malloc(static_cast<size_t>(size));
    if (b) std::memset(b, value, static_cast<size_t>(size));
    return b;
}

char* get_data_ptr_from_fragment(char* buf) { return buf + kHdr; }

int get_libec_version(char* buf, uint32_t* ver)
{
    if (!has_magic(buf)) return -1;
    *ver = hdr(buf)->libec_version;
    return 0;
}

int get_backend_id(char* buf, ec_backend_id_t* id)
{
    if (!has_magic(buf)) return -1;
    *id = static_cast<ec_backend_id_t>(hdr(buf)->meta.backend_id);
    return 0;
}

int get_backend_version(char* buf, uint32_t* version)
{
    if (!has_magic(buf)) return -1;
    *version = hdr(buf)->meta.backend_version;
    return 0;
}

int get_fragment_partition(int k, int m, char** fragments, int num_fragments, char** data,
                           char** parity, int* missing)
{
    for (int i = 0; i < k; i++) data[i] = nullptr;
    for (int i = 0; i < m; i++) parity[i] = nullptr;
    for (int i = 0; i < num_fragments; i++) {
        int idx = frag_idx(fragments[i]);
        if (idx < 0 || idx >= k + m) return -EBADHEADER;
        if (idx < k)
            data[idx] = fragments[i];
        else
            parity[idx - k] = fragments[i];
    }
    int n = 0;
    for (int i = 0; i < k; i++)
        if (!data[i]) missing[n++] = i;
    for (int i = 0; i < m; i++)
        if (!parity[i]) missing[n++] = k + i;
    return 0;
}

ec_backend_t liberasurecode_backend_instance_get_by_desc(int desc) { return find(desc); }

int liberasurecode_backend_available(const ec_backend_id_t backend_id)
{
    // the reference's C enum compares unsigned (gcc), so negative ids are out of range too
    if (static_cast<unsigned>(backend_id) >= EC_BACKENDS_MAX) return 0;
    void* so = open_backend(kBackends[backend_id]);
    if (!so) return 0;
    dlclose(so);
    return 1;
}

int liberasurecode_instance_create(const ec_backend_id_t id, struct ec_args* args)
{
    if (!args) return -EINVALIDPARAMS;
    // unsigned as in the reference's C (gcc gives ec_backend_id_t an unsigned type): -1 is
    // -EBACKENDNOTSUPP there (test/liberasurecode_test.c:630-631), not an index below the table
    if (static_cast<unsigned>(id) >= EC_BACKENDS_MAX) return -EBACKENDNOTSUPP;
    if (args->k < 0 || args->m < 0) return -EINVALIDPARAMS;
    if (args->k + args->m > EC_MAX_FRAGMENTS) {
        LOGE("Total number of fragments (k + m) must be less than %d\n", EC_MAX_FRAGMENTS);
        return -EINVALIDPARAMS;
    }
    auto* be = static_cast<ec_backend*>(std::calloc(1, sizeof(ec_backend)));
    if (!be) return -ENOMEM;
    fill_common(be->common, kBackends[id]);
    std::memcpy(&be->args.uargs, args, sizeof(ec_args));
    be->desc.backend_sohandle = open_backend(kBackends[id]);
    if (!be->desc.backend_sohandle) {
        const char* e = dlerror();
        LOGE("%s: dynamic linking error %s\n", __func__, e ? e : "(backend not built)");
        std::free(be);
        return -EBACKENDNOTAVAIL;
    }
    int desc = -1;
    if (pthread_rwlock_wrlock(&g_lock) != 0) {
        std::free(be);
        return -1;
    }
    be->desc.backend_desc = be->common.ops->init(&be->args, be->desc.backend_sohandle);
    if (!be->desc.backend_desc) {
        std::free(be);
        desc = -EBACKENDINITERR;
    } else {
        be->idesc = new_desc();
        be->link.sle_next = g_instances;
        g_instances = be;
        desc = be->idesc;
    }
    pthread_rwlock_unlock(&g_lock);
    return desc;
}

int liberasurecode_instance_destroy(int desc)
{
    int rc = pthread_rwlock_wrlock(&g_lock);
    if (rc != 0) return rc;
    ec_backend** pp = &g_instances;
    while (*pp && (*pp)->idesc != desc) pp = &(*pp)->link.sle_next;
    ec_backend* be = *pp;
    if (!be) {
        pthread_rwlock_unlock(&g_lock);
        return -EBACKENDNOTAVAIL;
    }
    be->common.ops->exit(be->desc.backend_desc);
    if (be->desc.backend_sohandle) {
        dlclose(be->desc.backend_sohandle);
        dlerror();
    }
    *pp = be->link.sle_next;
    std::free(be);
    pthread_rwlock_unlock(&g_lock);
    return 0;
}

int liberasurecode_encode_cleanup(int desc, char** encoded_data, char** encoded_parity)
{
    int k, m;
    {
        ReadLock lk;
        if (lk.rc) return lk.rc;
        ec_backend* be = find(desc);
        if (!be) return -EBACKENDNOTAVAIL;
        k = be->args.uargs.k;
        m = be->args.uargs.m;
    }
    if (encoded_data) {
        for (int i = 0; i < k; i++) buf_free(encoded_data[i]);
        std::free(encoded_data);
    }
    if (encoded_parity) {
        for (int i = 0; i < m; i++) buf_free(encoded_parity[i]);
        std::free(encoded_parity);
    }
    return 0;
}

int liberasurecode_encode(int desc, const char* orig_data, uint64_t orig_data_size,
                          char*** encoded_data, char*** encoded_parity, uint64_t* fragment_len)
{
    if (!orig_data || !encoded_data || !encoded_parity || !fragment_len) {
        LOGE("liberasurecode_encode: null argument");
        return -EINVALIDPARAMS;
    }
    int ret = 0;
    char** data = nullptr;
    char** parity = nullptr;
    int k = 0, m = 0;
    {
        ReadLock lk;
        if (lk.rc) return lk.rc < 0 ? lk.rc : -lk.rc;
        ec_backend* be = find(desc);
        if (!be) return -EBACKENDNOTAVAIL;
        k = be->args.uargs.k;
        m = be->args.uargs.m;
        data = static_cast<char**>(alloc_and_set_buffer(static_cast<int>(sizeof(char*)) * k, 0));
        parity = static_cast<char**>(alloc_and_set_buffer(static_cast<int>(sizeof(char*)) * m, 0));
        if (!data || !parity) {
            ret = -ENOMEM;
        } else {
            // prepare_fragments_for_encode (erasurecode_preprocessing.c:36-108)
            const int total = static_cast<int>(orig_data_size);
            const int bs = aligned_size(be, total) / k;
            const int meta = static_cast<int>(
                be->common.ops->get_backend_metadata_size(be->desc.backend_desc, bs));
            const int off = static_cast<int>(be->common.ops->get_encode_offset(be->desc.backend_desc, meta));
            int left = total;
            const char* src = orig_data;
            // In front of this repo's codecs only the data bytes the object copy does not cover are
            // zeroed (the reference zeroes every fragment first: 14 MiB of memset per 10 MiB object
            // at k=10 m=4).  Parity stays zeroed for flat_xor_hd, whose encode XORs into the parity
            // buffers as the reference's does (xor_code.c:141-191); this repo's rs_vand writes every
            // parity byte.  A foreign codec gets zeroed buffers throughout.
            const bool lean = hooks_of(be).ours() && !zero_all();
            const bool lean_parity = lean && be->common.id == EC_BACKEND_LIBERASURECODE_RS_VAND;
            // object -> data payloads: on the codec's staging pack when it offers tees
            TeeCopies cb(hooks_of(be));
            const bool tee = lean && tee_on();
            for (int i = 0; i < k + m && ret == 0; i++) {
                char* f = new_fragment(bs + meta, !(i < k ? lean : lean_parity));
                if (!f) {
                    ret = -ENOMEM;
                    break;
                }
                if (i < k) {
                    data[i] = f;
                    const int take = left > bs ? bs : left;
                    if (lean) {
                        const size_t lo = static_cast<size_t>(off);
                        zero_outside(payload(f), static_cast<size_t>(bs + meta), lo,
                                     lo + static_cast<size_t>(take > 0 ? take : 0));
                    }
                    if (left > 0) cb.add(payload(f) + off, payload(f) + off, src, take);
                    src += take;
                    left -= take;
                } else {
                    parity[i - k] = f;
                }
            }
            // with tees the copies happen inside the codec call (every data payload is its input;
            // the payloads start at offset 0 for both backends), else right here
            if (ret == 0) cb.start(tee && off == 0);
            CrcArm arm(be, be->args.uargs.ct == CHKSUM_CRC32);  // through the stamping below
            if (ret == 0) {
                std::vector<char*> dp(k), pp(m);
                for (int i = 0; i < k; i++) dp[i] = payload(data[i]);
                for (int i = 0; i < m; i++) pp[i] = payload(parity[i]);
                ret = be->common.ops->encode(be->desc.backend_desc, dp.data(), pp.data(), bs);
                if (ret > 0) ret = 0;  // only negative returns are failures (erasurecode.c:454-461)
                cb.finish();
            }
            if (ret == 0) {
                // finalize_fragments_after_encode (erasurecode_postprocessing.c:71-93)
                const ec_checksum_type_t ct = be->args.uargs.ct;
                for (int i = 0; i < k; i++) stamp(be, data[i], i, orig_data_size, bs, ct, true);
                for (int i = 0; i < m; i++) stamp(be, parity[i], k + i, orig_data_size, bs, ct, true);
                *fragment_len = static_cast<uint64_t>(frag_size(data[0])) +
                                hdr(data[0])->meta.frag_backend_metadata_size + kHdr;
            }
        }
    }
    if (ret) {
        LOGE("Error in liberasurecode_encode %d", ret);
        liberasurecode_encode_cleanup(desc, data, parity);
        data = parity = nullptr;
    }
    *encoded_data = data;
    *encoded_parity = parity;
    return ret;
}

int liberasurecode_decode_cleanup(int desc, char* data)
{
    {
        ReadLock lk;
        if (lk.rc) return lk.rc;
        if (!find(desc)) return -EBACKENDNOTAVAIL;
    }
    buf_free(data);
    return 0;
}

int liberasurecode_decode(int desc, char** available_fragments, int num_fragments,
                          uint64_t fragment_len, int force_metadata_checks, char** out_data,
                          uint64_t* out_data_len)
{
    ReadLock lk;
    if (lk.rc) return lk.rc;
    ec_backend* be = find(desc);
    if (!be) return -EBACKENDNOTAVAIL;
    if (!available_fragments || !out_data || !out_data_len) {
        LOGE("liberasurecode_decode: null argument");
        return -EINVALIDPARAMS;
    }
    const int k = be->args.uargs.k, m = be->args.uargs.m;
    if (num_fragments < k) {
        LOGE("Not enough fragments to decode, got %d, need %d!", num_fragments, k);
        return -EINSUFFFRAGS;
    }
    if (fragment_len < kHdr) {
        LOGE("Fragments not long enough to include headers!");
        return -EBADHEADER;
    }
    for (int i = 0; i < num_fragments; i++)
        if (is_invalid_fragment_header(hdr(available_fragments[i]))) {
            LOGE("Invalid fragment header information!");
            return -EBADHEADER;
        }
    if (be->common.ops->is_systematic &&
        assemble(k, available_fragments, num_fragments, out_data, out_data_len, &hooks_of(be)) == 0)
        return 0;  // every data fragment present: no backend work

    std::vector<char*> data(k), parity(m), owned;
    std::vector<int> missing(k + m, -1);
    if (force_metadata_checks) {
        int bad = 0;
        for (int i = 0; i < num_fragments; i++) bad += invalid_fragment(desc, available_fragments[i]);
        if (num_fragments - bad < k) {
            LOGE("Not enough valid fragments available for decode!");
            return -EINSUFFFRAGS;
        }
    }
    int ret = get_fragment_partition(k, m, available_fragments, num_fragments, data.data(),
                                     parity.data(), missing.data());
    int orig = 0, bs = 0;
    const bool realign = !(be->common.id == EC_BACKEND_LIBERASURECODE_RS_VAND && hooks_of(be).ours());
    if (ret == 0 && !realign && !zero_all() && decode_direct_on()) {
        const int d = decode_direct(be, data.data(), parity.data(), missing.data(), out_data, out_data_len);
        if (d <= 0) return d;  // else irregular fragments: the general path below
    }
    if (ret == 0)
        ret = prepare_decode(k, m, data.data(), parity.data(), missing.data(), &orig, &bs,
                             fragment_len, owned, realign);
    if (ret == 0) {
        std::vector<char*> dp(k), pp(m);
        for (int i = 0; i < k; i++) dp[i] = payload(data[i]);
        for (int i = 0; i < m; i++) pp[i] = payload(parity[i]);
        ret = be->common.ops->decode(be->desc.backend_desc, dp.data(), pp.data(), missing.data(), bs);
        if (ret < 0) LOGE("Encountered error in backend decode function!");
    }
    if (ret == 0) {
        for (int j = 0; missing[j] >= 0; j++) {
            if (missing[j] >= k) continue;
            char* f = data[missing[j]];
            hdr(f)->magic = LIBERASURECODE_FRAG_HEADER_MAGIC;  // init_fragment_header
            stamp(be, f, missing[j], static_cast<uint64_t>(orig), bs, be->args.uargs.ct, false);
        }
        ret = assemble(k, data.data(), k, out_data, out_data_len, &hooks_of(be));
        if (ret < 0) LOGE("Could not convert decoded fragments to a string!");
    }
    free_owned(owned);
    return ret;
}

int liberasurecode_reconstruct_fragment(int desc, char** available_fragments, int num_fragments,
                                        uint64_t fragment_len, int destination_idx,
                                        char* out_fragment)
{
    ReadLock lk;
    if (lk.rc) return lk.rc;
    ec_backend* be = find(desc);
    if (!be) return -EBACKENDNOTAVAIL;
    if (!available_fragments || !out_fragment) {
        LOGE("Can not reconstruct fragment: null argument");
        return -EINVALIDPARAMS;
    }
    const int k = be->args.uargs.k, m = be->args.uargs.m;
    if (destination_idx < 0 || destination_idx >= k + m) return -EINVALIDPARAMS;
    for (int i = 0; i < num_fragments; i++)
        if (is_invalid_fragment_header(hdr(available_fragments[i]))) {
            LOGE("Invalid fragment header information!");
            return -EBADHEADER;
        }
    std::vector<char*> data(k), parity(m), owned;
    std::vector<int> missing(k + m, -1);
    int ret = get_fragment_partition(k, m, available_fragments, num_fragments, data.data(),
                                     parity.data(), missing.data());
    if (ret < 0) return ret;
    bool dest_missing = false;
    for (int i = 0; missing[i] > -1; i++) dest_missing |= missing[i] == destination_idx;
    auto slot = [&](int idx) -> char* { return idx < k ? data[idx] : parity[idx - k]; };
    if (!dest_missing) {
        LOGW("Dest idx for reconstruction was supplied as available buffer!");
        std::memcpy(out_fragment, slot(destination_idx), fragment_len);
        return 0;
    }
    if (!be->common.ops->check_reconstruct_fragments) {
        if (num_fragments < k) return -EINSUFFFRAGS;
    } else {
        ret = be->common.ops->check_reconstruct_fragments(be->desc.backend_desc, missing.data(),
                                                          destination_idx);
        if (ret < 0) return ret;
    }
    int orig = 0, bs = 0;
    const bool realign = !(be->common.id == EC_BACKEND_LIBERASURECODE_RS_VAND && hooks_of(be).ours());
    ret = prepare_decode(k, m, data.data(), parity.data(), missing.data(), &orig, &bs,
                         fragment_len, owned, realign);
    CrcArm arm(be, be->args.uargs.ct == CHKSUM_CRC32);  // through the stamping below
    if (ret == 0) {
        std::vector<char*> dp(k), pp(m);
        for (int i = 0; i < k; i++) dp[i] = payload(data[i]);
        for (int i = 0; i < m; i++) pp[i] = payload(parity[i]);
        ret = be->common.ops->reconstruct(be->desc.backend_desc, dp.data(), pp.data(),
                                          missing.data(), destination_idx, bs);
        if (ret < 0) LOGE("Could not reconstruct fragment!");
    }
    if (ret == 0) {
        char* f = slot(destination_idx);
        hdr(f)->magic = LIBERASURECODE_FRAG_HEADER_MAGIC;
        stamp(be, f, destination_idx, static_cast<uint64_t>(orig), bs, be->args.uargs.ct, true);
        std::memcpy(out_fragment, f, fragment_len);
    }
    free_owned(owned);
    return ret;
}

int liberasurecode_fragments_needed(int desc, int* fragments_to_reconstruct,
                                    int* fragments_to_exclude, int* fragments_needed)
{
    ReadLock lk;
    if (lk.rc) return lk.rc;
    ec_backend* be = find(desc);
    if (!be) return -EBACKENDNOTAVAIL;
    if (!fragments_to_reconstruct || !fragments_to_exclude || !fragments_needed) {
        LOGE("Unable to determine list of fragments needed: null argument");
        return -EINVALIDPARAMS;
    }
    return be->common.ops->fragments_needed(be->desc.backend_desc, fragments_to_reconstruct,
                                            fragments_to_exclude, fragments_needed);
}

int liberasurecode_get_fragment_metadata(char* fragment, fragment_metadata_t* md)
{
    if (!fragment || !md) {
        LOGE("liberasurecode_get_fragment_metadata: null argument");
        return -EINVALIDPARAMS;
    }
    if (is_invalid_fragment_header(hdr(fragment))) {
        LOGE("Invalid fragment header information!");
        return -EBADHEADER;
    }
    std::memcpy(md, fragment, sizeof(fragment_metadata_t));
    if (hdr(fragment)->magic != LIBERASURECODE_FRAG_HEADER_MAGIC) {
        if (bswap32(hdr(fragment)->magic) != LIBERASURECODE_FRAG_HEADER_MAGIC) {
            LOGE("Invalid fragment, illegal magic value");
            return -EINVALIDPARAMS;
        }
        // written on an opposite-endian host (erasurecode.c:1050-1068); the reference swaps the
        // one-byte chksum_type through a 32-bit swap, which always leaves it 0
        md->idx = bswap32(md->idx);
        md->size = bswap32(md->size);
        md->frag_backend_metadata_size = bswap32(md->frag_backend_metadata_size);
        md->orig_data_size = bswap64(md->orig_data_size);
        md->chksum_type = static_cast<uint8_t>(bswap32(md->chksum_type));
        for (int i = 0; i < LIBERASURECODE_MAX_CHECKSUM_LEN; i++) md->chksum[i] = bswap32(md->chksum[i]);
        md->backend_version = bswap32(md->backend_version);
    }
    if (md->chksum_type == CHKSUM_CRC32) {
        const uint32_t stored = md->chksum[0];
        char* p = payload(fragment);
        const size_t n = md->size;
        md->chksum_mismatch =
            (stored != zcrc(p, n) &&
             stored != static_cast<uint32_t>(liberasurecode_crc32_alt(0, p, n))) ? 1 : 0;
    }
    return 0;
}

int is_invalid_fragment_header(fragment_header_t* header)
{
    if (header->libec_version == 0) return 1;
    uint32_t stored = header->metadata_chksum, ver = header->libec_version;
    if (header->magic != LIBERASURECODE_FRAG_HEADER_MAGIC) {
        if (bswap32(header->magic) != LIBERASURECODE_FRAG_HEADER_MAGIC) {
            LOGE("Invalid fragment header (get meta chksum)!");
            return 1;
        }
        stored = bswap32(stored);
        ver = bswap32(ver);
    }
    if (ver < _VERSION(1, 2, 0)) return 0;  // no metadata checksum before 1.2.0
    if (stored == zcrc(&header->meta, sizeof(fragment_metadata_t))) return 0;
    return stored != static_cast<uint32_t>(
                         liberasurecode_crc32_alt(0, &header->meta, sizeof(fragment_metadata_t)));
}

int liberasurecode_verify_fragment_metadata(ec_backend_t be, fragment_metadata_t* md)
{
    if (md->idx >= static_cast<uint32_t>(be->args.uargs.k + be->args.uargs.m)) return 1;
    if (md->backend_id != be->common.id) return 1;
    if (!be->common.ops->is_compatible_with(md->backend_version)) return 1;
    return 0;
}

int is_invalid_fragment(int desc, char* fragment)
{
    ReadLock lk;
    if (lk.rc) return lk.rc;
    return invalid_fragment(desc, fragment);
}

int liberasurecode_verify_stripe_metadata(int desc, char** fragments, int num_fragments)
{
    if (!fragments) {
        LOGE("Unable to verify stripe metadata: fragments missing.");
        return -EINVALIDPARAMS;
    }
    if (num_fragments <= 0) {
        LOGE("Unable to verify stripe metadata: number of fragments must be greater than 0.");
        return -EINVALIDPARAMS;
    }
    ReadLock lk;
    if (lk.rc) return lk.rc;
    for (int i = 0; i < num_fragments; i++) {
        int ret = check_metadata(desc, reinterpret_cast<fragment_metadata_t*>(fragments[i]));
        if (ret < 0) return ret;
    }
    return 0;
}

int liberasurecode_get_aligned_data_size(int desc, uint64_t data_len)
{
    ReadLock lk;
    if (lk.rc) return lk.rc < 0 ? lk.rc : -lk.rc;
    ec_backend* be = find(desc);
    if (!be) return -EBACKENDNOTAVAIL;
    const uint64_t a = static_cast<uint64_t>(be->args.uargs.k) *
                       static_cast<uint64_t>(be->common.ops->element_size(be->desc.backend_desc) / 8);
    return static_cast<int>(((data_len + a - 1) / a) * a);
}

int liberasurecode_get_minimum_encode_size(int desc) { return liberasurecode_get_aligned_data_size(desc, 1); }

int liberasurecode_get_fragment_size(int desc, int data_len)
{
    ReadLock lk;
    if (lk.rc) return lk.rc < 0 ? lk.rc : -lk.rc;
    ec_backend* be = find(desc);
    if (!be) return -EBACKENDNOTAVAIL;
    const int bs = aligned_size(be, data_len) / be->args.uargs.k;
    return bs + static_cast<int>(be->common.ops->get_backend_metadata_size(be->desc.backend_desc, bs));
}

uint32_t liberasurecode_get_version(void) { return LIBERASURECODE_VERSION; }

}  // extern "C"
