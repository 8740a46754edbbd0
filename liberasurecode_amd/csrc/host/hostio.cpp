// hostio.cpp -- synchronous host-buffer execution for the per-call drop-in ABIs
// (liberasurecode_rs_vand.so.1, libXorcode.so.1): the reference contract is "caller-owned host
// fragments in, results complete on return", called concurrently from many threads
// (src/erasurecode.c:414, 543, 769 hold only a shared read lock around the codec calls).
//
// Each call borrows a pooled staging context (2 HIP streams, 2 pinned host slabs, 2 device slabs)
// and walks the fragments in chunks: while the GPU runs chunk c (H2D -> kernel -> D2H on stream
// c&1), the CPU packs chunk c+1 into the other pinned slab and unpacks chunk c-1.  Fragment maps
// are cached by content, so callers may free() and rebuild matrices at will.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include <zlib.h>

#include "crc.hpp"
#include "ecamd.h"
#include "ecamd_host.h"

namespace {

// Per-call checksum handoff (ecamd_percall_crc_*): while armed on a thread, the chunked
// pipeline also checksums every fragment slab on the GPU and records (pointer, length, crc).
struct CrcRecord {
    bool armed = false;
    bool legacy = false;
    struct Entry {
        const void* ptr;
        int64_t len;
        uint32_t crc;
    };
    std::vector<Entry> entries;
};
thread_local CrcRecord t_crc;

// Per-call execution status (ecamd_percall_status): the first staging / copy / launch failure on
// this thread since ecamd_percall_reset.  The reference codec cannot fail mid-call, so its shim
// discards return codes (src/backends/rs_vand/liberasurecode_rs_vand.c:86-90); a GPU codec can,
// and the frontend reads this to fail the call instead of stamping stale parity.
thread_local int t_exec_rc = 0;

// Input tees of the calling thread (ecamd_percall_tee_arm): packing input `key` reads bytes
// [0, len) from `src` and also writes them to `dst2`.
struct Tee {
    const void* key;
    const char* src;
    char* dst2;
    int64_t len;
    int64_t done = 0;
};
thread_local std::vector<Tee> t_tee;

Tee* find_tee(const void* key)
{
    for (auto& t : t_tee)
        if (t.key == key) return &t;
    return nullptr;
}

int note_exec(int rc)
{
    if (rc != 0 && t_exec_rc == 0) t_exec_rc = rc;
    return rc;
}

// Fault injection (ecamd_fault_inject): the next N staging acquisitions fail as an allocation
// failure would, before any GPU work.
std::atomic<int> g_fail_staging{0};

// zlib crc32_combine: crc(A || B) = A^|B| crc(A) ^ crc(B) for both checksum machines.
uint32_t crc_combine(bool legacy, uint32_t a, uint32_t b, int64_t len_b)
{
    static std::mutex mu;
    static std::map<std::pair<bool, int64_t>, ecamd::Mat32> cache;
    ecamd::Mat32 m;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find({legacy, len_b});
        if (it == cache.end()) {
            if (cache.size() > 256) cache.clear();
            it = cache.emplace(std::make_pair(legacy, len_b),
                               ecamd::zero_shift(ecamd::CrcMachine(legacy),
                                                 static_cast<uint64_t>(len_b))).first;
        }
        m = it->second;
    }
    return m.apply(a) ^ b;
}

// bytes of all fragments per chunk (both directions); ECAMD_PERCALL_CHUNK_KIB overrides (A/B runs)
int64_t chunk_target()
{
    static const int64_t bytes = [] {
        const char* s = std::getenv("ECAMD_PERCALL_CHUNK_KIB");
        const long v = s && *s ? std::atol(s) : 0;
        return v >= 64 ? static_cast<int64_t>(v) << 10 : int64_t(8) << 20;
    }();
    return bytes;
}

// Waiting for a chunk: with ECAMD_PERCALL_SPIN_US > 0 the caller polls the stream for up to that
// many microseconds before it blocks in hipStreamSynchronize.  Only chunks of at least
// kSpinMinBytes of fragments poll: for 4-16 KiB calls polling measured 1-6 us SLOWER than
// blocking, while 4-16 MiB objects gained 15% with it (tools/latency_ab.py,
// profiles/r03_latency_ab2.log).
constexpr int64_t kSpinMinBytes = 64 << 10;
// Default: one-chunk calls (up to 8 MiB of fragments) let the kernel write its outputs straight into the
// pinned slab (mode 2), saving the D2H DMA and its queue round trip; the inputs still arrive by DMA -- a
// kernel READING pinned host memory over PCIe costs more than the DMA (mode 1 / 3: 4 KiB RS(10,4) encode
// 36.9 -> 49.1 us).  One thread, RS(10,4), two interleaved passes (tools/latency_bench.py,
// profiles/r05_lat_m{0,1,2,3}{a,b}.log): encode 4 KiB 36.9 -> 35.0 us, 64 KiB 69.7 -> 62.8, 256 KiB
// 82.7 -> 74.5, 1 MiB 135 -> 126; with CRC32 64 KiB 100.6 -> 79, 256 KiB 122 -> 101.
constexpr long kZeroCopyKibDefault = 8192;
constexpr int kZeroCopyModeDefault = 2;
// off by default: measured neutral (4 KiB encode 33.6-34.5 -> 33.2-33.4 us, 16 KiB 43.3 -> 42.2 us; the
// DMA is queued ahead of the launch and overlaps it -- the floor is the launch and its completion;
// profiles/r05_lat3_{def,bar}{a,b}.log)
constexpr long kBarKibDefault = 0;

// ECAMD_PERCALL_ZEROCOPY_KIB: a call whose fragments fit one chunk of at most this many KiB (all
// fragments) lets the kernel work on the pinned slab itself over PCIe (hipHostMalloc memory is
// device-accessible and coherent) instead of a DMA: its outputs (ECAMD_PERCALL_ZEROCOPY_MODE bit 1,
// default) and / or its inputs (bit 0) -- one queued operation fewer per direction.
int64_t zerocopy_bytes()
{
    static const int64_t v = [] {
        const char* env = std::getenv("ECAMD_PERCALL_ZEROCOPY_KIB");
        const long kib = env ? std::atol(env) : kZeroCopyKibDefault;
        return static_cast<int64_t>(std::max(0L, kib)) << 10;
    }();
    return v;
}

// ECAMD_PERCALL_ZEROCOPY_IN_KIB (default 64): one-chunk calls whose fragments are at most this many KiB
// let the kernel read its inputs from the pinned slab (no H2D DMA): the small-launch kernel's sizes
// (<= 4096 16-byte chunks), which stage them through LDS with 16-byte loads -- RS(10,4) 4 / 16 / 64 / 256
// KiB encodes 22.3 / 28.0 / 31.6 / 42.0 -> 21.5 / 23.4 / 24.9 / 34.0 us (profiles/r06_lat_zc.json).
int64_t zerocopy_in_bytes()
{
    static const int64_t v = [] {
        const char* env = std::getenv("ECAMD_PERCALL_ZEROCOPY_IN_KIB");
        const long kib = env ? std::atol(env) : 64;
        return static_cast<int64_t>(std::max(0L, kib)) << 10;
    }();
    return v;
}

// ECAMD_PERCALL_FUSE_CRC=0: never fold the CRC32s into the codec launch (A/B switch)
const bool g_fuse_crc = [] {
    const char* env = std::getenv("ECAMD_PERCALL_FUSE_CRC");
    return !(env && std::strcmp(env, "0") == 0);
}();

int zerocopy_mode()
{
    static const int v = [] {
        const char* env = std::getenv("ECAMD_PERCALL_ZEROCOPY_MODE");
        return env ? std::atoi(env) & 3 : kZeroCopyModeDefault;
    }();
    return v;
}

// ECAMD_PERCALL_BAR_KIB: a one-chunk call whose inputs are at most this many KiB packs them straight
// into host-writable device memory (ecamd_malloc_host_writable: the PCIe BAR, no DMA) -- a 4 KiB
// hipMemcpyAsync + wait costs ~13.5 us, the host's own 4 KiB write through the BAR ~0.7 us
// (tools/bar_probe.py) -- while the kernel writes its outputs into the pinned slab (zero copy, mode
// bit 1): the call is then one launch and one wait.  0 = off; platforms without a large BAR fall
// back to the DMA by themselves.
int64_t bar_bytes()
{
    static const int64_t v = [] {
        const char* env = std::getenv("ECAMD_PERCALL_BAR_KIB");
        const long kib = env ? std::atol(env) : kBarKibDefault;
        return static_cast<int64_t>(std::max(0L, kib)) << 10;
    }();
    return v;
}
std::atomic<int> g_bar_ok{1};  // 0 once an allocation found no host-visible device memory

int spin_us()
{
    static const int us = [] {
        const char* s = std::getenv("ECAMD_PERCALL_SPIN_US");
        return s && *s ? std::max(0, std::atoi(s)) : 0;
    }();
    return us;
}

int wait_stream(void* stream, bool poll)
{
    if (poll && spin_us() > 0) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us());
        do {
            const int q = ecamd_stream_query(stream);
            if (q <= 0) return q;
        } while (std::chrono::steady_clock::now() < until);
    }
    return ecamd_stream_synchronize(stream);
}

struct MapHolder {
    ecamd_map* map = nullptr;
    ~MapHolder() { ecamd_map_destroy(map); }
};
std::mutex g_map_mu;
std::map<std::vector<int>, std::shared_ptr<MapHolder>> g_maps;

std::shared_ptr<MapHolder> cached_map(int dev, const int* coeff, int R, int K, int* rc)
{
    std::vector<int> key = {dev, R, K};
    key.insert(key.end(), coeff, coeff + static_cast<size_t>(R) * K);
    {
        std::lock_guard<std::mutex> lk(g_map_mu);
        auto it = g_maps.find(key);
        if (it != g_maps.end()) return it->second;
    }
    auto h = std::make_shared<MapHolder>();
    *rc = ecamd_map_create(coeff, R, K, &h->map);
    if (*rc) return nullptr;
    std::lock_guard<std::mutex> lk(g_map_mu);
    if (g_maps.size() > 4096) g_maps.clear();  // holders in flight keep their map alive
    return g_maps.emplace(key, h).first->second;
}

struct Slot {
    void* stream = nullptr;
    void* event = nullptr;
    char* h_pin = nullptr;
    char* d_buf = nullptr;
    char* d_bar = nullptr;  // host-writable device memory for small calls' inputs (bar_bytes())
};

struct Staging {
    Slot slot[2];
    int64_t cap = 0;  // bytes per slab
    uint32_t seq = 0;  // completion-flag values handed out (per context: one caller at a time)
    int device = 0;   // every stream, event and buffer of this context lives there
    ~Staging()
    {
        for (auto& s : slot) {
            if (s.h_pin) ecamd_host_free(s.h_pin);
            if (s.d_buf) ecamd_free(s.d_buf);
            if (s.d_bar) ecamd_free(s.d_bar);
        }
    }
};

// The slot's host-writable input slab (kBarSlabBytes), allocated on first use; null when unavailable.
constexpr int64_t kBarSlabBytes = 1 << 20;
char* bar_slab(Slot& s)
{
    if (!s.d_bar && g_bar_ok.load(std::memory_order_relaxed)) {
        void* p = nullptr;
        if (ecamd_malloc_host_writable(&p, kBarSlabBytes) == 0)
            s.d_bar = static_cast<char*>(p);
        else
            g_bar_ok.store(0, std::memory_order_relaxed);
    }
    return s.d_bar;
}

// One pool of staging contexts per device; calls go round-robin over the planned devices
// (ecamd_percall_device_plan), so concurrent callers on an 8-GPU node use 8 PCIe links.
std::mutex g_pool_mu;
std::vector<std::vector<Staging*>> g_pool;  // by device

// ECAMD_PERCALL_DEVICES: device indices ("3", "0,2,4"), or "current" -- the device current on the
// thread whose call builds the plan, resolved ONCE: a worker thread that never selected a device
// would otherwise report device 0 and send a rank's calls to another rank's GPU (shard.py passes
// the rank's index explicitly).
struct DevicePlan {
    std::vector<int> devs;
    std::atomic<unsigned> next{0};
    DevicePlan()
    {
        const int n = ecamd_device_count();
        if (n <= 0) return;
        const char* spec = std::getenv("ECAMD_PERCALL_DEVICES");
        int cur = -1;
        if (spec && std::strcmp(spec, "current") == 0 && ecamd_get_device(&cur) == 0 && cur >= 0 && cur < n) {
            devs.assign(1, cur);
            return;
        }
        devs.resize(static_cast<size_t>(n));
        devs.resize(static_cast<size_t>(ecamd_percall_device_plan(n, spec, devs.data(), n)));
    }
};

int pick_device()
{
    static DevicePlan plan;  // thread-safe one-time initialisation
    if (plan.devs.empty()) return -1;
    return plan.devs[plan.next.fetch_add(1, std::memory_order_relaxed) % plan.devs.size()];
}

// Makes `dev` current for one call and restores the caller's device afterwards.
struct DeviceScope {
    int prev = -1;
    int rc = 0;
    explicit DeviceScope(int dev)
    {
        if ((rc = ecamd_get_device(&prev)) == 0 && prev != dev) rc = ecamd_set_device(dev);
    }
    ~DeviceScope()
    {
        int cur = -1;
        if (prev >= 0 && ecamd_get_device(&cur) == 0 && cur != prev) ecamd_set_device(prev);
    }
};

int grow(Staging* st, int64_t bytes)
{
    if (st->cap >= bytes) return 0;
    for (auto& s : st->slot) {
        if (s.h_pin) ecamd_host_free(s.h_pin);
        if (s.d_buf) ecamd_free(s.d_buf);
        s.h_pin = s.d_buf = nullptr;
        void* p = nullptr;
        int rc = ecamd_host_alloc(&p, bytes);
        if (rc) return rc;
        s.h_pin = static_cast<char*>(p);
        std::memset(s.h_pin + bytes - 512, 0, 512);  // the completion flag and chunk CRC words
        rc = ecamd_malloc(&p, bytes);
        if (rc) return rc;
        s.d_buf = static_cast<char*>(p);
    }
    st->cap = bytes;
    return 0;
}

Staging* acquire(int dev, int64_t bytes, int* rc)
{
    for (int left = g_fail_staging.load(); left > 0; left = g_fail_staging.load())
        if (g_fail_staging.compare_exchange_weak(left, left - 1)) {
            *rc = ECAMD_ENOMEM;
            return nullptr;
        }
    Staging* st = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (static_cast<int>(g_pool.size()) <= dev) g_pool.resize(static_cast<size_t>(dev) + 1);
        if (!g_pool[dev].empty()) {
            st = g_pool[dev].back();
            g_pool[dev].pop_back();
        }
    }
    if (!st) {
        st = new Staging();
        st->device = dev;
        for (auto& s : st->slot) {
            if ((*rc = ecamd_stream_create(&s.stream)) || (*rc = ecamd_event_create(&s.event))) {
                delete st;
                return nullptr;
            }
        }
    }
    if ((*rc = grow(st, bytes))) {
        delete st;
        return nullptr;
    }
    return st;
}

void release(Staging* st)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool[st->device].push_back(st);
}

// The completion-flag word of a slab (ecamd_done_flag_arm): 512 bytes before its end, apart from the
// chunk CRCs in the last 256.
uint32_t* done_word(char* h_pin, int64_t cap) { return reinterpret_cast<uint32_t*>(h_pin + cap - 512); }

// ECAMD_PERCALL_DONE_FLAG=0: synchronize the stream instead of polling the completion flag (A/B switch)
const bool g_done_flag = [] {
    const char* env = std::getenv("ECAMD_PERCALL_DONE_FLAG");
    return !(env && std::strcmp(env, "0") == 0);
}();
// ECAMD_PERCALL_SERVER=0: launch every small kernel instead of posting one-launch calls to the resident
// small server (ecamd_done_flag_arm_server; DESIGN.md §6, profiles/r06_lat_server.json)
const bool g_server = [] {
    const char* env = std::getenv("ECAMD_PERCALL_SERVER");
    return !(env && std::strcmp(env, "0") == 0);
}();
// ECAMD_PERCALL_OVERLAP_CRC=0: leave a small call's input CRC32s to the frontend, after the call (A/B switch)
const bool g_overlap_crc = [] {
    const char* env = std::getenv("ECAMD_PERCALL_OVERLAP_CRC");
    return !(env && std::strcmp(env, "0") == 0);
}();
constexpr int kDonePollUs = 200;  // then block in hipStreamSynchronize (a busy GPU, or a fault)

// Polls the flag word for `value` (the GPU writes it to pinned host memory); false after kDonePollUs.
bool poll_done(const uint32_t* flag, uint32_t value)
{
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(kDonePollUs);
    for (int i = 0;; i++) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == value) return true;
        if ((i & 63) == 63 && std::chrono::steady_clock::now() > until) return false;
    }
}

// Kernel launcher for one chunk: inputs at d + j*pitch, outputs at d + (K+r)*pitch.
// Inputs at din + j*pitch, outputs at dout + (K+r)*pitch.
// crc_dst (may be null): where a launcher that can fold the payload CRC32s into its kernel
// (ecamd_map_apply_strided_crc) writes them, all inputs then all outputs; *fused says whether it did.
using Launch = int (*)(const void* ctx, char* din, char* dout, int64_t pitch, int64_t bytes, void* stream,
                       uint32_t* crc_dst, bool legacy, bool* fused);

// staged_in: the launcher's small kernel stages its inputs through LDS with wide loads (gf16_small_kernel,
// xor_small_kernel; reading 2-4-byte lanes in place over PCIe costs more than the DMA), so small calls may
// leave the inputs in the pinned slab.
int run_chunked(int dev, int K, int R, const char* const* in, char* const* out, int64_t bs,
                const void* ctx, Launch launch, bool staged_in)
{
    const int64_t nfr = K + R;
    // The chunk is also the fragment pitch in the slab: a multiple of 128 puts every fragment
    // on a cache line (16-byte-aligned pitches cost the codec 13-19%).
    int64_t chunk = std::max<int64_t>(128, (chunk_target() / nfr) / 128 * 128);
    const int64_t padded = (bs + 127) / 128 * 128;
    chunk = std::min(chunk, padded);
    int rc = 0;
    // CRC32 of every fragment (ecamd_percall_crc_arm), from 16 KiB of fragments (below, zlib on the host
    // answers sooner; the frontend falls back to the CPU): a one-chunk call first offers it to the codec
    // launch, which folds it into the small-launch kernel when it can (ecamd_map_apply_strided_crc);
    // otherwise a separate ecamd_crc32 pass.
    const bool crc_armed = t_crc.armed && nfr <= 64;
    const bool crc_pass_ok = crc_armed && bs * nfr >= (16 << 10);
    const bool want_crc = crc_pass_ok;
    Staging* st = acquire(dev, chunk * nfr + 512, &rc);  // last 512 B of each slab: done flag, chunk CRCs
    if (!st) return rc;
    const int64_t crc_off = st->cap - 256;
    std::vector<uint32_t> crc(crc_armed ? nfr : 0, 0u);
    const int64_t nchunks = (bs + chunk - 1) / chunk;
    const bool zero_copy = nchunks == 1 && chunk * nfr <= zerocopy_bytes();
    // which side works on the pinned slab itself (ECAMD_PERCALL_ZEROCOPY_MODE, bit 0 inputs, bit 1
    // outputs; inputs also for fragments of at most ECAMD_PERCALL_ZEROCOPY_IN_KIB, the small-launch
    // kernel's sizes, whose inputs it stages through LDS with wide loads)
    const bool zc_in = zero_copy && ((zerocopy_mode() & 1) || (staged_in && bs <= zerocopy_in_bytes()));
    const bool zc_out = zero_copy && (zerocopy_mode() & 2);
    // inputs packed straight into host-writable device memory (no H2D DMA), outputs into the pinned slab
    const bool bar = zc_out && !zc_in && !want_crc && nchunks == 1 && K * chunk <= std::min(bar_bytes(), kBarSlabBytes);
    int64_t pending[2] = {-1, -1};  // chunk index in flight per slot
    // completion flag (one-chunk calls whose outputs land in the pinned slab): the kernel that ends the
    // operation stores a per-call value into the slab's flag word once its stores are visible; the
    // caller polls it instead of synchronizing the stream (falls back to that after kDonePollUs)
    bool flagged[2] = {false, false};
    bool served[2] = {false, false};  // posted to the resident small server: its stream, not the slot's
    uint32_t flag_val[2] = {0, 0};
    std::vector<void*> cdst(static_cast<size_t>(nfr));
    std::vector<const void*> csrc(static_cast<size_t>(nfr));
    std::vector<int64_t> clen(static_cast<size_t>(nfr));
    std::vector<void*> pdst, pdst2;  // the pack with tees
    std::vector<const void*> psrc;
    std::vector<int64_t> plen;
    auto drain = [&](int s) -> int {
        if (pending[s] < 0) return 0;
        int r = 0;
        if (served[s]) {
            const uint32_t* fw = done_word(st->slot[s].h_pin, st->cap);
            if (!poll_done(fw, flag_val[s])) r = ecamd_small_server_wait(fw, flag_val[s]);
        } else if (!(flagged[s] && poll_done(done_word(st->slot[s].h_pin, st->cap), flag_val[s]))) {
            r = wait_stream(st->slot[s].stream, chunk * nfr >= kSpinMinBytes);
        }
        flagged[s] = served[s] = false;
        if (r) return r;
        const int64_t off = pending[s] * chunk;
        const int64_t n = std::min(chunk, bs - off);
        for (int o = 0; o < R; o++) {
            cdst[o] = out[o] + off;
            csrc[o] = st->slot[s].h_pin + (K + o) * chunk;
            clen[o] = n;
        }
        ecamd_host_copy(R, cdst.data(), csrc.data(), clen.data());  // unpack (copy_pool.cpp)
        if (want_crc) {  // chunks drain in order, so the running CRCs extend by this chunk
            const auto* cc = reinterpret_cast<const uint32_t*>(st->slot[s].h_pin + crc_off);
            for (int f = 0; f < nfr; f++) crc[f] = crc_combine(t_crc.legacy, crc[f], cc[f], n);
        }
        pending[s] = -1;
        return 0;
    };
    for (int64_t c = 0; c < nchunks && rc == 0; c++) {
        const int s = static_cast<int>(c & 1);
        Slot& sl = st->slot[s];
        if ((rc = drain(s))) break;
        const int64_t off = c * chunk;
        const int64_t n = std::min(chunk, bs - off);
        // the pack's destination: the pinned slab, or (small calls) host-writable device memory
        char* const bar_in = bar ? bar_slab(sl) : nullptr;
        char* const pack = bar_in ? bar_in : sl.h_pin;
        if (t_tee.empty()) {
            for (int j = 0; j < K; j++) {
                cdst[j] = pack + j * chunk;
                csrc[j] = in[j] + off;
                clen[j] = n;
            }
            ecamd_host_copy(K, cdst.data(), csrc.data(), clen.data());  // pack
        } else {  // pack, the tees' bytes also to their second destination
            pdst.clear();
            pdst2.clear();
            psrc.clear();
            plen.clear();
            auto add = [&](void* d, void* d2, const void* sr, int64_t len) {
                pdst.push_back(d);
                pdst2.push_back(d2);
                psrc.push_back(sr);
                plen.push_back(len);
            };
            for (int j = 0; j < K; j++) {
                char* d = pack + j * chunk;
                Tee* te = find_tee(in[j]);
                const int64_t a = te && off < te->len ? std::min(n, te->len - off) : 0;
                if (a > 0) {
                    add(d, te->dst2 + off, te->src + off, a);
                    te->done += a;
                }
                if (a < n) add(d + a, nullptr, in[j] + off + a, n - a);
            }
            ecamd_host_copy2(static_cast<int>(pdst.size()), pdst.data(), pdst2.data(), psrc.data(), plen.data());
        }
        // One DMA each way per chunk (the slabs are [K inputs | R outputs] x chunk, contiguous):
        // for small fragments the per-call cost is API latency, not bytes.  A short last chunk
        // also moves the stale tail of each slot, which the kernel and the unpack never read.
        // zero copy: the kernel reads its inputs from / writes its outputs to the pinned slab itself
        char* const win = bar_in ? bar_in : zc_in ? sl.h_pin : sl.d_buf;
        char* const work = zc_out ? sl.h_pin : sl.d_buf;  // outputs (and the CRC pass)
        if (bar_in)  // the host's writes through the BAR reach the device before the launch's doorbell
            std::atomic_thread_fence(std::memory_order_seq_cst);
        else if (!zc_in)
            rc = ecamd_memcpy_async(sl.d_buf, sl.h_pin, (K - 1) * chunk + n, 0, sl.stream);
        auto* d_crc = reinterpret_cast<uint32_t*>(work + crc_off);
        bool fused = false;
        // fused only from 16 KiB of fragments as well: below, the fused epilogue (~5 us of kernel time)
        // costs more than zlib on the host (4 KiB RS(10,4) encode 27.8 vs 24.7 us, profiles/r06_lat_crc.json)
        const bool arm = g_done_flag && zc_out && nchunks == 1;
        if (arm) {
            flag_val[s] = ++st->seq;
            // the resident small server may take the launch when nothing else of this call is on the stream
            // (inputs read from the slab itself: no copy before it) -- with a checksum wanted, only a fused one
            // (a separate pass after it would run on the stream, unordered with the server)
            const int srv = g_server && zc_in && rc == 0 ? (want_crc ? 2 : 1) : 0;
            ecamd_done_flag_arm_server(done_word(sl.h_pin, st->cap), flag_val[s], srv);
        }
        if (rc == 0)
            rc = launch(ctx, win, work, chunk, n, sl.stream, crc_pass_ok && nchunks == 1 ? d_crc : nullptr,
                        t_crc.legacy, &fused);
        // the flag ends the call only when nothing follows the codec launch on the stream: a separate
        // CRC pass (want_crc, not fused) does
        if (arm) {
            const int taken = ecamd_done_flag_taken();
            flagged[s] = taken != 0 && rc == 0 && !(want_crc && !fused);
            served[s] = taken == 2;
        }
        if (rc == 0 && want_crc && !fused && zc_in && !zc_out)  // the CRC pass reads every fragment from the device slab
            rc = ecamd_memcpy_async(work, win, K * chunk, 0, sl.stream);
        if (rc == 0 && !zc_out)
            rc = ecamd_memcpy_async(sl.h_pin + K * chunk, sl.d_buf + K * chunk,
                                    (R - 1) * chunk + n, 1, sl.stream);
        if (rc == 0 && want_crc) {
            if (!fused)
                rc = ecamd_crc32(t_crc.legacy ? 1 : 0, work, 0, chunk, static_cast<int>(nfr), n, 1, d_crc, sl.stream);
            if (rc == 0 && !zc_out)
                rc = ecamd_memcpy_async(sl.h_pin + crc_off, d_crc, nfr * 4, 1, sl.stream);
        }
        pending[s] = c;
    }
    // below crc_pass_ok's size the frontend checksums the fragments with zlib after the call: the inputs'
    // CRC32s are taken here instead, while the kernel runs (the caller's buffers, which the call only
    // reads), and reach write_checksum through ecamd_percall_crc_lookup; the outputs' stay the frontend's
    std::vector<uint32_t> in_crc;
    if (rc == 0 && crc_armed && !want_crc && !t_crc.legacy && g_overlap_crc) {
        in_crc.resize(static_cast<size_t>(K));
        for (int j = 0; j < K; j++)
            in_crc[j] = static_cast<uint32_t>(::crc32(0, reinterpret_cast<const Bytef*>(in[j]), static_cast<uInt>(bs)));
    }
    for (int s = 0; s < 2; s++) {
        int r = drain(s);
        if (rc == 0) rc = r;
    }
    release(st);
    // the outputs' bytes changed: drop what was recorded for them (an earlier call's input, or an output
    // that is also an input: flat XOR applies in place)
    auto overlaps_out = [&](const void* p, int64_t len) {
        const char* a = static_cast<const char*>(p);
        for (int o = 0; o < R; o++)
            if (a < out[o] + bs && out[o] < a + len) return true;
        return false;
    };
    if (crc_armed) {
        auto& e = t_crc.entries;
        e.erase(std::remove_if(e.begin(), e.end(), [&](const auto& x) { return overlaps_out(x.ptr, x.len); }),
                e.end());
    }
    if (rc == 0 && want_crc) {  // outputs after inputs: a lookup takes the latest entry
        for (int j = 0; j < K; j++)
            if (!overlaps_out(in[j], bs)) t_crc.entries.push_back({in[j], bs, crc[j]});
        for (int o = 0; o < R; o++) t_crc.entries.push_back({out[o], bs, crc[K + o]});
    }
    if (rc == 0 && !in_crc.empty())
        for (int j = 0; j < K; j++)
            if (!overlaps_out(in[j], bs)) t_crc.entries.push_back({in[j], bs, in_crc[j]});
    return rc;
}

struct MapCtx {
    const ecamd_map* map;
    int K, R;
};

int launch_map(const void* vctx, char* din, char* dout, int64_t pitch, int64_t bytes, void* stream,
               uint32_t* crc_dst, bool legacy, bool* fused)
{
    const MapCtx* c = static_cast<const MapCtx*>(vctx);
    std::vector<int64_t> io(c->K), oo(c->R);
    for (int j = 0; j < c->K; j++) io[j] = j * pitch;
    for (int r = 0; r < c->R; r++) oo[r] = (c->K + r) * pitch;
    *fused = false;
    if (crc_dst && g_fuse_crc) {  // the codec launch with the checksums folded in, when the shape allows
        const int rc = ecamd_map_apply_strided_crc(c->map, din, io.data(), dout, oo.data(), bytes, legacy ? 1 : 0,
                                                   crc_dst, stream);
        if (rc <= 0) {
            *fused = rc == 0;
            return rc;
        }
    }
    return ecamd_map_apply_strided(c->map, din, 0, io.data(), dout, 0, oo.data(), bytes, 1, stream);
}

struct XorCtx {
    std::vector<uint32_t> masks;
    int K, R;
};

int launch_xor(const void* vctx, char* din, char* dout, int64_t pitch, int64_t bytes, void* stream,
               uint32_t* crc_dst, bool legacy, bool* fused)
{
    *fused = false;
    const XorCtx* c = static_cast<const XorCtx*>(vctx);
    std::vector<int64_t> io(c->K), oo(c->R);
    for (int j = 0; j < c->K; j++) io[j] = j * pitch;
    for (int r = 0; r < c->R; r++) oo[r] = (c->K + r) * pitch;
    if (crc_dst && g_fuse_crc) {  // the XOR launch with the checksums folded in, when the shape allows
        const int rc = ecamd_xor_apply_strided_crc(c->masks.data(), c->R, c->K, din, io.data(), dout, oo.data(),
                                                   bytes, legacy ? 1 : 0, crc_dst, stream);
        if (rc <= 0) {
            *fused = rc == 0;
            return rc;
        }
    }
    return ecamd_xor_apply_strided(c->masks.data(), c->R, c->K, din, 0, io.data(), dout, 0, oo.data(),
                                   bytes, 1, stream);
}

}  // namespace

extern "C" {

int ecamd_host_map_apply(const int* coeff, int R, int K, const void* const* in,
                         void* const* out, int64_t blocksize)
{
    if (R <= 0 || blocksize <= 0) return 0;
    if (K <= 0) {
        for (int r = 0; r < R; r++) std::memset(out[r], 0, static_cast<size_t>(blocksize));
        return 0;
    }
    const int dev = pick_device();
    if (dev < 0) return note_exec(ECAMD_ENODEV);
    DeviceScope scope(dev);
    if (scope.rc) return note_exec(scope.rc);
    int rc = 0;
    auto mh = cached_map(dev, coeff, R, K, &rc);
    if (!mh) return note_exec(rc ? rc : ECAMD_EINVAL);
    MapCtx ctx{mh->map, K, R};
    return note_exec(run_chunked(dev, K, R, reinterpret_cast<const char* const*>(in),
                                 reinterpret_cast<char* const*>(out), blocksize, &ctx, launch_map, true));
}

int ecamd_host_xor_apply(const uint64_t* sources, int R, int nbuf, const void* const* bufs,
                         void* const* out, int64_t blocksize)
{
    if (R <= 0 || blocksize <= 0) return 0;
    // compact the referenced originals into input slots 0..K-1
    uint64_t used = 0;
    for (int r = 0; r < R; r++) used |= sources[r];
    std::vector<const char*> in;
    std::vector<int> slot(64, -1);
    for (int b = 0; b < nbuf && b < 64; b++)
        if ((used >> b) & 1u) {
            slot[b] = static_cast<int>(in.size());
            in.push_back(static_cast<const char*>(bufs[b]));
        }
    if (in.size() > 32) return ECAMD_EINVAL;
    XorCtx ctx;
    ctx.K = static_cast<int>(in.size());
    ctx.R = R;
    for (int r = 0; r < R; r++) {
        uint32_t mk = 0;
        for (int b = 0; b < nbuf && b < 64; b++)
            if ((sources[r] >> b) & 1u) mk |= 1u << slot[b];
        ctx.masks.push_back(mk);
    }
    if (ctx.K == 0) {
        for (int r = 0; r < R; r++) std::memset(out[r], 0, static_cast<size_t>(blocksize));
        return 0;
    }
    // outputs may alias inputs: results land in pinned memory first and are copied back only
    // after the whole chunk's inputs were packed, so every output sees the ORIGINAL inputs.
    const int dev = pick_device();
    if (dev < 0) return note_exec(ECAMD_ENODEV);
    DeviceScope scope(dev);
    if (scope.rc) return note_exec(scope.rc);
    return note_exec(run_chunked(dev, ctx.K, R, in.data(), reinterpret_cast<char* const*>(out),
                                 blocksize, &ctx, launch_xor, true));
}

int ecamd_percall_crc_arm(int legacy)
{
    t_crc.armed = true;
    t_crc.legacy = legacy != 0;
    t_crc.entries.clear();
    return 0;
}

int ecamd_percall_crc_lookup(const void* ptr, int64_t len, uint32_t* crc)
{
    for (auto it = t_crc.entries.rbegin(); it != t_crc.entries.rend(); ++it)
        if (it->ptr == ptr && it->len == len) {
            *crc = it->crc;
            return 0;
        }
    return -1;
}

void ecamd_percall_crc_disarm(void)
{
    t_crc.armed = false;
    t_crc.entries.clear();
}

void ecamd_percall_reset(void) { t_exec_rc = 0; }

int ecamd_percall_tee_arm(int n, const void* const* key, const void* const* src, void* const* dst2,
                          const int64_t* len)
{
    t_tee.clear();
    if (n < 0 || n > 64 || (n > 0 && (!key || !src || !dst2 || !len))) return ECAMD_EINVAL;
    for (int i = 0; i < n; i++) {  // one entry per argument (done[i] of disarm); null ones never match
        const bool ok = key[i] && src[i] && dst2[i] && len[i] > 0;
        t_tee.push_back({ok ? key[i] : nullptr, static_cast<const char*>(src[i]), static_cast<char*>(dst2[i]),
                         ok ? len[i] : 0});
    }
    return 0;
}

void ecamd_percall_tee_disarm(int64_t* done)
{
    if (done)
        for (size_t i = 0; i < t_tee.size(); i++) done[i] = t_tee[i].done;
    t_tee.clear();
}

int ecamd_percall_status(void) { return t_exec_rc; }

int ecamd_fault_inject(const char* site, int count)
{
    if (!site || std::strcmp(site, "staging") != 0 || count < 0) return ECAMD_EINVAL;
    g_fail_staging.store(count);
    return 0;
}

}  // extern "C"
