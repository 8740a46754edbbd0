// copy_pool.cpp -- host copies of one per-call request spread over a few helper threads.
//
// A drop-in call (liberasurecode_encode / _decode, the per-call codec) moves every byte of the
// object through host memory three times: object -> fragments (frontend), fragments -> pinned
// staging (pack), staging -> fragments (unpack), and the reverse for decode.  One core copies
// ~10 GB/s, so a single caller -- a Swift proxy worker is one thread -- is bound by its own
// memcpy, not by PCIe.  ecamd_host_copy splits a batch of copies into pieces that the caller and
// ECAMD_COPY_THREADS helpers (default 4, 0 = off) take from a shared counter.  The helpers serve
// a process whose calls come from ONE thread at a time (a Swift proxy worker): when another
// thread called within the last few milliseconds, or another request holds the helpers, the
// caller copies alone -- with many concurrent callers every core already has a caller's copy to
// run, and the helpers only added contention (tools/percall_ab.py: 8 threads 29.6 -> 25 GiB/s).
// Helpers poll for the next request for a short while before they sleep, so the pack, unpack
// and object copies of one call do not each pay a thread wake-up.  After fork() the child copies
// alone (the helpers live in the parent only).
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <functional>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "ecamd.h"
#include "ecamd_host.h"

namespace {

constexpr int64_t kPiece = 256 << 10;     // bytes per piece handed to one thread
// Smaller batches are copied by the caller alone (ECAMD_COPY_MIN_KIB, default 2 MiB: 1 MiB objects,
// 10 x 100 KiB fragments, measured slower with the helpers than without before they polled)
int64_t parallel_min()
{
    static const int64_t bytes = [] {
        const char* s = std::getenv("ECAMD_COPY_MIN_KIB");
        const long v = s && *s ? std::atol(s) : 0;
        return v > 0 ? static_cast<int64_t>(v) << 10 : int64_t(2) << 20;
    }();
    return bytes;
}
constexpr auto kHelperPoll = std::chrono::microseconds(300);  // helper polling before it sleeps
constexpr int64_t kSoloNs = 5000000;  // another caller thread within 5 ms: copy alone

struct Piece {
    char* dst;
    const char* src;
    int64_t len;
    char* dst2;  // also written (ecamd_host_copy2), or null
};

// dst <- src, then dst2 <- src through the cache: the second copy reads the piece just written
// (256 KiB, resident in the core's L2), so the source leaves DRAM once for both destinations.
void copy_piece(const Piece& q)
{
    if (q.len <= 0) return;
    if (!q.dst2) {
        std::memcpy(q.dst, q.src, static_cast<size_t>(q.len));
        return;
    }
    for (int64_t off = 0; off < q.len; off += kPiece) {
        const size_t n = static_cast<size_t>(std::min(kPiece, q.len - off));
        std::memcpy(q.dst2 + off, q.src + off, n);
        std::memcpy(q.dst + off, q.dst2 + off, n);
    }
}

struct Pool {
    std::mutex busy;  // held by the one request using the helpers
    std::mutex mu;
    std::condition_variable wake, idle;
    std::vector<Piece> job;
    std::atomic<int64_t> next{0};
    std::atomic<int64_t> gen{0};  // written under mu, polled without it
    std::atomic<uint64_t> last_caller{0};
    std::atomic<int64_t> other_caller_ns{INT64_MIN / 2};  // when a second caller thread was last seen
    int working = 0;  // helpers inside the current generation
    int threads = 0;
    std::atomic<pid_t> owner{0};  // process that started the helpers
    std::atomic<bool> started{false};
};

Pool& pool()
{
    static Pool* p = new Pool();  // never destroyed: helpers may outlive static destructors
    return *p;
}

int configured_threads()
{
    const char* s = std::getenv("ECAMD_COPY_THREADS");
    if (!s || !*s) return 4;
    return std::max(0, std::min(64, std::atoi(s)));
}

void drain(Pool& p)
{
    const int64_t n = static_cast<int64_t>(p.job.size());
    for (int64_t i = p.next.fetch_add(1); i < n; i = p.next.fetch_add(1)) copy_piece(p.job[i]);
}

void helper(Pool* p)
{
    int64_t seen = 0;
    for (;;) {
        const auto until = std::chrono::steady_clock::now() + kHelperPoll;
        while (p->gen.load() == seen && std::chrono::steady_clock::now() < until) __builtin_ia32_pause();
        {
            std::unique_lock<std::mutex> lk(p->mu);
            p->wake.wait(lk, [&] { return p->gen.load() != seen; });
            seen = p->gen.load();
            p->working++;
        }
        drain(*p);
        {
            std::lock_guard<std::mutex> lk(p->mu);
            if (--p->working == 0) p->idle.notify_all();
        }
    }
}

// Starts the helpers once per process; false when there are none (disabled, forked child, or a
// thread could not be created).
bool ensure_started(Pool& p)
{
    // a forked child must not touch the mutexes: a parent thread may have held them at fork()
    if (p.started.load() && p.owner.load() != getpid()) return false;
    std::lock_guard<std::mutex> lk(p.mu);
    if (p.started.load()) return p.threads > 0;
    p.owner.store(getpid());
    p.started.store(true);
    const int want = configured_threads();
    for (int i = 0; i < want; i++) {
        try {
            std::thread(helper, &p).detach();
            p.threads++;
        } catch (...) {
            break;
        }
    }
    return p.threads > 0;
}

int64_t now_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// True while calls come from one thread only: records this caller and reports whether a
// different thread called within the last kSoloNs.
bool solo_caller(Pool& p)
{
    static thread_local const uint64_t me =
        std::hash<std::thread::id>()(std::this_thread::get_id()) | 1u;
    const int64_t t = now_ns();
    const uint64_t prev = p.last_caller.exchange(me);
    if (prev != 0 && prev != me) p.other_caller_ns.store(t);
    return t - p.other_caller_ns.load() > kSoloNs;
}

void copy_serial(int n, void* const* dst, void* const* dst2, const void* const* src, const int64_t* len)
{
    for (int i = 0; i < n; i++)
        copy_piece({static_cast<char*>(dst[i]), static_cast<const char*>(src[i]), len[i],
                    dst2 ? static_cast<char*>(dst2[i]) : nullptr});
}

int copy_batch(int n, void* const* dst, void* const* dst2, const void* const* src, const int64_t* len)
{
    if (n <= 0) return 0;
    if (!dst || !src || !len) return ECAMD_EINVAL;
    int64_t total = 0;
    for (int i = 0; i < n; i++) total += std::max<int64_t>(0, len[i]);
    Pool& p = pool();
    const bool solo = solo_caller(p);
    if (total < parallel_min() || !solo || !ensure_started(p) || !p.busy.try_lock()) {
        copy_serial(n, dst, dst2, src, len);
        return 0;
    }
    {
        std::unique_lock<std::mutex> lk(p.mu);
        // helpers still finishing the previous generation hold no piece of it any more (the
        // counter ran out), but wait for them so the job vector can be rebuilt safely
        p.idle.wait(lk, [&] { return p.working == 0; });
        p.job.clear();
        for (int i = 0; i < n; i++)
            for (int64_t off = 0; off < len[i]; off += kPiece)
                p.job.push_back({static_cast<char*>(dst[i]) + off,
                                 static_cast<const char*>(src[i]) + off,
                                 std::min(kPiece, len[i] - off),
                                 dst2 && dst2[i] ? static_cast<char*>(dst2[i]) + off : nullptr});
        p.next.store(0);
        p.gen++;
    }
    p.wake.notify_all();
    drain(p);
    {
        std::unique_lock<std::mutex> lk(p.mu);
        p.idle.wait(lk, [&] { return p.working == 0; });
    }
    p.busy.unlock();
    return 0;
}

}  // namespace

extern "C" int ecamd_host_copy(int n, void* const* dst, const void* const* src, const int64_t* len)
{
    return copy_batch(n, dst, nullptr, src, len);
}

extern "C" int ecamd_host_copy2(int n, void* const* dst, void* const* dst2, const void* const* src,
                                const int64_t* len)
{
    return copy_batch(n, dst, dst2, src, len);
}
