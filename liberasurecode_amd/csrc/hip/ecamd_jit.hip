// ecamd_jit.hip -- run-time specialised bitsliced GF(2^16) kernels (host/bitslice.hpp).
//
// The XOR network of a bitsliced map depends on every coefficient, so its kernel is generated for
// the matrix and compiled at run time.  Both steps -- the network search (tens to hundreds of ms)
// and the hiprtc compile (seconds) -- run in a child process (ecamd_jitc, next to this library),
// never on a caller's thread or in this process: a GPU process that exits while a compile is in
// flight simply abandons it, and hiprtc's runtime never shares an address space with the GPU
// work.  Code objects land in a disk cache ($ECAMD_JIT_CACHE, else /tmp/ecamd-jit-<uid>) keyed by
// a hash of the request and of the generator itself, so later processes load them at once.  Knob "bitslice": 1 (default)
// launches the LDS-table kernel until the code object is ready, 2 waits for it (tests, bench), 0
// never uses the bitsliced form; ecamd_bitslice_wait() waits for every compile started so far.
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../host/bitslice.hpp"
#include "ecamd.h"
#include "ecamd_internal.hpp"

extern char** environ;

namespace ecamd {
namespace {

// Temporaries per input, first choice first: 96 (the search stops by itself near 80 on C5 maps)
// fits the register file at 2 waves per SIMD for the C5 encode and decode networks (230-248 VGPRs,
// no scratch: each temporary is computed right before its first use); a network that spills (the
// compiler's schedule decides, not the count alone) is rebuilt with the next.
constexpr int kCaps[] = {96, 64, 40, 16};
constexpr int kNumCaps = static_cast<int>(sizeof(kCaps) / sizeof(kCaps[0]));

// First cap to try: the largest not above $ECAMD_JIT_CAP_MAX (A/B experiments), else kCaps[0].
int first_cap_index()
{
    static const int idx = [] {
        const char* env = std::getenv("ECAMD_JIT_CAP_MAX");
        const int v = env ? std::atoi(env) : 0;
        int i = 0;
        while (v > 0 && i + 1 < kNumCaps && kCaps[i] > v) i++;
        return i;
    }();
    return idx;
}

std::string helper_path()
{
    static std::string path;
    static std::once_flag once;
    std::call_once(once, [] {
        Dl_info info{};
        if (dladdr(reinterpret_cast<void*>(&helper_path), &info) && info.dli_fname) {
            std::string lib(info.dli_fname);
            const size_t slash = lib.rfind('/');
            path = (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/ecamd_jitc";
        }
        if (access(path.c_str(), X_OK) != 0) path.clear();
    });
    return path;
}

// Code objects shipped with the library (<libdir>/jit, written at build time by
// ecamd_bitslice_prebuild for the maps the BASELINE configurations run): looked up before the
// per-user cache, so those maps take the bitsliced kernel at their first launch without a compile
// -- and without ecamd_jitc or libhiprtc.  Used only if it is a real directory owned by this user
// or root that nobody else can write (its code objects run on the GPU, like the library beside it).
std::string shipped_dir()
{
    static std::string dir;
    static std::once_flag once;
    std::call_once(once, [] {
        Dl_info info{};
        if (!dladdr(reinterpret_cast<void*>(&shipped_dir), &info) || !info.dli_fname) return;
        std::string lib(info.dli_fname);
        const size_t slash = lib.rfind('/');
        const std::string d = (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/jit";
        struct stat st {};
        if (lstat(d.c_str(), &st) == 0 && S_ISDIR(st.st_mode) && (st.st_uid == getuid() || st.st_uid == 0) &&
            !(st.st_mode & 022))
            dir = d;
    });
    return dir;
}

// Keep the disk cache to the newest $ECAMD_JIT_CACHE_MAX (4096) code objects and drop temporaries
// older than an hour (a compile stopped mid-way): run once per process.
void prune_cache(const std::string& dir)
{
    const char* env = std::getenv("ECAMD_JIT_CACHE_MAX");
    const long cap = env && std::atol(env) > 0 ? std::atol(env) : 4096;
    std::vector<std::pair<time_t, std::string>> cos;
    if (DIR* d = opendir(dir.c_str())) {
        while (const dirent* ent = readdir(d)) {
            const std::string name(ent->d_name);
            if (name.compare(0, 3, "bs_") != 0) continue;
            struct stat st {};
            const std::string path = dir + "/" + name;
            if (stat(path.c_str(), &st) != 0) continue;
            if (name.find(".tmp.") != std::string::npos || name.find(".req.") != std::string::npos) {
                if (st.st_mtime + 3600 < time(nullptr)) std::remove(path.c_str());  // left by a killed compile
                continue;
            }
            if (name.size() > 3 && name.compare(name.size() - 3, 3, ".co") == 0) cos.emplace_back(st.st_mtime, path);
        }
        closedir(d);
    }
    if (static_cast<long>(cos.size()) <= cap) return;
    std::sort(cos.begin(), cos.end());
    for (size_t i = 0; i + static_cast<size_t>(cap) < cos.size(); i++) {
        std::remove(cos[i].second.c_str());
        std::remove((cos[i].second.substr(0, cos[i].second.size() - 3) + ".hip").c_str());
    }
}

std::string cache_dir()
{
    static std::string dir;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* env = std::getenv("ECAMD_JIT_CACHE");
        dir = env && *env ? env : "/tmp/ecamd-jit-" + std::to_string(getuid());
        mkdir(dir.c_str(), 0700);
        // Code objects from this directory run on the GPU: use it only if it is a real directory of
        // ours that nobody else can write; otherwise a fresh private one (no sharing across processes).
        struct stat st {};
        if (lstat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode) || st.st_uid != getuid() || (st.st_mode & 022)) {
            char tmpl[] = "/tmp/ecamd-jit-XXXXXX";
            dir = mkdtemp(tmpl) ? tmpl : "";
        }
        if (!dir.empty()) prune_cache(dir);
    });
    return dir;
}

uint64_t fnv1a(const std::string& s)
{
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h;
}

// The code object's target: the device's architecture name without feature flags ("gfx950"), so
// the cache key and the compile follow the GPU rather than the build (kept per device).
std::string device_arch(int dev)
{
    static std::mutex mu;
    static std::map<int, std::string> names;
    std::lock_guard<std::mutex> lk(mu);
    auto it = names.find(dev);
    if (it != names.end()) return it->second;
    std::string arch = "gfx950";
    hipDeviceProp_t p{};
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.gcnArchName[0]) {
        arch = p.gcnArchName;
        arch = arch.substr(0, arch.find(':'));
    }
    (void)hipGetLastError();
    return names[dev] = arch;
}

bool file_exists(const std::string& path)
{
    struct stat st {};
    return stat(path.c_str(), &st) == 0;
}

bool read_file(const std::string& path, std::string& out)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return !out.empty();
}

struct BsEntry {
    std::vector<int> coeff;
    int R = 0, K = 0;
    int depth = 0;        // bitslice_source: 0 register loads, 2 / 4 LDS ring
    bool copy = false;    // copy-through variant (framed paths)
    int crc = 0;          // copy-through + payload CRC32 variant: position table sets (1, 2, 4), 0 = none;
                          //   + 8: lane-shift fold, + 16: nibble piece tables
    bool wave = false;    // one-wave workgroups, 4 KiB tiles (BitsliceStyle::threads 64)
    std::vector<int> shifts;  // copy-through inputs' byte shifts (BitsliceStyle::in_shift), empty: none
    int prefetch = 0;         // one-wave form: chunks of the next input loaded ahead (BitsliceStyle::prefetch)
    BsOcc occ;                // one-wave form: amdgpu_waves_per_eu and input barrier (bitslice.hpp)
    int cap_index = 0;    // into kCaps: shared temporaries allowed (fewer: fewer registers)
    std::string arch;     // target of the code object (the requesting device's gcnArchName)
    std::string co_path;  // cache file of the code object
    pid_t pid = -1;       // compiler child while running
    time_t started = 0;   // when the child was spawned
    int state = 0;        // 0 compiling, 2 waiting for a compiler slot, 1 code object ready, -1 failed
    std::string code;
    bool shipped = false;  // code object from the library's own jit/ directory
    std::map<int, hipFunction_t> fn;  // per device; nullptr: unusable there
    std::vector<std::pair<int, hipModule_t>> modules;  // (device, module), spilled ones included
    uint64_t last_use = 0;
    // The last launch of this entry's kernels on each (device, stream): an event recorded after it
    // (bitslice_launch), so unloading waits for exactly those launches, not for whole devices.
    std::mutex ev_mu;
    std::map<std::pair<int, hipStream_t>, hipEvent_t> last_launch;

    // Reached only for an entry evicted from the cache (the cache itself is never destroyed, so
    // nothing here runs at process exit) once its last holder -- a launch in progress keeps one --
    // has let go, and never under g_jit_mu: no launch of its functions can still be enqueued; wait
    // for the recorded ones, then unload the modules.
    ~BsEntry()
    {
        int cur = -1;
        (void)hipGetDevice(&cur);
        for (const auto& kv : last_launch) {
            if (hipSetDevice(kv.first.first) != hipSuccess) continue;
            (void)hipEventSynchronize(kv.second);
            (void)hipEventDestroy(kv.second);
        }
        for (const auto& dm : modules) {
            if (hipSetDevice(dm.first) != hipSuccess) continue;
            (void)hipModuleUnload(dm.second);
        }
        if (cur >= 0) (void)hipSetDevice(cur);
        (void)hipGetLastError();
    }
};

std::atomic<long long> g_bs_launches{0};  // bitsliced kernel launches enqueued by this process

// Matrices with a bitsliced kernel (or one on the way), the least recently used evicted past the
// "bitslice_entries" knob (256); heap objects never destroyed, so no HIP call runs during static
// destruction.
std::mutex g_jit_mu;  // guards g_jit, g_running, g_clock and every entry
auto& g_jit = *new std::map<std::vector<int>, std::shared_ptr<BsEntry>>();
auto& g_running = *new std::vector<std::shared_ptr<BsEntry>>();  // entries whose compiler child runs
uint64_t g_clock = 0;

// Compiler children at once ($ECAMD_JIT_JOBS, default 2): a burst of new erasure patterns queues
// rather than loading the host with one compile per pattern.
size_t max_jobs()
{
    static size_t n = [] {
        const char* env = std::getenv("ECAMD_JIT_JOBS");
        const int v = env ? std::atoi(env) : 0;
        return static_cast<size_t>(v >= 1 && v <= 64 ? v : 2);
    }();
    return n;
}

// Identifies the generator: the sources it emits for a tiny map in both load modes, and the
// search settings -- a changed generator never reuses an old cache entry.
const std::string& generator_fingerprint()
{
    static std::string fp;
    static std::once_flag once;
    std::call_once(once, [] {
        const BitsliceNet tiny = bitslice_network({3}, 1, 1, 0);
        const BitsliceNet tiny5 = bitslice_network({3, 5, 7, 9, 11}, 5, 1, 0);  // the fold-each form
        BitsliceStyle copy, crc, lane, nib, wave;
        wave.threads = 64;
        wave.waves = 2;
        copy.copy_through = true;
        crc.copy_through = crc.crc = true;
        lane = crc;
        lane.crc_lane = true;
        nib = lane;
        nib.crc_nib = true;
        BitsliceStyle shifted = copy, crc_shifted = lane, wave_pf = wave, wave_ring = wave, wave_occ = wave,
                      crc_wave = lane;
        crc_wave.crc_wave = 6;
        crc_wave.crc_mix = true;
        crc_wave.crc_pos = 2;
        crc_wave.waves = 3;
        wave_occ.waves_max = 8;
        wave_occ.input_barrier = true;
        wave_pf.prefetch = 4;
        shifted.in_shift = {6};
        crc_shifted.in_shift = {10};
        BitsliceStyle copy_ring = shifted;  // the one-wave copy-through LDS ring (knob bs_copy_ring)
        copy_ring.threads = 64;
        copy_ring.waves = 2;
        fp = bitslice_source(tiny, 0) + bitslice_source(tiny, 2) + bitslice_source(tiny, 0, copy) +
             bitslice_source(tiny, 0, crc) + bitslice_source(tiny, 0, lane) + bitslice_source(tiny5, 0, crc) +
             bitslice_source(tiny5, 0, nib) + bitslice_source(tiny, 0, wave) + bitslice_source(tiny, 0, shifted) +
             bitslice_source(tiny, 0, crc_shifted) + bitslice_source(tiny5, 0, wave_pf) +
             bitslice_source(tiny, 2, wave_ring) + bitslice_source(tiny, 0, wave_occ) +
             bitslice_source(tiny, 0, crc_wave) + bitslice_source(tiny, 2, copy_ring) + kBsNetworkVersion;
    });
    return fp;
}

// At exit, stop the compilers this process started and has not reaped (their results would only
// land in the cache; a half-written one never does -- jitc renames whole files into place).  The
// exact PIDs, never a pattern; skipped if another thread holds the lock, or with
// ECAMD_JIT_DETACH=1 (short-lived processes that want later ones to find the kernels compiled).
void stop_children_at_exit()
{
    const char* detach = std::getenv("ECAMD_JIT_DETACH");
    if ((detach && std::atoi(detach)) || !g_jit_mu.try_lock()) return;
    for (const auto& ep : g_running)
        if (ep->pid > 0) kill(ep->pid, SIGTERM);
    g_jit_mu.unlock();
}

// The compile request of e's kernel at kCaps[e.cap_index], and the name of its code object (a hash
// of the request, the target and the generator: the same in the shipped and the per-user cache).
std::string request_of(const BsEntry& e)
{
    // (+ 16: crc_mix, + 32 * dwords of a piece on nibble tables, + 128: the last dword's lookups via L1)
    const int cw = (e.crc & 32) ? ((e.crc >> 6) & 15) | ((e.crc & 1024) ? 16 : 0) | (((e.crc >> 11) & 3) << 5) |
                                      ((e.crc & 8192) ? 128 : 0)
                                : 0;
    return bitslice_request(e.coeff, e.R, e.K, kCaps[e.cap_index], e.depth, e.copy, e.crc > 0,
                            e.crc > 0 ? (e.crc & 7) : 1, (e.crc & 8) != 0, (e.crc & 16) != 0, e.wave, &e.shifts,
                            e.prefetch, e.wave || e.occ.threads || cw ? &e.occ : nullptr, cw);
}
std::string object_name(const BsEntry& e)
{
    char name[40];
    std::snprintf(name, sizeof(name), "bs_%016llx",
                  static_cast<unsigned long long>(fnv1a(generator_fingerprint() + "arch " + e.arch + "\n" + request_of(e))));
    return name;
}

// Start (or skip, when shipped or cached) the build of e's kernel at kCaps[e.cap_index]; queue it
// (state 2) while max_jobs() compilers run, unless `force`.  Caller holds the lock.
void start_compile(const std::shared_ptr<BsEntry>& ep, bool force)
{
    BsEntry& e = *ep;
    const std::string req = request_of(e);
    const std::string name = object_name(e);
    e.pid = -1;
    e.code.clear();
    const std::string shipped = shipped_dir();
    if (!shipped.empty() && read_file(shipped + "/" + name + ".co", e.code)) {  // built with the library
        e.co_path = shipped + "/" + name + ".co";
        e.state = 1;
        e.shipped = true;
        return;
    }
    e.shipped = false;
    const std::string dir = cache_dir();
    if (dir.empty()) {  // no usable cache directory: the LDS tables serve this matrix
        e.state = -1;
        return;
    }
    const std::string base = dir + "/" + name;
    e.co_path = base + ".co";
    if (read_file(e.co_path, e.code)) {  // compiled before, here or by another process
        e.state = 1;
        return;
    }
    e.state = -1;
    const std::string helper = helper_path();
    if (helper.empty()) return;
    if (!force && g_running.size() >= max_jobs()) {
        e.state = 2;
        return;
    }
    const std::string req_path = base + ".req." + std::to_string(getpid());  // this process's; jitc consumes it
    {
        const std::string tmp = req_path + ".tmp." + std::to_string(getpid());
        std::ofstream f(tmp);
        f << req;
        f.close();
        if (!f || std::rename(tmp.c_str(), req_path.c_str()) != 0) return;
    }
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_addopen(&fa, 1, "/dev/null", O_WRONLY, 0);  // keep our stdout clean
    posix_spawn_file_actions_addclosefrom_np(&fa, 3);  // no GPU / socket descriptors in the child
    const char* argv[] = {helper.c_str(), req_path.c_str(), e.co_path.c_str(), e.arch.c_str(), nullptr};
    pid_t pid = -1;
    if (posix_spawn(&pid, helper.c_str(), &fa, nullptr, const_cast<char* const*>(argv), environ) == 0) {
        e.pid = pid;
        e.started = time(nullptr);
        e.state = 0;
        g_running.push_back(ep);
        static std::once_flag once;
        std::call_once(once, [] { std::atexit(stop_children_at_exit); });
    }
    posix_spawn_file_actions_destroy(&fa);
}

// A compile whose child cannot be waited for (reaped by the host process: SIGCHLD ignored, or a
// waitpid(-1) elsewhere) counts as running while its pid exists, for at most this long.
constexpr int kOrphanSeconds = 300;

// Advance an entry without blocking: reap its compiler child, or start a queued compile when a
// slot is free (or at once when `force`).  Caller holds the lock.
void poll_compile(const std::shared_ptr<BsEntry>& ep, bool force)
{
    BsEntry& e = *ep;
    if (e.state == 2) start_compile(ep, force);
    if (e.state != 0) return;
    int status = 0;
    pid_t r;
    do {
        r = waitpid(e.pid, &status, WNOHANG);
    } while (r < 0 && errno == EINTR);
    if (r == 0) return;  // still running
    if (r < 0 && errno == ECHILD && !file_exists(e.co_path) && kill(e.pid, 0) == 0 &&
        time(nullptr) - e.started < kOrphanSeconds)
        return;  // not ours to reap any more, but still there: keep waiting for its code object
    e.pid = -1;
    g_running.erase(std::remove(g_running.begin(), g_running.end(), ep), g_running.end());
    // a child reaped elsewhere, or another process compiling the same request, may still have
    // produced the code object
    e.state = read_file(e.co_path, e.code) ? 1 : -1;
}

// Block until the entry's compile (started now if queued) has finished, polling with the lock
// released so other threads' launches never wait behind a compile.  `lk` holds g_jit_mu.
void wait_compile(std::unique_lock<std::mutex>& lk, const std::shared_ptr<BsEntry>& ep)
{
    poll_compile(ep, true);
    while (ep->state == 0) {
        lk.unlock();
        usleep(2000);
        lk.lock();
        poll_compile(ep, true);
    }
}

// The canonical parameters of a request (and the entry's key): whatever the caller asked, equal
// kernels get equal requests.  Returns the key.
std::vector<int> normalize(const std::vector<int>& coeff, int R, int K, int& depth, bool& copy, int& crc,
                           bool& wave, const std::vector<int>* in_shift, int& prefetch, std::vector<int>& shifts,
                           BsOcc& occ)
{
    if (crc) {  // position sets 1 / 2 / 4, + 8 for the lane-shift fold, + 16 for nibble piece tables;
        // + 32 for one-wave tiles (with the lane fold, byte tables) in workgroups of (crc >> 6) waves
        const int pos = crc & 7;
        const int cw = (crc & 32) ? std::clamp((crc >> 6) & 15, 1, 15) : 0;
        crc = (pos >= 4 ? 4 : pos >= 2 ? 2 : 1) | (cw ? 8 | 32 | (cw << 6) | (crc & (1024 | 6144)) : crc & 24);
    }
    copy = copy || crc;
    wave = wave && !crc;
    // the LDS ring: plain maps, and copy-through maps in one-wave tiles (not the crc variant)
    depth = crc || (copy && !wave) ? 0 : bitslice_depth(depth, K);
    prefetch = depth ? 0
               : (wave || crc) && (prefetch == 2 || prefetch == 4) ? prefetch
               : (crc & 32) && prefetch == 3 ? 3  // the one-wave crc form: two inputs ahead
               : (copy && !crc && !wave && prefetch == 1) ? 1 : 0;
    if (crc & 32) {  // the one-wave crc form keeps its occupancy (waves per SIMD, cap, barrier)
        occ.threads = 0;
    } else if (!wave) {  // the multi-wave forms: only the plain register form's workgroup size
        const int th = occ.threads;
        occ = BsOcc{};
        if (!copy && !crc && depth == 0 && (th == 128 || th == 512)) occ.threads = th;
    }
    occ.wmin = std::clamp(occ.wmin, 1, 8);
    occ.wmax = std::clamp(occ.wmax, occ.wmin, 8);
    std::vector<int> key = {R, K, depth, (copy ? 1 : 0) | (crc << 1) | (wave ? 256 : 0) | (prefetch << 9),
                            occ.wmin, occ.wmax, occ.barrier ? 1 : 0, occ.threads};
    key.insert(key.end(), coeff.begin(), coeff.end());
    shifts.clear();  // realigned copy-through inputs: their own kernel (and cache entry)
    if (copy && in_shift)
        for (int j = 0; j < K; j++) {
            const int v = j < static_cast<int>(in_shift->size()) ? ((*in_shift)[static_cast<size_t>(j)] & 15) : 0;
            shifts.push_back(v);
        }
    if (std::find_if(shifts.begin(), shifts.end(), [](int v) { return v != 0; }) == shifts.end()) shifts.clear();
    if (!shifts.empty()) {
        key.push_back(-1);
        key.insert(key.end(), shifts.begin(), shifts.end());
    }
    return key;
}

// First kCaps index of a new entry: the 4-waves-per-SIMD build of maps with up to 4 outputs (16 KiB
// tiles) has half the registers, so it starts at 40 temporaries.
int first_cap(int R, int crc, bool wave)
{
    return std::max(first_cap_index(), bitslice_waves_per_simd(R, crc > 0) > 2 && !wave ? 2 : 0);
}

// The code object's private segment (scratch) size from its metadata note (msgpack: the key string
// ".private_segment_fixed_size" followed by an unsigned integer): > 0 means the network spilled.
long code_object_scratch(const std::string& code)
{
    static const std::string key = ".private_segment_fixed_size";
    size_t pos = code.find(key);
    if (pos == std::string::npos) return -1;
    pos += key.size();
    if (pos >= code.size()) return -1;
    const auto b = [&](size_t i) { return static_cast<unsigned char>(code[i]); };
    const unsigned char t = b(pos);
    if (t < 0x80) return t;
    if (t == 0xcc && pos + 1 < code.size()) return b(pos + 1);
    if (t == 0xcd && pos + 2 < code.size()) return (b(pos + 1) << 8) | b(pos + 2);
    if (t == 0xce && pos + 4 < code.size())
        return static_cast<long>((static_cast<unsigned long>(b(pos + 1)) << 24) | (b(pos + 2) << 16) |
                                 (b(pos + 3) << 8) | b(pos + 4));
    return -1;
}

}  // namespace

// Build time (no GPU): the code object of one map into `dir` (the library's jit/ directory), under the
// name the run-time lookup computes, through ecamd_jitc run synchronously; a network that spills is
// built again at the next cap, as the run time would ask for it.  1: present (built now or before),
// 0: this form never takes a bitsliced kernel, < 0: the helper is missing or failed.
int bitslice_prebuild(const std::vector<int>& coeff, int R, int K, int depth, bool copy, int crc, bool wave,
                      const std::vector<int>* in_shift, int prefetch, const BsOcc& occ_in, const std::string& arch,
                      const std::string& dir)
{
    if (R <= 0 || R > kBsMaxR || K <= 0 || K > kBsMaxK) return 0;
    const std::string helper = helper_path();
    if (helper.empty()) return -1;
    BsEntry e;
    std::vector<int> shifts;
    BsOcc occ = occ_in;
    normalize(coeff, R, K, depth, copy, crc, wave, in_shift, prefetch, shifts, occ);
    e.occ = occ;
    e.coeff = coeff;
    e.R = R;
    e.K = K;
    e.depth = depth;
    e.copy = copy;
    e.crc = crc;
    e.wave = wave;
    e.shifts = shifts;
    e.prefetch = prefetch;
    e.arch = arch;
    for (e.cap_index = first_cap(R, crc, wave); e.cap_index < kNumCaps; e.cap_index++) {
        const std::string co = dir + "/" + object_name(e) + ".co";
        std::string code;
        if (!read_file(co, code)) {
            // unique per call: prebuild.py runs several of these threads at once, and two of them (or a
            // cap retry) may resolve to the same code object; ecamd_jitc renames its output into place
            static std::atomic<unsigned> seq{0};
            const std::string req_path = co + ".req." + std::to_string(getpid()) + "." +
                                         std::to_string(seq.fetch_add(1, std::memory_order_relaxed));
            {
                std::ofstream f(req_path);
                f << request_of(e);
                if (!f) return -2;
            }
            const char* argv[] = {helper.c_str(), req_path.c_str(), co.c_str(), arch.c_str(), nullptr};
            pid_t pid = -1;
            int status = 0;
            if (posix_spawn(&pid, helper.c_str(), nullptr, nullptr, const_cast<char* const*>(argv), environ) != 0)
                return -3;
            while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
            }
            std::remove(req_path.c_str());
            if (!WIFEXITED(status) || WEXITSTATUS(status) != 0 || !read_file(co, code)) return -4;
        }
        const long scratch = code_object_scratch(code);
        if (scratch == 0) return 1;
        if (scratch < 0) return -5;
    }
    return -6;  // every cap spills: the run time keeps the LDS tables for this map
}

// Kernel for the R x K matrix on `dev`: nullptr while compiling (wait = false) or when the
// bitsliced form is unavailable; starts the compile the first time the matrix is seen.  `hold`
// keeps the kernel's module loaded until the caller has enqueued its launch.  `status` (optional):
// 1 the kernel is loaded, 0 compiling or queued, -1 unavailable (no code object can be had).
hipFunction_t bitslice_function(int dev, const std::vector<int>& coeff, int R, int K, int depth, bool wait,
                                std::shared_ptr<void>& hold, bool copy, int crc, bool wave,
                                const std::vector<int>* in_shift, int prefetch, int* status, const BsOcc* occ_in)
{
    if (status) *status = -1;
    if (R <= 0 || R > kBsMaxR || K <= 0 || K > kBsMaxK || (helper_path().empty() && shipped_dir().empty()))
        return nullptr;
    std::vector<int> shifts;
    BsOcc occ = occ_in ? *occ_in : BsOcc{};
    const std::vector<int> key = normalize(coeff, R, K, depth, copy, crc, wave, in_shift, prefetch, shifts, occ);
    std::vector<std::shared_ptr<BsEntry>> evicted;  // released after the lock (declared before it)
    std::unique_lock<std::mutex> lk(g_jit_mu);
    for (size_t i = 0; i < g_running.size();) {  // reap finished compilers, freeing their slots
        const auto ep = g_running[i];
        poll_compile(ep, false);
        if (ep->state == 0) i++;
    }
    const size_t max_entries = static_cast<size_t>(std::max(1, dev_tune("bitslice_entries")));
    while (g_jit.size() >= max_entries && !g_jit.count(key)) {  // evict the least recently used
        auto victim = g_jit.end();
        for (auto it = g_jit.begin(); it != g_jit.end(); ++it)
            if (it->second->state != 0 && (victim == g_jit.end() || it->second->last_use < victim->second->last_use))
                victim = it;
        if (victim == g_jit.end()) break;  // all compiling: let the map grow until they finish
        evicted.push_back(std::move(victim->second));
        g_jit.erase(victim);
    }
    auto& slot = g_jit[key];
    if (!slot) {
        slot = std::make_shared<BsEntry>();
        slot->coeff = coeff;
        slot->R = R;
        slot->K = K;
        slot->depth = depth;
        slot->copy = copy;
        slot->crc = crc;
        slot->wave = wave;
        slot->shifts = shifts;
        slot->prefetch = prefetch;
        slot->occ = occ;
        slot->arch = device_arch(dev);
        slot->cap_index = first_cap(R, crc, wave);
        start_compile(slot, wait);
    }
    const std::shared_ptr<BsEntry> ep = slot;
    BsEntry& e = *ep;
    e.last_use = ++g_clock;
    hold = ep;
    for (;;) {
        auto it = e.fn.find(dev);
        if (it != e.fn.end()) {
            if (status) *status = it->second ? 1 : -1;
            return it->second;
        }
        if (wait)
            wait_compile(lk, ep);
        else
            poll_compile(ep, false);
        if (e.state == 0 || e.state == 2) {
            if (status) *status = 0;
            return nullptr;
        }
        if ((it = e.fn.find(dev)) != e.fn.end()) {  // loaded while unlocked
            if (status) *status = it->second ? 1 : -1;
            return it->second;
        }
        hipFunction_t fn = nullptr;
        int spill = 0;
        if (e.state == 1) {
            hipModule_t mod = nullptr;
            int cur = -1;
            (void)hipGetDevice(&cur);
            if (cur != dev) (void)hipSetDevice(dev);  // the module belongs to the map's device
            const hipError_t lrc = hipModuleLoadData(&mod, e.code.data());
            if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
            if (lrc == hipSuccess) {
                e.modules.emplace_back(dev, mod);
                if (hipModuleGetFunction(&fn, mod, "ecamd_bs_kernel") != hipSuccess) fn = nullptr;
                if (fn && hipFuncGetAttribute(&spill, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, fn) == hipSuccess &&
                    spill > 0)
                    fn = nullptr;  // a spilling network runs slower than the LDS tables
            }
            (void)hipGetLastError();
        }
        if (!fn && spill > 0 && e.cap_index + 1 < kNumCaps) {  // rebuild with fewer temporaries
            e.cap_index++;
            e.fn.clear();
            start_compile(ep, wait);
            continue;
        }
        e.fn[dev] = fn;
        if (status) *status = fn ? 1 : -1;
        return fn;
    }
}

int bitslice_launch(hipFunction_t fn, const BsArgs& args, int grid, hipStream_t st,
                    const std::shared_ptr<void>& hold, int threads, unsigned lds)
{
    BsArgs a = args;
    void* params[] = {&a};
    // 64 / 128 / 256 / 512 lanes, or whole waves up to 1024 (the one-wave crc form's workgroups)
    const bool ok = threads > 0 && threads <= 1024 && threads % 64 == 0;
    const hipError_t e = hipModuleLaunchKernel(fn, static_cast<unsigned>(grid), 1, 1,
                                               static_cast<unsigned>(ok ? threads : 256), 1, 1, lds, st,
                                               params, nullptr);
    if (e != hipSuccess)
        return dev_fail(ECAMD_EHIP, "hipModuleLaunchKernel(bitslice): %s", hipGetErrorString(e));
    g_bs_launches.fetch_add(1, std::memory_order_relaxed);
    auto* entry = static_cast<BsEntry*>(hold.get());
    if (entry) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::lock_guard<std::mutex> lk(entry->ev_mu);
        // Callers that create and destroy streams (per-call slots, user streams) would grow the map
        // for as long as the entry stays cached: drop the events of other streams that completed.
        if (entry->last_launch.size() >= 8) {
            for (auto it = entry->last_launch.begin(); it != entry->last_launch.end();) {
                if (it->first != std::make_pair(dev, st) && it->second &&
                    hipEventQuery(it->second) == hipSuccess) {
                    (void)hipEventDestroy(it->second);
                    it = entry->last_launch.erase(it);
                } else {
                    ++it;
                }
            }
            (void)hipGetLastError();
        }
        hipEvent_t& ev = entry->last_launch[{dev, st}];
        if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
        if (ev) (void)hipEventRecord(ev, st);
        (void)hipGetLastError();
    }
    return 0;
}

}  // namespace ecamd

extern "C" int ecamd_bitslice_wait(void)
{
    std::unique_lock<std::mutex> lk(ecamd::g_jit_mu);
    std::vector<std::shared_ptr<ecamd::BsEntry>> all;
    for (auto& kv : ecamd::g_jit) all.push_back(kv.second);
    int failed = 0;
    for (const auto& ep : all) {
        ecamd::wait_compile(lk, ep);  // starts queued compiles too
        if (ep->state != 1) failed++;
    }
    return failed;
}

extern "C" long long ecamd_bitslice_launches(void)
{
    return ecamd::g_bs_launches.load(std::memory_order_relaxed);
}

extern "C" int ecamd_bitslice_entries(void)
{
    std::lock_guard<std::mutex> lk(ecamd::g_jit_mu);
    return static_cast<int>(ecamd::g_jit.size());
}

extern "C" int ecamd_bitslice_available(void) { return ecamd::helper_path().empty() ? 0 : 1; }
