// memcache.cpp — see memcache.h.
#include "memcache.h"

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

namespace kpw {

namespace {

size_t cap_gb(const char *env, size_t dflt)
{
    const char *e = getenv(env);
    if (!e || !*e) return dflt << 30;
    const long long v = atoll(e);
    return v > 0 ? (size_t)v << 30 : 0;
}
// Processes sharing this host (torchrun's LOCAL_WORLD_SIZE: one rank per GPU of the node).
size_t local_ranks()
{
    const char *e = getenv("LOCAL_WORLD_SIZE");
    const long long v = e ? atoll(e) : 1;
    return v > 1 ? (size_t)v : 1;
}
// idle memory kept (KPW_DEV_CACHE_GB per device / KPW_PIN_CACHE_GB; 0 = keep nothing idle).
// The device cap is per device, and each rank owns its device; pinned memory is the host's, so
// its default (48 GB) is shared by the ranks of the node: 48 / LOCAL_WORLD_SIZE per process
// (8 ranks: 6 GB each, on top of each rank's own pinned record batches).  An explicit
// KPW_PIN_CACHE_GB is per process.
size_t dev_cache_cap()
{
    static const size_t v = cap_gb("KPW_DEV_CACHE_GB", 96);
    return v;
}
bool dev_cap_explicit()
{
    static const bool v = [] { const char *e = getenv("KPW_DEV_CACHE_GB"); return e && *e; }();
    return v;
}
size_t pin_cache_cap()
{
    static const size_t v = [] {
        const char *e = getenv("KPW_PIN_CACHE_GB");
        if (e && *e) return cap_gb("KPW_PIN_CACHE_GB", 48);
        return (size_t)(48ull << 30) / local_ranks();
    }();
    return v;
}

double mono_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Pool {
    std::multimap<size_t, void *> free_;   // size -> block
    std::map<void *, size_t> size_;        // every block this pool allocated (live or free)
    size_t free_bytes = 0;
    size_t live = 0, peak = 0;             // bytes handed out now / at most (device pools)
    size_t total = 0;                      // the device's memory (0: not queried yet)
};

// a block handed back with dev_free_after: it rejoins its pool once `ev` has completed
struct Deferred {
    void *p;
    int dev;
    hipEvent_t ev;
};

std::mutex g_mu;
Pool g_dev[64];
Pool g_pin;
std::map<uintptr_t, size_t> g_pin_live;     // live pinned blocks (pin_contains)
std::map<void *, int> g_dev_of;             // device of every block dev_alloc handed out
                                            // (hipPointerGetAttributes per free cost ~0.3 ms)
std::vector<Deferred> g_deferred;
// allocator counters (kpw_cache_stats): calls into the HIP allocator and the host time they took
struct Counters {
    double dev_malloc_n = 0, dev_malloc_ms = 0, dev_free_n = 0, dev_free_ms = 0;
    double pin_malloc_n = 0, pin_malloc_ms = 0, pin_free_n = 0, pin_free_ms = 0;
    double dev_hits = 0, pin_hits = 0, dev_live = 0, pin_live = 0, dev_retry = 0;
    double dev_sync_n = 0, dev_sync_ms = 0;   // device-wide synchronisations of a buffer growth
} g_cnt;
double g_gate_wait_ms = 0, g_gate_waits = 0;   // EncodeGate admissions and their host wait (under g_mu)

hipError_t timed_malloc(void **q, size_t bytes)
{
    const double t = mono_ms();
    const hipError_t e = hipMalloc(q, bytes);
    g_cnt.dev_malloc_n++;
    g_cnt.dev_malloc_ms += mono_ms() - t;
    return e;
}
void timed_free(void *q)
{
    const double t = mono_ms();
    (void)hipFree(q);
    g_cnt.dev_free_n++;
    g_cnt.dev_free_ms += mono_ms() - t;
}
hipError_t timed_host_malloc(void **q, size_t bytes)
{
    const double t = mono_ms();
    const hipError_t e = hipHostMalloc(q, bytes, hipHostMallocDefault);
    g_cnt.pin_malloc_n++;
    g_cnt.pin_malloc_ms += mono_ms() - t;
    return e;
}
void timed_host_free(void *q)
{
    const double t = mono_ms();
    (void)hipHostFree(q);
    g_cnt.pin_free_n++;
    g_cnt.pin_free_ms += mono_ms() - t;
}

// best fit within 2x (and never more than 1 GiB of slack)
void *take(Pool &p, size_t bytes)
{
    auto it = p.free_.lower_bound(bytes);
    if (it == p.free_.end()) return nullptr;
    if (it->first > 2 * bytes && it->first - bytes > (1ull << 30)) return nullptr;
    if (it->first > 2 * bytes && bytes < (64ull << 20)) return nullptr;
    void *q = it->second;
    p.free_bytes -= it->first;
    p.free_.erase(it);
    return q;
}

template <class FreeFn>
void trim(Pool &p, size_t keep, FreeFn fn)
{
    // release the largest idle blocks first until at most `keep` bytes stay cached
    while (p.free_bytes > keep && !p.free_.empty()) {
        auto it = std::prev(p.free_.end());
        fn(it->second);
        p.free_bytes -= it->first;
        p.size_.erase(it->second);
        p.free_.erase(it);
    }
}

void dev_release(void *b)
{
    g_dev_of.erase(b);
    timed_free(b);
}

// a block of ours back into its pool (under g_mu)
// Idle bytes a device pool keeps: KPW_DEV_CACHE_GB when set; by default at least 96 GB and up
// to the pool's peak live bytes (capped at 3/4 of the device), so a workload that re-opens the
// same writers every file (C5: eight writers, ~110 GB live) finds every block again instead of
// re-allocating the part above a fixed cap each file.
size_t dev_keep(const Pool &p)
{
    if (dev_cap_explicit()) return dev_cache_cap();
    const size_t lim = p.total ? p.total / 4 * 3 : dev_cache_cap();
    return std::max(dev_cache_cap(), std::min(p.peak, lim));
}

void dev_return(void *q, int dev)
{
    Pool &p = g_dev[dev];
    auto it = p.size_.find(q);
    if (it == p.size_.end()) { timed_free(q); return; }
    p.free_.emplace(it->second, q);
    p.free_bytes += it->second;
    p.live -= it->second;
    g_cnt.dev_live -= (double)it->second;
    trim(p, dev_keep(p), dev_release);
}

// deferred blocks whose event completed rejoin their pools (under g_mu); wait: block on them
void reap(bool wait)
{
    size_t k = 0;
    for (size_t i = 0; i < g_deferred.size(); i++) {
        Deferred &d = g_deferred[i];
        const hipError_t e = wait ? hipEventSynchronize(d.ev) : hipEventQuery(d.ev);
        if (e == hipErrorNotReady) { g_deferred[k++] = d; continue; }
        (void)hipGetLastError();
        (void)hipEventDestroy(d.ev);
        dev_return(d.p, d.dev);
    }
    g_deferred.resize(k);
}

}  // namespace

void *dev_alloc(size_t bytes)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    if (bytes < 256) bytes = 256;
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_deferred.empty()) reap(false);
    Pool &p = g_dev[dev];
    if (!p.total) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) p.total = tot; else (void)hipGetLastError();
    }
    if (void *q = take(p, bytes)) {
        g_cnt.dev_hits++;
        g_cnt.dev_live += (double)p.size_[q];
        p.live += p.size_[q];
        p.peak = std::max(p.peak, p.live);
        return q;
    }
    void *q = nullptr;
    if (timed_malloc(&q, bytes) != hipSuccess) {
        (void)hipGetLastError();
        g_cnt.dev_retry++;
        reap(true);
        trim(p, 0, dev_release);   // give the idle blocks back and retry
        if (timed_malloc(&q, bytes) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
    }
    p.size_[q] = bytes;
    g_dev_of[q] = dev;
    g_cnt.dev_live += (double)bytes;
    p.live += bytes;
    p.peak = std::max(p.peak, p.live);
    return q;
}

void dev_free(void *q)
{
    if (!q) return;
    std::lock_guard<std::mutex> g(g_mu);
    auto d = g_dev_of.find(q);
    if (d == g_dev_of.end()) { timed_free(q); return; }   // not ours
    dev_return(q, d->second);
}

void dev_free_after(void *q, hipStream_t s)
{
    if (!q) return;
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, s) != hipSuccess) {
        (void)hipGetLastError();
        if (ev) (void)hipEventDestroy(ev);
        (void)hipStreamSynchronize(s);   // cannot defer: order the free after the stream the slow way
        dev_free(q);
        return;
    }
    std::lock_guard<std::mutex> g(g_mu);
    auto d = g_dev_of.find(q);
    if (d == g_dev_of.end()) {   // not ours: a plain free after the stream
        (void)hipEventSynchronize(ev);
        (void)hipEventDestroy(ev);
        timed_free(q);
        return;
    }
    g_deferred.push_back(Deferred{q, d->second, ev});
}

void *pin_alloc(size_t bytes)
{
    if (bytes < 4096) bytes = 4096;
    std::lock_guard<std::mutex> g(g_mu);
    void *q = take(g_pin, bytes);
    if (q) g_cnt.pin_hits++;
    if (!q) {
        if (timed_host_malloc(&q, bytes) != hipSuccess) {
            (void)hipGetLastError();
            trim(g_pin, 0, timed_host_free);
            if (timed_host_malloc(&q, bytes) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
        }
        g_pin.size_[q] = bytes;
    }
    g_pin_live[(uintptr_t)q] = g_pin.size_[q];
    g_cnt.pin_live += (double)g_pin.size_[q];
    return q;
}

void pin_free(void *q)
{
    if (!q) return;
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_pin.size_.find(q);
    if (it == g_pin.size_.end()) return;
    g_pin_live.erase((uintptr_t)q);
    g_cnt.pin_live -= (double)it->second;
    g_pin.free_.emplace(it->second, q);
    g_pin.free_bytes += it->second;
    trim(g_pin, pin_cache_cap(), timed_host_free);
}

size_t pin_size(const void *q)
{
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_pin_live.upper_bound((uintptr_t)q);
    if (it == g_pin_live.begin()) return 0;
    --it;
    return (uintptr_t)q < it->first + it->second ? it->second : 0;
}

bool pin_contains(const void *q, size_t n)
{
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_pin_live.upper_bound((uintptr_t)q);
    if (it == g_pin_live.begin()) return false;
    --it;
    return (uintptr_t)q >= it->first && (uintptr_t)q + n <= it->first + it->second;
}

void stream_sets_trim();

void device_sync_for_free()
{
    const double t = mono_ms();
    (void)hipDeviceSynchronize();
    const double dt = mono_ms() - t;
    std::lock_guard<std::mutex> g(g_mu);
    g_cnt.dev_sync_n++;
    g_cnt.dev_sync_ms += dt;
}

void trim_caches()
{
    {
        std::lock_guard<std::mutex> g(g_mu);
        reap(true);
        for (auto &p : g_dev) { trim(p, 0, dev_release); p.peak = p.live; }
        trim(g_pin, 0, timed_host_free);
    }
    stream_sets_trim();   // idle pooled stream sets too
}

int cache_stats(double *out, int cap)
{
    size_t dev_idle = 0;
    std::lock_guard<std::mutex> g(g_mu);
    for (auto &p : g_dev) dev_idle += p.free_bytes;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || cur < 0 || cur >= 64) cur = 0;
    const double v[] = {(double)dev_keep(g_dev[cur]), (double)pin_cache_cap(), g_cnt.dev_live, (double)dev_idle,
                        g_cnt.pin_live, (double)g_pin.free_bytes, g_cnt.dev_malloc_n, g_cnt.dev_malloc_ms,
                        g_cnt.dev_free_n, g_cnt.dev_free_ms, g_cnt.pin_malloc_n, g_cnt.pin_malloc_ms,
                        g_cnt.pin_free_n, g_cnt.pin_free_ms, g_cnt.dev_hits, g_cnt.pin_hits, g_cnt.dev_retry,
                        g_cnt.dev_sync_n, g_cnt.dev_sync_ms, g_gate_waits, g_gate_wait_ms};
    const int n = (int)(sizeof(v) / sizeof(v[0]));
    int k = 0;
    for (; k < n && k < cap; k++) out[k] = v[k];
    return k;
}

// ---------------------------------------------------------------- streams
namespace {
struct StreamSet {
    int dev, n;
    hipStream_t s[8];
};
std::mutex g_smu;
std::vector<StreamSet> g_sets;   // idle pooled sets
std::vector<hipStream_t> g_pads;   // pad streams (stream_set_acquire), under g_smu
int g_live_sets = 0;               // sets handed out and not yet released (under g_smu)
bool stream_pad_on()
{
    static const bool on = [] { const char *e = getenv("KPW_STREAM_PAD"); return !(e && e[0] == '0'); }();
    return on;
}
bool stream_pool_on()
{
    static const bool on = [] { const char *e = getenv("KPW_STREAM_POOL"); return !(e && e[0] == '0'); }();
    return on;
}
}  // namespace

hipError_t stream_set_acquire(int n, hipStream_t *s)
{
    if (n <= 0 || n > 8) return hipErrorInvalidValue;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    if (stream_pool_on()) {
        std::lock_guard<std::mutex> g(g_smu);
        for (size_t i = g_sets.size(); i-- > 0;)
            if (g_sets[i].dev == dev && g_sets[i].n == n) {
                for (int k = 0; k < n; k++) s[k] = g_sets[i].s[k];
                g_sets.erase(g_sets.begin() + (long)i);
                g_live_sets++;
                return hipSuccess;
            }
    }
    // one set's streams are created back to back (HIP hands hardware queues to streams in creation
    // order): concurrent writers opening at once (C5) would otherwise interleave their creations,
    // and a set could get two streams on one queue, serialising its two encode workers
    static std::mutex create_mu;
    std::lock_guard<std::mutex> cg(create_mu);
    for (int k = 0; k < n; k++) {
        const hipError_t e = hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking);
        if (e != hipSuccess) {
            for (int j = 0; j < k; j++) (void)hipStreamDestroy(s[j]);
            for (int j = 0; j < n; j++) s[j] = nullptr;
            return e;
        }
    }
    // HIP hands out its hardware queues round-robin in creation order, so with sets of four
    // streams on four (or eight) queues every writer's first engine stream lands on the same
    // queue, and so does every second one: eight concurrent writers' encodes then share two
    // queues (r06h kernel trace of C5: all engine dispatches on queues 2 and 3).  Sets of an odd
    // number of streams rotate over the queues by themselves; after an even-sized set one pad
    // stream (kept idle until trim_caches) shifts the next set by one queue (KPW_STREAM_PAD=0: none).
    hipStream_t pad = nullptr;
    if (stream_pad_on() && n % 2 == 0 && hipStreamCreateWithFlags(&pad, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        pad = nullptr;
    }
    std::lock_guard<std::mutex> g(g_smu);
    if (pad) g_pads.push_back(pad);
    g_live_sets++;
    return hipSuccess;
}

void stream_sets_trim()
{
    std::vector<StreamSet> idle;
    std::vector<hipStream_t> pads;
    {
        std::lock_guard<std::mutex> g(g_smu);
        idle.swap(g_sets);
        if (g_live_sets == 0) pads.swap(g_pads);   // (pads only when no set is in use)
    }
    for (auto &t : idle)
        for (int k = 0; k < t.n; k++) if (t.s[k]) (void)hipStreamDestroy(t.s[k]);
    for (hipStream_t p : pads) (void)hipStreamDestroy(p);
}

void stream_set_release(int n, const hipStream_t *s)
{
    if (n <= 0 || n > 8 || !s[0]) return;
    int dev = 0;   // (the streams' own device: the caller's current one may differ)
    const bool keep = stream_pool_on() && hipStreamGetDevice(s[0], &dev) == hipSuccess;
    {
        std::lock_guard<std::mutex> g(g_smu);
        g_live_sets--;
    }
    if (keep) {
        std::lock_guard<std::mutex> g(g_smu);
        if (g_sets.size() < 64) {   // (bounded)
            StreamSet t{dev, n, {}};
            for (int k = 0; k < n; k++) t.s[k] = s[k];
            g_sets.push_back(t);
            return;
        }
    }
    for (int k = 0; k < n; k++) if (s[k]) (void)hipStreamDestroy(s[k]);
}

// ---------------------------------------------------------------- device encode gate
namespace {
struct Gate {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t next_ticket = 0, serving = 0;   // FIFO admission
    int running = 0;
};
Gate g_gate[64];
int gate_cap()
{
    static const int v = [] {
        const char *e = getenv("KPW_DEVICE_ENCODES");
        const int x = e ? atoi(e) : 0;
        return x > 0 ? x : 1 << 20;   // 0 (default) or negative: no limit
    }();
    return v;
}
}  // namespace

EncodeGate::EncodeGate(int device) : dev_(device >= 0 && device < 64 ? device : 0)
{
    Gate &G = g_gate[dev_];
    const double t = mono_ms();
    std::unique_lock<std::mutex> lk(G.mu);
    const uint64_t my = G.next_ticket++;
    G.cv.wait(lk, [&] { return G.serving == my && G.running < gate_cap(); });
    G.serving++;
    G.running++;
    held_ = true;
    waited_ = mono_ms() - t;
    G.cv.notify_all();   // the next ticket may be admitted too
    lk.unlock();
    std::lock_guard<std::mutex> g(g_mu);
    g_gate_wait_ms += waited_;
    g_gate_waits += 1;
}

void EncodeGate::release()
{
    if (!held_) return;
    Gate &G = g_gate[dev_];
    {
        std::lock_guard<std::mutex> g(G.mu);
        G.running--;
        held_ = false;
    }
    G.cv.notify_all();
}

EncodeGate::~EncodeGate() { release(); }

}  // namespace kpw

extern "C" void kpw_trim_caches(void) { kpw::trim_caches(); }
extern "C" int kpw_cache_stats(double *out, int cap) { return out && cap > 0 ? kpw::cache_stats(out, cap) : 0; }
