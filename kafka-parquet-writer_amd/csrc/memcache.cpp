// memcache.cpp — see memcache.h.
#include "memcache.h"

#include <cstdint>
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
// idle memory kept (KPW_DEV_CACHE_GB per device / KPW_PIN_CACHE_GB; 0 = keep nothing idle)
size_t dev_cache_cap()
{
    static const size_t v = cap_gb("KPW_DEV_CACHE_GB", 96);
    return v;
}
size_t pin_cache_cap()
{
    static const size_t v = cap_gb("KPW_PIN_CACHE_GB", 48);
    return v;
}

struct Pool {
    std::multimap<size_t, void *> free_;   // size -> block
    std::map<void *, size_t> size_;        // every block this pool allocated (live or free)
    size_t free_bytes = 0;
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
    (void)hipFree(b);
}

// a block of ours back into its pool (under g_mu)
void dev_return(void *q, int dev)
{
    Pool &p = g_dev[dev];
    auto it = p.size_.find(q);
    if (it == p.size_.end()) { (void)hipFree(q); return; }
    p.free_.emplace(it->second, q);
    p.free_bytes += it->second;
    trim(p, dev_cache_cap(), dev_release);
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
    if (void *q = take(p, bytes)) return q;
    void *q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) {
        (void)hipGetLastError();
        reap(true);
        trim(p, 0, dev_release);   // give the idle blocks back and retry
        if (hipMalloc(&q, bytes) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
    }
    p.size_[q] = bytes;
    g_dev_of[q] = dev;
    return q;
}

void dev_free(void *q)
{
    if (!q) return;
    std::lock_guard<std::mutex> g(g_mu);
    auto d = g_dev_of.find(q);
    if (d == g_dev_of.end()) { (void)hipFree(q); return; }   // not ours
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
        (void)hipFree(q);
        return;
    }
    g_deferred.push_back(Deferred{q, d->second, ev});
}

void *pin_alloc(size_t bytes)
{
    if (bytes < 4096) bytes = 4096;
    std::lock_guard<std::mutex> g(g_mu);
    void *q = take(g_pin, bytes);
    if (!q) {
        if (hipHostMalloc(&q, bytes, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            trim(g_pin, 0, [](void *b) { (void)hipHostFree(b); });
            if (hipHostMalloc(&q, bytes, hipHostMallocDefault) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
        }
        g_pin.size_[q] = bytes;
    }
    g_pin_live[(uintptr_t)q] = g_pin.size_[q];
    return q;
}

void pin_free(void *q)
{
    if (!q) return;
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_pin.size_.find(q);
    if (it == g_pin.size_.end()) return;
    g_pin_live.erase((uintptr_t)q);
    g_pin.free_.emplace(it->second, q);
    g_pin.free_bytes += it->second;
    trim(g_pin, pin_cache_cap(), [](void *b) { (void)hipHostFree(b); });
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

void trim_caches()
{
    std::lock_guard<std::mutex> g(g_mu);
    reap(true);
    for (auto &p : g_dev) trim(p, 0, dev_release);
    trim(g_pin, 0, [](void *b) { (void)hipHostFree(b); });
}

// ---------------------------------------------------------------- streams
namespace {
struct StreamSet {
    int dev, n;
    hipStream_t s[8];
};
std::mutex g_smu;
std::vector<StreamSet> g_sets;   // idle pooled sets
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
                return hipSuccess;
            }
    }
    for (int k = 0; k < n; k++) {
        const hipError_t e = hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking);
        if (e != hipSuccess) {
            for (int j = 0; j < k; j++) (void)hipStreamDestroy(s[j]);
            for (int j = 0; j < n; j++) s[j] = nullptr;
            return e;
        }
    }
    return hipSuccess;
}

void stream_set_release(int n, const hipStream_t *s)
{
    if (n <= 0 || n > 8 || !s[0]) return;
    int dev = 0;   // (the streams' own device: the caller's current one may differ)
    const bool keep = stream_pool_on() && hipStreamGetDevice(s[0], &dev) == hipSuccess;
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

}  // namespace kpw

extern "C" void kpw_trim_caches(void) { kpw::trim_caches(); }
