// memcache.cpp — see memcache.h.
#include "memcache.h"

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <mutex>

namespace kpw {

namespace {

constexpr size_t kDevCacheCap = 96ull << 30;   // idle HBM kept per device (of 288 GB)
constexpr size_t kPinCacheCap = 48ull << 30;   // idle pinned host memory kept

struct Pool {
    std::multimap<size_t, void *> free_;   // size -> block
    std::map<void *, size_t> size_;        // every block this pool allocated (live or free)
    size_t free_bytes = 0;
};

std::mutex g_mu;
Pool g_dev[64];
Pool g_pin;
std::map<uintptr_t, size_t> g_pin_live;     // live pinned blocks (pin_contains)
std::map<void *, int> g_dev_of;             // device of every block dev_alloc handed out
                                            // (hipPointerGetAttributes per free cost ~0.3 ms)

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

}  // namespace

void *dev_alloc(size_t bytes)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    if (bytes < 256) bytes = 256;
    std::lock_guard<std::mutex> g(g_mu);
    Pool &p = g_dev[dev];
    if (void *q = take(p, bytes)) return q;
    void *q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) {
        (void)hipGetLastError();
        trim(p, 0, [](void *b) { g_dev_of.erase(b); (void)hipFree(b); });   // give the idle blocks back and retry
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
    Pool &p = g_dev[d->second];
    auto it = p.size_.find(q);
    if (it == p.size_.end()) { (void)hipFree(q); return; }
    p.free_.emplace(it->second, q);
    p.free_bytes += it->second;
    trim(p, kDevCacheCap, [](void *b) { g_dev_of.erase(b); (void)hipFree(b); });
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
    trim(g_pin, kPinCacheCap, [](void *b) { (void)hipHostFree(b); });
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

}  // namespace kpw
