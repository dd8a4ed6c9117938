// memcache.h — process-wide caching allocators for device (HBM) and pinned host memory.
//
// A writer is a file (the reference opens one ParquetFile per rotation, and C5 runs many at
// once), and hipMalloc / hipFree / hipHostMalloc / hipHostFree of its multi-GiB stage, scratch
// and page buffers cost more than encoding a row group (hipFree also synchronises the whole
// device).  Freed blocks are kept per device (per size, best fit within 2x) and handed to the
// next allocation.  A block goes back to the cache only when no queued work can still touch
// it: the callers free after synchronising the stream that used it (Engine / writer teardown),
// or hand it over with dev_free_after(stream) (buffer growth: the block returns once the
// stream's queued work has passed an event, without a device-wide synchronisation).
//
// Idle memory kept: KPW_DEV_CACHE_GB per device when set; by default 96 GB or the device pool's
// peak live bytes, whichever is larger, at most 3/4 of the device (C5 runs 8 writers per GPU,
// ~110 GB live, and re-opens them every file), and KPW_PIN_CACHE_GB of pinned host memory per
// process (default 48 GB shared by the node's ranks: 48 / LOCAL_WORLD_SIZE);
// kpw_trim_caches() (kpw_gpu.h) releases every idle block, e.g. before a co-located consumer
// allocates.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace kpw {

void *dev_alloc(size_t bytes);     // on the current device; nullptr on failure
void dev_free(void *p);            // nullptr ok
void dev_free_after(void *p, hipStream_t s);   // back to the cache once s has run what it queued so far
void *pin_alloc(size_t bytes);     // page-locked host memory; nullptr on failure
void pin_free(void *p);            // nullptr ok
size_t pin_size(const void *p);    // usable bytes of a pin_alloc block containing p (0 if none)
bool pin_contains(const void *p, size_t n);   // [p, p+n) inside one live pin_alloc block
void trim_caches();                // release every idle block (device pools, pinned, stream sets)
int cache_stats(double *out, int cap);   // kpw_cache_stats (kpw_gpu.h)
void device_sync_for_free();       // hipDeviceSynchronize before a plain free, counted (kpw_cache_stats)
// Sets of n non-blocking HIP streams of the current device, kept across writers:
// hipStreamDestroy takes ~2.5 ms (a writer tears down four streams per file, and the reference
// opens a file per rotation).  A set is created stream after stream and reused whole: HIP gives
// streams hardware queues in creation order, so a set's streams sit on different queues (single
// pooled streams mixed from different writers could share one and serialise two encode
// workers: C4 21.3 -> 15.7 GB/s after the per-record legs).  stream_set_release takes idle
// streams (their owner synchronised them) back (KPW_STREAM_POOL=0: created and destroyed).
hipError_t stream_set_acquire(int n, hipStream_t *s);
void stream_set_release(int n, const hipStream_t *s);

// Device encode gate: at most KPW_DEVICE_ENCODES writer jobs encode on one device at once,
// admitted in arrival order (tickets); default 0 = no limit.  Measured on C5 (eight concurrent
// writers, 16 encode workers; r06b, one box): unlimited 32.5 GB/s, 2 slots 25.4, 3 slots 28.3,
// 4 slots 28.9 — admitted jobs encode 3.4x faster each, but the chip is fuller with every
// writer's job in flight (a job's kernel chain alone leaves most CUs idle), so the default
// stays unlimited.  Kept for deployments that bound per-file latency or share the GPU.
class EncodeGate {
public:
    explicit EncodeGate(int device);   // blocks until admitted
    ~EncodeGate();                     // releases the slot (idempotent with release())
    void release();
    EncodeGate(const EncodeGate &) = delete;
    EncodeGate &operator=(const EncodeGate &) = delete;
    double waited_ms() const { return waited_; }

private:
    int dev_;
    bool held_ = false;
    double waited_ = 0;
};

}  // namespace kpw
