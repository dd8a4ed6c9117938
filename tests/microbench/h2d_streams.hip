// h2d_streams.hip — test infrastructure: pinned H2D throughput of 31 MB chunks (a C2 poll batch)
// on one stream against chunks alternated over 2 / 4 streams (does a second SDMA queue hide
// the per-copy gaps?), and single-stream 64 / 128 MiB chunks.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)

static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main()
{
    const size_t total = 3ull << 30;
    void *d, *h;
    CK(hipMalloc(&d, total));
    CK(hipHostMalloc(&h, total, hipHostMallocDefault));
    for (size_t i = 0; i < total; i += 4096) ((char *)h)[i] = (char)i;
    hipStream_t s[4];
    for (int i = 0; i < 4; i++) CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
    struct Cfg { size_t chunk; int ns; } cfgs[] = {{31000000, 1}, {31000000, 2}, {31000000, 4}, {64u << 20, 1}, {128u << 20, 1},
                                                  {31000000, 1}, {31000000, 2}};
    for (const Cfg &c : cfgs) {
        CK(hipMemcpyAsync(d, h, c.chunk, hipMemcpyHostToDevice, s[0]));
        CK(hipDeviceSynchronize());
        const double t0 = now_ms();
        int k = 0;
        size_t bytes = 0;
        for (size_t o = 0; o + c.chunk <= total; o += c.chunk, k++) {
            CK(hipMemcpyAsync((char *)d + o, (char *)h + o, c.chunk, hipMemcpyHostToDevice, s[k % c.ns]));
            bytes += c.chunk;
        }
        CK(hipDeviceSynchronize());
        const double ms = now_ms() - t0;
        printf("chunk %9zu B, %d stream(s): %8.2f ms, %.2f GB/s\n", c.chunk, c.ns, ms, bytes / ms / 1e6);
    }
    // the writer's async pattern: issue DMA k, record event k, wait for event k - depth
    hipEvent_t ev[8];
    for (int i = 0; i < 8; i++) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    hipEvent_t ev2;
    CK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
    for (int extra = 0; extra <= 1; extra++)
    for (int depth = 1; depth <= 1; depth++) {
        for (int rep = 0; rep < 2; rep++) {
            const size_t chunk = 31000000;
            CK(hipDeviceSynchronize());
            const double t0 = now_ms();
            size_t bytes = 0;
            int k = 0;
            for (size_t o = 0; o + chunk <= total; o += chunk, k++) {
                CK(hipMemcpyAsync((char *)d + o, (char *)h + o, chunk, hipMemcpyHostToDevice, s[0]));
                if (extra) CK(hipEventRecord(ev2, s[0]));   // the writer's second record (direct_ev)
                CK(hipEventRecord(ev[k % 8], s[0]));
                if (k >= depth) CK(hipEventSynchronize(ev[(k - depth) % 8]));
                bytes += chunk;
            }
            CK(hipDeviceSynchronize());
            const double ms = now_ms() - t0;
            printf("writer pattern, %d event records per DMA: %8.2f ms, %.2f GB/s\n", 1 + extra, ms, bytes / ms / 1e6);
        }
    }
    return 0;
}
