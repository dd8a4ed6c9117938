// h2d_probe.hip — test infrastructure: PCIe copy ceilings of the box (pinned H2D, D2H, and both
// at once on two streams), and which engine serves them (rocprofv3 kernel trace shows
// __amd_rocclr_copyBuffer when a shader blit is used instead of SDMA).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)

static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main()
{
    const size_t total = 1ull << 30;
    void *d, *d2; CK(hipMalloc(&d, total)); CK(hipMalloc(&d2, total));
    void *h, *h2; CK(hipHostMalloc(&h, total, hipHostMallocDefault)); CK(hipHostMalloc(&h2, total, hipHostMallocDefault));
    for (size_t i = 0; i < total; i += 4096) { ((char *)h)[i] = (char)i; ((char *)h2)[i] = 0; }
    hipStream_t s, s2; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const size_t chunks[3] = {32u << 20, 128u << 20, 1u << 30};
    for (size_t c : chunks) {
        for (int dir = 0; dir < 3; dir++) {   // 0 H2D, 1 D2H, 2 both (two streams)
            CK(hipMemcpyAsync(d, h, c, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
            const double t0 = now_ms();
            for (size_t o = 0; o < total; o += c) {
                if (dir != 1) CK(hipMemcpyAsync((char *)d + o, (char *)h + o, c, hipMemcpyHostToDevice, s));
                if (dir != 0) CK(hipMemcpyAsync((char *)h2 + o, (char *)d2 + o, c, hipMemcpyDeviceToHost, dir == 2 ? s2 : s));
            }
            CK(hipStreamSynchronize(s)); CK(hipStreamSynchronize(s2));
            const double ms = now_ms() - t0;
            const double gb = (dir == 2 ? 2.0 : 1.0) * total / 1e9;
            printf("%-5s chunk %5zu MiB: %.2f ms, %.1f GB/s\n", dir == 0 ? "H2D" : dir == 1 ? "D2H" : "both", c >> 20, ms,
                   gb / (ms * 1e-3));
        }
    }
    return 0;
}
