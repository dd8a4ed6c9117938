// d2h_kernel_probe.hip — test infrastructure: D2H into pinned host memory by a copy kernel with a
// limited number of workgroups (how few CUs reach the PCIe rate), vs hipMemcpyAsync.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)
static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void __launch_bounds__(256) k_copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) if (i + u * 256 < n16) v[u] = src[i + u * 256];
#pragma unroll
        for (int u = 0; u < 4; u++) if (i + u * 256 < n16) dst[i + u * 256] = v[u];
    }
}

int main()
{
    const size_t total = 330ull << 20;
    void *d; CK(hipMalloc(&d, total));
    CK(hipMemset(d, 1, total));
    void *h; CK(hipHostMalloc(&h, total, hipHostMallocDefault));
    void *hd; CK(hipHostGetDevicePointer(&hd, h, 0));
    printf("host %p device view %p\n", h, hd);
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int rep = 0; rep < 2; rep++) {
        double t0 = now_ms();
        CK(hipMemcpyAsync(h, d, total, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s));
        double ms = now_ms() - t0;
        printf("hipMemcpyAsync D2H 330 MiB: %.2f ms, %.1f GB/s\n", ms, total / (ms * 1e-3) / 1e9);
        const int grids[6] = {8, 16, 32, 64, 128, 512};
        for (int g : grids) {
            t0 = now_ms();
            hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, s, (const uint4 *)d, (uint4 *)hd, (uint64_t)(total / 16));
            CK(hipGetLastError());
            CK(hipStreamSynchronize(s));
            ms = now_ms() - t0;
            printf("kernel D2H %4d WGs: %.2f ms, %.1f GB/s\n", g, ms, total / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
