// h2d_probe.hip — test infrastructure: which engine serves pinned H2D copies (rocprofv3 kernel
// trace shows __amd_rocclr_copyBuffer when a shader blit is used) and at what rate.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)
int main()
{
    const size_t sz = 32u << 20, n = 8;
    void *d; CK(hipMalloc(&d, sz * n));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const unsigned flags[3] = {hipHostMallocDefault, hipHostMallocNonCoherent, hipHostMallocCoherent};
    const char *names[3] = {"default", "noncoherent", "coherent"};
    for (int k = 0; k < 3; k++) {
        void *h; CK(hipHostMalloc(&h, sz * n, flags[k]));
        for (size_t i = 0; i < sz * n; i += 4096) ((char *)h)[i] = (char)i;
        CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < n; i++) CK(hipMemcpyAsync((char *)d + i * sz, (char *)h + i * sz, sz, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        printf("%-12s %zu x %zu MiB H2D: %.2f ms, %.1f GB/s\n", names[k], n, sz >> 20, ms, sz * n / (ms * 1e-3) / 1e9);
        CK(hipHostFree(h));
    }
    return 0;
}
