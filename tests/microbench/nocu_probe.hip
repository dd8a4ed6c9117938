// nocu_probe.hip — does a small copy wait for the compute units?  A kernel holds one 1024-thread
// workgroup with 150 KiB of LDS on every CU for ~40 ms (bounded by the 100 MHz real-time
// counter); on a second stream, a 1 KiB device -> host copy is issued in three forms and its
// completion time measured against the busy kernel's:
//   pageable D2H, pinned D2H, and hipMemcpyDeviceToDeviceNoCU into the pinned buffer.
// A copy that completes long before the kernel ends ran without a CU (SDMA).
//   hipcc --offload-arch=gfx950 -O2 nocu_probe.hip -o nocu_probe && ./nocu_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void busy(unsigned long long ticks, int *sink)
{
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int acc = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        lds[threadIdx.x] = acc;
        acc += lds[(threadIdx.x + 1) & 1023];
    }
    if (acc == 12345) sink[0] = acc;
}

static double ms_since(std::chrono::steady_clock::time_point t)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    int *sink;
    uint8_t *dev, *pin;
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&dev, 1 << 20));
    CK(hipHostMalloc((void **)&pin, 1 << 20, hipHostMallocDefault));
    std::vector<uint8_t> pageable(1 << 20);
    std::vector<uint8_t> ref(1024);
    for (int i = 0; i < 1024; i++) ref[i] = (uint8_t)(i * 7 + 3);
    CK(hipMemcpy(dev, ref.data(), 1024, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void *)busy, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    const char *names[5] = {"pageable D2H", "pinned D2H", "NoCU into pinned", "pinned H2D", "NoCU from pinned"};
    uint8_t *dev2;
    CK(hipMalloc(&dev2, 1 << 20));
    for (int rep = 0; rep < 2; rep++) {
        for (int m = 0; m < 5; m++) {
            memset(pin, 0, 1024);
            if (m >= 3) { memcpy(pin, ref.data(), 1024); CK(hipMemset(dev2, 0, 1024)); }
            memset(pageable.data(), 0, 1024);
            hipEvent_t kdone, cdone;
            CK(hipEventCreate(&kdone));
            CK(hipEventCreate(&cdone));
            const auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(busy, dim3(cus), dim3(1024), 150 * 1024, a, 4000000ull, sink);   // 40 ms
            CK(hipGetLastError());
            CK(hipEventRecord(kdone, a));
            // let the busy grid occupy the CUs first
            while (ms_since(t0) < 5.0) {}
            const auto t1 = std::chrono::steady_clock::now();
            if (m == 0) CK(hipMemcpyAsync(pageable.data(), dev, 1024, hipMemcpyDeviceToHost, b));
            if (m == 1) CK(hipMemcpyAsync(pin, dev, 1024, hipMemcpyDeviceToHost, b));
            if (m == 2) CK(hipMemcpyAsync(pin, dev, 1024, hipMemcpyDeviceToDeviceNoCU, b));
            if (m == 3) CK(hipMemcpyAsync(dev2, pin, 1024, hipMemcpyHostToDevice, b));
            if (m == 4) CK(hipMemcpyAsync(dev2, pin, 1024, hipMemcpyDeviceToDeviceNoCU, b));
            CK(hipEventRecord(cdone, b));
            double tc = -1, tk = -1;
            while (tc < 0 || tk < 0) {
                if (tc < 0 && hipEventQuery(cdone) == hipSuccess) tc = ms_since(t1);
                if (tk < 0 && hipEventQuery(kdone) == hipSuccess) tk = ms_since(t1);
            }
            if (m >= 3) CK(hipMemcpy(pageable.data(), dev2, 1024, hipMemcpyDeviceToHost));
            const uint8_t *got = (m == 0 || m >= 3) ? pageable.data() : pin;
            printf("%-18s copy done %.3f ms after issue, busy kernel done %.3f ms after it, bytes %s\n", names[m], tc, tk,
                   memcmp(got, ref.data(), 1024) ? "WRONG" : "ok");
            CK(hipEventDestroy(kdone));
            CK(hipEventDestroy(cdone));
        }
    }
    return 0;
}
