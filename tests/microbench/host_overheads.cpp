// Per-call host costs on the per-record path (write + getDataSize per record): hipSetDevice,
// an uncontended std::mutex, hipGetDevice.  Build: hipcc -O2 -o host_overheads host_overheads.cpp
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <mutex>

static double ns_per(std::chrono::steady_clock::time_point a, long n)
{
    return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - a).count() / n;
}

int main()
{
    const long n = 2000000;
    if (hipSetDevice(0) != hipSuccess) return 1;
    auto t = std::chrono::steady_clock::now();
    for (long i = 0; i < n; i++) (void)hipSetDevice(0);
    printf("hipSetDevice: %.1f ns\n", ns_per(t, n));
    int d = 0;
    t = std::chrono::steady_clock::now();
    for (long i = 0; i < n; i++) (void)hipGetDevice(&d);
    printf("hipGetDevice: %.1f ns\n", ns_per(t, n));
    std::mutex mu;
    volatile long x = 0;
    t = std::chrono::steady_clock::now();
    for (long i = 0; i < n; i++) {
        std::lock_guard<std::mutex> g(mu);
        x = x + 1;
    }
    printf("mutex lock/unlock: %.1f ns\n", ns_per(t, n));
    return 0;
}
