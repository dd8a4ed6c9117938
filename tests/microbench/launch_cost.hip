// launch_cost.hip — test infrastructure: host cost of a kernel launch (empty kernel, by-value
// argument of 8 / 256 / 1024 bytes), on one stream, without and with a sync every 50 launches.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
template <int B> struct Arg { unsigned char b[B]; };
template <int B> __global__ void k_empty(Arg<B> a) { if (a.b[0] == 255 && threadIdx.x == 9999) a.b[1] = 0; }
template <int B> static void run(hipStream_t s)
{
    Arg<B> a{};
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_empty<B>, dim3(256), dim3(256), 0, s, a);
    hipStreamSynchronize(s);
    const int n = 20000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_empty<B>, dim3(256), dim3(256), 0, s, a);
    const double issue = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    hipStreamSynchronize(s);
    const double all = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) { hipLaunchKernelGGL(k_empty<B>, dim3(256), dim3(256), 0, s, a); if (i % 50 == 49) hipStreamSynchronize(s); }
    hipStreamSynchronize(s);
    const double chunked = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    printf("arg %4d B: issue %.2f us/launch, issue+drain %.2f, with a sync per 50 launches %.2f\n", B, issue, all, chunked);
}
int main()
{
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    run<8>(s); run<256>(s); run<1024>(s);
    return 0;
}
