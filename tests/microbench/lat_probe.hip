// lat_probe.hip — hardware probe (test infrastructure): dependent-chain latency, in shader
// clocks per step, of the scalar/lane primitives the K7 match loop is built from.
//   hipcc -O3 --offload-arch=gfx950 lat_probe.hip -o build/lat_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#pragma clang diagnostic ignored "-Winline-asm"
#define N 4096

template <int K>
__global__ void __launch_bounds__(64, 1) k_lat(const uint32_t *seed, uint64_t *cyc)
{
    uint32_t h = __builtin_amdgcn_readfirstlane(seed[0]);
    uint32_t v = seed[threadIdx.x + 1];
    asm volatile("v_mov_b32 v100, %0\n\tv_mov_b32 v101, %0\n\tv_accvgpr_write_b32 a0, %0\n\tv_accvgpr_write_b32 a1, %0\n\ts_nop 4"
                 : : "v"(v) : "v100", "v101", "a0", "a1");
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int k = 0; k < N; k++) {
        if (K == 0)   // SALU only: mul + shift + and
            asm volatile("s_mul_i32 %0, %0, 0x1e35a7bd\n\ts_lshr_b32 %0, %0, 18\n\ts_and_b32 %0, %0, 63" : "+s"(h));
        else if (K == 1)   // readlane of a fixed VGPR at the lane h, then SALU
            asm volatile("v_readlane_b32 %0, v100, %0\n\ts_and_b32 %0, %0, 63" : "+s"(h) :: "v100");
        else if (K == 2)   // indexed VGPR row read + readlane
            asm volatile("s_set_gpr_idx_on %0, gpr_idx(SRC0)\n\tv_mov_b32 v102, v100\n\ts_set_gpr_idx_off\n\ts_nop 1\n\t"
                         "v_readlane_b32 %0, v102, %0\n\ts_and_b32 %0, %0, 1" : "+s"(h) :: "v100", "v101", "v102", "m0");
        else if (K == 3)   // readlane then SALU then VALU writelane then readlane (table update shape)
            asm volatile("v_readlane_b32 %0, v100, %0\n\ts_and_b32 %0, %0, 63\n\ts_mov_b32 m0, %0\n\t"
                         "v_writelane_b32 v100, %0, m0\n\ts_nop 1" : "+s"(h) :: "v100", "m0");
        else if (K == 4)   // SALU chain with a taken branch each step
            asm volatile("s_add_u32 %0, %0, 1\n\ts_and_b32 %0, %0, 63\n\ts_branch 1f\n1:" : "+s"(h));
        else if (K == 5)   // indexed AGPR row read + readlane + and
            asm volatile("s_set_gpr_idx_on %0, gpr_idx(SRC0)\n\tv_accvgpr_read_b32 v102, a0\n\ts_set_gpr_idx_off\n\ts_nop 1\n\t"
                         "v_readlane_b32 %0, v102, %0\n\ts_and_b32 %0, %0, 1" : "+s"(h) :: "a0", "a1", "v102", "m0");
        else if (K == 8)   // static AGPR read + readlane + and
            asm volatile("v_accvgpr_read_b32 v102, a1\n\ts_nop 1\n\t"
                         "v_readlane_b32 %0, v102, %0\n\ts_and_b32 %0, %0, 1" : "+s"(h) :: "a0", "a1", "v102");
        else if (K == 9)   // readlane + s_mul hash + shift (lane from the hash), as in agpr_probe
            asm volatile("v_readlane_b32 %0, v100, %0\n\ts_mul_i32 %0, %0, 0x9e3779b1\n\ts_lshr_b32 %0, %0, 26" : "+s"(h) :: "v100");
        else if (K == 6)   // v_readfirstlane of a VALU result (VALU -> SGPR -> VALU round trip)
            asm volatile("v_add_u32 v102, %0, v100\n\ts_nop 1\n\tv_readfirstlane_b32 %0, v102\n\ts_and_b32 %0, %0, 63" : "+s"(h) :: "v100", "v102");
        else if (K == 7)   // s_cmp + conditional branch not taken
            asm volatile("s_add_u32 %0, %0, 1\n\ts_cmp_eq_u32 %0, 12345678\n\ts_cbranch_scc1 1f\n1:" : "+s"(h));
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) { cyc[K * 2] = t1 - t0; cyc[K * 2 + 1] = h; }
}

int main(int argc, char **argv)
{
    const int K = atoi(argv[1]);
    uint32_t *ds; uint64_t *dc;
    (void)hipMalloc(&ds, 65 * 4); (void)hipMalloc(&dc, 24 * 8);
    uint32_t hs[65]; for (int i = 0; i < 65; i++) hs[i] = i * 7 + 1;
    (void)hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
    switch (K) {
    case 0: hipLaunchKernelGGL(k_lat<0>, 1, 64, 0, 0, ds, dc); break;
    case 1: hipLaunchKernelGGL(k_lat<1>, 1, 64, 0, 0, ds, dc); break;
    case 2: hipLaunchKernelGGL(k_lat<2>, 1, 64, 0, 0, ds, dc); break;
    case 3: hipLaunchKernelGGL(k_lat<3>, 1, 64, 0, 0, ds, dc); break;
    case 4: hipLaunchKernelGGL(k_lat<4>, 1, 64, 0, 0, ds, dc); break;
    case 5: hipLaunchKernelGGL(k_lat<5>, 1, 64, 0, 0, ds, dc); break;
    case 6: hipLaunchKernelGGL(k_lat<6>, 1, 64, 0, 0, ds, dc); break;
    case 7: hipLaunchKernelGGL(k_lat<7>, 1, 64, 0, 0, ds, dc); break;
    case 8: hipLaunchKernelGGL(k_lat<8>, 1, 64, 0, 0, ds, dc); break;
    case 9: hipLaunchKernelGGL(k_lat<9>, 1, 64, 0, 0, ds, dc); break;
    }
    (void)hipDeviceSynchronize();
    uint64_t c[24]; (void)hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
    const char *names[] = {"salu mul+shr+and (3 dep)", "readlane + and", "idx VGPR row read + readlane + and", "readlane+and+m0+writelane",
                           "add+and+branch(taken)", "idx AGPR row read + readlane + and", "v_add + readfirstlane + and",
                           "add+cmp+cbranch(not taken)", "static AGPR read + readlane + and", "readlane + s_mul + s_lshr"};
    printf("%-38s %7.2f ticks/step (s_memtime)\n", names[K], (double)c[2 * K] / N);
    fflush(stdout);
    return 0;
}
