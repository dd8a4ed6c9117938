// idxrl_probe.hip — hardware probe (test infrastructure): does VGPR index mode (SRC0) apply
// to v_readlane_b32's vector source on gfx950, and does DPP wave_shl:1 shift lanes down by
// one?  Prints PASS/FAIL.
//   hipcc -O3 --offload-arch=gfx950 idxrl_probe.hip -o build/idxrl_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#pragma clang diagnostic ignored "-Winline-asm"

__global__ void __launch_bounds__(64, 1) k_probe(const uint32_t *sel, uint32_t *out)
{
    const uint32_t lane = threadIdx.x;
    // v106..v109 = lane * 16 + {0,1,2,3}
    asm volatile("v_lshlrev_b32 v106, 4, %0\n\t"
                 "v_add_u32 v107, 1, v106\n\t"
                 "v_add_u32 v108, 2, v106\n\t"
                 "v_add_u32 v109, 3, v106\n\ts_nop 4" : : "v"(lane) : "v106", "v107", "v108", "v109");
    for (int k = 0; k < 8; k++) {
        const uint32_t idx = __builtin_amdgcn_readfirstlane(sel[2 * k]);
        const uint32_t ln = __builtin_amdgcn_readfirstlane(sel[2 * k + 1]);
        uint32_t x;
        asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\t"
                     "v_readlane_b32 %0, v106, %2\n\t"
                     "s_set_gpr_idx_off\n\ts_nop 4"
                     : "=s"(x) : "s"(idx), "s"(ln) : "v106", "v107", "v108", "v109", "m0");
        if (lane == 0) out[k] = x;
    }
    uint32_t y;
    asm volatile("v_mov_b32_dpp %0, v106 wave_shl:1 row_mask:0xf bank_mask:0xf\n\ts_nop 1" : "=v"(y) : : "v106");
    out[8 + lane] = y;
}

int main()
{
    uint32_t hs[16] = {0, 5, 1, 5, 2, 63, 3, 0, 3, 63, 1, 17, 0, 0, 2, 40};
    uint32_t *ds, *dout;
    (void)hipMalloc(&ds, sizeof hs); (void)hipMalloc(&dout, 72 * 4);
    (void)hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, 1, 64, 0, 0, ds, dout);
    (void)hipDeviceSynchronize();
    uint32_t o[72];
    (void)hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int k = 0; k < 8; k++) {
        const uint32_t want = hs[2 * k + 1] * 16 + hs[2 * k];
        if (o[k] != want) { printf("readlane idx %u lane %u: got %u want %u\n", hs[2 * k], hs[2 * k + 1], o[k], want); bad++; }
    }
    int dbad = 0;
    for (int l = 0; l < 63; l++) if (o[8 + l] != (uint32_t)(l + 1) * 16) dbad++;
    printf("index-mode readlane: %s; DPP wave_shl:1: %s (lane 63 = %u)\n", bad ? "FAIL" : "PASS", dbad ? "FAIL" : "PASS", o[8 + 63]);
    if (dbad) for (int l = 0; l < 8; l++) printf("  lane %d: %u\n", l, o[8 + l]);
    return 0;
}
