// agpr_probe.hip — hardware probe (test infrastructure): does VGPR index mode
// (s_set_gpr_idx_on) apply to the AGPR operand of v_accvgpr_read/write on gfx950, and what
// does a dependent indexed read cost (AGPR and VGPR tables)?  Prints values and cycles.
//   hipcc -O3 --offload-arch=gfx950 agpr_probe.hip -o build/agpr_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define A_CLOBBERS "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207", "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223", "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239", "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255"

#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ uint32_t a_row(uint32_t r)
{
    uint32_t x;
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_accvgpr_read_b32 %0, a0\n\ts_set_gpr_idx_off" : "=v"(x) : "s"(r & 255u) : "m0");
    return x;
}
__device__ __forceinline__ void a_set_row(uint32_t r, uint32_t v)
{
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(DST)\n\tv_accvgpr_write_b32 a0, %0\n\ts_set_gpr_idx_off" : : "v"(v), "s"(r & 255u) : "m0");
}

__global__ void __launch_bounds__(64, 1) k_probe(const uint32_t *idx, uint32_t *out, int n, uint64_t *cyc)
{
    const uint32_t lane = threadIdx.x;
    asm volatile("; reserve a0..a255" ::: A_CLOBBERS);
    for (uint32_t r = 0; r < 256; r++) a_set_row(r, lane * 1000u + r);
    for (int k = 0; k < 8; k++) {
        const uint32_t r = __builtin_amdgcn_readfirstlane(idx[k]);
        out[k * 64 + lane] = a_row(r);
    }
    uint32_t s0, s77, s255;
    asm volatile("v_accvgpr_read_b32 %0, a0\n\tv_accvgpr_read_b32 %1, a77\n\tv_accvgpr_read_b32 %2, a255" : "=v"(s0), "=v"(s77), "=v"(s255));
    out[8 * 64 + lane] = s0;
    out[9 * 64 + lane] = s77;
    out[10 * 64 + lane] = s255;
    uint32_t h = __builtin_amdgcn_readfirstlane(idx[0]);
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int k = 0; k < n; k++) {
        const uint32_t x = a_row(h);
        h = (__builtin_amdgcn_readlane(x, h & 63) * 2654435761u) >> 24;
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = h; }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 2; } } while (0)
int main()
{
    uint32_t hidx[8] = {0, 1, 5, 77, 128, 200, 254, 255};
    uint32_t *didx, *dout; uint64_t *dcyc;
    CK(hipMalloc(&didx, 32)); CK(hipMalloc(&dout, 11 * 64 * 4)); CK(hipMalloc(&dcyc, 16));
    CK(hipMemcpy(didx, hidx, 32, hipMemcpyHostToDevice));
    const int n = 10000;
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, didx, dout, n, dcyc);
    CK(hipDeviceSynchronize());
    uint32_t o[11 * 64]; uint64_t c[2];
    CK(hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost)); CK(hipMemcpy(c, dcyc, 16, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int k = 0; k < 8; k++)
        for (int l = 0; l < 64; l++) if (o[k * 64 + l] != l * 1000u + hidx[k]) { if (bad < 10) printf("indexed read row %u lane %d got %u\n", hidx[k], l, o[k * 64 + l]); bad++; }
    const uint32_t st[3] = {0, 77, 255};
    for (int k = 0; k < 3; k++)
        for (int l = 0; l < 64; l++) if (o[(8 + k) * 64 + l] != l * 1000u + st[k]) { if (bad < 20) printf("static read a%u lane %d got %u\n", st[k], l, o[(8 + k) * 64 + l]); bad++; }
    printf("AGPR index mode: %s (%d bad); dependent indexed read+readlane chain: %.1f cycles/step\n", bad ? "FAIL" : "PASS", bad, (double)c[0] / n);
    return 0;
}
