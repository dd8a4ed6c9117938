// vtab_probe.hip — codegen probe (compile-only): a 128-VGPR table pinned to v128..v255
// (the allocator is capped at 128 registers), indexed with s_set_gpr_idx_on.  Checked:
// no scratch, and the kernel descriptor accounts for all 256 VGPRs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VT_CLOBBERS \
    "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", \
    "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", \
    "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", \
    "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", \
    "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", \
    "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", \
    "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", \
    "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", \
    "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", \
    "v254", "v255"

__device__ __forceinline__ uint32_t tab_row(uint32_t r)
{
    uint32_t x;
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_mov_b32 %0, v128\n\ts_set_gpr_idx_off" : "=v"(x) : "s"(r) : "m0");
    return x;
}
__device__ __forceinline__ void tab_set_row(uint32_t r, uint32_t v)
{
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(DST)\n\tv_mov_b32 v128, %0\n\ts_set_gpr_idx_off" : : "v"(v), "s"(r) : "m0");
}

__global__ void __launch_bounds__(64, 2) __attribute__((amdgpu_num_vgpr(128))) kC(const uint32_t *idx, uint32_t *out, int n)
{
    asm volatile("; table registers v128..v255 reserved" ::: VT_CLOBBERS);
    for (uint32_t r = 0; r < 128; r++) tab_set_row(r, 0);
    uint32_t acc = 0;
    for (int k = 0; k < n; k++) {
        uint32_t h = __builtin_amdgcn_readfirstlane(idx[k]);
        uint32_t r = h & 127, L = (h >> 10) & 63;
        uint32_t x = tab_row(r);
        acc += __builtin_amdgcn_readlane(x, L);
        uint32_t nv = threadIdx.x == L ? x + k : x;
        tab_set_row(r, nv);
    }
    out[threadIdx.x] = acc;
}
