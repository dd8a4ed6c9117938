// k_scan.hip — prefix sums used by the planner and the encoders.
//
//  * multi-job equal-length exclusive scans (reduce -> scan tile sums -> apply), 2048
//    elements per 256-thread tile, 16-byte-friendly sequential per-thread ranges;
//  * single-block segmented scans over tile aggregates (tile arrays are small: one entry
//    per 2048 positions / 256 elements), generic over the combine operator.
#include "kpw_device.h"
#include "kpw_kernels.h"
#include "kpw_scan.h"

namespace kpw {

// ------------------------------------------------------------------ functors

struct RawF {
    const uint32_t *raw; uint64_t *P;
    __device__ uint64_t get(uint32_t, uint64_t i) const { return raw[i]; }
    __device__ void put(uint32_t, uint64_t i, uint64_t v) const { P[i] = v; }
};
struct PcntF {
    const DevCol *cols; const uint32_t *opt;
    __device__ uint64_t get(uint32_t j, uint64_t w) const { return __popcll(cols[opt[j]].pres[w]); }
    __device__ void put(uint32_t j, uint64_t w, uint64_t v) const { cols[opt[j]].pcnt[w] = (uint32_t)v; }
};
struct EvF {
    const uint8_t *ev; uint32_t *E; uint64_t stride;
    __device__ uint64_t get(uint32_t j, uint64_t i) const { return ev[j * stride + i]; }
    __device__ void put(uint32_t j, uint64_t i, uint64_t v) const { E[j * stride + i] = (uint32_t)v; }
};

template <class F>
__global__ void __launch_bounds__(KPW_BLOCK) k_mj_tsum(F f, uint64_t len, uint32_t tpj, uint64_t *tsum)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x, j = t / tpj, tile = t % tpj;
    const uint64_t i0 = (uint64_t)tile * KPW_TILE_P + (uint64_t)threadIdx.x * 8;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) if (i0 + k < len) s += f.get(j, i0 + k);
    s = block_reduce<uint64_t, OpSum64>(s, lds);
    if (threadIdx.x == 0) tsum[t] = s;
}

// one block per job: exclusive scan of its tiles' sums; writes the job total to tsum[njobs*tpj + j]
__global__ void __launch_bounds__(KPW_BLOCK) k_mj_tscan(uint64_t *tsum, uint32_t tpj, uint32_t njobs)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t j = blockIdx.x;
    uint64_t carry = 0;
    for (uint32_t b = 0; b < tpj; b += KPW_BLOCK) {
        const uint32_t k = b + threadIdx.x;
        uint64_t v = k < tpj ? tsum[(uint64_t)j * tpj + k] : 0;
        uint64_t tot;
        uint64_t ex = block_scan_excl<uint64_t, OpSum64>(v, lds, &tot);
        if (k < tpj) tsum[(uint64_t)j * tpj + k] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) tsum[(uint64_t)njobs * tpj + j] = carry;
}

template <class F>
__global__ void __launch_bounds__(KPW_BLOCK) k_mj_tapply(F f, uint64_t len, uint32_t tpj, uint32_t njobs, const uint64_t *tsum)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x, j = t / tpj, tile = t % tpj;
    const uint64_t i0 = (uint64_t)tile * KPW_TILE_P + (uint64_t)threadIdx.x * 8;
    uint64_t v[8], s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) { v[k] = (i0 + k < len) ? f.get(j, i0 + k) : 0; s += v[k]; }
    uint64_t tot;
    uint64_t ex = block_scan_excl<uint64_t, OpSum64>(s, lds, &tot) + tsum[t];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (i0 + k < len) f.put(j, i0 + k, ex);
        ex += v[k];
    }
    if (tile == tpj - 1 && threadIdx.x == 0) f.put(j, len, tsum[(uint64_t)njobs * tpj + j]);
}

template <class F>
static void mj_scan(F f, uint64_t len, uint32_t njobs, uint64_t *tmp, hipStream_t s)
{
    if (!njobs) return;
    const uint32_t tpj = (uint32_t)((len + KPW_TILE_P - 1) / KPW_TILE_P) ? (uint32_t)((len + KPW_TILE_P - 1) / KPW_TILE_P) : 1;
    const uint32_t nt = tpj * njobs;
    hipLaunchKernelGGL(k_mj_tsum<F>, dim3(nt), dim3(KPW_BLOCK), 0, s, f, len, tpj, tmp);
    hipLaunchKernelGGL(k_mj_tscan, dim3(njobs), dim3(KPW_BLOCK), 0, s, tmp, tpj, njobs);
    hipLaunchKernelGGL(k_mj_tapply<F>, dim3(nt), dim3(KPW_BLOCK), 0, s, f, len, tpj, njobs, (const uint64_t *)tmp);
}

uint64_t mj_scan_tmp_words(uint64_t len, uint32_t njobs)
{
    uint64_t tpj = (len + KPW_TILE_P - 1) / KPW_TILE_P;
    if (!tpj) tpj = 1;
    return tpj * njobs + njobs + 1;
}

void launch_prefix_raw(const uint32_t *raw, uint64_t n, uint64_t *P, uint64_t *tmp, hipStream_t s)
{
    RawF f{raw, P};
    mj_scan(f, n, 1, tmp, s);
}

void launch_pcnt_scan(const DevCol *cols_d, const uint32_t *opt_d, uint32_t nopt, uint64_t nwords, uint64_t *tmp, hipStream_t s)
{
    PcntF f{cols_d, opt_d};
    mj_scan(f, nwords, nopt, tmp, s);
}

void launch_scan_events(const uint8_t *ev, uint32_t *E, uint64_t n, uint32_t njobs, uint64_t *tmp, hipStream_t s)
{
    EvF f{ev, E, n + 1};
    mj_scan(f, n, njobs, tmp, s);
}

// ------------------------------------------------------------------ single-block segmented tile scans
// Exclusive, segmented by job id (seg[t]); job totals written to tot[job] when tot != nullptr.

// Each thread owns SEG_PER consecutive elements: a sequential segmented scan in registers,
// then one Hillis-Steele segmented scan over the 256 thread aggregates per chunk of
// 256*SEG_PER elements, carrying (value, segment) between chunks.
constexpr int SEG_PER = 8;

template <typename T, typename Op>
__global__ void __launch_bounds__(KPW_BLOCK) k_seg_tile_scan(const T *in, T *out, const uint32_t *seg, uint32_t n, T *tot)
{
    __shared__ T lv[KPW_BLOCK];
    __shared__ uint32_t lh[KPW_BLOCK];
    __shared__ T lcarry;
    __shared__ uint32_t lcarry_seg;
    if (threadIdx.x == 0) { lcarry = Op::id(); lcarry_seg = 0xffffffffu; }
    __syncthreads();
    const uint32_t CH = KPW_BLOCK * SEG_PER;
    for (uint32_t b = 0; b < n; b += CH) {
        const uint32_t k0 = b + threadIdx.x * SEG_PER;
        T v[SEG_PER];
        uint32_t sg[SEG_PER];
        // local inclusive segmented scan; `head` = a segment starts inside my range
        T acc = Op::id();
        uint32_t head = 0;
        uint32_t prev = (k0 == 0) ? 0xffffffffu : (k0 - 1 < n ? seg[k0 - 1] : 0xfffffffeu);
        if (k0 == b && b != 0) prev = lcarry_seg;
        const uint32_t first_seg = k0 < n ? seg[k0] : 0xfffffffeu;
#pragma unroll
        for (int i = 0; i < SEG_PER; i++) {
            const uint32_t k = k0 + i;
            sg[i] = k < n ? seg[k] : 0xfffffffeu;
            v[i] = k < n ? in[k] : Op::id();
            const uint32_t p = i ? sg[i - 1] : prev;
            if (sg[i] != p) { head = 1; acc = v[i]; } else acc = Op::op(acc, v[i]);
        }
        // block scan over (acc, head) of the threads; thread t's aggregate covers its range
        lv[threadIdx.x] = acc;
        lh[threadIdx.x] = head;
        __syncthreads();
        for (int d = 1; d < KPW_BLOCK; d <<= 1) {
            T xv = Op::id();
            uint32_t xh = 0;
            const bool take = (int)threadIdx.x >= d;
            if (take) { xv = lv[threadIdx.x - d]; xh = lh[threadIdx.x - d]; }
            __syncthreads();
            if (take) {
                const uint32_t myh = lh[threadIdx.x];
                if (!myh) lv[threadIdx.x] = Op::op(xv, lv[threadIdx.x]);
                lh[threadIdx.x] = myh | xh;
            }
            __syncthreads();
        }
        // exclusive prefix entering my range (value continuing my first segment)
        T in_pre;
        if (threadIdx.x == 0) in_pre = lcarry;
        else in_pre = lv[threadIdx.x - 1];
        const uint32_t pre_head = threadIdx.x == 0 ? 0u : lh[threadIdx.x - 1];
        // fold the carry into everything before the chunk's first head
        if (threadIdx.x != 0 && !pre_head) in_pre = Op::op(lcarry, in_pre);
        // does my first element continue the incoming segment?
        const bool cont = (k0 < n) && (first_seg == prev);
        T run = cont ? in_pre : Op::id();
#pragma unroll
        for (int i = 0; i < SEG_PER; i++) {
            const uint32_t k = k0 + i;
            if (k >= n) break;
            const uint32_t p = i ? sg[i - 1] : prev;
            if (sg[i] != p) run = Op::id();
            out[k] = run;
            run = Op::op(run, v[i]);
            const bool last_of_seg = (k + 1 >= n) || (seg[k + 1] != sg[i]);
            if (last_of_seg && tot) tot[sg[i]] = run;
        }
        __syncthreads();
        // carry = inclusive value at the last valid element of this chunk
        const uint32_t last = (b + CH <= n) ? (b + CH - 1) : (n - 1);
        if (k0 <= last && last < k0 + SEG_PER) { lcarry = run; lcarry_seg = seg[last]; }
        __syncthreads();
    }
}

template <typename T, typename Op>
void seg_tile_scan(const T *in, T *out, const uint32_t *seg, uint32_t n, T *tot, hipStream_t s)
{
    if (!n) return;
    hipLaunchKernelGGL((k_seg_tile_scan<T, Op>), dim3(1), dim3(KPW_BLOCK), 0, s, in, out, seg, n, tot);
}

template void seg_tile_scan<uint32_t, OpSum32>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t, uint32_t *, hipStream_t);
template void seg_tile_scan<uint64_t, OpSum64>(const uint64_t *, uint64_t *, const uint32_t *, uint32_t, uint64_t *, hipStream_t);
template void seg_tile_scan<int64_t, OpMaxI64>(const int64_t *, int64_t *, const uint32_t *, uint32_t, int64_t *, hipStream_t);
template void seg_tile_scan<uint32_t, OpMapCompose>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t, uint32_t *, hipStream_t);

}  // namespace kpw
