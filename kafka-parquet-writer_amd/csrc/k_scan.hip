// k_scan.hip — prefix sums used by the planner and the encoders.
//
//  * multi-job equal-length exclusive scans (reduce -> scan tile sums -> apply), 2048
//    elements per 256-thread tile, 16-byte-friendly sequential per-thread ranges;
//  * multi-block segmented scans over tile aggregates (one entry per 2048 positions / 256
//    elements), generic over the combine operator.
#include "kpw_device.h"
#include "kpw_kernels.h"
#include "kpw_scan.h"
#include "memcache.h"

namespace kpw {

// ------------------------------------------------------------------ functors

struct RawF {
    const uint32_t *raw; uint64_t *P;
    __device__ uint64_t get(uint32_t, uint64_t i) const { return raw[i]; }
    __device__ void put(uint32_t, uint64_t i, uint64_t v) const { P[i] = v; }
};
// record lengths narrowed to T (u8 / u16) on the host; element 0 is `base` (the first boundary)
template <typename T>
struct NarrowF {
    const T *raw; uint64_t base; uint64_t *P;
    __device__ uint64_t get(uint32_t, uint64_t i) const { return i ? (uint64_t)raw[i] : base; }
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

void launch_prefix_narrow(const void *raw, int width, uint64_t base, uint64_t n, uint64_t *P, uint64_t *tmp, hipStream_t s)
{
    if (width == 1) mj_scan(NarrowF<uint8_t>{(const uint8_t *)raw, base, P}, n, 1, tmp, s);
    else mj_scan(NarrowF<uint16_t>{(const uint16_t *)raw, base, P}, n, 1, tmp, s);
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

// Multi-block, three phases over chunks of CH = 256 * SEG_PER elements (one block each):
//   1. per chunk, the segmented-scan pair (any head in the chunk, reduction since its last
//      head) — head = first element of a segment (seg[i] != seg[i-1]);
//   2. one thread scans the chunk pairs into each chunk's carry-in (running value of the
//      segment that continues into it);
//   3. per chunk, a sequential scan of SEG_PER elements per thread plus a Hillis-Steele scan
//      of the 256 thread aggregates, seeded with the carry-in; segment totals written at
//      each segment's last element.
constexpr int SEG_PER = 8;
constexpr uint32_t SEG_CH = KPW_BLOCK * SEG_PER;

// block-wide inclusive segmented scan of per-thread (value, head) pairs in LDS; returns
// nothing, leaves lv/lh holding the inclusive scan
template <typename T, typename Op>
__device__ __forceinline__ void seg_block_scan(T *lv, uint32_t *lh)
{
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
}

template <typename T, typename Op>
__global__ void __launch_bounds__(KPW_BLOCK) k_seg_reduce(const T *in, const uint32_t *seg, uint32_t n, T *bv, uint32_t *bh)
{
    __shared__ T lv[KPW_BLOCK];
    __shared__ uint32_t lh[KPW_BLOCK];
    const uint32_t k0 = blockIdx.x * SEG_CH + threadIdx.x * SEG_PER;
    T acc = Op::id();
    uint32_t head = 0;
    uint32_t prev = k0 == 0 ? 0xffffffffu : (k0 - 1 < n ? seg[k0 - 1] : 0xfffffffeu);
#pragma unroll
    for (int i = 0; i < SEG_PER; i++) {
        const uint32_t k = k0 + i;
        const uint32_t sg = k < n ? seg[k] : 0xfffffffeu;
        const T v = k < n ? in[k] : Op::id();
        if (sg != prev) { head = 1; acc = v; } else acc = Op::op(acc, v);
        prev = sg;
    }
    lv[threadIdx.x] = acc;
    lh[threadIdx.x] = head;
    __syncthreads();
    seg_block_scan<T, Op>(lv, lh);
    if (threadIdx.x == KPW_BLOCK - 1) { bv[blockIdx.x] = lv[threadIdx.x]; bh[blockIdx.x] = lh[threadIdx.x]; }
}

template <typename T, typename Op>
__global__ void k_seg_carry(T *bv, const uint32_t *bh, uint32_t nb)
{
    if (threadIdx.x != 0) return;
    T acc = Op::id();
    for (uint32_t b = 0; b < nb; b++) {
        const T v = bv[b];
        const uint32_t h = bh[b];
        bv[b] = acc;
        acc = h ? v : Op::op(acc, v);
    }
}

template <typename T, typename Op>
__global__ void __launch_bounds__(KPW_BLOCK) k_seg_apply(const T *in, T *out, const uint32_t *seg, uint32_t n, T *tot, const T *bv)
{
    __shared__ T lv[KPW_BLOCK];
    __shared__ uint32_t lh[KPW_BLOCK];
    const uint32_t b = blockIdx.x * SEG_CH;
    const T lcarry = bv[blockIdx.x];
    const uint32_t lcarry_seg = b == 0 ? 0xffffffffu : seg[b - 1];
    const uint32_t k0 = b + threadIdx.x * SEG_PER;
    T v[SEG_PER];
    uint32_t sg[SEG_PER];
    T acc = Op::id();
    uint32_t head = 0;
    const uint32_t prev = (k0 == 0) ? 0xffffffffu : (k0 - 1 < n ? seg[k0 - 1] : 0xfffffffeu);
    const uint32_t first_seg = k0 < n ? seg[k0] : 0xfffffffeu;
#pragma unroll
    for (int i = 0; i < SEG_PER; i++) {
        const uint32_t k = k0 + i;
        sg[i] = k < n ? seg[k] : 0xfffffffeu;
        v[i] = k < n ? in[k] : Op::id();
        const uint32_t p = i ? sg[i - 1] : prev;
        if (sg[i] != p) { head = 1; acc = v[i]; } else acc = Op::op(acc, v[i]);
    }
    lv[threadIdx.x] = acc;
    lh[threadIdx.x] = head;
    __syncthreads();
    seg_block_scan<T, Op>(lv, lh);
    // exclusive prefix entering my range, continuing my first segment
    T in_pre = threadIdx.x == 0 ? lcarry : lv[threadIdx.x - 1];
    const uint32_t pre_head = threadIdx.x == 0 ? 0u : lh[threadIdx.x - 1];
    if (threadIdx.x != 0 && !pre_head) in_pre = Op::op(lcarry, in_pre);
    (void)lcarry_seg;
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
}

void seg_scratch_free(SegScratch &sc)
{
    dev_free(sc.p);
    sc.p = nullptr;
    sc.bytes = 0;
}

template <typename T, typename Op>
void seg_tile_scan(const T *in, T *out, const uint32_t *seg, uint32_t n, T *tot, SegScratch *sc, hipStream_t s)
{
    if (!n) return;
    const uint32_t nb = (n + SEG_CH - 1) / SEG_CH;
    const size_t need = (size_t)nb * (sizeof(T) + sizeof(uint32_t)) + 64;
    if (need > sc->bytes) {
        // earlier scans of this handle may still read the old buffer on `s`
        if (sc->p) { (void)hipStreamSynchronize(s); dev_free(sc->p); }
        sc->bytes = need * 2;
        sc->p = dev_alloc(sc->bytes);
        if (!sc->p) { sc->bytes = 0; sc->failed = true; return; }
    }
    T *bv = (T *)sc->p;
    uint32_t *bh = (uint32_t *)((char *)sc->p + (((size_t)nb * sizeof(T) + 15) & ~(size_t)15));
    hipLaunchKernelGGL((k_seg_reduce<T, Op>), dim3(nb), dim3(KPW_BLOCK), 0, s, in, seg, n, bv, bh);
    hipLaunchKernelGGL((k_seg_carry<T, Op>), dim3(1), dim3(64), 0, s, bv, (const uint32_t *)bh, nb);
    hipLaunchKernelGGL((k_seg_apply<T, Op>), dim3(nb), dim3(KPW_BLOCK), 0, s, in, out, seg, n, tot, (const T *)bv);
}

template void seg_tile_scan<uint32_t, OpSum32>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t, uint32_t *, SegScratch *, hipStream_t);
template void seg_tile_scan<uint64_t, OpSum64>(const uint64_t *, uint64_t *, const uint32_t *, uint32_t, uint64_t *, SegScratch *, hipStream_t);
template void seg_tile_scan<int64_t, OpMaxI64>(const int64_t *, int64_t *, const uint32_t *, uint32_t, int64_t *, SegScratch *, hipStream_t);
template void seg_tile_scan<uint32_t, OpMapCompose>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t, uint32_t *, SegScratch *, hipStream_t);

}  // namespace kpw
