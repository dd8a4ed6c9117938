// k_scan.hip — prefix sums used by the planner and the encoders.
//
//  * multi-job equal-length exclusive scans (reduce -> scan tile sums -> apply), 2048
//    elements per 256-thread tile, 16-byte-friendly sequential per-thread ranges;
//  * multi-block segmented scans over tile aggregates (one entry per 2048 positions / 256
//    elements), generic over the combine operator.
#include <algorithm>

#include "kpw_device.h"
#include "kpw_kernels.h"
#include "kpw_scan.h"
#include "kpw_lookback.h"
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
// The planner's prefixes, one multi-job scan over groups of 8 positions: jobs [0, nev) the event
// streams (element g = the 8 event bytes of positions [8g, 8g + 8) summed from one 8-byte load;
// E8[j * (groups + 1) + g] = the prefix), job nev the raw record sizes (P8[g] = the bytes of
// records [0, 8g)) and job nev + 1, when val is given, the folded sizes (Q8).  A position's prefix
// is its group's plus up to 7 elements (k_plan pref8).
struct PlanPrefixF {
    const uint64_t *ev; uint32_t *E8; uint64_t groups; uint32_t nev;
    const uint32_t *raw, *val; uint64_t n; uint64_t *P8, *Q8;
    __device__ uint64_t get(uint32_t j, uint64_t g) const
    {
        if (j < nev) {
            uint64_t b = ev[j * groups + g];
            b = (b & 0x00ff00ff00ff00ffull) + ((b >> 8) & 0x00ff00ff00ff00ffull);
            b += b >> 16;
            b += b >> 32;
            return b & 0xffffu;
        }
        const uint32_t *x = j == nev ? raw : val;
        const uint64_t i0 = g * 8;
        uint64_t s = 0;
        if (i0 + 8 <= n) {
            const uint4 u = *(const uint4 *)(x + i0), v = *(const uint4 *)(x + i0 + 4);
            s = (uint64_t)u.x + u.y + u.z + u.w + v.x + v.y + v.z + v.w;
        } else {
            for (uint64_t i = i0; i < n; i++) s += x[i];
        }
        return s;
    }
    __device__ void put(uint32_t j, uint64_t g, uint64_t v) const
    {
        if (j < nev) E8[j * (groups + 1) + g] = (uint32_t)v;
        else (j == nev ? P8 : Q8)[g] = v;
    }
};

// Multi-job equal-length exclusive sums, reduce -> scan tile sums -> apply (three launches).
// r04: a single-pass look-back version measured 1.8x slower on the planner's 400 M-element
// event scans (each tile's look-back is a round trip of uncached agent-scope loads; these
// scans stream their input once more instead).  Tiles of KPW_TILE_P elements, 8 consecutive
// ones per thread.
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

// Two-launch version when the tile sums are few (MJ2_MAX_READS: all apply blocks together read
// about nt * tpj / 2 of them): each apply block sums the tile sums before it itself (L2-resident)
// instead of a third launch scanning them (the writer's record offsets: 4.4 k tiles per job).
// (r04: a single-pass look-back version of these scans took 0.48 ms per writer job on the
// record offsets where the three launches took 0.09: each tile's look-back polls its
// predecessors' status through uncached device-scope loads.)
constexpr uint64_t MJ2_MAX_READS = 16ull << 20;
template <class F>
__global__ void __launch_bounds__(KPW_BLOCK) k_mj_tapply_c(F f, uint64_t len, uint32_t tpj, const uint64_t *tsum)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x, j = t / tpj, tile = t % tpj;
    uint64_t c = 0;
    for (uint32_t k = threadIdx.x; k < tile; k += KPW_BLOCK) c += tsum[(uint64_t)j * tpj + k];
    const uint64_t carry = block_reduce<uint64_t, OpSum64>(c, lds);
    const uint64_t i0 = (uint64_t)tile * KPW_TILE_P + (uint64_t)threadIdx.x * 8;
    uint64_t v[8], s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) { v[k] = (i0 + k < len) ? f.get(j, i0 + k) : 0; s += v[k]; }
    uint64_t tot;
    uint64_t ex = block_scan_excl<uint64_t, OpSum64>(s, lds, &tot) + carry;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (i0 + k < len) f.put(j, i0 + k, ex);
        ex += v[k];
    }
    if (tile == tpj - 1 && threadIdx.x == 0) f.put(j, len, carry + tot);
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

// the reduce-then-scan scratch (tile sums): w == nullptr if it cannot grow (sc->failed set)
uint64_t *scan_tmp(SegScratch *sc, uint64_t words, hipStream_t s)
{
    const size_t need = (size_t)words * 8 + 64;
    if (need > sc->tmp_bytes) {
        if (sc->tmp) dev_free_after(sc->tmp, s);   // earlier scans may still use it on `s`
        sc->tmp_bytes = need * 2;
        sc->tmp = dev_alloc(sc->tmp_bytes);
        if (!sc->tmp) { sc->tmp_bytes = 0; sc->failed = true; return nullptr; }
    }
    return (uint64_t *)sc->tmp;
}

// Look-back fallbacks counted since the previous call (kpw_lookback.h), read and cleared: the
// count lives in its own word (SegScratch::fails), which the status words' growth and
// epoch-wrap clears never touch, so one early in an encode is still seen at its end.
int lb_failures(SegScratch *sc, hipStream_t s)
{
    if (!sc->fails) return 0;
    uint32_t n = 0;
    if (hipMemcpyAsync(&n, sc->fails, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    if (n && (hipMemsetAsync(sc->fails, 0, 4, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)) return -1;
    return (int)n;
}

// Status words of one single-pass launch (nwords: ntiles x scans; w == nullptr: allocation
// failed, sc->failed set).  Grown buffers start zeroed; the epoch wraps after 2^15 - 1
// launches with a clear.
LbView lb_prepare(SegScratch *sc, uint64_t nwords, hipStream_t s)
{
    const size_t need = 64 + (size_t)nwords * 8;
    if (!sc->fails) {
        sc->fails = (uint32_t *)dev_alloc(64);
        if (!sc->fails || hipMemsetAsync(sc->fails, 0, 64, s) != hipSuccess) {
            sc->failed = true; return LbView{nullptr, 0, nullptr, 0};
        }
    }
    if (need > sc->bytes) {
        // earlier scans of this handle may still use the old buffer on `s`
        if (sc->p) dev_free_after(sc->p, s);
        // (at least 16 MiB: one cleared buffer serves every scan of a typical job, instead of a
        // clear at each first larger scan)
        sc->bytes = std::max<size_t>(need * 2, 16u << 20);
        sc->p = dev_alloc(sc->bytes);
        if (!sc->p || hipMemsetAsync(sc->p, 0, sc->bytes, s) != hipSuccess) {
            sc->bytes = 0; sc->failed = true; return LbView{nullptr, 0, nullptr, 0};
        }
        sc->epoch = 0;
    }
    if (++sc->epoch >= (1u << 15)) {
        if (hipMemsetAsync(sc->p, 0, sc->bytes, s) != hipSuccess) { sc->failed = true; return LbView{nullptr, 0, nullptr, 0}; }
        sc->epoch = 1;
    }
    // polls before a look-back falls back (each an agent-scope load plus a short sleep; a
    // running predecessor publishes within microseconds).  KPW_LB_SPIN=0 falls back at once,
    // which the tests use to exercise every fallback.
    static const uint32_t spin = [] {
        const char *e = getenv("KPW_LB_SPIN");
        return e ? (uint32_t)strtoul(e, nullptr, 10) : (1u << 13);
    }();
    return LbView{(uint64_t *)sc->p, sc->epoch, sc->fails, spin};
}

template <class F>
static void mj_scan(F f, uint64_t len, uint32_t njobs, SegScratch *sc, hipStream_t s)
{
    if (!njobs) return;
    const uint32_t tpj = (uint32_t)std::max<uint64_t>(1, (len + KPW_TILE_P - 1) / KPW_TILE_P);
    const uint32_t nt = tpj * njobs;
    uint64_t *tmp = scan_tmp(sc, (uint64_t)nt + njobs + 1, s);
    if (!tmp) return;
    hipLaunchKernelGGL(k_mj_tsum<F>, dim3(nt), dim3(KPW_BLOCK), 0, s, f, len, tpj, tmp);
    if ((uint64_t)nt * tpj / 2 <= MJ2_MAX_READS) {
        hipLaunchKernelGGL(k_mj_tapply_c<F>, dim3(nt), dim3(KPW_BLOCK), 0, s, f, len, tpj, (const uint64_t *)tmp);
        return;
    }
    hipLaunchKernelGGL(k_mj_tscan, dim3(njobs), dim3(KPW_BLOCK), 0, s, tmp, tpj, njobs);
    hipLaunchKernelGGL(k_mj_tapply<F>, dim3(nt), dim3(KPW_BLOCK), 0, s, f, len, tpj, njobs, (const uint64_t *)tmp);
}

void launch_prefix_raw(const uint32_t *raw, uint64_t n, uint64_t *P, SegScratch *sc, hipStream_t s)
{
    RawF f{raw, P};
    mj_scan(f, n, 1, sc, s);
}

void launch_prefix_narrow(const void *raw, int width, uint64_t base, uint64_t n, uint64_t *P, SegScratch *sc, hipStream_t s)
{
    if (width == 1) mj_scan(NarrowF<uint8_t>{(const uint8_t *)raw, base, P}, n, 1, sc, s);
    else mj_scan(NarrowF<uint16_t>{(const uint16_t *)raw, base, P}, n, 1, sc, s);
}

void launch_pcnt_scan(const DevCol *cols_d, const uint32_t *opt_d, uint32_t nopt, uint64_t nwords, SegScratch *sc, hipStream_t s)
{
    PcntF f{cols_d, opt_d};
    mj_scan(f, nwords, nopt, sc, s);
}

void launch_plan_prefix(const uint8_t *ev, uint32_t *E8, uint32_t nev, uint64_t ev_stride, const uint32_t *raw, const uint32_t *val,
                        uint64_t n, uint64_t *P8, uint64_t *Q8, SegScratch *sc, hipStream_t s)
{
    PlanPrefixF f{(const uint64_t *)ev, E8, ev_stride / 8, nev, raw, val, n, P8, Q8};
    mj_scan(f, ev_stride / 8, nev + 1 + (val ? 1 : 0), sc, s);
}

// ------------------------------------------------------------------ segmented tile scans
// Exclusive, segmented by job id (seg[t]); job totals written to tot[job] when tot != nullptr.
// One launch: per chunk of CH = 256 * SEG_PER elements, a sequential scan of SEG_PER elements
// per thread plus a block scan of the 256 (value, head) pairs; a chunk that contains a segment
// head publishes its inclusive value at once (the value leaving it does not depend on earlier
// chunks), others publish their aggregate and look back for their carry-in.
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

// Fallback: chunk q's segmented aggregate (from its last segment head) recomputed
// sequentially, as k_seg_scan's block scan leaves it; inclusive when the chunk has a head.
template <typename T, typename Op>
struct SegFb {
    const T *in;
    const uint32_t *seg;
    uint32_t n;
    __device__ void operator()(uint32_t q, T &v, bool &inc) const
    {
        const uint32_t b = q * SEG_CH;
        uint32_t p = (b == 0) ? 0xffffffffu : (b - 1 < n ? seg[b - 1] : 0xfffffffeu);
        T acc = Op::id();
        bool head = false;
        for (uint32_t k = b; k < b + SEG_CH; k++) {
            const uint32_t sg = k < n ? seg[k] : 0xfffffffeu;
            const T x = k < n ? in[k] : Op::id();
            if (sg != p) { head = true; acc = x; } else acc = Op::op(acc, x);
            p = sg;
        }
        v = acc;
        inc = q == 0 || head;
    }
};

template <typename T, typename Op>
__global__ void __launch_bounds__(KPW_BLOCK) k_seg_scan(const T *in, T *out, const uint32_t *seg, uint32_t n, T *tot, uint32_t nb,
                                                        LbView L)
{
    __shared__ T lv[KPW_BLOCK];
    __shared__ uint32_t lh[KPW_BLOCK];
    __shared__ T lcarry_s;
    const uint32_t blk = blockIdx.x;
    const uint32_t b = blk * SEG_CH;
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
    const T agg = lv[KPW_BLOCK - 1];
    const bool has_head = lh[KPW_BLOCK - 1] != 0;
    // the chunk's first element continues a segment of an earlier chunk: it needs a carry-in
    const bool need = b > 0 && b < n && seg[b] == seg[b - 1];
    const T lcarry = lb_tile<T, Op>(L, 0, blk, 0, agg, blk == 0 || has_head, need, &lcarry_s, SegFb<T, Op>{in, seg, n});
    // exclusive prefix entering my range, continuing my first segment
    T in_pre = threadIdx.x == 0 ? lcarry : lv[threadIdx.x - 1];
    const uint32_t pre_head = threadIdx.x == 0 ? 0u : lh[threadIdx.x - 1];
    if (threadIdx.x != 0 && !pre_head) in_pre = Op::op(lcarry, in_pre);
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
    dev_free(sc.tmp);
    dev_free(sc.fails);
    sc.p = sc.tmp = nullptr;
    sc.fails = nullptr;
    sc.bytes = sc.tmp_bytes = 0;
}

template <typename T, typename Op>
void seg_tile_scan(const T *in, T *out, const uint32_t *seg, uint32_t n, T *tot, SegScratch *sc, hipStream_t s)
{
    if (!n) return;
    const uint32_t nb = (n + SEG_CH - 1) / SEG_CH;
    const LbView L = lb_prepare(sc, nb, s);
    if (!L.w) return;
    hipLaunchKernelGGL((k_seg_scan<T, Op>), dim3(nb), dim3(KPW_BLOCK), 0, s, in, out, seg, n, tot, nb, L);
}

template void seg_tile_scan<uint32_t, OpSum32>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t, uint32_t *, SegScratch *, hipStream_t);
template void seg_tile_scan<uint64_t, OpSum64>(const uint64_t *, uint64_t *, const uint32_t *, uint32_t, uint64_t *, SegScratch *, hipStream_t);
template void seg_tile_scan<int64_t, OpMaxI64>(const int64_t *, int64_t *, const uint32_t *, uint32_t, int64_t *, SegScratch *, hipStream_t);
template void seg_tile_scan<uint32_t, OpMapCompose>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t, uint32_t *, SegScratch *, hipStream_t);

}  // namespace kpw
