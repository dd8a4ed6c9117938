// k_plan.hip — A9: row-group boundary planner.
//
// Restates parquet-mr 1.10.1 InternalParquetRecordWriter.checkBlockSizeReached exactly:
// check when recordCount >= recordCountForNextMemCheck (100 at a row-group start, also
// after a flush because flushRowGroupToStore zeroes recordCount first); memSize =
// columnStore.getBufferedSize(); recordSize = memSize / recordCount; flush iff
// memSize > nextRowGroupSize - 2*recordSize; otherwise next check at
// min(max(100, (recordCount + (long)(nextRowGroupSize / (float)recordSize)) / 2),
//     recordCount + 10000) (Java float division, saturating float->long cast, wrapping add).
//
// memSize for the single-page-per-chunk regime (every column's page check stays below
// pageSize; verified on the host from the encoded chunk sizes) is
//   sum over columns of  rl(0) + dl.getBufferedSize() + data.getBufferedSize()
// = [P[r]-P[s]]                         FallbackValuesWriter.rawDataByteSize / PlainValuesWriter
// + sum_bool ceil(count/8)              v1: BooleanPlainValuesWriter (ByteBasedBitPackingEncoder)
// + sum_stream E_s(q)                   RunLengthBitPackingHybridEncoder baos.size() of each RLE
//                                       stream written since the row-group start: the
//                                       definition levels of optional columns (q = r) and, in
//                                       v2, the boolean values (q = r, or the value rank r'
//                                       for an optional column); a width-0 REQUIRED level
//                                       encoder never emits before toBytes.
// E_s(q) comes from the global RLE parse (E_g, started at position 0) once the local parse
// started at s re-synchronises with it (both end an RLE run at the same position; from
// there on the encoders are in identical states), and from a short local walk before.
//
// One block walks the row groups sequentially; its 1024 threads split the streams / boolean
// columns (every thread takes the same decisions from block-wide sums).
//
// Folding: once every record-indexed stream's walker has converged in a row group, their sum
// is sum_s (E_g,s(r) + delta_s) = sum_s E_g,s(r) + D, so memSize(r) = Q[r] - P[s] + D (+ the
// value-rank streams and v1 booleans), with Q = P + sum_s E_g,s precomputed for every r
// (k_plan_fold + one scan): one load per evaluation instead of one per stream (C3: 199).
#include "kpw_device.h"
#include "kpw_kernels.h"

namespace kpw {

struct Walker {
    int64_t p;          // next group start
    int64_t conv_pos;   // position of the RLE event where the parse re-synchronised
    int64_t delta;      // E_s - E_g after conv_pos
    uint64_t eacc;      // bytes emitted by events consumed so far
    int64_t pend_pos;   // pending element event position (-1 none)
    int64_t pend_next;
    uint32_t pend_bytes, pend_rle;
    uint32_t grp;       // groups in the current bit-packed run
    uint32_t state;     // 0 walking, 1 converged, 2 no more events in the batch
#ifdef KPW_PLAN_PROF
    uint32_t steps;     // profiling build: walk iterations
#endif
};

__device__ __forceinline__ int32_t java_f2i(float f)
{
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int32_t)f;
}
__device__ __forceinline__ int64_t java_f2l(float f)
{
    if (f != f) return 0;
    if (f >= 9223372036854775808.0f) return 9223372036854775807ll;
    if (f <= -9223372036854775808.0f) return (-9223372036854775807ll - 1);
    return (int64_t)f;
}
__device__ __forceinline__ int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

__device__ __forceinline__ uint64_t wave_sum(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// the global parse's emitted bytes of one stream before position x: the group-of-8 prefix plus
// the event bytes of the positions before x in its group
struct EvView {
    const uint32_t *E8;
    const uint8_t *ev;
};
__device__ __forceinline__ uint64_t ev_prefix(const EvView &v, uint64_t x)
{
    const uint64_t g = x >> 3;
    uint64_t s = v.E8[g];
    if (x & 7) {
        uint64_t b = *(const uint64_t *)(v.ev + 8 * g) & ((1ull << (8 * (x & 7))) - 1);
        b = (b & 0x00ff00ff00ff00ffull) + ((b >> 8) & 0x00ff00ff00ff00ffull);
        b += b >> 16;
        b += b >> 32;
        s += b & 0xffffu;
    }
    return s;
}
template <class A> __device__ __forceinline__ EvView ev_view(const A &a, uint32_t k)
{
    return EvView{a.E8 + (uint64_t)k * (a.ev_stride / 8 + 1), a.ev + (uint64_t)k * a.ev_stride};
}

// A walker's bits: the stream's 64-bit windows and the global parse's run-end flags.
struct SrcDirect {
    const uint64_t *bits, *gend;
    __device__ uint64_t win(uint64_t p) const { return bits_window(bits, p); }
    __device__ bool gend_at(uint64_t b) const { return (gend[b >> 6] >> (b & 63)) & 1; }
};
// E_s(r) for one optional column (dl width 1).
template <class Src>
__device__ uint64_t walker_query(Walker &w, int64_t r, const Src &src, uint64_t n, const EvView &Eg)
{
    while (w.state == 0) {
#ifdef KPW_PLAN_PROF
        w.steps++;
#endif
        if (w.pend_pos < 0) {
            const int64_t p = w.p;
            if (p + 8 > (int64_t)n) { w.state = 2; break; }
            const uint64_t x64 = src.win((uint64_t)p);
            const uint32_t x8 = (uint32_t)(x64 & 0xffu);
            if (x8 != 0 && x8 != 0xffu && p + 7 < r) {
                // bit-packed groups straight from the 64-bit window: the mixed groups before the
                // first pure byte (0x00 / 0xff: SWAR zero-byte tests of x and ~x), that end before
                // r and inside the batch, are consumed at once (1 byte each, +1 for a new run
                // header every 63 groups); the next group goes to the general path below
                const uint64_t lo7 = 0x0101010101010101ull, hi7 = 0x8080808080808080ull;
                const uint64_t nx = ~x64;
                const uint64_t pm = ((x64 - lo7) & nx & hi7) | ((nx - lo7) & x64 & hi7);
                int64_t k = pm ? (int64_t)(__builtin_ctzll(pm) >> 3) : 8;   // >= 1: byte 0 is mixed
                const int64_t kn = ((int64_t)n - p) >> 3, kr = (r - p) >> 3;
                k = k < kn ? k : kn;
                k = k < kr ? k : kr;
                w.eacc += (uint64_t)k + (w.grp + (uint32_t)k + 62) / 63 - (w.grp + 62) / 63;
                w.grp += (uint32_t)k;
                w.p = p + 8 * k;
                continue;
            }
            if (x8 == 0 || x8 == 0xffu) {
                const uint64_t fill = x8 ? ~0ull : 0ull;
                int64_t pos = p + 8, b = (int64_t)n;
                while (pos < (int64_t)n) {
                    uint64_t d = src.win((uint64_t)pos) ^ fill;
                    if (d) { b = pos + __ffsll((long long)d) - 1; break; }
                    pos += 64;
                }
                if (b > (int64_t)n) b = (int64_t)n;
                if (b >= (int64_t)n) { w.state = 2; break; }
                w.pend_pos = b;
                w.pend_next = b;
                w.pend_bytes = varint_len32((uint32_t)(b - p) << 1) + 1;
                w.pend_rle = 1;
            } else {
                w.pend_pos = p + 7;
                w.pend_next = p + 8;
                w.pend_bytes = 1 + ((w.grp % 63) == 0 ? 1 : 0);
                w.pend_rle = 0;
            }
        }
        if (w.pend_pos >= r) break;
        w.eacc += w.pend_bytes;
        w.p = w.pend_next;
        if (w.pend_rle) {
            w.grp = 0;
            const uint64_t b = (uint64_t)w.pend_pos;
            if (src.gend_at(b)) {
                w.state = 1;
                w.conv_pos = (int64_t)b;
                w.delta = (int64_t)w.eacc - (int64_t)ev_prefix(Eg, b + 1);
            }
        } else {
            w.grp++;
        }
        w.pend_pos = -1;
    }
    if (w.state == 1 && r > w.conv_pos) return (uint64_t)((int64_t)ev_prefix(Eg, (uint64_t)r) + w.delta);
    return w.eacc;
}

__device__ __forceinline__ uint64_t pc_at(const DevCol &c, uint64_t x)
{
    const uint64_t wi = x >> 6;
    const uint64_t m = (x & 63) ? (c.pres[wi] & ((1ull << (x & 63)) - 1)) : 0ull;
    return (uint64_t)c.pcnt[wi] + (uint64_t)__popcll(m);
}

// prefix at position r of a sequence scanned per group of 8 (k_scan.hip PlanPrefixF): the
// group's prefix plus the group's elements before r (independent loads)
__device__ __forceinline__ uint64_t pref8(const uint64_t *X8, const uint32_t *x, int64_t r)
{
    const uint64_t g = (uint64_t)r >> 3;
    uint64_t s = X8[g];
    const uint32_t k = (uint32_t)r & 7;
#pragma unroll
    for (uint32_t i = 0; i < 7; i++) s += i < k ? x[8 * g + i] : 0u;
    return s;
}

// k_plan's copies of the stream and boolean-column tables in LDS: every evaluation reads
// them, and from global memory each read added a dependent load ahead of the stream's own
// (C3: 199 streams, ~20 evaluations per row group)
struct PlanSt {
    const uint64_t *rpres;   // rank-indexed stream: the presence bits and counts of its column
    const uint32_t *rpcnt;
    const uint32_t *lra, *lrb;   // the stream's long runs (K3 structure of the planning jobs)
    const uint32_t *lroff;       // per long-run tile of the stream: its first long run ending there
    const uint8_t *lrle;         // per long run: the global parse took it as an RLE run
    uint32_t nlong, ntiles;
    int64_t len;
};

// k_plan's walker: the parse started at the row group's first position, stepped over the long
// runs (maximal runs of >= 8 equal values, k_rle.hip) rather than over positions.  Its groups
// start at gs, gs + 8, ... (phase gs mod 8) until an RLE run: a long run [a, b) is one iff its
// first group start g = a + ((gs - a) mod 8) has g + 8 <= b; the (g - gs) / 8 groups before it
// cost 1 byte each (+1 run header per 63), the run varint((b - g) << 1) + 1 at position b, and
// the next gap starts at b.  The parse has converged with the global one (started at 0) once
// both take the same long run as an RLE run (lr_rle), and from there E_s = E_g + delta.
struct LWalker {
    int64_t gs;         // start of the open gap (bit-packed groups from here)
    uint64_t eacc;      // bytes of the events before gs
    int64_t conv_pos;
    int64_t delta;
    uint32_t cur;       // next long run
    uint32_t state;     // 0 walking, 1 converged, 2 no long runs left (closed form)
};
__device__ __forceinline__ uint64_t bp_bytes(uint64_t G) { return G + (G + 62) / 63; }
constexpr uint32_t LW_BATCH = 8;   // long runs per load round of a walker (16 measured slower)

__device__ __forceinline__ void lw_init(LWalker &w, const PlanSt &S, int64_t p)
{
    w.gs = p; w.eacc = 0; w.conv_pos = -1; w.delta = 0; w.state = 0;
    // first long run ending after p: a binary search among the runs ending in p's tile
    const uint32_t t = (uint32_t)((uint64_t)p / KPW_TILE_L);
    uint32_t lo = t < S.ntiles ? S.lroff[t] : S.nlong;
    uint32_t hi = t + 1 < S.ntiles ? S.lroff[t + 1] : S.nlong;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((int64_t)S.lrb[mid] <= p) lo = mid + 1; else hi = mid;
    }
    w.cur = lo;
}

// the walker's value at r once it no longer walks: converged, or the closed-form final gap
__device__ __forceinline__ uint64_t lw_value(const LWalker &w, int64_t r, int64_t n, const EvView &Eg)
{
    if (w.state == 1) return (uint64_t)((int64_t)ev_prefix(Eg, (uint64_t)r) + w.delta);
    const int64_t lim = r < n ? r : n;
    return w.eacc + (lim > w.gs ? bp_bytes((uint64_t)(lim - w.gs) >> 3) : 0);
}

// E_s(r): the bytes the parse started at the row group's start emitted before position r
// (queries come in increasing r)
__device__ uint64_t lw_query(LWalker &w, int64_t r, const PlanSt &S, const EvView &Eg)
{
    const int64_t n = S.len;
    uint64_t cap = ~0ull;   // groups of the open gap before the next RLE run
    bool stop = false;
    while (!stop && w.state == 0) {
        if (w.cur >= S.nlong) { w.state = 2; break; }
        // 8 long runs per round: their loads issue together (one latency per 8 runs; C3 walks
        // ~150 runs before the parses meet)
        const uint32_t nb = S.nlong - w.cur < LW_BATCH ? S.nlong - w.cur : LW_BATCH;
        uint32_t A[LW_BATCH], B[LW_BATCH], Fl[LW_BATCH];
#pragma unroll
        for (int i = 0; i < (int)LW_BATCH; i++) {
            const bool v = (uint32_t)i < nb;
            A[i] = v ? S.lra[w.cur + i] : 0;
            B[i] = v ? S.lrb[w.cur + i] : 0;
            Fl[i] = v ? S.lrle[w.cur + i] : 0;
        }
#pragma unroll
        for (int i = 0; i < (int)LW_BATCH; i++) {
            if ((uint32_t)i >= nb) break;
            const int64_t b = B[i];
            int64_t a = A[i];
            if (a >= r) { stop = true; break; }        // every later event of the gap's groups: >= r
            if (a < w.gs) a = w.gs;                    // the run the row group starts in
            const int64_t g = a + ((w.gs - a) & 7);
            if (g + 8 > b) { w.cur++; continue; }      // bit-packed in this phase
            const uint64_t G = (uint64_t)(g - w.gs) >> 3;
            if (r <= b) { cap = G; stop = true; break; }   // the run's event (at b) is not before r
            w.eacc += bp_bytes(G) + varint_len32((uint32_t)(b - g) << 1) + 1;
            w.gs = b;
            w.cur++;
            if (Fl[i]) {   // the global parse ends an RLE run at b too
                w.state = 1;
                w.conv_pos = b;
                w.delta = (int64_t)w.eacc - (int64_t)ev_prefix(Eg, (uint64_t)b + 1);
                stop = true;
                break;
            }
        }
    }
    if (w.state != 0) return lw_value(w, r, n, Eg);
    const int64_t lim = r < n ? r : n;
    uint64_t G = lim > w.gs ? (uint64_t)(lim - w.gs) >> 3 : 0;
    if (G > cap) G = cap;
    return w.eacc + bp_bytes(G);
}
struct PlanBool {
    const uint64_t *pres;    // null: REQUIRED
    const uint32_t *pcnt;
};
__device__ __forceinline__ uint64_t pc_at_p(const uint64_t *pres, const uint32_t *pcnt, uint64_t x)
{
    const uint64_t wi = x >> 6;
    const uint64_t m = (x & 63) ? (pres[wi] & ((1ull << (x & 63)) - 1)) : 0ull;
    return (uint64_t)pcnt[wi] + (uint64_t)__popcll(m);
}
// position of record r in stream k (the record itself, or its value rank)
__device__ __forceinline__ int64_t st_pos(const PlanSt &S, int64_t r)
{
    return S.rpres ? (int64_t)pc_at_p(S.rpres, S.rpcnt, (uint64_t)r) : r;
}
__device__ __forceinline__ uint64_t bool_bytes(const PlanBool &B, int64_t s, int64_t r)
{
    const uint64_t cnt = B.pres ? pc_at_p(B.pres, B.pcnt, (uint64_t)r) - pc_at_p(B.pres, B.pcnt, (uint64_t)s) : (uint64_t)(r - s);
    return (cnt + 7) / 8;
}

// k_plan block: PLAN_T threads, each owning streams tid, tid + PLAN_T, ...; 1024 (16 waves) for
// many streams (C3: 199, so the clamp-point evaluation takes 13 per lane instead of 50 with 4
// waves; 1.72 -> 1.46 ms per job), 256 for few (C2: 4 streams, where 16 waves only add barrier
// cost: resident plan stage 13.1 -> 17.2 ms per 100 M records with 1024)

// folded (F = D - P[s]): the record-indexed streams are in Q[r] + F
template <int PLAN_T>
__device__ uint64_t eval_mem(const PlanArgs &a, LWalker *W, const PlanSt *St, const PlanBool *Bo, int64_t s, int64_t r, bool folded,
                             int64_t F)
{
    __shared__ uint64_t red[PLAN_T / 64];
    const int tid = threadIdx.x;
    uint64_t part = 0;   // issued first: its latency overlaps the streams'
    if (tid == 0) part = folded ? (uint64_t)((int64_t)pref8(a.Q8, a.qv, r) + F) : pref8(a.P8, a.raw, r) - pref8(a.P8, a.raw, s);
    for (int k = tid; k < a.nstreams; k += PLAN_T) {
        const PlanSt &S = St[k];
        if (folded && !S.rpres) continue;
        LWalker w = W[k];   // in registers for the walk
        part += lw_query(w, st_pos(S, r), S, ev_view(a, k));
        W[k] = w;
    }
    for (int k = tid; k < a.nbool; k += PLAN_T) part += bool_bytes(Bo[k], s, r);
    part = wave_sum(part);
    if ((tid & 63) == 0) red[tid >> 6] = part;
    __syncthreads();   // also publishes the walkers to eval_mem_points
    uint64_t tot = 0;
#pragma unroll
    for (int i = 0; i < PLAN_T / 64; i++) tot += red[i];
    __syncthreads();
    return tot;
}

// memSize at the 64 clamp-step check points s + rc + 10000*j, valid only when every walker is
// past its convergence point (or has no further events): E_s(q) is then one lookup per stream.
// The block splits (point, stream) pairs: lane j of every wave owns point j, wave g the streams
// g, g + 16, ... (independent loads, no walking), and the 16 partial sums meet in LDS; every
// lane j returns the memSize of point j.
template <int PLAN_T>
__device__ uint64_t eval_mem_points(const PlanArgs &a, const LWalker *W, const PlanSt *St, const PlanBool *Bo, int64_t s,
                                    int64_t rc, bool folded, int64_t F)
{
    __shared__ uint64_t red[PLAN_T];
    constexpr int NW = PLAN_T / 64;
    const int tid = threadIdx.x;
    const int j = tid & 63, g = tid >> 6;
    const int64_t r = s + rc + 10000 * (int64_t)j;
    uint64_t part = 0;
    if (r <= (int64_t)a.n) {
        if (g == 0) part = folded ? (uint64_t)((int64_t)pref8(a.Q8, a.qv, r) + F) : pref8(a.P8, a.raw, r) - pref8(a.P8, a.raw, s);
        for (int k = g; k < a.nstreams; k += NW) {
            if (folded && !St[k].rpres) continue;
            part += lw_value(W[k], st_pos(St[k], r), St[k].len, ev_view(a, k));
        }
        for (int k = g; k < a.nbool; k += NW) part += bool_bytes(Bo[k], s, r);
    }
    red[tid] = part;
    __syncthreads();
    uint64_t tot = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) tot += red[i * 64 + j];
    __syncthreads();
    return tot;
}

template <int PLAN_T>
__device__ __forceinline__ bool walkers_converged(const PlanArgs &a, const LWalker *W, const PlanSt *St, int64_t r)
{
    bool ok = true;
    for (int k = threadIdx.x; k < a.nstreams; k += PLAN_T)
        ok = ok && (W[k].state == 2 || (W[k].state == 1 && W[k].conv_pos < st_pos(St[k], r)));
    return __syncthreads_and(ok ? 1 : 0) != 0;
}

// Every record-indexed stream's walker converged: F = D - P[s] (D = the sum of their deltas).
template <int PLAN_T>
__device__ bool try_fold(const PlanArgs &a, const LWalker *W, const PlanSt *St, int64_t s, int64_t &F)
{
    __shared__ uint64_t red[PLAN_T / 64];
    const int tid = threadIdx.x;
    bool ok = true;
    int64_t d = 0;
    for (int k = tid; k < a.nstreams; k += PLAN_T)
        if (!St[k].rpres) { ok = ok && W[k].state == 1; d += W[k].delta; }
    if (!__syncthreads_and(ok ? 1 : 0)) return false;
    const uint64_t w = wave_sum((uint64_t)d);
    if ((tid & 63) == 0) red[tid >> 6] = w;
    __syncthreads();
    uint64_t D = 0;
#pragma unroll
    for (int i = 0; i < PLAN_T / 64; i++) D += red[i];
    __syncthreads();
    F = (int64_t)D - (int64_t)pref8(a.P8, a.raw, s);
    return true;
}

template <int PLAN_T>
__global__ void __launch_bounds__(PLAN_T) k_plan(PlanArgs a)
{
    __shared__ LWalker W[MAX_STREAMS];
    __shared__ PlanSt St[MAX_STREAMS];
    __shared__ PlanBool Bo[MAX_COLS];
    const int tid = threadIdx.x;
    for (int k = tid; k < a.nstreams; k += PLAN_T) {
        const PlanStream S = a.streams[k];
        const RleJob &J = a.jobs[k];
        PlanSt t;
        t.rpres = nullptr; t.rpcnt = nullptr;
        if (S.rank_col >= 0) { t.rpres = a.cols[S.rank_col].pres; t.rpcnt = a.cols[S.rank_col].pcnt; }
        t.lra = a.lr_a + J.e0; t.lrb = a.lr_b + J.e0; t.lroff = a.lr_off + J.ltile0;
        t.lrle = a.lr_rle + J.e0;
        t.nlong = J.n_long; t.ntiles = J.nltiles; t.len = J.len;
        St[k] = t;
    }
    for (int k = tid; k < a.nbool; k += PLAN_T) {
        const DevCol &c = a.cols[a.bool_cols[k]];
        Bo[k] = PlanBool{c.optional ? c.pres : nullptr, c.optional ? c.pcnt : nullptr};
    }
    __syncthreads();
    const int lane = tid & 63;
    const int64_t n = (int64_t)a.n;
    const int64_t T = a.next_rg_size;
    int64_t s = 0;
    int32_t nrg = 0;
    int64_t overflow = 0;
#ifdef KPW_PLAN_PROF
    // profiling build (tests/microbench): wall-clock ticks (100 MHz) per evaluation kind in
    // out[5..7]: total, walking evaluations, counts
    const uint64_t pp_t0 = wall_clock64();
    uint64_t pp_unc = 0, pp_cnv = 0, pp_nu = 0, pp_nc = 0, pp_np = 0;
#define PP_OUT()                                                                                   \
    if (tid == 0) {                                                                                \
        a.out[5] = (int64_t)(wall_clock64() - pp_t0); a.out[6] = (int64_t)pp_unc;                  \
        a.out[7] = (int64_t)(pp_nu | pp_nc << 21 | pp_np << 42);                                   \
    }
#else
#define PP_OUT()
#endif
    for (;;) {
        for (int k = tid; k < a.nstreams; k += PLAN_T) lw_init(W[k], St[k], st_pos(St[k], s));
        __syncthreads();
        int64_t rc = 100;
        bool cut = false;
        bool clamp = true;   // the previous decision took the recordCount + 10000 clamp
        bool folded = false;
        int64_t F = 0;
        int64_t r = 0;
        while (s + rc <= n) {
            if (a.Q8 && !folded) folded = try_fold<PLAN_T>(a, W, St, s, F);
            // Far from the cut every next check is recordCount + 10000 (the clamp): once the
            // walkers are converged, the block evaluates memSize at the next 64 clamp-step
            // check points and takes parquet-mr's decisions over them (one lane each), stopping
            // where a decision leaves the clamp path (or cuts).  Near the cut (the
            // estimate halves the distance each check) one point at a time is cheaper.
            if (clamp && walkers_converged<PLAN_T>(a, W, St, s + rc)) {
#ifdef KPW_PLAN_PROF
                pp_np++;
#endif
                const uint64_t Mj = eval_mem_points<PLAN_T>(a, W, St, Bo, s, rc, folded, F);
                // parquet-mr's decision at every point, lane j for point j (each depends only on
                // its own memSize); the replay stops at the first point past the batch, that cuts,
                // or whose next check leaves the clamp path
                const int64_t rcv = rc + 10000 * (int64_t)lane;
                const bool past = s + rcv > n;
                bool cut_j = false;
                int64_t nc = rcv + 10000;
                if (!past) {
                    const int64_t M = (int64_t)Mj;
                    const int64_t rs = M / rcv;
                    cut_j = M > T - 2 * rs;
                    if (!cut_j) {
                        const float q = __fdiv_rn((float)T, (float)rs);
                        const int64_t est = jadd(rcv, java_f2l(q)) / 2;
                        const int64_t lo = est > 100 ? est : 100;
                        const int64_t hi = jadd(rcv, 10000);
                        nc = lo < hi ? lo : hi;
                        if (nc < rcv + 1) nc = rcv + 1;
                    }
                }
                const uint64_t stop = __ballot(past || cut_j || nc != rcv + 10000);
                if (!stop) { rc += 10000 * 64; continue; }
                const int js = __builtin_ctzll(stop);   // uniform
                const int64_t rcs = rc + 10000 * (int64_t)js;
                if (s + rcs > n) { rc = rcs; continue; }   // leaves the loop
                if (__builtin_amdgcn_readlane((int)cut_j, js)) { cut = true; r = s + rcs; break; }
                const uint32_t nlo = __builtin_amdgcn_readlane((uint32_t)nc, js);
                const uint32_t nhi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)nc >> 32), js);
                rc = (int64_t)(((uint64_t)nhi << 32) | nlo);
                clamp = false;
                continue;
            }
            r = s + rc;
#ifdef KPW_PLAN_PROF
            bool pp_walk = false;
            for (int k = tid; k < a.nstreams; k += PLAN_T) pp_walk = pp_walk || W[k].state == 0;
            pp_walk = __syncthreads_or(pp_walk ? 1 : 0) != 0;
            const uint64_t pp_e0 = wall_clock64();
#endif
            const int64_t M = (int64_t)eval_mem<PLAN_T>(a, W, St, Bo, s, r, folded, F);
#ifdef KPW_PLAN_PROF
            if (pp_walk) { pp_unc += wall_clock64() - pp_e0; pp_nu++; }
            else { pp_cnv += wall_clock64() - pp_e0; pp_nc++; }
#endif
            const int64_t rs = M / rc;
            if (M > T - 2 * rs) { cut = true; break; }
            const float q = __fdiv_rn((float)T, (float)rs);
            const int64_t est = jadd(rc, java_f2l(q)) / 2;
            const int64_t lo = est > 100 ? est : 100;
            const int64_t hi = jadd(rc, 10000);
            int64_t nc = lo < hi ? lo : hi;
            if (nc < rc + 1) nc = rc + 1;
            clamp = nc == rc + 10000;
            rc = nc;
        }
        if (cut) {
            if (nrg < a.max_rgs) { if (tid == 0) { a.rg[2 * nrg] = s; a.rg[2 * nrg + 1] = r; } }
            else overflow = 1;
            nrg++;
            s = r;
            if (a.max_cuts > 0 && nrg >= a.max_cuts) {   // the caller re-plans from s with the next limit
                if (tid == 0) { a.out[0] = nrg; a.out[1] = s; a.out[2] = 0; a.out[3] = overflow; a.out[4] = (int64_t)*a.err; }
                PP_OUT();
                break;
            }
            __syncthreads();
            continue;
        }
        // the open row group [s, n)
        int64_t open_buf = 0;
        if (s < n) {
            if (a.Q8 && !folded) folded = try_fold<PLAN_T>(a, W, St, s, F);
            open_buf = (int64_t)eval_mem<PLAN_T>(a, W, St, Bo, s, n, folded, F);
        }
        if (a.final_flush && s < n) {
            if (nrg < a.max_rgs) { if (tid == 0) { a.rg[2 * nrg] = s; a.rg[2 * nrg + 1] = n; } }
            else overflow = 1;
            nrg++;
            s = n;
            open_buf = 0;
        }
        if (tid == 0) {
            a.out[0] = nrg;
            a.out[1] = s;
            a.out[2] = open_buf;
            a.out[3] = overflow;
            a.out[4] = (int64_t)*a.err;
        }
        PP_OUT();
        break;
    }
#undef PP_OUT
}

// val[x] = raw[x] + the event bytes at position x of every record-indexed stream (the input
// of Q's scan); one thread per group of 8 positions, one 8-byte load per stream, byte lanes
// summed as u16 (< 2^16: at most MAX_STREAMS streams x 6 bytes)
__global__ void __launch_bounds__(256) k_plan_fold(const uint8_t *ev, uint64_t ev_stride, const PlanStream *streams, uint32_t nstreams,
                                                   const uint32_t *raw, uint64_t n, uint32_t *val)
{
    const uint64_t x0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (x0 >= n) return;
    uint64_t lo = 0, hi = 0;
#pragma unroll 4
    for (uint32_t k = 0; k < nstreams; k++) {
        if (streams[k].rank_col >= 0) continue;
        const uint64_t b = *(const uint64_t *)(ev + (uint64_t)k * ev_stride + x0);
        lo += b & 0x00ff00ff00ff00ffull;
        hi += (b >> 8) & 0x00ff00ff00ff00ffull;
    }
    uint32_t e[8];
#pragma unroll
    for (int i = 0; i < 4; i++) { e[2 * i] = (uint32_t)(lo >> (16 * i)) & 0xffffu; e[2 * i + 1] = (uint32_t)(hi >> (16 * i)) & 0xffffu; }
    if (x0 + 8 <= n) {
        const uint4 r0 = *(const uint4 *)(raw + x0), r1 = *(const uint4 *)(raw + x0 + 4);
        *(uint4 *)(val + x0) = make_uint4(r0.x + e[0], r0.y + e[1], r0.z + e[2], r0.w + e[3]);
        *(uint4 *)(val + x0 + 4) = make_uint4(r1.x + e[4], r1.y + e[5], r1.z + e[6], r1.w + e[7]);
    } else {
        for (uint64_t i = 0; x0 + i < n; i++) val[x0 + i] = raw[x0 + i] + e[i];
    }
}

void launch_plan_fold(const uint8_t *ev, uint64_t ev_stride, const PlanStream *streams, uint32_t nstreams, const uint32_t *raw,
                      uint64_t n, uint32_t *val, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_plan_fold, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, s, ev, ev_stride, streams, nstreams, raw, n, val);
}

void launch_plan(const PlanArgs &a, hipStream_t s)
{
    if (a.nstreams > 64) hipLaunchKernelGGL(k_plan<1024>, dim3(1), dim3(1024), 0, s, a);
    else hipLaunchKernelGGL(k_plan<256>, dim3(1), dim3(256), 0, s, a);
}

// ------------------------------------------------------------------ multi-page (v1)

// (4 + len) of present BYTE_ARRAY values, 0 for nulls (input of the per-column size prefix)
__global__ void __launch_bounds__(256) k_str_sizes(const DevCol *cols, int c, uint64_t n, uint32_t *sz)
{
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const DevCol &col = cols[c];
    const bool pres = !col.optional || ((col.pres[r >> 6] >> (r & 63)) & 1ull);
    sz[r] = pres ? 4u + col.slen[r] : 0u;
}

__device__ __forceinline__ void walker_init(Walker &w, int64_t p)
{
    w.p = p; w.conv_pos = -1; w.delta = 0; w.eacc = 0; w.pend_pos = -1; w.pend_next = 0;
    w.pend_bytes = 0; w.pend_rle = 0; w.grp = 0; w.state = 0;
}
// v2 BOOLEAN column c: RLE bytes its value stream emitted since the page start (walker wb,
// started by bool_walker_init at the page's first record); stream position = value rank for an
// optional column
// A column's inputs to the multi-page checks, loaded once per kernel (each check used to reload
// the descriptor fields from global memory ahead of the data loads: one more dependent latency
// per check, r04 bulk multi-page ~2 us per check)
struct MpColInfo {
    const uint64_t *pres;    // null: REQUIRED
    const uint32_t *pcnt;
    const uint64_t *sp;      // BYTE_ARRAY size prefix
    const uint64_t *gdl;     // definition-level stream: run-end bits, events (kdl < 0: none)
    EvView edl;
    const uint64_t *bbits;   // v2 BOOLEAN value stream: bits, run-end bits, events, length (kb < 0: none)
    const uint64_t *gb;
    EvView eb;
    uint64_t blen;
    int32_t phys, vsize, kdl, kb;
};
__device__ __forceinline__ MpColInfo mp_col_info(const PageCutArgs &a, int c)
{
    const DevCol col = a.cols[c];
    MpColInfo I;
    I.pres = col.optional ? col.pres : nullptr;
    I.pcnt = col.pcnt;
    I.sp = col.phys == 6 ? a.sp[c] : nullptr;
    I.phys = col.phys; I.vsize = col.vsize;
    I.kdl = a.col_stream[c];
    I.gdl = nullptr; I.gb = nullptr; I.bbits = nullptr; I.blen = 0;
    I.edl = EvView{nullptr, nullptr}; I.eb = EvView{nullptr, nullptr};
    if (I.kdl >= 0) { I.gdl = a.gend + (uint64_t)I.kdl * a.gend_stride; I.edl = ev_view(a, I.kdl); }
    I.kb = a.col_bstream ? a.col_bstream[c] : -1;
    if (I.kb >= 0) {
        const PlanStream S = a.streams[I.kb];
        I.bbits = S.bits; I.blen = S.len;
        I.gb = a.gend + (uint64_t)I.kb * a.gend_stride; I.eb = ev_view(a, I.kb);
    }
    return I;
}
__device__ __forceinline__ uint64_t mp_rank(const MpColInfo &I, int64_t r)
{
    return I.pres ? pc_at_p(I.pres, I.pcnt, (uint64_t)r) : (uint64_t)r;
}
// v2 BOOLEAN column: RLE bytes its value stream emitted since the page start (walker wb,
// started by bool_walker_init at the page's first record); stream position = value rank for an
// optional column
__device__ __forceinline__ void bool_walker_init(const MpColInfo &I, Walker &wb, int64_t q) { walker_init(wb, (int64_t)mp_rank(I, q)); }
__device__ __forceinline__ uint64_t col_bool_rle(const MpColInfo &I, Walker &wb, int64_t r)
{
    return walker_query(wb, (int64_t)mp_rank(I, r), SrcDirect{I.bbits, I.gb}, I.blen, I.eb);
}
// rl(0) + dl + data buffered sizes of column c over the page [q, r):
// dl = RunLengthBitPackingHybridEncoder bytes emitted since q (walker), data =
// FallbackValuesWriter.rawDataByteSize / PlainValuesWriter size / boolean bit count (v1) or
// boolean RLE bytes (v2, walker wb).
__device__ __forceinline__ uint64_t col_data_bytes(const PageCutArgs &a, const MpColInfo &I, Walker &wb, int64_t q, int64_t r)
{
    if (I.phys == 0 && a.v2) return col_bool_rle(I, wb, r);
    if (I.phys == 6) return I.sp[r] - I.sp[q];
    const uint64_t cnt = mp_rank(I, r) - mp_rank(I, q);
    if (I.phys == 0) return (cnt + 7) / 8;
    return cnt * (uint64_t)I.vsize;
}
__device__ __forceinline__ uint64_t col_dl_bytes(const PageCutArgs &a, const MpColInfo &I, Walker &w, int64_t r)
{
    if (I.kdl < 0) return 0;
    return walker_query(w, r, SrcDirect{I.pres, I.gdl}, a.n, I.edl);
}

// ColumnWriterV1.accountForValueWritten (estimateNextSizeCheck = true), one thread per
// column: valueCountForNextSizeCheck starts at 100 (also after a row-group flush); after
// record x the page holds vc = x - q + 1 values; a check (vc > next) cuts when memSize >
// pageSize (next = vc / 2, count restarts), else next = (int)(vc + (float)vc * pageSize /
// memSize) / 2 + 1 in Java float arithmetic.
// the non-cutting branch of the page check: next = (int)(vc + (float)vc * pageSize / memSize) / 2 + 1
__device__ __forceinline__ int32_t pc_next(int32_t vc, int64_t page_size, uint64_t mem)
{
    float t = __fmul_rn((float)vc, (float)page_size);
    t = __fdiv_rn(t, (float)mem);
    return java_f2i(__fadd_rn((float)vc, t)) / 2 + 1;
}
__device__ __forceinline__ int64_t shfl64(int64_t v, int k)
{
    const int lo = __shfl((int)(uint32_t)v, k, 64), hi = __shfl((int)(uint32_t)((uint64_t)v >> 32), k, 64);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// A REQUIRED BYTE_ARRAY column's checks (memSize = sp[x + 1] - sp[q], one dependent load each;
// ~1900 per C2 row group at 1 MiB pages) in speculative batches: lane k follows the chain k
// checks ahead with memSize predicted from the page's bytes per value so far and loads sp at
// its check, all lanes in one round trip; the chain then takes the loaded values as long as
// the predicted positions are the actual ones (lane 0's always is: at least one check per trip)
constexpr int PC_SPEC = 8;
__device__ void page_cuts_str(const PageCutArgs &a, const MpColInfo &I, int c)
{
    const int lane = (int)threadIdx.x;
    int64_t q = a.s;
    int32_t next = 100;
    uint32_t nc = 0;
    uint64_t sq = I.sp[q];
    double bpv;   // bytes per value of the open page (prediction only)
    {
        const int64_t r = a.h < q + 4096 ? a.h : q + 4096;
        bpv = r > q ? (double)(I.sp[r] - sq) / (double)(r - q) : 1.0;
    }
    for (;;) {
        int64_t xk = -1;
        if (lane < PC_SPEC) {
            int64_t pq = q;
            int32_t pn = next;
            for (int j = 0;; j++) {
                const int64_t x = pq + (int64_t)pn;
                if (x >= a.h) break;
                if (j == lane) { xk = x; break; }
                const int32_t vc = pn + 1;
                const uint64_t memp = (uint64_t)(bpv * (double)vc) + 1;
                if (memp > (uint64_t)a.page_size) { pq = x + 1; pn = vc / 2; }
                else pn = pc_next(vc, a.page_size, memp);
            }
        }
        const uint64_t val = xk >= 0 ? I.sp[xk + 1] : 0;
        bool done = false;
        for (int k = 0; k < PC_SPEC; k++) {
            const int64_t x = q + (int64_t)next;
            if (x >= a.h) { done = true; break; }
            if (shfl64(xk, k) != x) break;
            const uint64_t mem = (uint64_t)shfl64((int64_t)val, k) - sq;
            const int32_t vc = next + 1;
            if (mem > (uint64_t)a.page_size) {
                if (lane == 0) {
                    if (nc < a.cap) a.cuts[(uint64_t)c * a.cap + nc] = x + 1;
                    else atomicOr(a.overflow, 1);
                }
                nc++;
                next = vc / 2;
                q = x + 1;
                sq += mem;
            } else {
                next = pc_next(vc, a.page_size, mem);
            }
            if (mem) bpv = (double)mem / (double)vc;
        }
        if (done) break;
    }
    if (lane == 0) a.ncuts[c] = nc < a.cap ? nc : a.cap;
}

__global__ void __launch_bounds__(64) k_page_cuts(PageCutArgs a)
{
    const int c = blockIdx.x;   // one wave per column: a column's chain waits only for its own loads
    const MpColInfo I = mp_col_info(a, c);
    if (I.phys == 6 && I.kdl < 0 && a.str_spec) { page_cuts_str(a, I, c); return; }
    if (threadIdx.x) return;
    Walker w, wb;
    int64_t q = a.s;
    walker_init(w, q);
    int32_t next = 100;
    uint32_t nc = 0;
#ifdef KPW_PLAN_PROF
    uint32_t pp_checks = 0, pp_steps = 0;
    const uint64_t pp_t0 = wall_clock64();
    w.steps = 0;
#endif
    for (;;) {
#ifdef KPW_PLAN_PROF
        pp_checks++;
#endif
        const int64_t x = q + (int64_t)next;
        if (x >= a.h) break;
        const int32_t vc = next + 1;
        const uint64_t mem = col_dl_bytes(a, I, w, x + 1) + col_data_bytes(a, I, wb, q, x + 1);
        if (mem > (uint64_t)a.page_size) {
            if (nc < a.cap) a.cuts[(uint64_t)c * a.cap + nc] = x + 1;
            else atomicOr(a.overflow, 1);
            nc++;
            next = vc / 2;
            q = x + 1;
#ifdef KPW_PLAN_PROF
            pp_steps += w.steps;
#endif
            walker_init(w, q);
#ifdef KPW_PLAN_PROF
            w.steps = 0;
#endif
        } else {
            float t = __fmul_rn((float)vc, (float)a.page_size);
            t = __fdiv_rn(t, (float)mem);
            const float sf = __fadd_rn((float)vc, t);
            next = java_f2i(sf) / 2 + 1;
        }
    }
    a.ncuts[c] = nc < a.cap ? nc : a.cap;
#ifdef KPW_PLAN_PROF
    printf("[page_cuts] s %lld h %lld col %d cuts %u checks %u walk steps %u ticks %llu\n", (long long)a.s, (long long)a.h, c, nc,
           pp_checks, pp_steps + w.steps, (unsigned long long)(wall_clock64() - pp_t0));
#endif
}

// ColumnWriteStoreV2.sizeCheck (PARQUET_2_0), one wave for the whole store, lanes own columns:
// the check runs after rowCount records once rowCount >= rowCountForNextSizeCheck (100 at a
// row-group start).  Per column usedMem = rl + dl + data buffered since its page start (the
// width-0 repetition / REQUIRED definition encoders emit nothing before toBytes); a column with
// pageSize - usedMem <= (long)(pageSize * 0.1f) writes its page at rowCount; rowsToFillPage =
// usedMem == 0 ? 10000 : (long)((float)rows) / usedMem * remainingMem (remainingMem = pageSize
// after a write); the next check at rowCount + min(max(min over columns / 2, 100), 10000).
__global__ void __launch_bounds__(64) k_page_cuts_v2(PageCutArgs a)
{
    __shared__ Walker Wd[MAX_COLS], Wb[MAX_COLS];
    __shared__ MpColInfo CI[MAX_COLS];
    __shared__ int64_t Q[MAX_COLS];
    __shared__ uint32_t NC[MAX_COLS];
    const int lane = threadIdx.x;
    for (int c = lane; c < a.ncols; c += 64) {
        CI[c] = mp_col_info(a, c);
        Q[c] = a.s;
        NC[c] = 0;
        walker_init(Wd[c], a.s);
        if (CI[c].kb >= 0) bool_walker_init(CI[c], Wb[c], a.s);
    }
    const int64_t ps = a.page_size;
    const int64_t tol = (int64_t)__fmul_rn((float)ps, 0.1f);
    int64_t rc = 100;
    while (a.s + rc <= a.h) {
        const int64_t x1 = a.s + rc;   // rowCount = rc: records [s, x1) written
        int64_t mn = INT64_MAX;
        for (int c = lane; c < a.ncols; c += 64) {
            const int64_t q = Q[c];
            const MpColInfo &I = CI[c];
            const int64_t used = (int64_t)(col_dl_bytes(a, I, Wd[c], x1) + col_data_bytes(a, I, Wb[c], q, x1));
            const int64_t rows = x1 - q;
            int64_t rem = ps - used;
            if (rem <= tol) {   // ColumnWriterV2.writePage(rowCount)
                if (NC[c] < a.cap) a.cuts[(uint64_t)c * a.cap + NC[c]] = x1;
                else atomicOr(a.overflow, 1);
                NC[c]++;
                Q[c] = x1;
                walker_init(Wd[c], x1);
                if (I.kb >= 0) bool_walker_init(I, Wb[c], x1);
                rem = ps;
            }
            const int64_t fill = used == 0 ? 10000 : ((int64_t)(float)rows / used) * rem;
            mn = fill < mn ? fill : mn;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int64_t v = __shfl_xor(mn, o, 64);
            mn = v < mn ? v : mn;
        }
        int64_t half = mn / 2;
        half = half < 100 ? 100 : (half > 10000 ? 10000 : half);
        rc += half;
    }
    for (int c = lane; c < a.ncols; c += 64) a.ncuts[c] = NC[c] < a.cap ? NC[c] : a.cap;
}

// checkBlockSizeReached over one row group from s with the page cuts above: memSize at
// record count rc = sum over columns of (open page rl+dl+data) + (header + compressed
// bytes of the pages already flushed to the ColumnChunkPageWriter).  One wave; lanes own
// columns; r only grows, so each column's page cursor and walker advance monotonically.
struct MpCol {
    Walker w, wb;       // definition levels; v2 boolean values
    MpColInfo I;
    int64_t q;
    int64_t next_cut;   // the column's next page end (INT64_MAX: none)
    uint64_t pb;
    uint32_t ci, nc;
};

__device__ uint64_t mp_mem(const PageCutArgs &a, MpCol *S, int64_t r)
{
    uint64_t part = 0;
    for (int c = threadIdx.x; c < a.ncols; c += 64) {
        MpCol &m = S[c];
        while (m.next_cut <= r) {
            m.pb += a.pbytes[a.pb_off[c] + m.ci];
            m.q = m.next_cut;
            m.ci++;
            m.next_cut = m.ci < m.nc ? a.cuts[(uint64_t)c * a.cap + m.ci] : INT64_MAX;
            walker_init(m.w, m.q);
            if (a.v2 && m.I.kb >= 0) bool_walker_init(m.I, m.wb, m.q);
        }
        part += m.pb + col_dl_bytes(a, m.I, m.w, r) + col_data_bytes(a, m.I, m.wb, m.q, r);
    }
    return wave_sum(part);
}

// A walker's value at r with a bounded walk (<= 16 windows of 4096 positions; false: over budget)
template <class Src>
__device__ __forceinline__ bool walker_query_capped(Walker &w, int64_t r, const Src &src, uint64_t n, const EvView &Eg, uint64_t &val)
{
    for (int k = 0; k < 16; k++) {
        const int64_t t = (w.state == 0 && r - w.p > 4096) ? w.p + 4096 : r;
        val = walker_query(w, t, src, n, Eg);
        if (t == r) return true;
        if (w.state != 0) { val = walker_query(w, r, src, n, Eg); return true; }
    }
    return false;
}

// memSize at record r evaluated by one lane alone (v1), for the clamp points ahead of the
// sequential cursor S (read only): each column's pages between the cursor and r, and its
// definition-level walker from the open page's start (the cursor's walker when it is the same
// page).  false: a walk over its budget (the point is then left to the sequential evaluation).
__device__ bool mp_mem_point(const PageCutArgs &a, const MpCol *S, int64_t r, uint64_t &M)
{
    uint64_t tot = 0;
    for (int c = 0; c < a.ncols; c++) {
        const MpCol &m = S[c];
        uint32_t ci = m.ci;
        int64_t q = m.q, nxt = m.next_cut;
        uint64_t pb = m.pb;
        while (nxt <= r) {
            pb += a.pbytes[a.pb_off[c] + ci];
            q = nxt;
            ci++;
            nxt = ci < m.nc ? a.cuts[(uint64_t)c * a.cap + ci] : INT64_MAX;
        }
        uint64_t dl = 0;
        if (m.I.kdl >= 0) {
            Walker w;
            if (q == m.q) w = m.w; else walker_init(w, q);
            if (!walker_query_capped(w, r, SrcDirect{m.I.pres, m.I.gdl}, a.n, m.I.edl, dl)) return false;
        }
        Walker wb;   // (v1: unused)
        tot += pb + dl + col_data_bytes(a, m.I, wb, q, r);
    }
    M = tot;
    return true;
}

__global__ void __launch_bounds__(64) k_plan_mp(PageCutArgs a)
{
    __shared__ MpCol S[MAX_COLS];
    for (int c = threadIdx.x; c < a.ncols; c += 64) {
        MpCol &m = S[c];
        m.I = mp_col_info(a, c);
        walker_init(m.w, a.s);
        if (a.v2 && m.I.kb >= 0) bool_walker_init(m.I, m.wb, a.s);
        m.q = a.s; m.pb = 0; m.ci = 0;
        m.nc = a.ncuts[c];
        m.next_cut = m.nc ? a.cuts[(uint64_t)c * a.cap] : INT64_MAX;
    }
    __syncthreads();
    const int64_t T = a.next_rg_size;
    const int64_t s = a.s;
    int64_t rc = 100, cut = -1;
#ifdef KPW_PLAN_PROF
    uint32_t pp_checks = 0;
    const uint64_t pp_t0 = wall_clock64();
#endif
    const int lane = threadIdx.x;
    bool clamp = false;   // the previous decision took the recordCount + 10000 clamp
    while (s + rc <= a.h) {
        if (clamp && !a.v2) {
            // (as k_plan) the next 64 clamp-step points at once, lane j for point j: its memSize
            // and parquet-mr's decision there; the first point past the horizon, that cuts, that
            // leaves the clamp path or whose walk ran over budget ends the batch
            __syncthreads();   // the cursor's state, written by every lane, is read by each
            const int64_t rcv = rc + 10000 * (int64_t)lane;
            const bool past = s + rcv > a.h;
            bool ok = true, cut_j = false;
            int64_t nc = rcv + 10000;
            if (!past) {
                uint64_t Mu = 0;
                ok = mp_mem_point(a, S, s + rcv, Mu);
                if (ok) {
                    const int64_t M = (int64_t)Mu;
                    const int64_t rs = M / rcv;
                    cut_j = M > T - 2 * rs;
                    if (!cut_j) {
                        const float qf = __fdiv_rn((float)T, (float)rs);
                        const int64_t est = jadd(rcv, java_f2l(qf)) / 2;
                        const int64_t lo = est > 100 ? est : 100;
                        const int64_t hi = jadd(rcv, 10000);
                        nc = lo < hi ? lo : hi;
                        if (nc < rcv + 1) nc = rcv + 1;
                    }
                }
            }
#ifdef KPW_PLAN_PROF
            pp_checks++;
#endif
            const uint64_t stop = __ballot(past || !ok || cut_j || nc != rcv + 10000);
            if (!stop) { rc += 10000 * 64; continue; }
            const int js = __builtin_ctzll(stop);   // uniform
            const int64_t rcs = rc + 10000 * (int64_t)js;
            if (s + rcs > a.h) { rc = rcs; continue; }   // leaves the loop
            clamp = false;
            if (!__builtin_amdgcn_readlane((int)ok, js)) { rc = rcs; continue; }   // the sequential check, at rcs
            if (__builtin_amdgcn_readlane((int)cut_j, js)) { cut = s + rcs; break; }
            const uint32_t nlo = __builtin_amdgcn_readlane((uint32_t)nc, js);
            const uint32_t nhi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)nc >> 32), js);
            rc = (int64_t)(((uint64_t)nhi << 32) | nlo);
            continue;
        }
#ifdef KPW_PLAN_PROF
        pp_checks++;
#endif
        const int64_t M = (int64_t)mp_mem(a, S, s + rc);
        const int64_t rs = M / rc;
        if (M > T - 2 * rs) { cut = s + rc; break; }
        const float qf = __fdiv_rn((float)T, (float)rs);
        const int64_t est = jadd(rc, java_f2l(qf)) / 2;
        const int64_t lo = est > 100 ? est : 100;
        const int64_t hi = jadd(rc, 10000);
        int64_t nc = lo < hi ? lo : hi;
        if (nc < rc + 1) nc = rc + 1;
        clamp = nc == rc + 10000;
        rc = nc;
    }
    int64_t open_buf = 0;
    if (cut < 0 && a.h == (int64_t)a.n && s < a.h) open_buf = (int64_t)mp_mem(a, S, a.h);
    if (threadIdx.x == 0) { a.out[0] = cut; a.out[1] = open_buf; }
#ifdef KPW_PLAN_PROF
    if (threadIdx.x == 0)
        printf("[plan_mp] s %lld h %lld cut %lld checks %u ticks %llu\n", (long long)a.s, (long long)a.h, (long long)cut, pp_checks,
               (unsigned long long)(wall_clock64() - pp_t0));
#endif
}

void launch_str_sizes(const DevCol *cols, int c, uint64_t n, uint32_t *sz, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_str_sizes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, cols, c, n, sz);
}
void launch_page_cuts(const PageCutArgs &a, hipStream_t s)
{
    if (a.v2) hipLaunchKernelGGL(k_page_cuts_v2, dim3(1), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(k_page_cuts, dim3(a.ncols), dim3(64), 0, s, a);
}
void launch_plan_mp(const PageCutArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(k_plan_mp, dim3(1), dim3(64), 0, s, a);
}

}  // namespace kpw
