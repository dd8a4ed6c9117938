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

// E_s(r) for one optional column (dl width 1).
__device__ uint64_t walker_query(Walker &w, int64_t r, const uint64_t *pres, uint64_t n, const EvView &Eg,
                                 const uint64_t *gend)
{
    while (w.state == 0) {
        if (w.pend_pos < 0) {
            const int64_t p = w.p;
            if (p + 8 > (int64_t)n) { w.state = 2; break; }
            const uint64_t x64 = bits_window(pres, (uint64_t)p);
            const uint32_t x8 = (uint32_t)(x64 & 0xffu);
            if (x8 != 0 && x8 != 0xffu && p + 7 < r) {
                // bit-packed groups straight from the 64-bit window: every mixed group that ends
                // before r is consumed (1 byte, +1 for a new run header every 63 groups) without
                // reloading; the first group that is not is left to the general path below
                int64_t q = p;
                int k = 0;
                do {
                    w.eacc += 1 + ((w.grp % 63) == 0 ? 1 : 0);
                    w.grp++;
                    q += 8;
                    k++;
                    if (k == 8 || q + 8 > (int64_t)n || q + 7 >= r) break;
                    const uint32_t y8 = (uint32_t)((x64 >> (8 * k)) & 0xffu);
                    if (y8 == 0 || y8 == 0xffu) break;
                } while (true);
                w.p = q;
                continue;
            }
            if (x8 == 0 || x8 == 0xffu) {
                const uint64_t fill = x8 ? ~0ull : 0ull;
                int64_t pos = p + 8, b = (int64_t)n;
                while (pos < (int64_t)n) {
                    uint64_t d = bits_window(pres, (uint64_t)pos) ^ fill;
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
            if ((gend[b >> 6] >> (b & 63)) & 1) {
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

// position of record r in stream k (the record itself, or its value rank)
__device__ __forceinline__ int64_t stream_pos(const PlanArgs &a, const PlanStream &S, int64_t r)
{
    return S.rank_col < 0 ? r : (int64_t)pc_at(a.cols[S.rank_col], (uint64_t)r);
}

// k_plan block: PLAN_T threads, each owning streams tid, tid + PLAN_T, ...; 1024 (16 waves) for
// many streams (C3: 199, so the clamp-point evaluation takes 13 per lane instead of 50 with 4
// waves; 1.72 -> 1.46 ms per job), 256 for few (C2: 4 streams, where 16 waves only add barrier
// cost: resident plan stage 13.1 -> 17.2 ms per 100 M records with 1024)

template <int PLAN_T>
__device__ uint64_t eval_mem(const PlanArgs &a, Walker *W, int64_t s, int64_t r)
{
    __shared__ uint64_t red[PLAN_T / 64];
    const int tid = threadIdx.x;
    uint64_t part = 0;
    for (int k = tid; k < a.nstreams; k += PLAN_T) {
        const PlanStream &S = a.streams[k];
        part += walker_query(W[k], stream_pos(a, S, r), S.bits, S.len, ev_view(a, k),
                             a.gend + (uint64_t)k * a.gend_stride);
    }
    for (int k = tid; k < a.nbool; k += PLAN_T) {
        const DevCol &c = a.cols[a.bool_cols[k]];
        const uint64_t cnt = c.optional ? pc_at(c, (uint64_t)r) - pc_at(c, (uint64_t)s) : (uint64_t)(r - s);
        part += (cnt + 7) / 8;
    }
    part = wave_sum(part);
    if ((tid & 63) == 0) red[tid >> 6] = part;
    __syncthreads();   // also publishes the walkers to eval_mem_points
    uint64_t tot = 0;
#pragma unroll
    for (int i = 0; i < PLAN_T / 64; i++) tot += red[i];
    __syncthreads();
    return tot + (a.P[r] - a.P[s]);
}

// memSize at the 64 clamp-step check points s + rc + 10000*j, valid only when every walker is
// past its convergence point (or has no further events): E_s(q) is then one lookup per stream.
// The block splits (point, stream) pairs: lane j of every wave owns point j, wave g the streams
// g, g + 16, ... (independent loads, no walking), and the 16 partial sums meet in LDS; every
// lane j returns the memSize of point j.
template <int PLAN_T>
__device__ uint64_t eval_mem_points(const PlanArgs &a, const Walker *W, int64_t s, int64_t rc)
{
    __shared__ uint64_t red[PLAN_T];
    constexpr int NW = PLAN_T / 64;
    const int tid = threadIdx.x;
    const int j = tid & 63, g = tid >> 6;
    const int64_t r = s + rc + 10000 * (int64_t)j;
    uint64_t part = 0;
    if (r <= (int64_t)a.n) {
        if (g == 0) part = a.P[r] - a.P[s];
        for (int k = g; k < a.nstreams; k += NW) {
            const Walker &w = W[k];
            part += w.state == 1 ? (uint64_t)((int64_t)ev_prefix(ev_view(a, k), (uint64_t)stream_pos(a, a.streams[k], r)) + w.delta)
                                 : w.eacc;
        }
        for (int k = g; k < a.nbool; k += NW) {
            const DevCol &c = a.cols[a.bool_cols[k]];
            const uint64_t cnt = c.optional ? pc_at(c, (uint64_t)r) - pc_at(c, (uint64_t)s) : (uint64_t)(r - s);
            part += (cnt + 7) / 8;
        }
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
__device__ __forceinline__ bool walkers_converged(const PlanArgs &a, const Walker *W, int64_t r)
{
    bool ok = true;
    for (int k = threadIdx.x; k < a.nstreams; k += PLAN_T)
        ok = ok && (W[k].state == 2 || (W[k].state == 1 && W[k].conv_pos < stream_pos(a, a.streams[k], r)));
    return __syncthreads_and(ok ? 1 : 0) != 0;
}

template <int PLAN_T>
__global__ void __launch_bounds__(PLAN_T) k_plan(PlanArgs a)
{
    __shared__ Walker W[MAX_STREAMS];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int64_t n = (int64_t)a.n;
    const int64_t T = a.next_rg_size;
    int64_t s = 0;
    int32_t nrg = 0;
    int64_t overflow = 0;
    for (;;) {
        for (int k = tid; k < a.nstreams; k += PLAN_T) {
            Walker w;
            w.p = stream_pos(a, a.streams[k], s); w.conv_pos = -1; w.delta = 0; w.eacc = 0; w.pend_pos = -1; w.pend_next = 0;
            w.pend_bytes = 0; w.pend_rle = 0; w.grp = 0; w.state = 0;
            W[k] = w;
        }
        __syncthreads();
        int64_t rc = 100;
        bool cut = false;
        bool clamp = true;   // the previous decision took the recordCount + 10000 clamp
        int64_t r = 0;
        while (s + rc <= n) {
            // Far from the cut every next check is recordCount + 10000 (the clamp): once the
            // walkers are converged, the block evaluates memSize at the next 64 clamp-step
            // check points and the scalar replay below takes parquet-mr's decisions over them,
            // stopping where a decision leaves the clamp path (or cuts).  Near the cut (the
            // estimate halves the distance each check) one point at a time is cheaper.
            if (clamp && walkers_converged<PLAN_T>(a, W, s + rc)) {
                const uint64_t Mj = eval_mem_points<PLAN_T>(a, W, s, rc);
                bool left = false;
                for (int j = 0; j < 64; j++) {
                    const int64_t rcv = rc + 10000 * (int64_t)j;
                    if (s + rcv > n) { rc = rcv; left = true; break; }
                    const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)Mj, j);
                    const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(Mj >> 32), j);
                    const int64_t M = (int64_t)(((uint64_t)mhi << 32) | mlo);
                    const int64_t rs = M / rcv;
                    if (M > T - 2 * rs) { cut = true; r = s + rcv; left = true; break; }
                    const float q = __fdiv_rn((float)T, (float)rs);
                    const int64_t est = jadd(rcv, java_f2l(q)) / 2;
                    const int64_t lo = est > 100 ? est : 100;
                    const int64_t hi = jadd(rcv, 10000);
                    int64_t nc = lo < hi ? lo : hi;
                    if (nc < rcv + 1) nc = rcv + 1;
                    if (nc != rcv + 10000) { rc = nc; left = true; clamp = false; break; }
                }
                if (cut) break;
                if (!left) rc += 10000 * 64;
                continue;
            }
            r = s + rc;
            const int64_t M = (int64_t)eval_mem<PLAN_T>(a, W, s, r);
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
                if (tid == 0) { a.out[0] = nrg; a.out[1] = s; a.out[2] = 0; a.out[3] = overflow; }
                break;
            }
            __syncthreads();
            continue;
        }
        // the open row group [s, n)
        int64_t open_buf = 0;
        if (s < n) open_buf = (int64_t)eval_mem<PLAN_T>(a, W, s, n);
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
        }
        break;
    }
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
__device__ __forceinline__ void bool_walker_init(const PageCutArgs &a, int c, Walker &wb, int64_t q)
{
    const DevCol &col = a.cols[c];
    walker_init(wb, col.optional ? (int64_t)pc_at(col, (uint64_t)q) : q);
}
__device__ __forceinline__ uint64_t col_bool_rle(const PageCutArgs &a, int c, Walker &wb, int64_t r)
{
    const int k = a.col_bstream[c];
    const DevCol &col = a.cols[c];
    const PlanStream &S = a.streams[k];
    const int64_t pos = col.optional ? (int64_t)pc_at(col, (uint64_t)r) : r;
    return walker_query(wb, pos, S.bits, S.len, ev_view(a, k), a.gend + (uint64_t)k * a.gend_stride);
}
// rl(0) + dl + data buffered sizes of column c over the page [q, r):
// dl = RunLengthBitPackingHybridEncoder bytes emitted since q (walker), data =
// FallbackValuesWriter.rawDataByteSize / PlainValuesWriter size / boolean bit count (v1) or
// boolean RLE bytes (v2, walker wb).
__device__ __forceinline__ uint64_t col_data_bytes(const PageCutArgs &a, int c, Walker &wb, int64_t q, int64_t r)
{
    const DevCol &col = a.cols[c];
    if (col.phys == 0 && a.v2) return col_bool_rle(a, c, wb, r);
    const uint64_t cnt = col.optional ? pc_at(col, (uint64_t)r) - pc_at(col, (uint64_t)q) : (uint64_t)(r - q);
    if (col.phys == 0) return (cnt + 7) / 8;
    if (col.phys == 6) return a.sp[c][r] - a.sp[c][q];
    return cnt * (uint64_t)col.vsize;
}
__device__ __forceinline__ uint64_t col_dl_bytes(const PageCutArgs &a, int c, Walker &w, int64_t r)
{
    const int k = a.col_stream[c];
    if (k < 0) return 0;
    const DevCol &col = a.cols[c];
    return walker_query(w, r, col.pres, a.n, ev_view(a, k), a.gend + (uint64_t)k * a.gend_stride);
}

// ColumnWriterV1.accountForValueWritten (estimateNextSizeCheck = true), one thread per
// column: valueCountForNextSizeCheck starts at 100 (also after a row-group flush); after
// record x the page holds vc = x - q + 1 values; a check (vc > next) cuts when memSize >
// pageSize (next = vc / 2, count restarts), else next = (int)(vc + (float)vc * pageSize /
// memSize) / 2 + 1 in Java float arithmetic.
__global__ void __launch_bounds__(64) k_page_cuts(PageCutArgs a)
{
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c >= a.ncols) return;
    Walker w, wb;
    int64_t q = a.s;
    walker_init(w, q);
    int32_t next = 100;
    uint32_t nc = 0;
    for (;;) {
        const int64_t x = q + (int64_t)next;
        if (x >= a.h) break;
        const int32_t vc = next + 1;
        const uint64_t mem = col_dl_bytes(a, c, w, x + 1) + col_data_bytes(a, c, wb, q, x + 1);
        if (mem > (uint64_t)a.page_size) {
            if (nc < a.cap) a.cuts[(uint64_t)c * a.cap + nc] = x + 1;
            else atomicOr(a.overflow, 1);
            nc++;
            next = vc / 2;
            q = x + 1;
            walker_init(w, q);
        } else {
            float t = __fmul_rn((float)vc, (float)a.page_size);
            t = __fdiv_rn(t, (float)mem);
            const float sf = __fadd_rn((float)vc, t);
            next = java_f2i(sf) / 2 + 1;
        }
    }
    a.ncuts[c] = nc < a.cap ? nc : a.cap;
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
    __shared__ int64_t Q[MAX_COLS];
    __shared__ uint32_t NC[MAX_COLS];
    const int lane = threadIdx.x;
    for (int c = lane; c < a.ncols; c += 64) {
        Q[c] = a.s;
        NC[c] = 0;
        walker_init(Wd[c], a.s);
        if (a.col_bstream[c] >= 0) bool_walker_init(a, c, Wb[c], a.s);
    }
    const int64_t ps = a.page_size;
    const int64_t tol = (int64_t)__fmul_rn((float)ps, 0.1f);
    int64_t rc = 100;
    while (a.s + rc <= a.h) {
        const int64_t x1 = a.s + rc;   // rowCount = rc: records [s, x1) written
        int64_t mn = INT64_MAX;
        for (int c = lane; c < a.ncols; c += 64) {
            const int64_t q = Q[c];
            const int64_t used = (int64_t)(col_dl_bytes(a, c, Wd[c], x1) + col_data_bytes(a, c, Wb[c], q, x1));
            const int64_t rows = x1 - q;
            int64_t rem = ps - used;
            if (rem <= tol) {   // ColumnWriterV2.writePage(rowCount)
                if (NC[c] < a.cap) a.cuts[(uint64_t)c * a.cap + NC[c]] = x1;
                else atomicOr(a.overflow, 1);
                NC[c]++;
                Q[c] = x1;
                walker_init(Wd[c], x1);
                if (a.col_bstream[c] >= 0) bool_walker_init(a, c, Wb[c], x1);
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
    int64_t q;
    uint64_t pb;
    uint32_t ci, pad;
};

__device__ uint64_t mp_mem(const PageCutArgs &a, MpCol *S, int64_t r)
{
    uint64_t part = 0;
    for (int c = threadIdx.x; c < a.ncols; c += 64) {
        MpCol &m = S[c];
        const uint32_t nc = a.ncuts[c];
        while (m.ci < nc && a.cuts[(uint64_t)c * a.cap + m.ci] <= r) {
            m.pb += a.pbytes[a.pb_off[c] + m.ci];
            m.q = a.cuts[(uint64_t)c * a.cap + m.ci];
            m.ci++;
            walker_init(m.w, m.q);
            if (a.v2 && a.col_bstream[c] >= 0) bool_walker_init(a, c, m.wb, m.q);
        }
        part += m.pb + col_dl_bytes(a, c, m.w, r) + col_data_bytes(a, c, m.wb, m.q, r);
    }
    return wave_sum(part);
}

__global__ void __launch_bounds__(64) k_plan_mp(PageCutArgs a)
{
    __shared__ MpCol S[MAX_COLS];
    for (int c = threadIdx.x; c < a.ncols; c += 64) {
        walker_init(S[c].w, a.s);
        if (a.v2 && a.col_bstream[c] >= 0) bool_walker_init(a, c, S[c].wb, a.s);
        S[c].q = a.s; S[c].pb = 0; S[c].ci = 0;
    }
    __syncthreads();
    const int64_t T = a.next_rg_size;
    const int64_t s = a.s;
    int64_t rc = 100, cut = -1;
    while (s + rc <= a.h) {
        const int64_t M = (int64_t)mp_mem(a, S, s + rc);
        const int64_t rs = M / rc;
        if (M > T - 2 * rs) { cut = s + rc; break; }
        const float qf = __fdiv_rn((float)T, (float)rs);
        const int64_t est = jadd(rc, java_f2l(qf)) / 2;
        const int64_t lo = est > 100 ? est : 100;
        const int64_t hi = jadd(rc, 10000);
        int64_t nc = lo < hi ? lo : hi;
        if (nc < rc + 1) nc = rc + 1;
        rc = nc;
    }
    int64_t open_buf = 0;
    if (cut < 0 && a.h == (int64_t)a.n && s < a.h) open_buf = (int64_t)mp_mem(a, S, a.h);
    if (threadIdx.x == 0) { a.out[0] = cut; a.out[1] = open_buf; }
}

void launch_str_sizes(const DevCol *cols, int c, uint64_t n, uint32_t *sz, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(k_str_sizes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, cols, c, n, sz);
}
void launch_page_cuts(const PageCutArgs &a, hipStream_t s)
{
    if (a.v2) hipLaunchKernelGGL(k_page_cuts_v2, dim3(1), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(k_page_cuts, dim3((a.ncols + 63) / 64), dim3(64), 0, s, a);
}
void launch_plan_mp(const PageCutArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(k_plan_mp, dim3(1), dim3(64), 0, s, a);
}

}  // namespace kpw
