// k_rle.hip — K3: RLE / bit-packing hybrid, byte-identical to parquet-mr 1.10.1
// RunLengthBitPackingHybridEncoder (writeInt / writeOrAppendBitPackedRun / writeRleRun /
// endPreviousBitPackedRun / toBytes), reformulated for a data-parallel GPU.
//
// The sequential encoder's behaviour is fully determined by where its 8-value groups
// start.  Group starts form an arithmetic progression (phase = start mod 8) that only
// changes after an RLE run; an RLE run starts at a group start g iff v[g..g+7] are equal,
// and then extends to the end b of that maximal run of equal values (the next group
// starts at b).  Hence only "long runs" (maximal runs of >= 8 equal values) matter: for a
// long run [a, b) entered with phase phi, the first group start inside it is
// g = a + ((phi - a) mod 8); it becomes an RLE run iff g + 8 <= b, and the phase after it
// is b mod 8 (else phi is unchanged).  Each long run is therefore an 8-state transfer map;
// an exclusive composition scan over long runs yields every decision in parallel.
// Bit-packed groups fill the gaps between RLE runs; a gap of G groups costs G*bw bytes
// plus ceil(G/63) run headers ((groups<<1)|1, at most 63 groups per run); the final
// partial group is zero padded (toBytes).  An RLE run costs varint(len<<1) +
// ceil(bw/8) value bytes.
//
// Pipeline per batch of jobs (launched back to back, no host sync; every scan a single-pass
// decoupled look-back inside the kernel that needs it, kpw_lookback.h):
//   bounds -> [max-scan] -> longruns(count) -> [sum-scan] -> longruns(write) -> phase
//   (compose-scan, RLE runs, sum-scan, write) -> sizes (two sum-scans, job totals) -> write
//   (runs + groups) | events
#include "kpw_device.h"
#include "kpw_kernels.h"
#include "kpw_scan.h"
#include "kpw_lookback.h"

namespace kpw {

__device__ __forceinline__ ValSrc job_src(const RleJob &J)
{
    ValSrc s;
    s.kind = J.src.kind;
    s.pad = 0;
    s.ptr = J.src.ptr;
    s.base = J.src.base;
    return s;
}

__device__ __forceinline__ uint32_t run_map(uint32_t a, uint32_t b)
{
    uint32_t m = 0;
#pragma unroll
    for (uint32_t phi = 0; phi < 8; phi++) {
        uint32_t g = a + ((phi - a) & 7u);
        uint32_t o = (g + 8 <= b) ? (b & 7u) : phi;
        m |= o << (3 * phi);
    }
    return m;
}

// ------------------------------------------------------------------ long runs
// Over the long-run tiles (KPW_TILE_L = 16384 positions: 64 per thread, so a bit stream's tile
// is one 2 KiB slice of its bitmask): the last value break per tile, a segmented max-scan of
// those (the break before each tile), the long runs ending in each tile counted, a sum-scan of
// the counts, then the runs written as (a, b); the job's last tile stores n_long.  Each thread
// works on the 64-bit break mask of its positions, so the long-run ends are bit operations
// (a break whose previous break is >= 8 positions back) rather than a loop over positions.
// (Round 5: 8 positions per thread and 2048 per tile before: C3's 199 planning streams were
// ~75 k blocks per launch, each mostly block-scan overhead.  r04: one launch with both scans as
// in-kernel look-backs measured 2x slower here: every tile has full work, and its look-back
// round trips are exposed; the element-tile kernels below keep theirs, since most of their
// tiles are past the job's runs and exit at once.)

// The break mask of a thread's 64 positions [p0, p0 + 64), p0 = wb + 64 * lane (wb: the wave's
// first position, uniform): bit k set iff p0 + k < len and the value there starts a new run
// (position 0, or a value unlike the one before it).  Bits: the lane's own 64 bits (lanes read
// consecutive words).  u32 values: the wave loads its 4096 positions row by row (row k =
// positions wb + 64k .. + 63, one coalesced load per lane), a row's breaks are one ballot, and
// lane k keeps row k's.
__device__ __forceinline__ uint64_t brk_mask64(const ValSrc &s, int64_t wb, int64_t len)
{
    const uint32_t lane = threadIdx.x & 63;
    if (wb >= len) return 0;   // (uniform per wave)
    const int64_t p0 = wb + 64 * (int64_t)lane;
    if (s.kind == 0) {
        if (p0 >= len) return 0;
        const uint64_t *w = (const uint64_t *)s.ptr;
        const uint64_t b = s.base + (uint64_t)p0;
        const uint32_t sh = (uint32_t)(b & 63);
        uint64_t cur = w[b >> 6] >> sh;
        if (sh) cur |= w[(b >> 6) + 1] << (64 - sh);
        uint64_t before;   // the value before p0, in bit 0; at position 0 its complement (a break)
        if (p0 == 0) before = ~cur & 1ull;
        else before = (w[(b - 1) >> 6] >> ((b - 1) & 63)) & 1ull;
        uint64_t m = cur ^ ((cur << 1) | before);
        if (len - p0 < 64) m &= (1ull << (len - p0)) - 1;
        return m;
    }
    const uint32_t *q = (const uint32_t *)s.ptr + s.base;
    uint32_t carry = wb > 0 ? q[wb - 1] : 0u;   // the value before the current row
    uint64_t mine = 0;
    for (uint32_t k0 = 0; k0 < 64; k0 += 8) {
        uint32_t v[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const int64_t pos = wb + 64 * (int64_t)(k0 + j) + lane;
            v[j] = pos < len ? q[pos] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const int64_t pos = wb + 64 * (int64_t)(k0 + j) + lane;
            uint32_t pv = (uint32_t)__shfl_up((int)v[j], 1);
            if (lane == 0) pv = carry;
            carry = (uint32_t)__shfl((int)v[j], 63);
            const uint64_t row = __ballot(pos < len && (pos == 0 || v[j] != pv));
            if (lane == k0 + j) mine = row;
        }
    }
    return mine;
}

__device__ __forceinline__ int64_t hi_bit_pos(uint64_t m, int64_t p0) { return p0 + 63 - (int64_t)__clzll((long long)m); }

__global__ void __launch_bounds__(KPW_BLOCK) k_rle_bounds(const RleJob *jobs, const uint32_t *ltile_job, int64_t *last_brk)
{
    __shared__ int64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x;
    const RleJob &J = jobs[ltile_job[t]];
    const ValSrc src = job_src(J);
    const int64_t len = J.len;
    const int64_t wb = (int64_t)(t - J.ltile0) * KPW_TILE_L + (int64_t)(threadIdx.x >> 6) * 4096;
    const uint64_t m = brk_mask64(src, wb, len);
    int64_t last = m ? hi_bit_pos(m, wb + 64 * (int64_t)(threadIdx.x & 63)) : -1;
    last = block_reduce<int64_t, OpMaxI64>(last, lds);
    if (threadIdx.x == 0) last_brk[t] = last;
}

// write = 0: long runs per tile into cnt[t]; write = 1: the runs at their offsets off[t]
__global__ void __launch_bounds__(KPW_BLOCK) k_rle_longruns(RleJob *jobs, const uint32_t *ltile_job, const int64_t *prev_brk,
                                                            uint32_t *cnt, const uint32_t *off, uint32_t *lr_a, uint32_t *lr_b,
                                                            int write)
{
    __shared__ int64_t ldsi[KPW_BLOCK];
    __shared__ uint32_t ldsu[KPW_BLOCK];
    const uint32_t t = blockIdx.x;
    RleJob &J = jobs[ltile_job[t]];
    const ValSrc src = job_src(J);
    const int64_t len = J.len;
    const int64_t wb = (int64_t)(t - J.ltile0) * KPW_TILE_L + (int64_t)(threadIdx.x >> 6) * 4096;
    const int64_t p0 = wb + 64 * (int64_t)(threadIdx.x & 63);
    const uint64_t m = brk_mask64(src, wb, len);
    int64_t tot_i;
    int64_t incoming = block_scan_excl<int64_t, OpMaxI64>(m ? hi_bit_pos(m, p0) : -1, ldsi, &tot_i);
    const int64_t pb = (t == J.ltile0) ? -1 : prev_brk[t];
    if (pb > incoming) incoming = pb;

    // long-run ends: breaks whose previous break is >= 8 positions back (inside the mask for all
    // but the lowest break; the lowest one's previous break is `incoming`; position 0 never ends
    // one: 0 - (-1) < 8)
    uint64_t le = m & ~((m << 1) | (m << 2) | (m << 3) | (m << 4) | (m << 5) | (m << 6) | (m << 7));
    if (m) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        if (p0 + (int64_t)l - incoming < 8) le &= ~(1ull << l);
    }
    // the final run of the stream ends at len, in the thread holding position len - 1
    const bool has_last = p0 < len && len - 1 < p0 + 64;
    const int64_t lastb = m ? hi_bit_pos(m, p0) : incoming;
    const bool fin = has_last && len - lastb >= 8;
    const uint32_t c = (uint32_t)__popcll(le) + (fin ? 1u : 0u);
    if (write) {
        uint32_t tot;
        const uint32_t ex = block_scan_excl<uint32_t, OpSum32>(c, ldsu, &tot);
        if (t == J.ltile0 + J.nltiles - 1 && threadIdx.x == 0) J.n_long = off[t] + tot;
        uint64_t o = J.e0 + off[t] + ex;
        for (uint64_t r = le; r; r &= r - 1) {
            const uint32_t i = (uint32_t)__builtin_ctzll(r);
            const uint64_t lower = m & ((1ull << i) - 1);
            lr_a[o] = (uint32_t)(lower ? hi_bit_pos(lower, p0) : incoming);
            lr_b[o] = (uint32_t)(p0 + i);
            o++;
        }
        if (fin) { lr_a[o] = (uint32_t)lastb; lr_b[o] = (uint32_t)len; }
    } else {
        const uint32_t sum = block_reduce<uint32_t, OpSum32>(c, ldsu);
        if (threadIdx.x == 0) cnt[t] = sum;
    }
}

// ------------------------------------------------------------------ phase scan over long runs
// One launch over the element tiles: the phase entering each long run (an 8-state map
// composition scan, look-back 0), the RLE runs among them, placed (sum-scan, look-back 1) and
// written as (g, b).  The job's last element tile stores n_rle.

// Fallbacks of k_phase's two scans (kpw_lookback.h): tile q's composed run maps, and its RLE
// run count, which needs the phase entering q: the scan-0 words of tiles [first, q) read
// backwards to the nearest inclusive one (each recomputed when it is not out).
struct PhaseFb0 {
    const uint32_t *a, *b;   // the job's long runs (lr_a + e0, lr_b + e0)
    uint32_t et0, nlong;
    __device__ void operator()(uint32_t q, uint32_t &v, bool &inc) const
    {
        uint32_t m = OpMapCompose::id();
        const uint64_t k0 = (uint64_t)(q - et0) * KPW_TILE_E;
        for (uint64_t k = k0; k < k0 + KPW_TILE_E && k < nlong; k++) m = OpMapCompose::op(m, run_map(a[k], b[k]));
        v = m;
        inc = q == et0;
    }
};
struct PhaseFb1 {
    PhaseFb0 f0;
    LbView L;
    __device__ void operator()(uint32_t q, uint32_t &v, bool &inc) const
    {
        uint32_t pre = OpMapCompose::id();
        for (uint32_t r = q; r-- > f0.et0;) {
            uint32_t m;
            bool ri;
            lb_peek<uint32_t, EncU32>(L, r, r, f0, m, ri);
            pre = OpMapCompose::op(m, pre);
            if (ri) break;
        }
        uint32_t phi = pm_get(pre, 0), cnt = 0;
        const uint64_t k0 = (uint64_t)(q - f0.et0) * KPW_TILE_E;
        for (uint64_t k = k0; k < k0 + KPW_TILE_E && k < f0.nlong; k++) {
            const uint32_t a = f0.a[k], b = f0.b[k];
            const uint32_t g = a + ((phi - a) & 7u);
            if (g + 8 <= b) { cnt++; phi = b & 7u; }
        }
        v = cnt;
        inc = q == f0.et0;
    }
};

__global__ void __launch_bounds__(KPW_BLOCK) k_phase(RleJob *jobs, const uint32_t *etile_job, const uint32_t *lr_a,
                                                     const uint32_t *lr_b, uint32_t *r_g, uint32_t *r_b, uint8_t *lr_rle, uint32_t nt,
                                                     LbView L)
{
    __shared__ uint32_t lds[KPW_BLOCK];
    __shared__ uint32_t c0, c1;
    const uint32_t u = blockIdx.x;
    RleJob &J = jobs[etile_job[u]];
    const uint32_t et0 = J.etile0;
    const uint32_t nlong = J.n_long;
    // element tiles are laid out for the job's capacity (len / 8 + 2); past its long runs a
    // tile has nothing to scan or write, and no later tile of the job needs its status
    const uint32_t last = et0 + (nlong ? (nlong - 1) / KPW_TILE_E : 0);
    if (u > last) return;
    const uint64_t k = (uint64_t)(u - et0) * KPW_TILE_E + threadIdx.x;
    const bool valid = k < nlong;
    uint32_t a = 0, b = 0, m = OpMapCompose::id();
    if (valid) { a = lr_a[J.e0 + k]; b = lr_b[J.e0 + k]; m = run_map(a, b); }
    uint32_t tot;
    const uint32_t ex = block_scan_excl<uint32_t, OpMapCompose>(m, lds, &tot);
    const PhaseFb0 fb0{lr_a + J.e0, lr_b + J.e0, et0, nlong};
    const uint32_t pre = lb_tile<uint32_t, OpMapCompose>(L, 0, u, et0, tot, u == et0, u != et0, &c0, fb0);
    const uint32_t phi = pm_get(ex, pm_get(pre, 0));
    const uint32_t g = a + ((phi - a) & 7u);
    const uint32_t rle = (valid && g + 8 <= b) ? 1u : 0u;
    if (lr_rle && valid) lr_rle[J.e0 + k] = (uint8_t)rle;
    uint32_t t2;
    const uint32_t idx = block_scan_excl<uint32_t, OpSum32>(rle, lds, &t2);
    const uint32_t off = lb_tile<uint32_t, OpSum32>(L, nt, u, et0, t2, u == et0, u != et0, &c1, PhaseFb1{fb0, L});
    if (rle) {
        const uint64_t o = J.e0 + off + idx;
        r_g[o] = g;
        r_b[o] = b;
    }
    if (u == last && threadIdx.x == 0) J.n_rle = off + t2;
}

// ------------------------------------------------------------------ sizes / offsets

__device__ __forceinline__ uint64_t gap_bytes(uint64_t G, uint32_t bw) { return G * bw + (G + 62) / 63; }
__device__ __forceinline__ uint32_t rle_bytes(uint32_t L, uint32_t bw) { return varint_len32(L << 1) + (bw + 7) / 8; }

// One launch over the element tiles: per RLE run the bytes and groups of (gap before it + the
// run), their offsets (two sum-scans, look-backs 0 and 1), and the job totals (the job's last
// run, or its first tile when it has none).
// Fallback of k_r_sizes' scans: tile q's bytes (groups = false) or groups of its RLE runs.
struct SizesFb {
    const uint32_t *g, *b;   // r_g + e0, r_b + e0
    uint32_t et0, nrle, bw;
    bool groups;
    __device__ void operator()(uint32_t q, uint64_t &v, bool &inc) const
    {
        uint64_t sum = 0;
        const uint64_t k0 = (uint64_t)(q - et0) * KPW_TILE_E;
        for (uint64_t k = k0; k < k0 + KPW_TILE_E && k < nrle; k++) {
            const uint32_t pe = k ? b[k - 1] : 0;
            const uint64_t gr = (g[k] - pe) >> 3;
            sum += groups ? gr : gap_bytes(gr, bw) + rle_bytes(b[k] - g[k], bw);
        }
        v = sum;
        inc = q == et0;
    }
};

__global__ void __launch_bounds__(KPW_BLOCK) k_r_sizes(RleJob *jobs, const uint32_t *etile_job, const uint32_t *r_g,
                                                       const uint32_t *r_b, uint64_t *r_boff, uint64_t *r_goff, uint32_t nt,
                                                       LbView L)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    __shared__ uint64_t c0, c1;
    const uint32_t u = blockIdx.x;
    RleJob &J = jobs[etile_job[u]];
    const uint32_t et0 = J.etile0;
    const uint64_t k = (uint64_t)(u - et0) * KPW_TILE_E + threadIdx.x;
    const uint32_t nrle = J.n_rle;
    if (u > et0 + (nrle ? (nrle - 1) / KPW_TILE_E : 0)) return;   // past the job's RLE runs
    const bool valid = k < nrle;
    uint64_t by = 0, gr = 0;
    if (valid) {
        const uint32_t g = r_g[J.e0 + k], b = r_b[J.e0 + k];
        const uint32_t pe = k ? r_b[J.e0 + k - 1] : 0;
        gr = (g - pe) >> 3;
        by = gap_bytes(gr, J.bw) + rle_bytes(b - g, J.bw);
    }
    uint64_t t1, t2;
    const uint64_t eb = block_scan_excl<uint64_t, OpSum64>(by, lds, &t1);
    const uint64_t eg = block_scan_excl<uint64_t, OpSum64>(gr, lds, &t2);
    const SizesFb fb{r_g + J.e0, r_b + J.e0, et0, nrle, J.bw, false};
    const uint64_t boff = lb_tile<uint64_t, OpSum64>(L, 0, u, et0, t1, u == et0, u != et0, &c0, fb);
    const uint64_t goff = lb_tile<uint64_t, OpSum64>(L, nt, u, et0, t2, u == et0, u != et0, &c1,
                                                     SizesFb{fb.g, fb.b, et0, nrle, J.bw, true});
    if (valid) {
        r_boff[J.e0 + k] = boff + eb;
        r_goff[J.e0 + k] = goff + eg;
    }
    const bool owner = (nrle == 0) ? (u == et0 && threadIdx.x == 0) : (k == (uint64_t)nrle - 1);
    if (owner) {
        const uint64_t last_end = nrle ? r_b[J.e0 + nrle - 1] : 0;
        const uint64_t fg = (J.len > last_end) ? ((uint64_t)J.len - last_end + 7) / 8 : 0;
        const uint64_t rb = nrle ? boff + eb + by : 0;
        const uint64_t rg = nrle ? goff + eg + gr : 0;
        J.final_gap_start = last_end;
        J.final_gap_off = rb;
        J.final_gap_groups = fg;
        J.total_bytes = rb + gap_bytes(fg, J.bw);
        J.total_groups = rg + fg;
    }
}

// ------------------------------------------------------------------ writers

__device__ __forceinline__ void rle_write_runs(const RleJob *jobs, const uint32_t *etile_job, const uint32_t *r_g,
                                               const uint32_t *r_b, const uint64_t *r_boff, uint8_t *out, uint32_t u)
{
    const RleJob &J = jobs[etile_job[u]];
    const uint64_t k = (uint64_t)(u - J.etile0) * KPW_TILE_E + threadIdx.x;
    if (k >= J.n_rle) return;
    const uint32_t g = r_g[J.e0 + k], b = r_b[J.e0 + k];
    const uint32_t pe = k ? r_b[J.e0 + k - 1] : 0;
    const uint64_t G = (g - pe) >> 3;
    uint8_t *o = out + J.out_off + r_boff[J.e0 + k] + gap_bytes(G, J.bw);
    uint32_t v = (b - g) << 1;
    while (v >= 0x80u) { *o++ = (uint8_t)(v | 0x80u); v >>= 7; }
    *o++ = (uint8_t)v;
    const uint32_t val = src_get(job_src(J), g);
    for (uint32_t i = 0; i < (J.bw + 7) / 8; i++) o[i] = (uint8_t)(val >> (8 * i));
}

struct GroupLoc { uint64_t gs, within, G, gap_off; };

__device__ __forceinline__ GroupLoc locate_group(const RleJob &J, uint64_t q, const uint32_t *r_g, const uint32_t *r_b,
                                                 const uint64_t *r_boff, const uint64_t *r_goff)
{
    GroupLoc L;
    const uint64_t fstart = J.total_groups - J.final_gap_groups;
    if (q >= fstart) {
        L.gs = J.final_gap_start; L.within = q - fstart; L.G = J.final_gap_groups; L.gap_off = J.final_gap_off;
        return L;
    }
    // largest k with r_goff[k] <= q
    uint64_t lo = 0, hi = J.n_rle;  // invariant: answer in [lo, hi)
    while (hi - lo > 1) {
        uint64_t mid = (lo + hi) >> 1;
        if (r_goff[J.e0 + mid] <= q) lo = mid; else hi = mid;
    }
    const uint64_t k = lo;
    L.gs = k ? r_b[J.e0 + k - 1] : 0;
    L.within = q - r_goff[J.e0 + k];
    L.G = (r_g[J.e0 + k] - L.gs) >> 3;
    L.gap_off = r_boff[J.e0 + k];
    return L;
}

__device__ __forceinline__ void rle_write_groups(const RleJob *jobs, const uint32_t *ptile_job, const uint32_t *r_g,
                                                 const uint32_t *r_b, const uint64_t *r_boff, const uint64_t *r_goff, uint8_t *out,
                                                 uint32_t t)
{
    const RleJob &J = jobs[ptile_job[t]];
    const uint64_t q = (uint64_t)(t - J.tile0) * KPW_BLOCK + threadIdx.x;
    if (q >= J.total_groups) return;
    const GroupLoc L = locate_group(J, q, r_g, r_b, r_boff, r_goff);
    const uint32_t bw = J.bw;
    const uint64_t m = L.within / 63, wi = L.within % 63;
    uint8_t *base = out + J.out_off + L.gap_off + m * (63ull * bw + 1);
    if (wi == 0) {
        const uint64_t ng = (L.G - 63 * m) < 63 ? (L.G - 63 * m) : 63;
        base[0] = (uint8_t)((ng << 1) | 1);
    }
    const ValSrc src = job_src(J);
    uint64_t w[4] = {0, 0, 0, 0};
    const uint64_t p = L.gs + L.within * 8;
    const uint64_t mask = bw >= 32 ? 0xffffffffull : ((1ull << bw) - 1);
#pragma unroll
    for (int v = 0; v < 8; v++) {
        const uint64_t pos = p + v;
        const uint64_t x = (pos < J.len) ? (src_get(src, pos) & mask) : 0;
        const uint32_t bp = v * bw;
        if (bw) {
            w[bp >> 6] |= x << (bp & 63);
            if ((bp & 63) + bw > 64) w[(bp >> 6) + 1] |= x >> (64 - (bp & 63));
        }
    }
    uint8_t *o = base + 1 + wi * bw;
    for (uint32_t i = 0; i < bw; i++) o[i] = (uint8_t)(w[i >> 3] >> (8 * (i & 7)));
}

// Planning mode: per-position emitted-byte events (event at the position whose write
// emits the bytes) and a bitmask of RLE-run end positions (gend; null: not kept).
__device__ __forceinline__ void rle_ev_runs(const RleJob *jobs, const uint32_t *etile_job, const uint32_t *r_g,
                                            const uint32_t *r_b, uint8_t *ev, uint64_t *gend, uint64_t gend_stride, uint32_t u)
{
    const uint32_t j = etile_job[u];
    const RleJob &J = jobs[j];
    const uint64_t k = (uint64_t)(u - J.etile0) * KPW_TILE_E + threadIdx.x;
    if (k >= J.n_rle) return;
    const uint32_t g = r_g[J.e0 + k], b = r_b[J.e0 + k];
    if (b >= J.len) return;  // emitted only by toBytes()
    ev[J.out_off + b] = (uint8_t)rle_bytes(b - g, J.bw);
    if (gend) atomicOr((unsigned long long *)&gend[j * gend_stride + (b >> 6)], 1ull << (b & 63));
}

__device__ __forceinline__ void rle_ev_groups(const RleJob *jobs, const uint32_t *ptile_job, const uint32_t *r_g,
                                              const uint32_t *r_b, const uint64_t *r_boff, const uint64_t *r_goff, uint8_t *ev,
                                              uint32_t t)
{
    const RleJob &J = jobs[ptile_job[t]];
    const uint64_t q = (uint64_t)(t - J.tile0) * KPW_BLOCK + threadIdx.x;
    if (q >= J.total_groups) return;
    const GroupLoc L = locate_group(J, q, r_g, r_b, r_boff, r_goff);
    const uint64_t last = L.gs + L.within * 8 + 7;
    if (last >= J.len) return;  // partial group: emitted only by toBytes()
    ev[J.out_off + last] = (uint8_t)(J.bw + ((L.within % 63) == 0 ? 1 : 0));
}

// one launch each: blocks [0, n_etiles) the RLE runs, the rest the bit-packed groups
__global__ void __launch_bounds__(KPW_BLOCK) k_rle_write(const RleJob *jobs, const uint32_t *etile_job, const uint32_t *ptile_job,
                                                         const uint32_t *r_g, const uint32_t *r_b, const uint64_t *r_boff,
                                                         const uint64_t *r_goff, uint8_t *out, uint32_t n_etiles)
{
    if (blockIdx.x < n_etiles) rle_write_runs(jobs, etile_job, r_g, r_b, r_boff, out, blockIdx.x);
    else rle_write_groups(jobs, ptile_job, r_g, r_b, r_boff, r_goff, out, blockIdx.x - n_etiles);
}
__global__ void __launch_bounds__(KPW_BLOCK) k_rle_ev(const RleJob *jobs, const uint32_t *etile_job, const uint32_t *ptile_job,
                                                      const uint32_t *r_g, const uint32_t *r_b, const uint64_t *r_boff,
                                                      const uint64_t *r_goff, uint8_t *ev, uint64_t *gend, uint64_t gend_stride,
                                                      uint32_t n_etiles)
{
    if (blockIdx.x < n_etiles) rle_ev_runs(jobs, etile_job, r_g, r_b, ev, gend, gend_stride, blockIdx.x);
    else rle_ev_groups(jobs, ptile_job, r_g, r_b, r_boff, r_goff, ev, blockIdx.x - n_etiles);
}

// ------------------------------------------------------------------ host launchers

// Long runs (5 launches: bounds, max-scan, count, sum-scan, write), then phases and sizes (one
// launch each, chaining two look-back scans); a launch whose scan scratch cannot grow is
// skipped with sc.seg->failed set (the engine fails the encode).
void launch_rle_structure(RleJob *jobs_d, int njobs, uint32_t n_ptiles, uint32_t n_etiles, const RleScratch &sc,
                          hipStream_t s)
{
    if (!njobs || !n_ptiles) return;
    const uint32_t nlt = sc.n_ltiles;
    hipLaunchKernelGGL(k_rle_bounds, dim3(nlt), dim3(KPW_BLOCK), 0, s, jobs_d, sc.ltile_job, sc.last_brk);
    seg_tile_scan<int64_t, OpMaxI64>(sc.last_brk, sc.prev_brk, sc.ltile_job, nlt, nullptr, sc.seg, s);
    hipLaunchKernelGGL(k_rle_longruns, dim3(nlt), dim3(KPW_BLOCK), 0, s, jobs_d, sc.ltile_job, (const int64_t *)sc.prev_brk,
                       sc.lr_cnt, (const uint32_t *)sc.lr_off, sc.lr_a, sc.lr_b, 0);
    seg_tile_scan<uint32_t, OpSum32>(sc.lr_cnt, sc.lr_off, sc.ltile_job, nlt, nullptr, sc.seg, s);
    hipLaunchKernelGGL(k_rle_longruns, dim3(nlt), dim3(KPW_BLOCK), 0, s, jobs_d, sc.ltile_job, (const int64_t *)sc.prev_brk,
                       sc.lr_cnt, (const uint32_t *)sc.lr_off, sc.lr_a, sc.lr_b, 1);
    LbView L = lb_prepare(sc.seg, 2ull * n_etiles, s);
    if (!L.w) return;
    hipLaunchKernelGGL(k_phase, dim3(n_etiles), dim3(KPW_BLOCK), 0, s, jobs_d, sc.etile_job, sc.lr_a, sc.lr_b, sc.r_g, sc.r_b,
                       sc.lr_rle, n_etiles, L);
    L = lb_prepare(sc.seg, 2ull * n_etiles, s);
    if (!L.w) return;
    hipLaunchKernelGGL(k_r_sizes, dim3(n_etiles), dim3(KPW_BLOCK), 0, s, jobs_d, sc.etile_job, sc.r_g, sc.r_b, sc.r_boff, sc.r_goff,
                       n_etiles, L);
}

void launch_rle_write(RleJob *jobs_d, uint32_t n_ptiles, uint32_t n_etiles, const RleScratch &sc, uint8_t *out, hipStream_t s)
{
    if (!n_ptiles) return;
    hipLaunchKernelGGL(k_rle_write, dim3(n_etiles + n_ptiles), dim3(KPW_BLOCK), 0, s, jobs_d, sc.etile_job, sc.ptile_job, sc.r_g,
                       sc.r_b, sc.r_boff, sc.r_goff, out, n_etiles);
}

void launch_rle_events(RleJob *jobs_d, uint32_t n_ptiles, uint32_t n_etiles, const RleScratch &sc, uint8_t *ev,
                       uint64_t *gend, uint64_t gend_stride, hipStream_t s)
{
    if (!n_ptiles) return;
    hipLaunchKernelGGL(k_rle_ev, dim3(n_etiles + n_ptiles), dim3(KPW_BLOCK), 0, s, jobs_d, sc.etile_job, sc.ptile_job, sc.r_g,
                       sc.r_b, sc.r_boff, sc.r_goff, ev, gend, gend_stride, n_etiles);
}

}  // namespace kpw
