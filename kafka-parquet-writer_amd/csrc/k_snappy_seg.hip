// k_snappy_seg.hip — K7 main kernel: segment-parallel Snappy fragment compression, byte-identical
// to the sequential algorithm the oracle pins (Google Snappy 1.1.2 CompressFragment,
// oracle/oracle_snappy.c).  CPU model + exactness check: tests/microbench/snappy_seg_proto.c.
//
// Why: the sequential match loop is one dependent chain per 64 KiB fragment (~1-2 k cycles per
// decision on a wave), so one wave per fragment leaves the chip latency-bound.
// Here one 1024-thread workgroup compresses one fragment; thread k owns the 64-byte segment
// [64k, 64k+64).
//
// The sequential parse is a chain of decisions (probe ip with skip; after a copy, probe its
// end).  Its only memory is the hash table, and entry h of that table is always the largest
// INSERTED position q < ip with hash(q) = h, or 0 (insertions happen in increasing position
// order).  So given the set I of inserted positions, every lookup is a pure function:
//   cand[p] = max { q in I : q < p, hash(q) = hash(p) }   (0 if none).
// cand[] is computed for all positions at once by a segmented max-scan over the positions
// sorted by (hash, position) (the sort is done once per fragment).  Rounds (Jacobi):
//   1. cand[] from the previous round's I (round 0: every position inserted);
//   2. every thread parses its segment from its entry state with cand[] -> exit state, the
//      positions it inserted, whether it found a match;
//   3. fixed point?  every entry equals the left neighbour's exit and I reproduced itself.
//      Then, by induction over decisions in position order, every lookup saw exactly the
//      sequential table, so the parse IS the sequential parse: emit.
//   4. otherwise entry(k) = the exit of the nearest thread to the left that found a match,
//      advanced arithmetically over the match-free segments in between (the positions a
//      match-free search probes do not depend on the data: ip += skip++ >> 5), and repeat.
// A fragment that needs more than SEG_MAXR rounds, a copy longer than SEG_MAXLEN bytes
// (long repeats: cheap for the sequential kernels) or whose sort check fails is marked
// SEG_ABORTED and compressed by k_snappy_v / k_snappy_s_rest instead (same bytes).
//
// LDS: cand u16[65536] (128 KiB; the staged fragment and the bucket counters during setup),
// the inserted-position bitmask (8 KiB), entry and exit states (8 KiB each): one workgroup per
// CU; the grid is one workgroup per CU and pulls fragments from a counter.
#include "kpw_device.h"
#include "kpw_chunk.h"

namespace kpw {

namespace {

constexpr uint32_t SG_SEG = 64;          // bytes per thread segment
constexpr uint32_t SG_T = 1024;          // threads per workgroup (segments per 64 KiB fragment)
constexpr uint32_t SG_W = SG_T / 64;     // waves
#ifndef SG_MAXR
#define SG_MAXR 128u             // rounds before a fragment is handed to the sequential kernels
#endif
constexpr uint32_t SG_MAXLEN = 512;
constexpr uint32_t SG_RECS = 16;         // copies per segment (each >= 4 bytes, starting inside it)
constexpr uint32_t SG_LITCOPY = 128;     // longer literals are copied by the whole workgroup
#ifndef SG_PB
#define SG_PB 4u                 // search probes in flight per parse step
#endif
#ifndef SG_LITW
#define SG_LITW 1                // emit: short literals stored as dwords
#endif
#ifndef SG_SW
#define SG_SW 4u                 // sort scatter: waves (each owns the hashes h % SG_SW)
#endif

constexpr uint32_t SG_NOMATCH = 0xffff;  // cand[]: the table entry's 4 bytes differ (positions < 65521)

enum : uint32_t { MS = 0, MP = 1, MT = 2 };
struct PS {
    uint32_t mode, ip, skip, ne;
};
// packed: mode 2 | ip 17 | skip 17 | ne 17 ; states are kept canonical (P: ne = ip, skip 0;
// T: ip = skip = 0) so equality is equality of the packed words
__device__ __forceinline__ uint64_t pk(PS s)
{
    return (uint64_t)s.mode | ((uint64_t)s.ip << 2) | ((uint64_t)s.skip << 19) | ((uint64_t)s.ne << 36);
}
__device__ __forceinline__ PS upk(uint64_t v)
{
    return PS{(uint32_t)(v & 3), (uint32_t)((v >> 2) & 0x1ffff), (uint32_t)((v >> 19) & 0x1ffff), (uint32_t)((v >> 36) & 0x1ffff)};
}
__device__ __forceinline__ PS st_T(uint32_t ne) { return PS{MT, 0, 0, ne}; }
__device__ __forceinline__ PS st_P(uint32_t ip) { return PS{MP, ip, 0, ip}; }

__device__ __forceinline__ uint32_t sg_hash(uint32_t b, int shift) { return (b * 0x1e35a7bdu) >> shift; }

__device__ __forceinline__ uint32_t sg_skip_sum(uint32_t v)
{
    const uint32_t q = v >> 5, r = v & 31;
    return 16u * q * (q - 1u) + r * q;
}

// a state advanced over match-free decisions to its first decision at or after s
__device__ PS sg_ff(PS x, uint32_t s, uint32_t ip_limit)
{
    if (x.mode == MT || x.ip >= s) return x;
    if (x.mode == MP) {   // the probe at the copy's end finds nothing; search from ip + 1
        x = PS{MS, x.ip + 1, 32, x.ip};
        if (x.ip >= s) return x;
    }
    const uint32_t b = sg_skip_sum(x.skip);
    uint32_t lo = 0, hi = 70000;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (x.ip + sg_skip_sum(x.skip + m) - b >= s) hi = m; else lo = m + 1;
    }
    const uint32_t ipm = x.ip + sg_skip_sum(x.skip + lo) - b;
    if (ipm > ip_limit) return st_T(x.ne);   // the probe before it stops the search
    return PS{MS, ipm, x.skip + lo, x.ne};
}

// global-memory views (explicit address space: global_load, not flat_load, whose waits also
// cover the LDS counter)
typedef const __attribute__((address_space(1))) uint32_t sgg_cu32;
typedef const __attribute__((address_space(1))) uint16_t sgg_cu16;
typedef unsigned int sg_u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) sg_u32x4 sgg_cu4;
typedef __attribute__((address_space(1))) sg_u32x4 sgg_u4;
typedef __attribute__((address_space(1))) uint16_t sgg_u16;
typedef const __attribute__((address_space(1))) uint8_t sgg_cu8;
typedef __attribute__((address_space(1))) uint8_t sgg_u8;

// fragment bytes through aligned dword loads (the page buffer is padded past its last page)
struct FIn {
    const uint8_t *base;
    __device__ __forceinline__ uint32_t ld32(uint32_t p) const
    {
        const uintptr_t a = (uintptr_t)(base + p);
        sgg_cu32 *w = (sgg_cu32 *)(a & ~(uintptr_t)3);
        return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3));
    }
    __device__ __forceinline__ uint64_t ld64(uint32_t p) const
    {
        const uintptr_t a = (uintptr_t)(base + p);
        sgg_cu32 *w = (sgg_cu32 *)(a & ~(uintptr_t)3);
        const uint32_t s = (uint32_t)(a & 3);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, s) << 32);
    }
    __device__ __forceinline__ uint8_t ld8(uint32_t p) const { return ((sgg_cu8 *)base)[p]; }
    // D dwords starting at byte p (D + 1 aligned loads, all in flight together)
    template <int D> __device__ __forceinline__ void ldw(uint32_t p, uint32_t *o) const
    {
        const uintptr_t a = (uintptr_t)(base + p);
        sgg_cu32 *w = (sgg_cu32 *)(a & ~(uintptr_t)3);
        const uint32_t s = (uint32_t)(a & 3);
        uint32_t v[D + 1];
#pragma unroll
        for (int i = 0; i <= D; i++) v[i] = w[i];
#pragma unroll
        for (int i = 0; i < D; i++) o[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], s);
    }
};

// FindMatchLength(s1, s2, limit); stops early (returns > cap) past cap bytes.  Past the first
// 16 bytes the comparison runs SG_FMLW bytes per dependent load round trip (r04: 32 bytes,
// C4 parse 578 -> 561 K cycles per fragment; 64 measured slower, and re-using the previous
// round's length of the same copy cost more in record loads than it saved).
#ifndef SG_FMLW
#define SG_FMLW 32
#endif
__device__ __forceinline__ uint32_t sg_fml(const FIn &in, uint32_t s1, uint32_t s2, uint32_t limit, uint32_t cap)
{
    uint32_t m = 0;
    if (s2 + 16 <= limit) {
        const uint64_t x0 = in.ld64(s1) ^ in.ld64(s2);
        const uint64_t x1 = in.ld64(s1 + 8) ^ in.ld64(s2 + 8);
        if (x0) return (uint32_t)__builtin_ctzll(x0) >> 3;
        if (x1) return 8 + ((uint32_t)__builtin_ctzll(x1) >> 3);
        m = 16;
#if SG_FMLW > 16
        constexpr int D = SG_FMLW / 4;   // dwords compared per step
        while (s2 + m + SG_FMLW <= limit) {
            uint32_t a[D], b[D];
            in.ldw<D>(s1 + m, a);
            in.ldw<D>(s2 + m, b);
            uint32_t r = 0xffffffffu;
#pragma unroll
            for (int i = D - 1; i >= 0; i--) {
                const uint32_t x = a[i] ^ b[i];
                if (x) r = (uint32_t)i * 4 + ((uint32_t)__builtin_ctz(x) >> 3);
            }
            if (r != 0xffffffffu) return m + r;
            m += SG_FMLW;
            if (m > cap) return m;
        }
#endif
    }
    while (s2 + m + 16 <= limit) {   // 16 bytes per step: both words' loads in flight together
        const uint64_t x0 = in.ld64(s1 + m) ^ in.ld64(s2 + m);
        const uint64_t x1 = in.ld64(s1 + m + 8) ^ in.ld64(s2 + m + 8);
        if (x0) return m + ((uint32_t)__builtin_ctzll(x0) >> 3);
        if (x1) return m + 8 + ((uint32_t)__builtin_ctzll(x1) >> 3);
        m += 16;
        if (m > cap) return m;
    }
    while (s2 + m + 8 <= limit) {
        const uint64_t x = in.ld64(s1 + m) ^ in.ld64(s2 + m);
        if (x) return m + ((uint32_t)__builtin_ctzll(x) >> 3);
        m += 8;
        if (m > cap) return m;
    }
    while (s2 + m < limit && in.ld8(s1 + m) == in.ld8(s2 + m)) m++;
    return m;
}

__device__ __forceinline__ uint32_t lit_size(uint32_t len)
{
    const uint32_t n = len - 1;
    return len + 1 + (n < 60 ? 0 : n < 256 ? 1 : n < 65536 ? 2 : n < (1u << 24) ? 3 : 4);
}
__device__ __forceinline__ uint32_t copy_size(uint32_t off, uint32_t len)
{
    uint32_t s = 0;
    while (len >= 68) { s += 3; len -= 64; }
    if (len > 64) { s += 3; len -= 60; }
    return s + ((len < 12 && off < 2048) ? 2 : 3);
}
__device__ __forceinline__ uint32_t put_copy_lt64(sgg_u8 *o, uint32_t op, uint32_t off, uint32_t len)
{
    if (len < 12 && off < 2048) {
        o[op] = (uint8_t)(1 + ((len - 4) << 2) + ((off >> 8) << 5));
        o[op + 1] = (uint8_t)(off & 0xff);
        return op + 2;
    }
    o[op] = (uint8_t)(2 + ((len - 1) << 2));
    o[op + 1] = (uint8_t)(off & 0xff);
    o[op + 2] = (uint8_t)(off >> 8);
    return op + 3;
}
__device__ __forceinline__ uint32_t put_copy(sgg_u8 *o, uint32_t op, uint32_t off, uint32_t len)
{
    while (len >= 68) { op = put_copy_lt64(o, op, off, 64); len -= 64; }
    if (len > 64) { op = put_copy_lt64(o, op, off, 60); len -= 60; }
    return put_copy_lt64(o, op, off, len);
}
__device__ __forceinline__ uint32_t put_lit_tag(sgg_u8 *o, uint32_t op, uint32_t len)
{
    uint32_t n = len - 1;
    if (n < 60) { o[op] = (uint8_t)(n << 2); return op + 1; }
    const uint32_t b = op++;
    int c = 0;
    while (n > 0) { o[op++] = (uint8_t)(n & 0xff); n >>= 8; c++; }
    o[b] = (uint8_t)((59 + c) << 2);
    return op;
}

// per-workgroup global scratch.  Lane-major layouts where a thread owns a row: the c-th 4 keys
// of thread t's 64 sorted entries sit at key4[c * SG_T + t], the r-th copy record of segment t
// at rec[r * SG_T + t], so a wave's loads and stores cover contiguous 1 KiB / 512 B spans.
struct SgScratch {
    uint4 sig4[8 * SG_T];         // positions sorted by (hash, position), 8 entries per piece
    uint4 key4[16 * SG_T];        // the 4 bytes at each sorted entry's position
    uint64_t bflag[SG_T];         // bit j of word t: sorted entry 64t+j starts a hash bucket
    uint64_t rec[SG_T * SG_RECS]; // copies found by the last parse, per segment
    uint32_t job[2 * SG_T][4];    // long literals: src, dst, len
};

// uint16 slot of sorted entry i
__device__ __forceinline__ uint32_t sig_slot(uint32_t i) { return i; }

constexpr uint32_t SG_DATA = 65536 + 64;   // setup: the fragment's bytes (+ read padding)
struct SgShared {
    union {
        uint16_t cand[65536];     // rounds: candidate (table entry) per position
        struct {
            uint32_t data[SG_DATA / 4];   // setup: the fragment, staged for the sort
            uint32_t cnt[8192 + 2];       // setup: bucket counters, two uint16 per word; + a dummy
        } su;
    } a;
    struct {
        uint64_t entry[SG_T];
        uint64_t exitst[SG_T];
    } b;
    uint64_t ibits[SG_T];         // inserted positions (bit q of word q/64); bucket starts during setup
    uint64_t found[SG_W];
    uint32_t lfl[SG_T / 32];      // thread k inserted 64k-1
    uint32_t wf[SG_W], wv[SG_W];  // block scan
    uint32_t njobs;
    int frag;
    uint64_t prof[16];            // microbench phase counters (thread 0)
};

// 4 bytes at position p of the LDS-staged fragment
__device__ __forceinline__ uint32_t lds_ld32(const SgShared &S, uint32_t p)
{
    const uint32_t d = p >> 2;
    return __builtin_amdgcn_alignbyte(S.a.su.data[d + 1], S.a.su.data[d], p & 3);
}

__device__ __forceinline__ uint32_t cnt_add(SgShared &S, uint32_t h)
{
    const uint32_t sh = (h & 1) * 16;
    return (atomicAdd(&S.a.su.cnt[h >> 1], 1u << sh) >> sh) & 0xffffu;
}

// exclusive scan of u32 over the workgroup; *total = sum
__device__ __forceinline__ uint32_t sg_scan_excl(uint32_t v, SgShared &S, uint32_t *total)
{
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += o;
    }
    if (lane == 63) S.wv[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t i = 0; i < SG_W; i++) { const uint32_t x = S.wv[i]; if (i < w) pre += x; tot += x; }
    __syncthreads();
    *total = tot;
    return pre + inc - v;
}

// exclusive segmented max-scan over the workgroup: carry into thread t from threads < t
// (flag = the thread's range starts a new bucket somewhere; val = running max at its end)
__device__ __forceinline__ uint32_t sg_segmax_carry(uint32_t flag, uint32_t val, SgShared &S)
{
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t f = flag, v = val;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t fo = __shfl_up(f, d, 64), vo = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) { if (!f) v = v > vo ? v : vo; f |= fo; }
    }
    uint32_t ef = __shfl_up(f, 1, 64), ev = __shfl_up(v, 1, 64);
    if (lane == 0) { ef = 0; ev = 0; }
    if (lane == 63) { S.wf[w] = f; S.wv[w] = v; }
    __syncthreads();
    uint32_t cv = 0;
    for (uint32_t i = 0; i < w; i++) {
        const uint32_t fi = S.wf[i], vi = S.wv[i];
        cv = fi ? vi : (cv > vi ? cv : vi);
    }
    __syncthreads();
    return ef ? ev : (ev > cv ? ev : cv);
}

// one parse of segment [sk, sk+64) from entry `st` with the current cand[]; REC: record the
// copies (for the emit) in G.rec
struct ParseOut {
    PS st;
    uint64_t own;
    bool lfl, fnd, lng;
    uint32_t nrec;
};
__device__ __forceinline__ ParseOut sg_parse(const SgShared &S, SgScratch &G, const FIn &in, PS st, uint32_t t, uint32_t n,
                                             uint32_t ip_limit)
{
    const uint32_t sk = t * SG_SEG, sk1 = sk + SG_SEG;
    ParseOut o{st, 0, false, false, false, 0};
    while (st.mode != MT && st.ip < sk1) {
        uint32_t base, c;
        bool lit;
        if (st.mode == MP) {
            const uint32_t ipe = st.ip;
            if (ipe - 1 >= sk) o.own |= 1ull << (ipe - 1 - sk); else o.lfl = true;
            c = S.a.cand[ipe];
            o.own |= 1ull << (ipe - sk);
            if (c == SG_NOMATCH) { st = PS{MS, ipe + 1, 32, ipe}; continue; }
            base = ipe; lit = false;
        } else {
            // SG_PB probes of the search at once: their positions (ip += skip++ >> 5) do not
            // depend on the data, so the cand[] reads of the next SG_PB decisions overlap (a
            // cand[] entry already says whether the candidate's 4 bytes match); the first probe
            // that matches is the one the sequential loop takes, and every probe up to it is
            // inserted (the same state as SG_PB sequential steps)
            uint32_t q[SG_PB], cc[SG_PB];
            bool v[SG_PB];
            uint32_t ipk = st.ip, skk = st.skip;
            bool alive = true, term = false;
#pragma unroll
            for (int k = 0; k < (int)SG_PB; k++) {
                const bool inseg = ipk < sk1;
                const uint32_t nx = ipk + (skk >> 5);
                v[k] = alive && inseg && nx <= ip_limit;
                term |= alive && inseg && nx > ip_limit;   // the sequential loop stops before probing
                alive = v[k];
                q[k] = v[k] ? ipk : st.ip;                 // (an always-valid address when unused)
                if (v[k]) { ipk = nx; skk++; }
            }
#pragma unroll
            for (int k = 0; k < (int)SG_PB; k++) cc[k] = S.a.cand[q[k]];
            int hit = -1;
#pragma unroll
            for (int k = (int)SG_PB - 1; k >= 0; k--)
                if (v[k] && cc[k] != SG_NOMATCH) hit = k;
#pragma unroll
            for (int k = 0; k < (int)SG_PB; k++)
                if (v[k] && (hit < 0 || k <= hit)) o.own |= 1ull << (q[k] - sk);
            if (hit < 0) {
                if (term) { st = st_T(st.ne); break; }
                st.ip = ipk; st.skip = skk;
                continue;
            }
            base = q[0]; c = cc[0];
#pragma unroll
            for (int k = 1; k < (int)SG_PB; k++) if (hit == k) { base = q[k]; c = cc[k]; }
            lit = true;
        }
        const uint32_t len = 4 + sg_fml(in, c + 4, base + 4, n, SG_MAXLEN);
        if (len > SG_MAXLEN) { o.lng = true; break; }
        o.fnd = true;
        G.rec[(o.nrec++) * SG_T + t] = (uint64_t)base | ((uint64_t)(base - c) << 16) | ((uint64_t)len << 32) | ((uint64_t)lit << 48);
        const uint32_t ipe = base + len;
        st = ipe >= ip_limit ? st_T(ipe) : st_P(ipe);
    }
    o.st = st;
    return o;
}

}  // namespace

constexpr size_t SEG_SCRATCH_BYTES = sizeof(SgScratch);

template <bool PROF>
__device__ __forceinline__ void k_snappy_seg_t(const SnappyArgs &a)
{
    __shared__ SgShared S;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    SgScratch &G = ((SgScratch *)a.seg_scratch)[blockIdx.x];
    // phase counters (thread 0): 0 setup, 1 scan, 2 parse, 3 check, 4 emit (cycles), 5 rounds,
    // 6 fragments, 7 handed on, 8.. setup sub-phases
    uint64_t *prof = S.prof;
    const bool pf = PROF && a.seg_prof && t == 0;
    if (PROF && a.seg_prof && t < 16) S.prof[t] = 0;
    uint64_t plast = 0;
#define PMARK(i) do { if (pf) { const uint64_t now_ = clock64(); prof[i] += now_ - plast; plast = now_; } if (a.seg_dbg && t == 0) a.seg_dbg[blockIdx.x * 4 + 2] = (i); } while (0)

    for (;;) {
        if (t == 0) {
            // every workgroup draws once past the last fragment, so the draw numbered
            // nfrags + grid - 1 is the launch's last: it leaves the counter at 0 for the next
            // launch (no fill before each launch)
            const uint32_t d = atomicAdd(a.seg_counter, 1u);
            if (d == a.nfrags + gridDim.x - 1) atomicExch(a.seg_counter, 0u);
            S.frag = (int)d;
        }
        __syncthreads();
        const uint32_t fslot = (uint32_t)S.frag;
        __syncthreads();
        if (fslot >= a.nfrags) break;
        const uint32_t f = a.order ? a.order[fslot] : fslot;
        if (a.seg_only_marked && a.frag_len[f] != SEG_TODO) continue;
        if (a.ftime && t == 0) a.ftime[2 * f] = wall_clock64();
        const uint32_t pg = a.frag_page[f], fi = a.frag_idx[f];
        const uint64_t plen = a.page_len[pg];
        const uint64_t fstart = (uint64_t)fi * SNAPPY_FRAG;
        const uint32_t n = (uint32_t)((plen - fstart) < SNAPPY_FRAG ? (plen - fstart) : SNAPPY_FRAG);
        const FIn in{a.in + a.page_off[pg] + fstart};
        sgg_u8 *out = (sgg_u8 *)(a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP);
        if (pf) { plast = clock64(); prof[6]++; }
        if (a.seg_dbg && t == 0) { a.seg_dbg[blockIdx.x * 4] = f; a.seg_dbg[blockIdx.x * 4 + 1] = 0; }

        if (n < 15) {   // no match loop: one literal
            if (t == 0) {
                uint32_t op = 0;
                if (n) {
                    op = put_lit_tag(out, 0, n);
                    for (uint32_t i = 0; i < n; i++) out[op + i] = in.ld8(i);
                    op += n;
                }
                a.frag_len[f] = op;
                if (a.ftime) a.ftime[2 * f + 1] = wall_clock64();
            }
            continue;
        }
        const uint32_t ip_limit = n - 15;
        const uint32_t npos = ip_limit;                 // positions 1..ip_limit -> sorted entries 0..npos-1
        const uint32_t nseg = (n + SG_SEG - 1) / SG_SEG;
        uint32_t tsize = 256;
        while (tsize < 16384 && tsize < n) tsize <<= 1;
        int shift = 32;
        for (uint32_t x = tsize; x > 1; x >>= 1) shift--;
        const uint64_t c_setup = pf ? clock64() : 0;

        // ------------------------------------------------ setup: sort positions by (hash, position)
        // The fragment is staged in LDS; counting sort with uint16 counters.  A histogram wave
        // instruction covers 64 consecutive positions (periodic data spreads over several
        // counters).  The scatter is one wave walking the positions in order: LDS atomics of one
        // instruction on the same counter return in lane order (checked below; a violation
        // hands the fragment on).  Sorted entries go to the lane-major global layout.
        {
            const uintptr_t fb = (uintptr_t)in.base;
            sgg_cu32 *src = (sgg_cu32 *)(fb & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)(fb & 3);
            // only the dwords that cover [0, n) (+ the 16 bytes of read padding the page buffer
            // has) are loaded: a short fragment may end near the end of the buffer
            const uint32_t nw = (n + sh + 3) / 4 + 1;    // source dwords covering the fragment (+1)
            uint32_t v[17];
#pragma unroll
            for (int i = 0; i < 17; i++) v[i] = (t * 16 + i < nw) ? src[t * 16 + i] : 0u;
#pragma unroll
            for (int i = 0; i < 16; i++) S.a.su.data[t * 16 + i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], sh);
            if (t < 16) S.a.su.data[SG_T * 16 + t] = 0;
            for (uint32_t i = t; i <= tsize / 2; i += SG_T) S.a.su.cnt[i] = 0;
            S.ibits[t] = 0;   // bucket-start bits during the sort
        }
        __syncthreads();
        PMARK(8);
#pragma unroll 8
        for (uint32_t j = 0; j < SG_SEG; j++) {
            const uint32_t p = j * SG_T + t;
            if (p >= 1 && p <= ip_limit) (void)cnt_add(S, sg_hash(lds_ld32(S, p), shift));
        }
        __syncthreads();
        PMARK(9);
        uint64_t bf = 0;
        {   // exclusive scan of the counters: thread t owns counter words [t*wpt, t*wpt + wpt)
            const uint32_t words = tsize / 2, wpt = (words + SG_T - 1) / SG_T, w0 = t * wpt;
            uint32_t loc = 0;
            for (uint32_t i = 0; i < wpt; i++)
                if (w0 + i < words) { const uint32_t x = S.a.su.cnt[w0 + i]; loc += (x & 0xffffu) + (x >> 16); }
            uint32_t tot;
            uint32_t run = sg_scan_excl(loc, S, &tot);
            for (uint32_t i = 0; i < wpt; i++)
                if (w0 + i < words) {
                    const uint32_t x = S.a.su.cnt[w0 + i], lo = x & 0xffffu, hi = x >> 16;
                    S.a.su.cnt[w0 + i] = run | ((run + lo) << 16);
                    if (lo) atomicOr((unsigned long long *)&S.ibits[run >> 6], 1ull << (run & 63));   // bucket starts
                    if (hi) atomicOr((unsigned long long *)&S.ibits[(run + lo) >> 6], 1ull << ((run + lo) & 63));
                    run += lo + hi;
                }
        }
        __syncthreads();
        PMARK(10);
        if (w < SG_SW) {
            // SG_SW waves walk the positions in order, wave w placing the hashes h with
            // h % SG_SW == w: a bucket belongs to one wave, so its entries stay in position
            // order; the other lanes issue no atomic (a returning LDS atomic costs per active lane)
            sgg_u16 *sig = (sgg_u16 *)G.sig4;
            const uint32_t ngr = ip_limit / 64 + 1;
            for (uint32_t g0 = 0; g0 < ngr; g0 += 16) {
                uint32_t h[16], idx[16];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const uint32_t p = (g0 + u) * 64 + lane;
                    const uint32_t hv = sg_hash(lds_ld32(S, p & 0xffffu), shift);
                    h[u] = (p >= 1 && p <= ip_limit && (hv % SG_SW) == w) ? hv : 0xffffffffu;
                }
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    idx[u] = 0;
                    if (h[u] != 0xffffffffu) idx[u] = atomicAdd(&S.a.su.cnt[h[u] >> 1], 1u << ((h[u] & 1) * 16));
                }
#pragma unroll
                for (int u = 0; u < 16; u++) asm volatile("" : "+v"(idx[u]));   // one wait for the batch
#pragma unroll
                for (int u = 0; u < 16; u++)
                    if (h[u] != 0xffffffffu) sig[sig_slot((idx[u] >> ((h[u] & 1) * 16)) & 0xffffu)] = (uint16_t)((g0 + u) * 64 + lane);
            }
        }
        __threadfence_block();
        __syncthreads();
        PMARK(11);
        // order check, bucket-start bits -> global (every round reads its 64 entries and bits)
        int bad = 0;
        {
            const uint32_t i0 = t * SG_SEG;
            bf = S.ibits[t];
            uint32_t prevp = (i0 > 0 && i0 <= npos) ? ((sgg_cu16 *)G.sig4)[sig_slot(i0 - 1)] : 0;
            // with the check, the 4 bytes at every sorted entry's position, from the staged
            // fragment: the rounds compare a position with its candidate there, so the parse's
            // probes are LDS reads
            sgg_cu4 *sp4 = (sgg_cu4 *)(G.sig4 + t * 8);
            sgg_u4 *kp = (sgg_u4 *)(G.key4 + t);
#pragma unroll
            for (int q0 = 0; q0 < 8; q0 += 4) {
            sg_u32x4 vq[4];
#pragma unroll
            for (int q = 0; q < 4; q++) vq[q] = sp4[q0 + q];
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const int q = q0 + qq;
                uint32_t pp[8], kk[8];
#pragma unroll
                for (int e = 0; e < 8; e++) pp[e] = (vq[qq][e >> 1] >> ((e & 1) * 16)) & 0xffffu;
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    const uint32_t j = q * 8 + e;
                    if (i0 + j < npos && !((bf >> j) & 1) && pp[e] <= prevp) bad = 1;
                    prevp = pp[e];
                    kk[e] = lds_ld32(S, pp[e]);
                }
                kp[(2 * q) * SG_T] = sg_u32x4{kk[0], kk[1], kk[2], kk[3]};
                kp[(2 * q + 1) * SG_T] = sg_u32x4{kk[4], kk[5], kk[6], kk[7]};
            }
            }
            G.bflag[t] = bf;
        }
        const uint32_t key0 = lds_ld32(S, 0);   // the empty table's candidate is position 0
        __syncthreads();
        // round 0: every position inserted; entries advanced from the start over match-free segments
        const PS init{MS, 1, 32, 0};
        S.ibits[t] = t < nseg ? ~0ull : 0ull;
        S.b.entry[t] = pk(t == 0 ? init : sg_ff(init, t * SG_SEG, ip_limit));
        if (t < SG_T / 32) S.lfl[t] = 0;
        if (t < SG_W) S.found[t] = 0;
        __threadfence_block();
        bad = __syncthreads_or(bad);
        PMARK(12);
        bool converged = false;
        uint32_t rounds = 0;
        uint64_t sc_ins = 0;      // the scan's inserted bits and carry-in of the previous round
        uint32_t sc_carry = 0;
        const uint32_t sk = t * SG_SEG;
        if (pf) prof[0] += clock64() - c_setup;
        ParseOut po{};

        while (!bad && rounds < SG_MAXR) {
            rounds++;
            if (a.seg_dbg && t == 0) a.seg_dbg[blockIdx.x * 4 + 1] = rounds;
            // ---------------------------------------------- cand[] from ibits (segmented max-scan)
            {
                const uint32_t i0 = t * SG_SEG;
                uint32_t sg2[SG_SEG / 2];
                {
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const uint4 v = G.sig4[t * 8 + q];
                        sg2[4 * q] = v.x; sg2[4 * q + 1] = v.y; sg2[4 * q + 2] = v.z; sg2[4 * q + 3] = v.w;
                    }
                }
                const uint64_t bf = G.bflag[t];
                uint32_t m = 0;
                uint64_t insm = 0;   // bit j: sorted entry i0+j is an inserted position
                const uint32_t *ib32 = (const uint32_t *)S.ibits;
#pragma unroll
                for (int j0 = 0; j0 < (int)SG_SEG; j0 += 16) {   // 16 LDS reads in flight per batch
                    uint32_t wv[16];
#pragma unroll
                    for (int u = 0; u < 16; u++) {
                        const int j = j0 + u;
                        const uint32_t p = (sg2[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
                        wv[u] = ib32[p >> 5];
                    }
#pragma unroll
                    for (int u = 0; u < 16; u++) asm volatile("" : "+v"(wv[u]));
#pragma unroll
                    for (int u = 0; u < 16; u++) {
                        const int j = j0 + u;
                        const uint32_t p = (sg2[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
                        const uint32_t ins = (i0 + j < npos) ? ((wv[u] >> (p & 31)) & 1) : 0u;
                        insm |= (uint64_t)ins << j;
                        if ((bf >> j) & 1) m = 0;
                        if (ins) m = p;
                    }
                }
                PMARK(13);
                m = sg_segmax_carry(i0 < npos && bf != 0, i0 < npos ? m : 0, S);
                PMARK(14);
                // cand[p] = the candidate when its 4 bytes equal p's, else SG_NOMATCH.  The
                // thread's cand[] values are a function of its inserted bits and its carry-in
                // alone: when neither changed since the last round they are already in LDS
                const bool same = rounds > 1 && insm == sc_ins && m == sc_carry;
                sc_ins = insm;
                sc_carry = m;
                uint32_t km = (!same && m) ? in.ld32(m) : key0;
#pragma unroll
                for (int q = 0; q < (int)SG_SEG / 2; q++) asm volatile("" : "+v"(sg2[q]));   // re-extract, do not keep 64 values live
                if (!same) {
                    // keys in 4 chunks of 4 pieces, the next chunk's loads in flight while one is
                    // used (the base is re-derived every round: hoisted per-piece addresses spill)
                    sgg_cu4 *kp = (sgg_cu4 *)(G.key4 + t);
                    asm volatile("" : "+v"(kp));
                    sg_u32x4 kb[2][4];
#pragma unroll
                    for (int i = 0; i < 4; i++) kb[0][i] = kp[i * SG_T];
#pragma unroll
                    for (int c4 = 0; c4 < 4; c4++) {
                        if (c4 < 3) {
#pragma unroll
                            for (int i = 0; i < 4; i++) kb[(c4 + 1) & 1][i] = kp[((c4 + 1) * 4 + i) * SG_T];
                        }
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const sg_u32x4 k4 = kb[c4 & 1][i];
                            const uint32_t kk[4] = {k4.x, k4.y, k4.z, k4.w};
#pragma unroll
                            for (int e = 0; e < 4; e++) {
                                const int j = (c4 * 4 + i) * 4 + e;
                                const uint32_t p = (sg2[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
                                if ((bf >> j) & 1) { m = 0; km = key0; }
                                if (i0 + j < npos) S.a.cand[p] = (uint16_t)(km == kk[e] ? m : SG_NOMATCH);
                                if ((insm >> j) & 1) { m = p; km = kk[e]; }
                            }
                        }
                    }
                }
            }
            PMARK(15);
            __syncthreads();
            PMARK(1);
            // ---------------------------------------------- parse my segment
            po = t < nseg ? sg_parse(S, G, in, upk(S.b.entry[t]), t, n, ip_limit)
                          : ParseOut{upk(S.b.entry[t]), 0, false, false, false, 0};
            S.b.exitst[t] = pk(po.st);
            if (po.lfl) atomicOr(&S.lfl[t >> 5], 1u << (t & 31));
            {
                const uint64_t fm = __ballot(po.fnd);
                if (lane == 0) S.found[w] = fm;
            }
            __syncthreads();
            PMARK(2);
            // ---------------------------------------------- fixed point?
            bool diff = false;
            uint64_t nb = 0;
            if (t < nseg) {
                const uint32_t k1 = t + 1;
                nb = po.own | ((k1 < SG_T && ((S.lfl[k1 >> 5] >> (k1 & 31)) & 1)) ? (1ull << 63) : 0ull);
                diff = nb != S.ibits[t];
                if (t + 1 < nseg && S.b.exitst[t] != S.b.entry[t + 1]) diff = true;
            }
            __syncthreads();
            if (t < nseg) S.ibits[t] = nb;
            if (__syncthreads_or((int)po.lng)) { bad = 1; break; }
            if (!__syncthreads_or((int)diff)) { converged = true; break; }
            // ---------------------------------------------- next entries
            if (t < nseg) {
                int j = -1;
                {
                    const uint64_t mine = S.found[w] & ((1ull << lane) - 1);
                    if (mine) j = (int)(w * 64 + 63 - __builtin_clzll(mine));
                    else
                        for (int ww = (int)w - 1; ww >= 0; ww--)
                            if (S.found[ww]) { j = ww * 64 + 63 - __builtin_clzll(S.found[ww]); break; }
                }
                const PS e = t == 0 ? init : sg_ff(j >= 0 ? upk(S.b.exitst[j]) : init, sk, ip_limit);
                S.b.entry[t] = pk(e);
            }
            __syncthreads();
            if (t < SG_T / 32) S.lfl[t] = 0;
            __syncthreads();
            PMARK(3);
        }
        if (pf) prof[5] += rounds;

        if (!converged) {
            if (pf) prof[7]++;
            if (t == 0) a.frag_len[f] = SEG_ABORTED;
            continue;
        }
        // ---------------------------------------------- emit the converged parse's copies
        const PS e0 = upk(S.b.entry[t]);
        uint32_t osz = 0;
        uint32_t ne = e0.ne;
        for (uint32_t r = 0; r < po.nrec; r++) {
            const uint64_t rc = G.rec[r * SG_T + t];
            const uint32_t base = (uint32_t)(rc & 0xffff), off = (uint32_t)((rc >> 16) & 0xffff);
            const uint32_t len = (uint32_t)((rc >> 32) & 0xffff), lit = (uint32_t)(rc >> 48) & 1;
            if (lit) osz += lit_size(base - ne);
            osz += copy_size(off, len);
            ne = base + len;
        }
        // the thread whose parse ends the fragment emits the remainder literal
        const bool tail = t < nseg && po.st.mode == MT && e0.mode != MT;
        if (tail && po.st.ne < n) osz += lit_size(n - po.st.ne);
        if (t == 0) S.njobs = 0;
        uint32_t total;
        const uint32_t obase = sg_scan_excl(osz, S, &total);
        if (t < nseg) {
            uint32_t op = obase;
            ne = e0.ne;
            auto lit_out = [&](uint32_t src, uint32_t len) {
                op = put_lit_tag(out, op, len);
                if (len <= SG_LITCOPY) {
#if SG_LITW
                    // dword stores once the output is aligned (the thread owns [op, op + len))
                    uint32_t i = 0;
                    for (; i < len && ((op + i) & 3); i++) out[op + i] = in.ld8(src + i);
                    for (; i + 4 <= len; i += 4) *(__attribute__((address_space(1))) uint32_t *)(out + op + i) = in.ld32(src + i);
                    for (; i < len; i++) out[op + i] = in.ld8(src + i);
#else
                    for (uint32_t i = 0; i < len; i++) out[op + i] = in.ld8(src + i);
#endif
                } else {
                    const uint32_t jx = atomicAdd(&S.njobs, 1u);
                    G.job[jx][0] = src; G.job[jx][1] = op; G.job[jx][2] = len;
                }
                op += len;
            };
            for (uint32_t r = 0; r < po.nrec; r++) {
                const uint64_t rc = G.rec[r * SG_T + t];
                const uint32_t base = (uint32_t)(rc & 0xffff), off = (uint32_t)((rc >> 16) & 0xffff);
                const uint32_t len = (uint32_t)((rc >> 32) & 0xffff), lit = (uint32_t)(rc >> 48) & 1;
                if (lit) lit_out(ne, base - ne);
                op = put_copy(out, op, off, len);
                ne = base + len;
            }
            if (tail && po.st.ne < n) lit_out(po.st.ne, n - po.st.ne);
        }
        __threadfence_block();
        __syncthreads();
        {   // long literals, copied by the whole workgroup
            const uint32_t nj = S.njobs;
            for (uint32_t jx = 0; jx < nj; jx++) {
                const uint32_t src = G.job[jx][0], dst = G.job[jx][1], len = G.job[jx][2];
                for (uint32_t i = t; i < len; i += SG_T) out[dst + i] = in.ld8(src + i);
            }
        }
        if (t == 0) {
            a.frag_len[f] = total;
            if (a.ftime) a.ftime[2 * f + 1] = wall_clock64();
        }
        __syncthreads();
        PMARK(4);
    }
#undef PMARK
    if (a.seg_dbg && t == 0) a.seg_dbg[blockIdx.x * 4 + 3] = 1;   // done
    if (pf)
        for (int i = 0; i < 16; i++) atomicAdd((unsigned long long *)&a.seg_prof[i], (unsigned long long)prof[i]);
}

// one instantiation, profiling gated at run time (a.seg_prof): the PROF=false instantiation hung
// after a fragment's last round on gfx950 (a barrier issue in the compiled code, not reproduced
// with the counters in; tests/microbench/seg_bench.hip SEG_DEBUG=2)
__global__ void __launch_bounds__(1024) k_snappy_seg(SnappyArgs a) { k_snappy_seg_t<true>(a); }

size_t snappy_seg_scratch_bytes(uint32_t grid) { return (size_t)grid * SEG_SCRATCH_BYTES; }

}  // namespace kpw
