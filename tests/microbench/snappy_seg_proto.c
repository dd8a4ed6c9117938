/*
 * snappy_seg_proto.c — test infrastructure: CPU model of the segment-parallel Snappy fragment
 * compressor that K7 (k_snappy_seg, csrc/k_snappy.hip) runs on the GPU, checked byte-for-byte
 * against the oracle's sequential compressor (oracle/oracle_snappy.c, Snappy 1.1.2).
 *
 * The sequential parse of a fragment is a chain of decisions (probe ip with skip; after a copy,
 * probe its end).  Its only memory is the hash table, whose entry for hash h is the largest
 * INSERTED position q < ip with hash(q) = h (insertions happen in increasing position order),
 * or 0.  So with prev[p] = the previous position with the same hash (a chain over all
 * positions) and the set I of inserted positions, candidate(p) = first q on p's chain with q in
 * I.  The fragment is cut into 64-byte segments, one lane each.  Every lane parses its segment
 * from a guessed entry state, with lookups of positions before its segment taken from the
 * previous round's I.  Rounds repeat (Jacobi) until every lane's entry state equals its left
 * neighbour's exit state and I reproduces itself: that fixed point is the sequential parse
 * (induction over segments), so the output is identical.  Between rounds a lane's entry is
 * the exit of the nearest lane to its left that found a match, advanced arithmetically over
 * the match-free lanes in between (the probe positions of a match-free search do not depend
 * on the data).
 *
 *   gcc -O2 -I../../include snappy_seg_proto.c ../../oracle/oracle_snappy.c -o /tmp/segp && /tmp/segp
 *   /tmp/segp -f pages.bin   (pages from dump_any.py): per page rounds, and a rounds histogram
 *
 * Options (environment):
 *   GPUF=1   every lookup reads the previous round's inserted set (k_snappy_seg before round 6);
 *            default: a lane's lookups inside its own segment see its live insertions of this parse
 *   GPUF=2   k_snappy_seg's live lookup (live_lookup: in-segment links with key-equality bits,
 *            CHAINCAP steps, undecided -> the previous round's candidate)
 *   MODE=4   in-round forwarding, bounded: after the Jacobi parse, every lane whose entry differs
 *            from the forwarded exit of its left neighbours re-parses once in the same round
 *   MODE=1/2 in-round forwarding, unbounded (Gauss-Seidel: lanes re-parse left to right until
 *            consistent; 2 also lets them see the left lanes' live insertions): one round, but
 *            the re-parses form a chain ("maxchain" = its longest run per round)
 *   TRACE=1  per round: lanes whose exit changed, entries changed, first inconsistent lane
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int64_t kpwo_snappy_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);

#define SEG 64
#define MAXSEG 1024
#define MAXIT 64
static int GPUF = 0;
static int HOPCAP = 1 << 30;

enum { M_S = 0, M_P = 1, M_T = 2 };
typedef struct { uint32_t mode, ip, skip, ne; } St;

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint32_t hsh(uint32_t b, int shift) { return (b * 0x1e35a7bdu) >> shift; }
static inline uint32_t skip_sum(uint32_t v) { uint32_t q = v >> 5, r = v & 31; return 16u * q * (q - 1u) + r * q; }

/* advance a state over match-free decisions to the first decision at or after s */
static St ff(St x, uint32_t s, uint32_t ip_limit)
{
    if (x.mode == M_T || x.ip >= s) return x;
    if (x.mode == M_P) { St y = {M_S, x.ip + 1, 32, x.ip}; x = y; if (x.ip >= s) return x; }
    /* smallest m with ip + D(m) >= s, D(m) = skip_sum(skip+m) - skip_sum(skip) */
    const uint32_t b = skip_sum(x.skip);
    uint32_t lo = 0, hi = 70000;
    while (lo < hi) { uint32_t m = (lo + hi) / 2; if (x.ip + (uint64_t)skip_sum(x.skip + m) - b >= s) hi = m; else lo = m + 1; }
    const uint64_t ipm = x.ip + (uint64_t)skip_sum(x.skip + lo) - b;
    if (ipm > ip_limit) { St t = {M_T, 0, 0, x.ne}; return t; }
    St y = {M_S, (uint32_t)ipm, x.skip + lo, x.ne};
    return y;
}

typedef struct { uint32_t ne, base, off, len; } Match;

typedef struct {
    const uint8_t *in;
    uint32_t n, ip_limit;
    int shift;
    uint16_t *prev;           /* [ip_limit+1] */
    uint64_t *iprev;          /* bitmask of inserted positions (previous round) */
} Frag;

typedef struct {
    St exit;
    uint64_t own;             /* insertions at sk..sk+63 */
    int flag_left;            /* inserted sk-1 */
    int found;                /* found a match */
    int aborted;              /* a lookup ran past HOPCAP hops */
    int nm;
    Match m[SEG];
    uint64_t lookups, hops;
} Lane;

static int bit(const uint64_t *bm, uint32_t q) { return (bm[q >> 6] >> (q & 63)) & 1; }

/* GPUF=2: k_snappy_seg's live lookup.  creg(x) = the previous round's candidate with its key
 * check (cand[x]: a position, or NOMATCH); links = the previous same-hash position inside x's
 * segment with a key-equality bit; walk them to the nearest own-inserted position, or to the
 * segment's first same-hash position, whose cand[] lies before the segment; an undecided key
 * comparison or a chain past CHAINCAP steps falls back to creg(x) (both agree at the fixed point) */
#define NOMATCH 0xffffffffu
static int CHAINCAP = 8;
static uint64_t st_live, st_linked, st_steps, st_fallback;
static uint32_t creg(const Frag *F, uint32_t x)
{
    uint32_t c = F->prev[x];
    while (c && !bit(F->iprev, c)) c = F->prev[c];
    return ld32(F->in + x) == ld32(F->in + c) ? c : NOMATCH;
}
/* GPUF=3: only the nearest same-hash position at distance d in LIVE_D (bit d-1) is looked at:
 * inserted -> decided by key equality; otherwise the previous round's candidate */
static int LIVE_D = 1;
static uint32_t live_short(const Frag *F, uint32_t x, uint32_t sk, uint64_t own)
{
    const uint32_t c = creg(F, x);
    const uint32_t q = F->prev[x];
    if (!q || q < sk || x - q > 8 || !((LIVE_D >> (x - q - 1)) & 1)) return c;
    if (!((own >> (q - sk)) & 1)) return c;
    return ld32(F->in + x) == ld32(F->in + q) ? q : NOMATCH;
}
static uint32_t live_lookup(const Frag *F, uint32_t x, uint32_t sk, uint64_t own)
{
    if (GPUF == 3) return live_short(F, x, sk, own);
    const uint32_t c = creg(F, x);
    uint32_t q = F->prev[x];
    st_live++;
    if (!q || q < sk) return c;                      /* no link: hasl bit clear */
    st_linked++;
    int rel = ld32(F->in + x) == ld32(F->in + q);    /* 1 EQ, 0 NE */
    for (int s = 0; s < CHAINCAP; s++) {
        st_steps++;
        if ((own >> (q - sk)) & 1) return rel ? q : NOMATCH;
        const uint32_t q2 = F->prev[q];
        if (!q2 || q2 < sk) {
            const uint32_t co = creg(F, q);
            if (rel) return co;
            return co != NOMATCH ? NOMATCH : c;
        }
        const int eq = ld32(F->in + q) == ld32(F->in + q2);
        if (rel) rel = eq;
        else if (!eq) return c;
        q = q2;
    }
    return c;
}

static void lane_parse(const Frag *F, uint32_t k, St st, Lane *L)
{
    const uint32_t sk = k * SEG, sk1 = sk + SEG;
    L->own = 0; L->flag_left = 0; L->found = 0; L->aborted = 0; L->nm = 0; L->lookups = 0; L->hops = 0;
#define INSERT(q) do { uint32_t q_ = (q); if (q_ >= sk) L->own |= 1ull << (q_ - sk); else L->flag_left = 1; } while (0)
#define INS(q) ((q) >= sk && !GPUF ? (int)((L->own >> ((q) - sk)) & 1) : bit(F->iprev, (q)))
    while (st.mode != M_T && st.ip < sk1) {
        uint32_t base, ne;
        uint32_t c;
        if (st.mode == M_P) {
            const uint32_t ipe = st.ip;
            INSERT(ipe - 1);
            if (GPUF >= 2) {
                c = live_lookup(F, ipe, sk, L->own); L->lookups++;
                INSERT(ipe);
                if (c == NOMATCH) { St y = {M_S, ipe + 1, 32, ipe}; st = y; continue; }
            } else {
            c = F->prev[ipe]; L->lookups++;
            { int h = 0; while (c && !INS(c)) { c = F->prev[c]; L->hops++; if (++h > HOPCAP) { L->aborted = 1; goto out; } } }
            INSERT(ipe);
            if (ld32(F->in + ipe) != ld32(F->in + c)) { St y = {M_S, ipe + 1, 32, ipe}; st = y; continue; }
            }
            base = ipe; ne = ipe;
        } else {
            const uint32_t ip = st.ip;
            const uint32_t next_ip = ip + (st.skip >> 5);
            if (next_ip > F->ip_limit) { St t = {M_T, 0, 0, st.ne}; st = t; break; }
            if (GPUF >= 2) {
                c = live_lookup(F, ip, sk, L->own); L->lookups++;
                INSERT(ip);
                if (c == NOMATCH) { st.ip = next_ip; st.skip++; continue; }
            } else {
            c = F->prev[ip]; L->lookups++;
            { int h = 0; while (c && !INS(c)) { c = F->prev[c]; L->hops++; if (++h > HOPCAP) { L->aborted = 1; goto out; } } }
            INSERT(ip);
            if (ld32(F->in + ip) != ld32(F->in + c)) { st.ip = next_ip; st.skip++; continue; }
            }
            base = ip; ne = st.ne;
        }
        /* match: FindMatchLength(c+4, base+4, n) */
        uint32_t len = 4;
        while (base + len < F->n && F->in[c + len] == F->in[base + len]) len++;
        L->found = 1;
        Match mm = {ne, base, base - c, len};
        L->m[L->nm++] = mm;
        const uint32_t ipe = base + len;
        if (ipe >= F->ip_limit) { St t = {M_T, 0, 0, ipe}; st = t; }
        else { St p = {M_P, ipe, 0, ipe}; st = p; }
    }
out:
    L->exit = st;
#undef INSERT
#undef INS
}

static uint8_t *emit_literal(uint8_t *op, const uint8_t *lit, uint32_t len)
{
    uint32_t n = len - 1;
    if (n < 60) *op++ = (uint8_t)(n << 2);
    else { uint8_t *b = op++; int c = 0; while (n > 0) { *op++ = (uint8_t)(n & 0xff); n >>= 8; c++; } *b = (uint8_t)((59 + c) << 2); }
    memcpy(op, lit, len);
    return op + len;
}
static uint8_t *emit_copy_lt64(uint8_t *op, uint32_t offset, uint32_t len)
{
    if (len < 12 && offset < 2048) { *op++ = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 8) << 5)); *op++ = (uint8_t)(offset & 0xff); }
    else { *op++ = (uint8_t)(2 + ((len - 1) << 2)); *op++ = (uint8_t)(offset & 0xff); *op++ = (uint8_t)(offset >> 8); }
    return op;
}
static uint8_t *emit_copy(uint8_t *op, uint32_t offset, uint32_t len)
{
    while (len >= 68) { op = emit_copy_lt64(op, offset, 64); len -= 64; }
    if (len > 64) { op = emit_copy_lt64(op, offset, 60); len -= 60; }
    return emit_copy_lt64(op, offset, len);
}

static int st_eq(St a, St b)
{
    if (a.mode != b.mode) return 0;
    if (a.mode == M_T) return a.ne == b.ne;
    if (a.mode == M_P) return a.ip == b.ip;
    return a.ip == b.ip && a.skip == b.skip && a.ne == b.ne;
}

static Lane lanes[MAXSEG];
static St entry[MAXSEG];
static uint64_t stat_lookups, stat_hops, stat_cost, stat_reparse, stat_chain;
static int MODE = 0; static int TRACE = 0;

/* returns output length, or -1 when the rounds do not converge; *rounds = rounds run */
static long seg_fragment(const uint8_t *in, uint32_t n, uint8_t *out, int *rounds)
{
    uint8_t *op = out;
    *rounds = 0;
    if (n < 15) { if (n) op = emit_literal(op, in, n); return op - out; }
    uint32_t ts = 256;
    while (ts < (1u << 14) && ts < n) ts <<= 1;
    int shift = 32; for (uint32_t t = ts; t > 1; t >>= 1) shift--;
    Frag F;
    F.in = in; F.n = n; F.ip_limit = n - 15; F.shift = shift;
    static uint16_t prev[65536], last[1 << 14];
    static uint64_t bm[1024], bm2[1024];
    memset(last, 0, sizeof last);
    for (uint32_t p = 1; p <= F.ip_limit; p++) { uint32_t h = hsh(ld32(in + p), shift); prev[p] = last[h]; last[h] = (uint16_t)p; }
    F.prev = prev;
    const uint32_t nseg = (n + SEG - 1) / SEG;
    memset(bm, 0xff, sizeof bm);           /* round 0: every position inserted */
    F.iprev = bm;
    const St init = {M_S, 1, 32, 0};
    for (uint32_t k = 0; k < nseg; k++) entry[k] = ff(init, k * SEG, F.ip_limit);
    entry[0] = init;
    for (int it = 0; it < MAXIT; it++) {
        *rounds = it + 1;
        uint64_t mx = 0;
        for (uint32_t k = 0; k < nseg; k++) {
            lane_parse(&F, k, entry[k], &lanes[k]); stat_lookups += lanes[k].lookups; stat_hops += lanes[k].hops;
            uint64_t c = lanes[k].lookups + lanes[k].hops;
            for (int i = 0; i < lanes[k].nm; i++) c += lanes[k].m[i].len / 16;
            if (c > mx) mx = c;
        }
        if (MODE == 4) {   /* one extra Jacobi parse of the mismatched segments, same cand */
            static St ent2[MAXSEG];
            int32_t j = -1;
            const St init0 = {M_S, 1, 32, 0};
            for (uint32_t k = 1; k < nseg; k++) {
                if (lanes[k - 1].found) j = (int32_t)k - 1;
                ent2[k] = j >= 0 ? ff(lanes[j].exit, k * SEG, F.ip_limit) : ff(init0, k * SEG, F.ip_limit);
            }
            for (uint32_t k = 1; k < nseg; k++)
                if (!st_eq(entry[k], ent2[k])) { entry[k] = ent2[k]; lane_parse(&F, k, entry[k], &lanes[k]); stat_reparse++; }
        }
        if (MODE >= 1 && MODE <= 2) {
            int chain = 0, maxchain = 0;
            for (uint32_t k = 1; k < nseg; k++) {
                if (!st_eq(entry[k], lanes[k - 1].exit)) {
                    entry[k] = lanes[k - 1].exit;
                    if (MODE == 2) {   /* live I of the segments to the left */
                        memset(bm2, 0, sizeof bm2);
                        for (uint32_t q = 0; q < k; q++) { bm2[q] |= lanes[q].own; if (lanes[q].flag_left && q) bm2[q - 1] |= 1ull << 63; }
                        for (uint32_t q = k; q < 1024; q++) bm2[q] = bm[q];
                        F.iprev = bm2;
                    }
                    lane_parse(&F, k, entry[k], &lanes[k]);
                    F.iprev = bm;
                    chain++; stat_reparse++;
                    if (chain > maxchain) maxchain = chain;
                } else chain = 0;
            }
            stat_chain += maxchain;
        }
        if (TRACE) {
            static St pex[MAXSEG]; static uint64_t pown[MAXSEG]; static St pent[MAXSEG];
            int ch = 0, che = 0;
            for (uint32_t k = 0; k < nseg; k++) {
                if (it > 0 && (!st_eq(pex[k], lanes[k].exit) || pown[k] != lanes[k].own)) ch++;
                if (it > 0 && !st_eq(pent[k], entry[k])) che++;
                pex[k] = lanes[k].exit; pown[k] = lanes[k].own; pent[k] = entry[k];
            }
            int bad = 0; for (uint32_t k = 1; k < nseg; k++) if (!st_eq(entry[k], lanes[k-1].exit)) bad++;
            /* first inconsistent segment */
            int front = -1; for (uint32_t k = 1; k < nseg; k++) if (!st_eq(entry[k], lanes[k-1].exit)) { front = k; break; }
            fprintf(stderr, "  it %d changed %d entry-changed %d entry-mismatch %d front %d\n", it, ch, che, bad, front);
        }
        memset(bm2, 0, sizeof bm2);
        for (uint32_t k = 0; k < nseg; k++) {
            bm2[k] |= lanes[k].own;
            if (lanes[k].flag_left && k) bm2[k - 1] |= 1ull << 63;
        }
        int ok = memcmp(bm, bm2, nseg * 8) == 0;
        for (uint32_t k = 0; k < nseg; k++) if (lanes[k].aborted) { ok = 0; lanes[k].exit = ff(entry[k], (k + 1) * SEG, F.ip_limit); lanes[k].found = 0; }
        for (uint32_t k = 1; k < nseg && ok; k++) ok = st_eq(entry[k], lanes[k - 1].exit);
        if (ok) break;
        if (it == MAXIT - 1) return -1;
        memcpy(bm, bm2, sizeof bm);
        int32_t j = -1;
        for (uint32_t k = 1; k < nseg; k++) {
            if (lanes[k - 1].found) j = (int32_t)k - 1;
            entry[k] = j >= 0 ? ff(lanes[j].exit, k * SEG, F.ip_limit) : ff(init, k * SEG, F.ip_limit);
        }
    }
    /* output */
    St fin = init;
    for (uint32_t k = 0; k < nseg; k++) {
        for (int i = 0; i < lanes[k].nm; i++) {
            const Match *m = &lanes[k].m[i];
            if (m->base > m->ne) op = emit_literal(op, in + m->ne, m->base - m->ne);
            op = emit_copy(op, m->off, m->len);
        }
        fin = lanes[k].exit;
    }
    if (fin.mode != M_T) { fprintf(stderr, "parse did not terminate\n"); exit(3); }
    if (fin.ne < n) op = emit_literal(op, in + fin.ne, n - fin.ne);
    return op - out;
}

static uint64_t mix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; }

static size_t make_page(const char *kind, uint8_t *p, size_t target, uint64_t seed)
{
    size_t o = 0; uint64_t i = 0;
    while (o < target + 600) {
        const uint64_t r = mix(i * 0x9E3779B97F4A7C15ull + seed);
        if (!strcmp(kind, "ts")) { uint64_t v = 1700000000000ull + i + r % 1000; memcpy(p + o, &v, 8); o += 8; }
        else if (!strcmp(kind, "price")) { double d = (double)(r >> 11) * (1.0 / 9007199254740992.0) * 1000.0; memcpy(p + o, &d, 8); o += 8; }
        else if (!strcmp(kind, "user_id")) { uint32_t v = (uint32_t)(r & 0xFFFFF); memcpy(p + o, &v, 4); o += 4; }
        else if (!strcmp(kind, "random")) { memcpy(p + o, &r, 8); o += 8; }
        else if (!strcmp(kind, "zeros")) { p[o++] = 0; }
        else if (!strcmp(kind, "key16")) {
            static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
            uint64_t k = mix(0xA5A5 + r % 10000); uint32_t len = 16; memcpy(p + o, &len, 4); o += 4;
            for (int j = 0; j < 16; j++) p[o++] = (uint8_t)A[(k >> (j * 3 % 58)) % 62];
        } else if (!strcmp(kind, "json")) {
            char buf[256];
            int n = snprintf(buf, sizeof buf, "{\"id\":%llu,\"event\":\"%s\",\"value\":%u,\"tags\":[\"a%u\",\"b%u\"]}",
                             (unsigned long long)i, (r & 1) ? "click" : "view", (unsigned)(r >> 40) % 100000,
                             (unsigned)(r >> 20) % 50, (unsigned)(r >> 30) % 7);
            uint32_t len = (uint32_t)n; memcpy(p + o, &len, 4); o += 4; memcpy(p + o, buf, n); o += n;
        } else if (!strcmp(kind, "defl")) { p[o++] = (uint8_t)((r & 3) ? 0xFF : (r >> 8)); }
        else if (!strcmp(kind, "mixed")) {   /* stretches of random, zeros and repeats */
            uint32_t typ = (uint32_t)((i / 700) % 3);
            p[o++] = typ == 0 ? (uint8_t)r : typ == 1 ? 0 : (uint8_t)("abcdefg"[i % 7]);
        } else if (!strcmp(kind, "sparse")) {   /* random with rare short repeats */
            if ((r & 255) == 0 && o >= 64) { memcpy(p + o, p + o - 37, 6); o += 6; }
            else p[o++] = (uint8_t)(r >> 16);
        } else { fprintf(stderr, "kind?\n"); exit(2); }
        i++;
    }
    return target;
}

static int file_mode(const char *path)
{
    FILE *f = fopen(path, "rb");
    if (!f) return 2;
    static uint8_t buf[1 << 28], o1[80000], o2[80000];
    uint64_t len; int bad = 0; long frags = 0, hist[70] = {0}, fail = 0; double seqcost = 0;
    int pg = 0;
    while (fread(&len, 8, 1, f) == 1) {
        if (len > sizeof buf || fread(buf, 1, len, f) != len) return 2;
        long pf = 0, pr = 0, pmax = 0; uint64_t c0 = stat_cost;
        for (uint64_t pos = 0; pos < len; pos += 65536) {
            uint32_t n = (uint32_t)(len - pos < 65536 ? len - pos : 65536);
            int64_t L1 = kpwo_snappy_compress(buf + pos, n, o1, sizeof o1);
            int pre = 1; { uint32_t v = n; while (v >= 0x80) { v >>= 7; pre++; } }
            int r; long L2 = seg_fragment(buf + pos, n, o2, &r);
            frags++; pf++;
            if (L2 < 0) { fail++; hist[MAXIT]++; continue; }
            if (L2 != L1 - pre || memcmp(o1 + pre, o2, L2)) bad++;
            hist[r]++; pr += r; if (r > pmax) pmax = r;
            seqcost += n;
        }
        printf("page %3d len %9llu frags %5ld rounds avg %5.2f max %2ld  cost/frag %.0f\n", pg++, (unsigned long long)len, pf, pf ? (double)pr / pf : 0, pmax, pf ? (double)(stat_cost - c0) / pf : 0);
    }
    printf("frags %ld mismatches %d nonconverged %ld; rounds histogram:", frags, bad, fail);
    for (int i = 0; i <= MAXIT; i++) if (hist[i]) printf(" %d:%ld", i, hist[i]);
    if (GPUF == 2) printf("\nlive lookups %llu, linked %.4f, chain steps per linked %.2f", (unsigned long long)st_live, st_live ? (double)st_linked / st_live : 0.0, st_linked ? (double)st_steps / st_linked : 0.0);
    printf("\ncost/frag %.1f reparses/frag %.1f maxchain-sum/frag %.1f\n", (double)stat_cost / frags, (double)stat_reparse/frags, (double)stat_chain/frags);
    return bad != 0;
}

int main(int argc, char **argv)
{
    if (getenv("HOPCAP")) HOPCAP = atoi(getenv("HOPCAP"));
    if (getenv("MODE")) MODE = atoi(getenv("MODE")); if (getenv("TRACE")) TRACE = atoi(getenv("TRACE")); if (getenv("GPUF")) GPUF = atoi(getenv("GPUF"));
    if (getenv("CHAINCAP")) CHAINCAP = atoi(getenv("CHAINCAP"));
    if (getenv("LIVE_D")) LIVE_D = atoi(getenv("LIVE_D"));
    if (argc > 2 && !strcmp(argv[1], "-f")) return file_mode(argv[2]);
    const char *kinds[] = {"ts", "price", "user_id", "random", "zeros", "key16", "json", "defl", "mixed", "sparse"};
    static uint8_t page[65536 + 4096], o1[200000], o2[200000];
    const uint32_t sizes[] = {65536, 65536, 40000, 5000, 300, 16, 15, 14};
    int bad = 0;
    for (unsigned kk = 0; kk < sizeof kinds / sizeof *kinds; kk++) {
        int maxr = 0; double sumr = 0; int cnt = 0;
        stat_lookups = stat_hops = 0;
        for (unsigned si = 0; si < sizeof sizes / sizeof *sizes; si++) {
            for (uint64_t seed = 1; seed <= (argc > 1 ? (uint64_t)atoi(argv[1]) : 3); seed++) {
                const uint32_t n = sizes[si];
                make_page(kinds[kk], page, n, seed * 1000 + si);
                /* oracle: strip the varint length prefix */
                int64_t L1 = kpwo_snappy_compress(page, n, o1, sizeof o1);
                int pre = 1; { uint32_t v = n; while (v >= 0x80) { v >>= 7; pre++; } }
                int r;
                long L2 = seg_fragment(page, n, o2, &r);
                if (L2 < 0) { printf("%-8s n=%u seed=%llu: no convergence\n", kinds[kk], n, (unsigned long long)seed); bad++; continue; }
                if (L2 != L1 - pre || memcmp(o1 + pre, o2, L2)) {
                    printf("%-8s n=%u seed=%llu: MISMATCH len %ld vs %lld\n", kinds[kk], n, (unsigned long long)seed, L2, (long long)(L1 - pre));
                    bad++;
                }
                if (r > maxr) maxr = r;
                sumr += r; cnt++;
            }
        }
        printf("%-8s rounds avg %.2f max %d  hops/lookup %.3f\n", kinds[kk], sumr / cnt, maxr,
               stat_lookups ? (double)stat_hops / stat_lookups : 0.0);
    }
    printf(bad ? "FAIL %d\n" : "ALL OK\n", bad);
    return bad != 0;
}
