/*
 * deflate_seg_proto.c — test infrastructure: CPU model of a segment-parallel lazy parse for
 * K7' (zlib 1.2.11 level-6 deflate_slow, csrc/k_deflate.hip).
 *
 * At level 6 every position is inserted into the hash chains whatever the parse does, so the
 * longest match at each position (chain 128, or 32 after a match >= good_length) is a pure
 * function of the position: k_dfl_prev / k_dfl_match precompute them.  What is left sequential
 * is deflate_slow's loop, a small state machine over positions: at each loop top p the state is
 * (p, match_length, match_start, match_available), and a step emits at most one symbol (a literal
 * or the previous match) and moves p by 1 or to the end of the match.  The window slides only
 * decide which blocks may be stored; block flushes do not change the parse.
 *
 * Segment-parallel: cut the positions into segments of S; lane k parses the loop tops in
 * [kS, (k+1)S) from an entry state (round 0: a fresh state at kS), its exit = the first loop top
 * >= (k+1)S.  Rounds (Jacobi) set entry(k+1) = exit(k) until every entry equals its left
 * neighbour's exit; the symbols are then the sequential parse's (induction over segments).
 * This model checks that on dumped pages (tests/microbench/dump_any.py format) against the
 * sequential loop over the same precomputed matches, and reports the rounds.
 *   gcc -O2 deflate_seg_proto.c -o /tmp/dsp && /tmp/dsp pages.bin [S]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WSIZE 32768u
#define MIN_MATCH 3u
#define MAX_MATCH 258u
#define MAX_DIST (WSIZE - (MAX_MATCH + MIN_MATCH + 1))
#define TOO_FAR 4096u
#define GOOD 8u
#define LAZY 16u
#define NICE 128u
#define CHAIN 128u

static uint32_t hash3(const uint8_t *b) { return (((uint32_t)b[0] << 10) ^ ((uint32_t)b[1] << 5) ^ b[2]) & 0x7fffu; }

/* pdist[q] = q - (previous position with the same hash), 0 when none within MAX_DIST or it is 0 */
static void prev_dist(const uint8_t *in, uint64_t n, uint16_t *pdist)
{
    static int64_t head[1 << 15];
    for (int i = 0; i < (1 << 15); i++) head[i] = -1;
    for (uint64_t q = 0; q < n; q++) {
        pdist[q] = 0;
        if (n < 3 || q > n - 3) continue;
        const uint32_t h = hash3(in + q);
        const int64_t pq = head[h];
        if (pq > 0 && q - (uint64_t)pq <= MAX_DIST) pdist[q] = (uint16_t)(q - (uint64_t)pq);
        head[h] = (int64_t)q;
    }
}

static uint32_t mlen(const uint8_t *in, uint64_t c, uint64_t p, uint32_t maxlen)
{
    uint32_t l = 0;
    while (l < maxlen && in[c + l] == in[p + l]) l++;
    return l;
}

static void matches(const uint8_t *in, uint64_t n, const uint16_t *pdist, uint32_t *m128, uint32_t *m32)
{
    for (uint64_t p = 0; p < n; p++) {
        uint32_t r128 = 0, r32 = 0;
        const uint32_t d0 = (n >= 3 && p + 3 <= n) ? pdist[p] : 0;
        if (d0) {
            const uint64_t rem = n - p;
            const uint32_t maxlen = rem < MAX_MATCH ? (uint32_t)rem : MAX_MATCH;
            const uint32_t nice = rem < NICE ? (uint32_t)rem : NICE;
            const uint64_t limit = p > MAX_DIST ? p - MAX_DIST : 0;
            uint64_t c = p - d0;
            uint32_t best = MIN_MATCH - 1, bdist = 0, k = 0;
            int snap = 0;
            for (;;) {
                k++;
                const uint32_t l = mlen(in, c, p, maxlen);
                if (l > best) { best = l; bdist = (uint32_t)(p - c); if (l >= nice) break; }
                if (k == 32) { r32 = best > MIN_MATCH - 1 ? best | (bdist << 9) : 0; snap = 1; }
                if (k == CHAIN) break;
                const uint32_t d = pdist[c];
                if (!d) break;
                c -= d;
                if (c <= limit) break;
            }
            r128 = best > MIN_MATCH - 1 ? best | (bdist << 9) : 0;
            if (!snap) r32 = r128;
        }
        m128[p] = r128;
        m32[p] = r32;
    }
}

typedef struct { uint64_t p; uint32_t ml, ms, ma; } St;   /* loop-top state */

static int st_eq(St a, St b) { return a.p == b.p && a.ml == b.ml && a.ma == b.ma && (a.ml < MIN_MATCH || a.ms == b.ms); }

/* parse loop tops in [from state, until p >= end); symbols stored at sym[loop top] (1 + lc | dist << 8
   in the low bits... here: (dist << 9) | (lc << 1) | 1), cleared where no symbol */
static St parse(const uint8_t *in, uint64_t n, const uint16_t *pdist, const uint32_t *m128, const uint32_t *m32,
                St s, uint64_t begin, uint64_t end, uint64_t *sym)
{
    /* a segment owns the symbol slots [begin, end): the ones before its entry (inside the
       previous segment's last match) and the ones its matches jump over hold no symbol */
    for (uint64_t q = begin; q < s.p && q < end; q++) sym[q] = 0;
    uint64_t p = s.p;
    uint32_t match_length = s.ml, match_start = s.ms, match_available = s.ma;
    while (p < end && p < n) {
        uint64_t hash_head = 0;
        if (n - p >= MIN_MATCH && pdist[p]) hash_head = p - pdist[p];
        const uint32_t prev_length = match_length, prev_match = match_start;
        match_length = MIN_MATCH - 1;
        if (hash_head != 0 && prev_length < LAZY) {
            const uint32_t r = prev_length >= GOOD ? m32[p] : m128[p];
            const uint32_t rl = r & 0x1ff;
            if (r && rl > prev_length) { match_length = rl; match_start = (uint32_t)(p - (r >> 9)); }
            else match_length = prev_length;
            if (match_length == MIN_MATCH && p - match_start > TOO_FAR) match_length = MIN_MATCH - 1;
        }
        if (prev_length >= MIN_MATCH && match_length <= prev_length) {
            sym[p] = ((uint64_t)(p - 1 - prev_match) << 9) | ((uint64_t)(prev_length - MIN_MATCH) << 1) | 1;
            for (uint64_t q = p + 1; q < p + prev_length - 1 && q < end; q++) sym[q] = 0;
            p += prev_length - 1;
            match_available = 0;
            match_length = MIN_MATCH - 1;
        } else if (match_available) {
            sym[p] = ((uint64_t)in[p - 1] << 1) | 1;
            p++;
        } else {
            sym[p] = 0;
            match_available = 1;
            p++;
        }
    }
    St e = {p, match_length, match_length >= MIN_MATCH ? match_start : 0, match_available};
    return e;
}

int main(int argc, char **argv)
{
    if (argc < 2) { fprintf(stderr, "usage: dsp pages.bin [segment]\n"); return 2; }
    const uint64_t S = argc > 2 ? (uint64_t)atoll(argv[2]) : 2048;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint64_t len;
    int pg = 0, bad = 0;
    long hist[200] = {0};
    while (fread(&len, 8, 1, f) == 1) {
        uint8_t *in = malloc(len + 1);
        if (fread(in, 1, len, f) != len) return 2;
        uint16_t *pdist = malloc((len + 1) * 2);
        uint32_t *m128 = malloc((len + 1) * 4), *m32 = malloc((len + 1) * 4);
        uint64_t *seq = calloc(len + 2, 8), *par = calloc(len + 2, 8);
        prev_dist(in, len, pdist);
        matches(in, len, pdist, m128, m32);
        const St fresh0 = {0, MIN_MATCH - 1, 0, 0};
        St fin = parse(in, len, pdist, m128, m32, fresh0, 0, len, seq);
        if (fin.ma) seq[len] = ((uint64_t)in[len - 1] << 1) | 1;   /* the final literal (loop top n) */
        const uint64_t nseg = len ? (len + S - 1) / S : 1;
        St *entry = malloc(nseg * sizeof(St)), *exitst = malloc(nseg * sizeof(St));
        for (uint64_t k = 0; k < nseg; k++) { St e = {k * S, MIN_MATCH - 1, 0, 0}; entry[k] = e; }
        int rounds = 0;
        char *dirty = malloc(nseg);
        memset(dirty, 1, nseg);
        for (;;) {
            rounds++;
            for (uint64_t k = 0; k < nseg; k++)
                if (dirty[k]) exitst[k] = parse(in, len, pdist, m128, m32, entry[k], k * S, (k + 1) * S, par);
            int changed = 0;
            memset(dirty, 0, nseg);
            for (uint64_t k = 1; k < nseg; k++)
                if (!st_eq(entry[k], exitst[k - 1])) { entry[k] = exitst[k - 1]; dirty[k] = 1; changed = 1; }
            if (!changed) break;
            if (rounds > 150) { fprintf(stderr, "page %d: no convergence\n", pg); break; }
        }
        if (exitst[nseg - 1].ma && len) par[len] = ((uint64_t)in[len - 1] << 1) | 1;
        /* symbols: only at loop tops a parse reached; the skipped positions inside matches are 0
           in both (each segment's parse clears what it jumps over) */
        uint64_t nsym = 0, mism = 0;
        for (uint64_t q = 0; q <= len; q++) {
            if (seq[q] != par[q]) mism++;
            nsym += seq[q] & 1;
        }
        if (mism) bad++;
        hist[rounds < 199 ? rounds : 199]++;
        printf("page %3d len %9llu segments %7llu rounds %3d symbols %9llu mismatching positions %llu\n", pg, (unsigned long long)len,
               (unsigned long long)nseg, rounds, (unsigned long long)nsym, (unsigned long long)mism);
        free(in); free(pdist); free(m128); free(m32); free(seq); free(par); free(entry); free(exitst); free(dirty);
        pg++;
    }
    printf("rounds histogram:");
    for (int i = 0; i < 200; i++) if (hist[i]) printf(" %d:%ld", i, hist[i]);
    printf("\n%s\n", bad ? "MISMATCH" : "ALL MATCH");
    return bad != 0;
}
