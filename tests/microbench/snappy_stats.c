// snappy_stats.c — test-infrastructure tool: per-page statistics of the Snappy 1.1.2
// fragment loop (same algorithm as oracle/oracle_snappy.c, restated with counters) over a
// page dump written by tests/microbench/dump_pages.py.  Used to decide where K7's time goes:
// literal-search probes, copies, match-loop continuations, matched/literal bytes.
//   gcc -O2 -o build/snappy_stats snappy_stats.c && build/snappy_stats pages.bin
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ld64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

typedef struct { uint64_t probes, copies, cont, lit_bytes, lit_runs, match_bytes, long_lit, far_cand, frags, bytes; } st_t;

static void frag(const uint8_t *in, uint32_t n, uint16_t *table, int shift, st_t *S)
{
    const uint8_t *ip = in, *ip_end = in + n, *next_emit = in;
    S->frags++; S->bytes += n;
    if (n < 15) goto rem;
    const uint8_t *ip_limit = in + n - 15;
    uint32_t next_hash = (ld32(++ip) * 0x1e35a7bdu) >> shift;
    for (;;) {
        uint32_t skip = 32;
        const uint8_t *next_ip = ip, *cand;
        do {
            ip = next_ip;
            uint32_t h = next_hash;
            next_ip = ip + (skip++ >> 5);
            if (next_ip > ip_limit) goto rem;
            next_hash = (ld32(next_ip) * 0x1e35a7bdu) >> shift;
            cand = in + table[h];
            table[h] = (uint16_t)(ip - in);
            S->probes++;
        } while (ld32(ip) != ld32(cand));
        if (ip > next_emit) { S->lit_runs++; S->lit_bytes += ip - next_emit; if (ip - next_emit > 64) S->long_lit++; }
        uint64_t ib;
        uint32_t cb;
        int first = 1;
        do {
            if (!first) S->cont++;
            first = 0;
            const uint8_t *b = ip;
            uint32_t m = 4;
            while (ip + m < ip_end && cand[m] == ip[m]) m++;
            if (b - cand > 256) S->far_cand++;
            ip += m; S->copies++; S->match_bytes += m;
            next_emit = ip;
            if (ip >= ip_limit) goto rem;
            ib = ld64(ip - 1);
            table[(((uint32_t)ib) * 0x1e35a7bdu) >> shift] = (uint16_t)(ip - in - 1);
            uint32_t ch = (((uint32_t)(ib >> 8)) * 0x1e35a7bdu) >> shift;
            cand = in + table[ch];
            cb = ld32(cand);
            table[ch] = (uint16_t)(ip - in);
        } while ((uint32_t)(ib >> 8) == cb);
        next_hash = (((uint32_t)(ib >> 16)) * 0x1e35a7bdu) >> shift;
        ++ip;
    }
rem:
    if (next_emit < ip_end) { S->lit_runs++; S->lit_bytes += ip_end - next_emit; }
}

int main(int argc, char **argv)
{
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    static uint16_t table[1 << 14];
    uint64_t len;
    int pg = 0;
    st_t T = {0};
    while (fread(&len, 8, 1, f) == 1) {
        uint8_t *buf = malloc(len + 16);
        if (fread(buf, 1, len, f) != len) return 2;
        st_t S = {0};
        for (uint64_t pos = 0; pos < len; pos += 65536) {
            uint32_t n = (uint32_t)((len - pos) < 65536 ? (len - pos) : 65536);
            uint32_t ts = 256;
            int lg = 8;
            while (ts < (1u << 14) && ts < n) { ts <<= 1; lg++; }
            memset(table, 0, ts * 2);
            frag(buf + pos, n, table, 32 - lg, &S);
        }
        printf("page %2d %10llu B  probes/KB %6.1f copies/KB %6.1f cont %5.1f%% litB %5.1f%% runs/KB %5.1f longlit %llu mlen %5.1f far %4.1f%%\n", pg,
               (unsigned long long)len, S.probes * 1024.0 / len, S.copies * 1024.0 / len, 100.0 * S.cont / (S.copies + 1),
               100.0 * S.lit_bytes / len, S.lit_runs * 1024.0 / len, (unsigned long long)S.long_lit,
               (double)S.match_bytes / (S.copies + 1), 100.0 * S.far_cand / (S.copies + 1));
        T.probes += S.probes; T.copies += S.copies; T.cont += S.cont; T.lit_bytes += S.lit_bytes; T.bytes += len;
        T.lit_runs += S.lit_runs; T.match_bytes += S.match_bytes;
        free(buf);
        pg++;
    }
    printf("TOTAL %llu B probes/KB %.1f copies/KB %.1f cont %.1f%% litB %.1f%% runs/KB %.1f mlen %.1f\n", (unsigned long long)T.bytes,
           T.probes * 1024.0 / T.bytes, T.copies * 1024.0 / T.bytes, 100.0 * T.cont / (T.copies + 1), 100.0 * T.lit_bytes / T.bytes,
           T.lit_runs * 1024.0 / T.bytes, (double)T.match_bytes / (T.copies + 1));
    return 0;
}
