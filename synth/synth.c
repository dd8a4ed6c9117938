/*
 * synth.c — deterministic synthetic Kafka record values (proto2 wire bytes) for tests and
 * bench.py.  Stand-in for the reference's embedded-Kafka producer
 * (KafkaProtoParquetWriterTest.java:247-270): no broker runs here, records are generated
 * in memory, counter-based (record i depends only on (seed, i)) so any slice can be
 * produced in parallel and the CPU and GPU legs see identical bytes.
 *
 * Schemas:
 *   SAMPLE  : SampleMessage{required string query=1; required int64 timestamp=2;
 *             optional int32 page_number=3; optional int32 result_per_page=4}
 *             (src/test/resources/test-message.proto:5-10)
 *   REC8    : ts, user_id, status?, price, score?, key16, region?, flag?  (~62 B)
 *   HIGHCARD: ts, uuid (36 B), blob (JSON 64..512 B), code? (C4)
 *   WIDE    : ts + 199 optional columns at 30% nulls (C3)
 */
#include <stdint.h>
#include <string.h>

#define SYN_SAMPLE 0
#define SYN_REC8 1
#define SYN_HIGHCARD 2
#define SYN_WIDE 3

static inline uint64_t sm64(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
static inline uint64_t rnd(uint64_t seed, uint64_t i, uint64_t f) { return sm64(sm64(seed ^ (i * 0x100000001b3ull)) + f * 0x9e3779b97f4a7c15ull); }

typedef struct { uint8_t *p; uint64_t n; int dry; } out_t;
static inline void put(out_t *o, uint8_t b) { if (!o->dry) o->p[o->n] = b; o->n++; }
static inline void put_varint(out_t *o, uint64_t v) { while (v >= 0x80) { put(o, (uint8_t)(v | 0x80)); v >>= 7; } put(o, (uint8_t)v); }
static inline void put_tag(out_t *o, int f, int wt) { put_varint(o, ((uint64_t)f << 3) | (uint64_t)wt); }
static inline void put_fixed64(out_t *o, uint64_t v) { for (int i = 0; i < 8; i++) put(o, (uint8_t)(v >> (8 * i))); }
static inline void put_bytes(out_t *o, const uint8_t *s, uint64_t n) { if (!o->dry) memcpy(o->p + o->n, s, n); o->n += n; }

static const char ALNUM[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
static void alnum_from(uint64_t key, uint8_t *s, int n)
{
    uint64_t h = sm64(key);
    for (int i = 0; i < n; i++) { if ((i % 8) == 0 && i) h = sm64(h); s[i] = (uint8_t)ALNUM[(h >> (8 * (i % 8))) % 62]; }
}
static double u01(uint64_t r) { return ((double)(r >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

/* one code point -> UTF-8, valid scalar values only (no surrogates) */
static int utf8_cp(uint64_t r, uint8_t *s)
{
    uint32_t k = (uint32_t)(r % 100), cp;
    if (k < 40) cp = 0x20 + (uint32_t)((r >> 8) % 0x5f);
    else if (k < 65) cp = 0x80 + (uint32_t)((r >> 8) % (0x800 - 0x80));
    else if (k < 90) { cp = 0x800 + (uint32_t)((r >> 8) % (0x10000 - 0x800)); if (cp >= 0xD800 && cp < 0xE000) cp -= 0x800; }
    else cp = 0x10000 + (uint32_t)((r >> 8) % (0x110000 - 0x10000));
    if (cp < 0x80) { s[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { s[0] = (uint8_t)(0xC0 | (cp >> 6)); s[1] = (uint8_t)(0x80 | (cp & 63)); return 2; }
    if (cp < 0x10000) { s[0] = (uint8_t)(0xE0 | (cp >> 12)); s[1] = (uint8_t)(0x80 | ((cp >> 6) & 63)); s[2] = (uint8_t)(0x80 | (cp & 63)); return 3; }
    s[0] = (uint8_t)(0xF0 | (cp >> 18)); s[1] = (uint8_t)(0x80 | ((cp >> 12) & 63)); s[2] = (uint8_t)(0x80 | ((cp >> 6) & 63)); s[3] = (uint8_t)(0x80 | (cp & 63));
    return 4;
}

/* null_pct: SAMPLE uses it for its two optional fields (the reference test always sets them). */
static void gen_sample(out_t *o, uint64_t seed, uint64_t i, int null_pct)
{
    uint8_t s[256];
    int n = 0;
    for (int k = 0; k < 30; k++) n += utf8_cp(rnd(seed, i, 100 + k), s + n);
    put_tag(o, 1, 2); put_varint(o, (uint64_t)n); put_bytes(o, s, (uint64_t)n);
    put_tag(o, 2, 0); put_varint(o, 1700000000000ull + i);
    uint64_t r3 = rnd(seed, i, 3), r4 = rnd(seed, i, 4);
    if ((int)(r3 % 100) >= null_pct) { put_tag(o, 3, 0); put_varint(o, (uint64_t)(int64_t)(int32_t)(uint32_t)(r3 >> 32)); }
    if ((int)(r4 % 100) >= null_pct) { put_tag(o, 4, 0); put_varint(o, (uint64_t)(int64_t)(int32_t)(uint32_t)(r4 >> 32)); }
}

static void gen_rec8(out_t *o, uint64_t seed, uint64_t i)
{
    static const int32_t STATUS[5] = {200, 201, 301, 404, 500};
    uint8_t s[16];
    uint64_t r;
    r = rnd(seed, i, 1); put_tag(o, 1, 0); put_varint(o, 1700000000000ull + i + r % 1000);
    r = rnd(seed, i, 2); put_tag(o, 2, 0); put_varint(o, r & 0xFFFFF);
    r = rnd(seed, i, 3); if (r % 100 >= 10) { put_tag(o, 3, 0); put_varint(o, (uint64_t)STATUS[(r >> 32) % 5]); }
    r = rnd(seed, i, 4); { double d = u01(r) * 1000.0; uint64_t b; memcpy(&b, &d, 8); put_tag(o, 4, 1); put_fixed64(o, b); }
    r = rnd(seed, i, 5); if (r % 100 >= 20) { double d = ((double)((r >> 32) % 1024) + 0.5) / 8.0; uint64_t b; memcpy(&b, &d, 8); put_tag(o, 5, 1); put_fixed64(o, b); }
    r = rnd(seed, i, 6); alnum_from(0xA5A5000000000000ull + r % 10000, s, 16); put_tag(o, 6, 2); put_varint(o, 16); put_bytes(o, s, 16);
    r = rnd(seed, i, 7); if (r % 100 >= 30) { alnum_from(0x5A5A000000000000ull + (r >> 32) % 64, s, 16); put_tag(o, 7, 2); put_varint(o, 16); put_bytes(o, s, 16); }
    r = rnd(seed, i, 8); if (r % 100 >= 30) { put_tag(o, 8, 0); put_varint(o, (r >> 32) & 1); }
}

static void gen_highcard(out_t *o, uint64_t seed, uint64_t i)
{
    static const char HEX[] = "0123456789abcdef";
    uint8_t u[36], b[600];
    uint64_t r;
    r = rnd(seed, i, 1); put_tag(o, 1, 0); put_varint(o, 1700000000000ull + i + r % 1000);
    uint64_t a = rnd(seed, i, 2), c = rnd(seed, i, 3);
    for (int k = 0, h = 0; k < 36; k++) {
        if (k == 8 || k == 13 || k == 18 || k == 23) { u[k] = '-'; continue; }
        uint64_t src = h < 16 ? a : c;
        int nib = (int)((src >> (4 * (h % 16))) & 15);
        if (k == 14) nib = 4;               /* version 4 */
        if (k == 19) nib = 8 | (nib & 3);   /* variant */
        u[k] = (uint8_t)HEX[nib];
        h++;
    }
    put_tag(o, 2, 2); put_varint(o, 36); put_bytes(o, u, 36);
    /* templated JSON blob, 64..512 B, Snappy-friendly (~2-3x) */
    r = rnd(seed, i, 4);
    int target = 64 + (int)(r % 449);
    int n = 0;
    static const char *KEYS[8] = {"\"event\":", "\"user\":", "\"session\":", "\"page\":", "\"ref\":", "\"agent\":", "\"value\":", "\"tags\":"};
    b[n++] = '{';
    for (int k = 0; n < target - 2; k++) {
        const char *key = KEYS[k % 8];
        int kl = (int)strlen(key);
        for (int j = 0; j < kl && n < target - 2; j++) b[n++] = (uint8_t)key[j];
        uint64_t rv = rnd(seed, i, 10 + (uint64_t)k);
        int vl = 4 + (int)(rv % 12);
        if (n < target - 2) b[n++] = '"';
        uint8_t tmp[16];
        alnum_from((rv >> 20) % 256, tmp, vl); /* low-cardinality values: compressible */
        for (int j = 0; j < vl && n < target - 2; j++) b[n++] = tmp[j];
        if (n < target - 2) b[n++] = '"';
        if (n < target - 2) b[n++] = ',';
    }
    b[n++] = '}';
    put_tag(o, 3, 2); put_varint(o, (uint64_t)n); put_bytes(o, b, (uint64_t)n);
    r = rnd(seed, i, 5); if (r % 100 >= 10) { put_tag(o, 4, 0); put_varint(o, (uint64_t)(int64_t)(int32_t)((r >> 32) % 1000)); }
}

/* WIDE: field 1 ts required; fields 2..81 int64 counters (Zipf-ish small ints);
 * 82..141 doubles (1024 distinct); 142..200 strings 8..24 B with 8..64 distinct each.
 * All 199 optional columns are null 30% of the time. */
static void gen_wide(out_t *o, uint64_t seed, uint64_t i)
{
    uint8_t s[24];
    uint64_t r = rnd(seed, i, 1);
    put_tag(o, 1, 0); put_varint(o, 1700000000000ull + i + r % 1000);
    for (int f = 2; f <= 200; f++) {
        r = rnd(seed, i, (uint64_t)f);
        if (r % 100 < 30) continue;
        uint64_t q = r >> 32;
        if (f <= 81) {
            uint64_t z = q % 1000;  /* Zipf-ish: 1000/(z+1) */
            put_tag(o, f, 0); put_varint(o, 1000 / (z + 1));
        } else if (f <= 141) {
            double d = ((double)(q % 1024) - 300.25) * 0.125;
            uint64_t b; memcpy(&b, &d, 8);
            put_tag(o, f, 1); put_fixed64(o, b);
        } else {
            int card = 8 + (f * 7) % 57;
            int len = 8 + (f * 5) % 17;
            alnum_from(((uint64_t)f << 32) + q % (uint64_t)card, s, len);
            put_tag(o, f, 2); put_varint(o, (uint64_t)len); put_bytes(o, s, (uint64_t)len);
        }
    }
}

static void gen_one(int kind, out_t *o, uint64_t seed, uint64_t i, int param)
{
    switch (kind) {
    case SYN_SAMPLE: gen_sample(o, seed, i, param); break;
    case SYN_REC8: gen_rec8(o, seed, i); break;
    case SYN_HIGHCARD: gen_highcard(o, seed, i); break;
    default: gen_wide(o, seed, i); break;
    }
}

/* sizes[k] = wire size of record start+k */
int synth_sizes(int kind, uint64_t seed, uint64_t start, uint64_t n, int param, uint32_t *sizes)
{
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)n; k++) {
        out_t o = {0, 0, 1};
        gen_one(kind, &o, seed, start + (uint64_t)k, param);
        sizes[k] = (uint32_t)o.n;
    }
    return 0;
}

/* writes record start+k at out + offsets[k] - offsets[0] */
int synth_fill(int kind, uint64_t seed, uint64_t start, uint64_t n, int param, const uint64_t *offsets, uint8_t *out)
{
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)n; k++) {
        out_t o = {out + (offsets[k] - offsets[0]), 0, 0};
        gen_one(kind, &o, seed, start + (uint64_t)k, param);
    }
    return 0;
}
