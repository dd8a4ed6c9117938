/*
 * oracle_core.c — CPU ORACLE (test infrastructure only; see kpw_oracle.h header).
 *
 * A value-by-value restatement of the reference write path:
 *   KafkaProtoParquetWriter.WorkerThread.run  (KPW = src/main/java/ir/sahab/kafka/reader/
 *       KafkaProtoParquetWriter.java:253-292): parseFrom -> ParquetFile.write -> size check
 *   ParquetFile (PF = .../ParquetFile.java:36-83): ParquetWriter built with rowGroupSize,
 *       codec, OVERWRITE, pageSize, dictionary (PF:42-51), ProtoWriteSupport (PF:96-99)
 * and of the upstream parquet-mr 1.10.1 classes it delegates to (pinned by pom.xml:44-48,
 * not vendored; each function below names the class/method it restates):
 *   ProtoWriteSupport / ProtoSchemaConverter, InternalParquetRecordWriter,
 *   ColumnWriteStoreV1 / ColumnWriterV1, FallbackValuesWriter, Plain*DictionaryValuesWriter,
 *   PlainValuesWriter, BooleanPlainValuesWriter, RunLengthBitPackingHybridEncoder,
 *   Int/Long/Float/Double/Boolean/BinaryStatistics, ColumnChunkPageWriteStore,
 *   ParquetFileWriter, ParquetMetadataConverter (Thrift compact via parquet-format).
 * Proto decoding restates protobuf-java CodedInputStream + the generated parse loop
 * (src/test/java/ir/sahab/kafka/test/proto/TestMessage.java:85-139, isInitialized :263-278).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "kpw_oracle.h"

/* ------------------------------------------------------------------ utilities */

static void *xmalloc(size_t n) { void *p = malloc(n ? n : 1); if (!p) { fprintf(stderr, "oracle OOM\n"); abort(); } return p; }
static void *xrealloc(void *p, size_t n) { p = realloc(p, n ? n : 1); if (!p) { fprintf(stderr, "oracle OOM\n"); abort(); } return p; }

typedef struct { uint8_t *p; uint64_t n, cap; } buf_t;

static void buf_reserve(buf_t *b, uint64_t extra)
{
    if (b->n + extra <= b->cap) return;
    uint64_t c = b->cap ? b->cap : 256;
    while (c < b->n + extra) c *= 2;
    b->p = (uint8_t *)xrealloc(b->p, c);
    b->cap = c;
}
static void buf_put(buf_t *b, const void *d, uint64_t n) { buf_reserve(b, n); if (n) memcpy(b->p + b->n, d, n); b->n += n; }
static void buf_u8(buf_t *b, uint8_t v) { buf_reserve(b, 1); b->p[b->n++] = v; }
static void buf_le32(buf_t *b, uint32_t v) { uint8_t t[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)}; buf_put(b, t, 4); }
static void buf_le64(buf_t *b, uint64_t v) { for (int i = 0; i < 8; i++) buf_u8(b, (uint8_t)(v >> (8 * i))); }
static void buf_free(buf_t *b) { free(b->p); b->p = NULL; b->n = b->cap = 0; }

/* BytesUtils.getWidthFromMaxInt: 32 - Integer.numberOfLeadingZeros(bound). */
static int width_from_max_int(int32_t bound)
{
    uint32_t u = (uint32_t)bound;
    int w = 0;
    while (u) { w++; u >>= 1; }
    return w;
}

/* Java (int)f / (long)f: NaN -> 0, saturate, truncate toward zero. */
static int32_t java_f2i(float f)
{
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}
static int64_t java_f2l(float f)
{
    if (f != f) return 0;
    if (f >= 9223372036854775808.0f) return INT64_MAX;
    if (f <= -9223372036854775808.0f) return INT64_MIN;
    return (int64_t)f;
}
static int64_t jadd64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

/* ------------------------------------------------------------------ schema */

typedef struct {
    char *name;
    int32_t field_number, proto_type, label;
    int phys;       /* kpw_physical_type */
    int optional;   /* max definition level 1 */
    int utf8;       /* ConvertedType UTF8 */
    int wire_type;  /* expected proto wire type */
} colinfo_t;

static int proto_to_phys(int pt, int *wt, int *utf8)
{
    *utf8 = 0;
    switch (pt) {
    case KPW_PT_DOUBLE: *wt = 1; return KPW_DOUBLE;
    case KPW_PT_FLOAT: *wt = 5; return KPW_FLOAT;
    case KPW_PT_INT64: case KPW_PT_UINT64: case KPW_PT_SINT64: *wt = 0; return KPW_INT64;
    case KPW_PT_FIXED64: case KPW_PT_SFIXED64: *wt = 1; return KPW_INT64;
    case KPW_PT_INT32: case KPW_PT_UINT32: case KPW_PT_SINT32: *wt = 0; return KPW_INT32;
    case KPW_PT_FIXED32: case KPW_PT_SFIXED32: *wt = 5; return KPW_INT32;
    case KPW_PT_BOOL: *wt = 0; return KPW_BOOLEAN;
    case KPW_PT_STRING: *wt = 2; *utf8 = 1; return KPW_BYTE_ARRAY;
    case KPW_PT_BYTES: *wt = 2; return KPW_BYTE_ARRAY;
    default: return -1;
    }
}

/* ------------------------------------------------------------------ proto decode
 * protobuf-java CodedInputStream semantics for the generated proto2 parse loop. */

typedef struct { int present; uint64_t bits; const uint8_t *ptr; uint32_t len; } pval_t;

typedef struct { const uint8_t *p; uint64_t pos, end; } pin_t;

/* readRawVarint64: at most 10 bytes else malformedVarint; truncated -> error. */
static int rd_varint64(pin_t *in, uint64_t *out)
{
    uint64_t r = 0;
    for (int i = 0; i < 10; i++) {
        if (in->pos >= in->end) return -1;
        uint8_t b = in->p[in->pos++];
        if (i < 9 || 1) r |= (uint64_t)(b & 0x7f) << (7 * i);
        if (!(b & 0x80)) { *out = r; return 0; }
    }
    return -1;
}
/* readRawVarint32: low 32 bits of a <=10 byte varint. */
static int rd_varint32(pin_t *in, uint32_t *out)
{
    uint64_t v;
    if (rd_varint64(in, &v)) return -1;
    *out = (uint32_t)v;
    return 0;
}

static int skip_field(pin_t *in, uint32_t tag, int depth);

/* UnknownFieldSet.mergeFieldFrom / CodedInputStream.skipField semantics.
 * Returns 0 ok, 1 = end-group seen (caller decides), -1 = error. */
static int skip_field(pin_t *in, uint32_t tag, int depth)
{
    uint32_t wt = tag & 7;
    uint64_t v;
    uint32_t len;
    switch (wt) {
    case 0: return rd_varint64(in, &v);
    case 1: if (in->end - in->pos < 8) return -1; in->pos += 8; return 0;
    case 2:
        if (rd_varint32(in, &len)) return -1;
        if ((int32_t)len < 0) return -1;
        if (in->end - in->pos < len) return -1;
        in->pos += len;
        return 0;
    case 3: {
        if (depth >= 100) return -1; /* recursion limit */
        for (;;) {
            if (in->pos >= in->end) return -1;
            uint32_t t;
            if (rd_varint32(in, &t)) return -1;
            if ((t >> 3) == 0) return -1;
            if ((t & 7) == 4) {
                if ((t >> 3) != (tag >> 3)) return -1; /* invalidEndTag */
                return 0;
            }
            int r = skip_field(in, t, depth + 1);
            if (r) return -1;
        }
    }
    case 4: return 1;
    case 5: if (in->end - in->pos < 4) return -1; in->pos += 4; return 0;
    default: return -1; /* invalidWireType */
    }
}

/* parseFrom(bytes): returns 0 or -1 (InvalidProtocolBufferException). */
static int proto_decode(const colinfo_t *cols, int ncols, const uint8_t *rec, uint64_t len, pval_t *vals)
{
    pin_t in = {rec, 0, len};
    for (int c = 0; c < ncols; c++) vals[c].present = 0;
    while (in.pos < in.end) {
        uint32_t tag;
        if (rd_varint32(&in, &tag)) return -1;
        if ((tag >> 3) == 0) return -1; /* invalidTag */
        uint32_t fno = tag >> 3, wt = tag & 7;
        int c;
        for (c = 0; c < ncols; c++)
            if ((uint32_t)cols[c].field_number == fno && (uint32_t)cols[c].wire_type == wt) break;
        if (c == ncols) {
            int r = skip_field(&in, tag, 0);
            if (r) return -1; /* error, or a top-level END_GROUP (checkLastTagWas fails) */
            continue;
        }
        pval_t *pv = &vals[c];
        uint64_t v;
        switch (wt) {
        case 0:
            if (rd_varint64(&in, &v)) return -1;
            switch (cols[c].proto_type) {
            case KPW_PT_INT32: case KPW_PT_UINT32: pv->bits = (uint32_t)v; break;
            case KPW_PT_SINT32: { uint32_t u = (uint32_t)v; pv->bits = (uint32_t)((u >> 1) ^ (0u - (u & 1))); break; }
            case KPW_PT_SINT64: pv->bits = (v >> 1) ^ (0ull - (v & 1)); break;
            case KPW_PT_BOOL: pv->bits = v != 0; break;
            default: pv->bits = v; break;
            }
            break;
        case 1:
            if (in.end - in.pos < 8) return -1;
            v = 0;
            for (int i = 0; i < 8; i++) v |= (uint64_t)in.p[in.pos + i] << (8 * i);
            in.pos += 8;
            pv->bits = v;
            break;
        case 5:
            if (in.end - in.pos < 4) return -1;
            v = 0;
            for (int i = 0; i < 4; i++) v |= (uint64_t)in.p[in.pos + i] << (8 * i);
            in.pos += 4;
            pv->bits = v;
            break;
        case 2: {
            uint32_t l;
            if (rd_varint32(&in, &l)) return -1;
            if ((int32_t)l < 0) return -1;
            if (in.end - in.pos < l) return -1;
            pv->ptr = in.p + in.pos;
            pv->len = l;
            in.pos += l;
            break;
        }
        default: return -1;
        }
        pv->present = 1;
    }
    for (int c = 0; c < ncols; c++)
        if (!cols[c].optional && !vals[c].present) return -1; /* missing required field */
    return 0;
}

/* Canonicalise floating bits the way the Java writers observe them:
 * Double.doubleToLongBits / Float.floatToIntBits (NaN -> canonical NaN). */
static uint64_t canon_bits(int phys, uint64_t bits)
{
    if (phys == KPW_DOUBLE) {
        if ((bits & 0x7ff0000000000000ull) == 0x7ff0000000000000ull && (bits & 0x000fffffffffffffull))
            return 0x7ff8000000000000ull;
    } else if (phys == KPW_FLOAT) {
        uint32_t b = (uint32_t)bits;
        if ((b & 0x7f800000u) == 0x7f800000u && (b & 0x007fffffu)) return 0x7fc00000u;
        return b;
    }
    return bits;
}

/* ------------------------------------------------------------------ RLE / bit-packing hybrid
 * RunLengthBitPackingHybridEncoder (parquet-column 1.10.1). */

typedef struct {
    int bw;
    buf_t out;
    uint32_t prev;
    uint32_t bufv[8];
    int nbuf;
    int32_t rc;
    int groups;
    int64_t hdr;
} rle_t;

static void rle_init(rle_t *r, int bw) { memset(r, 0, sizeof(*r)); r->bw = bw; r->hdr = -1; }
static void rle_reset(rle_t *r) { int bw = r->bw; buf_t o = r->out; o.n = 0; memset(r, 0, sizeof(*r)); r->out = o; r->bw = bw; r->hdr = -1; }

/* Packer.LITTLE_ENDIAN pack8Values: LSB-first. */
static void pack8(const uint32_t *v, int bw, uint8_t *out)
{
    memset(out, 0, (size_t)bw);
    for (int i = 0; i < 8; i++) {
        uint64_t x = bw == 32 ? v[i] : (v[i] & ((1u << bw) - 1));
        for (int b = 0; b < bw; b++)
            if ((x >> b) & 1) { int bit = i * bw + b; out[bit >> 3] |= (uint8_t)(1u << (bit & 7)); }
    }
}

static void rle_end_bp(rle_t *r)
{
    if (r->hdr == -1) return;
    r->out.p[r->hdr] = (uint8_t)((r->groups << 1) | 1);
    r->hdr = -1;
    r->groups = 0;
}

static void rle_write_or_append_bp(rle_t *r)
{
    if (r->groups >= 63) rle_end_bp(r);
    if (r->hdr == -1) { buf_u8(&r->out, 0); r->hdr = (int64_t)r->out.n - 1; }
    uint8_t pk[32];
    pack8(r->bufv, r->bw, pk);
    buf_put(&r->out, pk, (uint64_t)r->bw);
    r->nbuf = 0;
    r->rc = 0;
    ++r->groups;
}

static void write_uvarint(buf_t *b, uint32_t v)
{
    while (v & 0xFFFFFF80u) { buf_u8(b, (uint8_t)((v & 0x7F) | 0x80)); v >>= 7; }
    buf_u8(b, (uint8_t)(v & 0x7F));
}
static void write_uvarint64(buf_t *b, uint64_t v)
{
    while (v & ~0x7Full) { buf_u8(b, (uint8_t)((v & 0x7F) | 0x80)); v >>= 7; }
    buf_u8(b, (uint8_t)(v & 0x7F));
}

static void rle_write_rle_run(rle_t *r)
{
    rle_end_bp(r);
    write_uvarint(&r->out, (uint32_t)r->rc << 1);
    int nb = (r->bw + 7) / 8;
    for (int i = 0; i < nb; i++) buf_u8(&r->out, (uint8_t)(r->prev >> (8 * i)));
    r->rc = 0;
    r->nbuf = 0;
}

static void rle_write(rle_t *r, uint32_t v)
{
    if (v == r->prev) {
        ++r->rc;
        if (r->rc >= 8) return;
    } else {
        if (r->rc >= 8) rle_write_rle_run(r);
        r->rc = 1;
        r->prev = v;
    }
    r->bufv[r->nbuf++] = v;
    if (r->nbuf == 8) rle_write_or_append_bp(r);
}

static void rle_finish(rle_t *r) /* toBytes() */
{
    if (r->rc >= 8) {
        rle_write_rle_run(r);
    } else if (r->nbuf > 0) {
        for (int i = r->nbuf; i < 8; i++) r->bufv[i] = 0;
        rle_write_or_append_bp(r);
        rle_end_bp(r);
    } else {
        rle_end_bp(r);
    }
}

int64_t kpwo_rle_encode(const uint32_t *vals, uint64_t n, int bit_width, uint8_t *out, uint64_t cap)
{
    if (bit_width < 0 || bit_width > 32) return -1;
    rle_t r;
    rle_init(&r, bit_width);
    for (uint64_t i = 0; i < n; i++) rle_write(&r, vals[i]);
    rle_finish(&r);
    int64_t n_out = (int64_t)r.out.n;
    if ((uint64_t)n_out > cap) { buf_free(&r.out); return -1; }
    if (n_out) memcpy(out, r.out.p, (size_t)n_out);
    buf_free(&r.out);
    return n_out;
}

/* ------------------------------------------------------------------ DELTA_BINARY_PACKED
 * DeltaBinaryPackingValuesWriterForInteger / ForLong (parquet-column 1.10.1), config
 * blockSizeInValues 128, miniBlockNumInABlock 4 (32 values per miniblock).
 *   writeInteger/Long: the first value is kept aside (firstValue); every later value adds
 *     delta = v - previousValue (Java int/long wrapping) to deltaBlockBuffer and lowers
 *     minDeltaInCurrentBlock; a full block of 128 deltas is flushed.
 *   flushBlockBuffer: deltas -= minDelta (wrapping); zigzag varint(minDelta); bit width of
 *     each of the ceil(n/32) miniblocks present (32/64 - nlz(OR of its deltas)); ALL four
 *     width bytes are written from bitWidths[], which is never cleared: the widths of
 *     miniblocks a partial last block does not have are the previous block's.  Each present
 *     miniblock is packed as 4 pack8Values calls (LSB first, values masked to the width);
 *     the last miniblock's padding slots pack whatever deltaBlockBuffer still holds there
 *     (the previous block's min-reduced deltas, zeros in a fresh writer).
 *   getBytes: varint(128) varint(4) varint(totalValueCount) zigzag(firstValue) blocks.
 *   getBufferedSize = flushed block bytes (baos.size()); reset() keeps bitWidths and
 *     deltaBlockBuffer. */
typedef struct {
    int is_long;
    buf_t out;            /* baos: flushed blocks */
    int32_t total;        /* totalValueCount */
    uint64_t first, prev; /* firstValue, previousValue (int version: low 32 bits) */
    uint64_t dbuf[128];   /* deltaBlockBuffer */
    int nbuf;             /* deltaValuesToFlush */
    int64_t min;          /* minDeltaInCurrentBlock (int version: sign-extended int) */
    int bw[4];            /* bitWidths */
} deltaw_t;

static void delta_init(deltaw_t *d, int is_long) { memset(d, 0, sizeof(*d)); d->is_long = is_long; d->min = is_long ? INT64_MAX : INT32_MAX; }
static void delta_reset(deltaw_t *d) { d->total = 0; d->out.n = 0; d->nbuf = 0; d->min = d->is_long ? INT64_MAX : INT32_MAX; }
static void delta_free(deltaw_t *d) { buf_free(&d->out); }
static uint32_t zz32(int32_t v) { return ((uint32_t)v << 1) ^ (uint32_t)(v >> 31); }
static uint64_t zzl(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }

static void delta_flush_block(deltaw_t *d)
{
    const uint64_t wmask = d->is_long ? ~0ull : 0xffffffffull;
    for (int i = 0; i < d->nbuf; i++) d->dbuf[i] = (d->dbuf[i] - (uint64_t)d->min) & wmask;
    if (d->is_long) write_uvarint64(&d->out, zzl(d->min)); else write_uvarint(&d->out, zz32((int32_t)d->min));
    const int nmb = (d->nbuf + 31) / 32;   /* getMiniBlockCountToFlush */
    for (int m = 0; m < nmb; m++) {
        uint64_t mask = 0;
        const int e = (m + 1) * 32 < d->nbuf ? (m + 1) * 32 : d->nbuf;
        for (int i = m * 32; i < e; i++) mask |= d->dbuf[i];
        int w = 0;
        while (mask) { w++; mask >>= 1; }
        d->bw[m] = w;
    }
    for (int m = 0; m < 4; m++) buf_u8(&d->out, (uint8_t)d->bw[m]);
    for (int m = 0; m < nmb; m++) {
        const int w = d->bw[m];
        const uint64_t vm = w >= 64 ? ~0ull : ((1ull << w) - 1);
        uint8_t pk[256];
        memset(pk, 0, sizeof pk);
        for (int i = 0; i < 32; i++) {
            const uint64_t x = d->dbuf[m * 32 + i] & vm;
            for (int b = 0; b < w; b++)
                if ((x >> b) & 1) { const int bit = i * w + b; pk[bit >> 3] |= (uint8_t)(1u << (bit & 7)); }
        }
        buf_put(&d->out, pk, (uint64_t)(4 * w));
    }
    d->min = d->is_long ? INT64_MAX : INT32_MAX;
    d->nbuf = 0;
}

static void delta_write(deltaw_t *d, uint64_t v)
{
    if (!d->is_long) v = (uint32_t)v;
    d->total++;
    if (d->total == 1) { d->first = d->prev = v; return; }
    uint64_t delta;
    int64_t sd;
    if (d->is_long) { delta = v - d->prev; sd = (int64_t)delta; }
    else { delta = (uint32_t)((uint32_t)v - (uint32_t)d->prev); sd = (int32_t)(uint32_t)delta; }
    d->prev = v;
    d->dbuf[d->nbuf++] = delta;
    if (sd < d->min) d->min = sd;
    if (d->nbuf == 128) delta_flush_block(d);
}

static void delta_get_bytes(deltaw_t *d, buf_t *out)
{
    if (d->nbuf != 0) delta_flush_block(d);
    write_uvarint(out, 128);
    write_uvarint(out, 4);
    write_uvarint(out, (uint32_t)d->total);
    if (d->is_long) write_uvarint64(out, zzl((int64_t)d->first)); else write_uvarint(out, zz32((int32_t)(uint32_t)d->first));
    buf_put(out, d->out.p, d->out.n);
}

int64_t kpwo_delta_encode(const uint64_t *vals, uint64_t n, int is_long, uint8_t *out, uint64_t cap)
{
    deltaw_t d;
    delta_init(&d, is_long);
    for (uint64_t i = 0; i < n; i++) delta_write(&d, vals[i]);
    buf_t b = {0};
    delta_get_bytes(&d, &b);
    int64_t n_out = (int64_t)b.n;
    if ((uint64_t)n_out > cap) n_out = -1;
    else if (n_out) memcpy(out, b.p, (size_t)n_out);
    buf_free(&b);
    delta_free(&d);
    return n_out;
}

/* DeltaByteArrayWriter (prefix lengths: DeltaBinaryPackingValuesWriterForInteger; suffixes:
 * DeltaLengthByteArrayValuesWriter = lengths DELTA_BINARY_PACKED + concatenated bytes).
 * writeBytes: prefix = common leading bytes with the previous value; getBytes = prefix
 * lengths | suffix lengths | suffix bytes; reset() forgets the previous value. */
typedef struct { deltaw_t pre, len; buf_t sfx; buf_t prev; } dbaw_t;

static void dba_init(dbaw_t *w) { memset(w, 0, sizeof(*w)); delta_init(&w->pre, 0); delta_init(&w->len, 0); }
static void dba_free(dbaw_t *w) { delta_free(&w->pre); delta_free(&w->len); buf_free(&w->sfx); buf_free(&w->prev); }
static void dba_reset(dbaw_t *w) { delta_reset(&w->pre); delta_reset(&w->len); w->sfx.n = 0; w->prev.n = 0; }
static int64_t dba_buffered(const dbaw_t *w) { return (int64_t)(w->pre.out.n + w->len.out.n + w->sfx.n); }
static void dba_write(dbaw_t *w, const uint8_t *p, uint32_t n)
{
    uint32_t m = (uint32_t)w->prev.n < n ? (uint32_t)w->prev.n : n, i = 0;
    while (i < m && w->prev.p[i] == p[i]) i++;
    delta_write(&w->pre, i);
    delta_write(&w->len, n - i);
    buf_put(&w->sfx, p + i, n - i);
    w->prev.n = 0;
    buf_put(&w->prev, p, n);
}
static void dba_get_bytes(dbaw_t *w, buf_t *out)
{
    delta_get_bytes(&w->pre, out);
    delta_get_bytes(&w->len, out);
    buf_put(out, w->sfx.p, w->sfx.n);
}

/* ------------------------------------------------------------------ statistics
 * Int/Long/Float/Double/Boolean/BinaryStatistics with the 1.10 PrimitiveComparators:
 * signed for INT32/INT64, Boolean.compare, Float/Double.compare, unsigned lexicographic
 * for BINARY. */

typedef struct {
    int phys;
    int has;
    int64_t nulls;
    uint64_t min, max;     /* fixed-width canonical bits */
    buf_t bmin, bmax;      /* binary */
} stats_t;

static int java_double_compare(uint64_t a, uint64_t b)
{
    double x, y;
    memcpy(&x, &a, 8); memcpy(&y, &b, 8);
    if (x < y) return -1;
    if (x > y) return 1;
    int64_t la = (int64_t)a, lb = (int64_t)b; /* doubleToLongBits (already canonical) */
    return la == lb ? 0 : (la < lb ? -1 : 1);
}
static int java_float_compare(uint32_t a, uint32_t b)
{
    float x, y;
    memcpy(&x, &a, 4); memcpy(&y, &b, 4);
    if (x < y) return -1;
    if (x > y) return 1;
    int32_t ia = (int32_t)a, ib = (int32_t)b;
    return ia == ib ? 0 : (ia < ib ? -1 : 1);
}
static int bin_compare(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb)
{
    uint32_t m = la < lb ? la : lb;
    for (uint32_t i = 0; i < m; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return la == lb ? 0 : (la < lb ? -1 : 1);
}
static int fixed_compare(int phys, uint64_t a, uint64_t b)
{
    switch (phys) {
    case KPW_INT32: { int32_t x = (int32_t)(uint32_t)a, y = (int32_t)(uint32_t)b; return x < y ? -1 : x > y; }
    case KPW_INT64: { int64_t x = (int64_t)a, y = (int64_t)b; return x < y ? -1 : x > y; }
    case KPW_BOOLEAN: return (int)(a != 0) - (int)(b != 0);
    case KPW_DOUBLE: return java_double_compare(a, b);
    case KPW_FLOAT: return java_float_compare((uint32_t)a, (uint32_t)b);
    }
    return 0;
}

static void stats_reset(stats_t *s, int phys) { s->phys = phys; s->has = 0; s->nulls = 0; s->bmin.n = 0; s->bmax.n = 0; }
static void stats_update_fixed(stats_t *s, uint64_t v)
{
    if (!s->has) { s->min = s->max = v; s->has = 1; return; }
    if (fixed_compare(s->phys, s->min, v) > 0) s->min = v;
    if (fixed_compare(s->phys, s->max, v) < 0) s->max = v;
}
static void stats_update_bin(stats_t *s, const uint8_t *p, uint32_t n)
{
    if (!s->has) {
        s->bmin.n = 0; buf_put(&s->bmin, p, n);
        s->bmax.n = 0; buf_put(&s->bmax, p, n);
        s->has = 1;
        return;
    }
    if (bin_compare(s->bmin.p, (uint32_t)s->bmin.n, p, n) > 0) { s->bmin.n = 0; buf_put(&s->bmin, p, n); }
    if (bin_compare(s->bmax.p, (uint32_t)s->bmax.n, p, n) < 0) { s->bmax.n = 0; buf_put(&s->bmax, p, n); }
}
/* Statistics.mergeStatistics */
static void stats_merge(stats_t *dst, const stats_t *src)
{
    if (src->has) {
        if (dst->phys == KPW_BYTE_ARRAY) {
            stats_update_bin(dst, src->bmin.p, (uint32_t)src->bmin.n);
            stats_update_bin(dst, src->bmax.p, (uint32_t)src->bmax.n);
        } else {
            stats_update_fixed(dst, src->min);
            stats_update_fixed(dst, src->max);
        }
    }
    dst->nulls += src->nulls;
}
static void stats_copy(stats_t *dst, const stats_t *src)
{
    stats_reset(dst, src->phys);
    dst->has = src->has; dst->nulls = src->nulls; dst->min = src->min; dst->max = src->max;
    buf_put(&dst->bmin, src->bmin.p, src->bmin.n);
    buf_put(&dst->bmax, src->bmax.p, src->bmax.n);
}
static void stats_free(stats_t *s) { buf_free(&s->bmin); buf_free(&s->bmax); }
static int stats_empty(const stats_t *s) { return !s->has && s->nulls == 0; }

static void fixed_le_bytes(int phys, uint64_t v, buf_t *b)
{
    switch (phys) {
    case KPW_INT32: case KPW_FLOAT: buf_le32(b, (uint32_t)v); break;
    case KPW_INT64: case KPW_DOUBLE: buf_le64(b, v); break;
    case KPW_BOOLEAN: buf_u8(b, (uint8_t)(v != 0)); break;
    }
}

/* ------------------------------------------------------------------ Thrift compact writer */

typedef struct { buf_t *b; int16_t last[16]; int depth; } tc_t;

static void tc_varint(buf_t *b, uint64_t v) { while (v >= 0x80) { buf_u8(b, (uint8_t)(v | 0x80)); v >>= 7; } buf_u8(b, (uint8_t)v); }
static uint64_t zz64(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }
static void tc_field(tc_t *t, int16_t id, uint8_t type)
{
    int16_t delta = (int16_t)(id - t->last[t->depth]);
    if (delta > 0 && delta <= 15) buf_u8(t->b, (uint8_t)((delta << 4) | type));
    else { buf_u8(t->b, type); tc_varint(t->b, zz64(id)); }
    t->last[t->depth] = id;
}
static void tc_i32(tc_t *t, int16_t id, int32_t v) { tc_field(t, id, 5); tc_varint(t->b, zz64(v)); }
static void tc_i64(tc_t *t, int16_t id, int64_t v) { tc_field(t, id, 6); tc_varint(t->b, zz64(v)); }
static void tc_bin(tc_t *t, int16_t id, const void *p, uint64_t n) { tc_field(t, id, 8); tc_varint(t->b, n); buf_put(t->b, p, n); }
static void tc_struct_begin(tc_t *t, int16_t id) { tc_field(t, id, 12); t->depth++; t->last[t->depth] = 0; }
static void tc_struct_end(tc_t *t) { buf_u8(t->b, 0); t->depth--; }
static void tc_list_begin(tc_t *t, int16_t id, uint8_t etype, uint32_t n)
{
    tc_field(t, id, 9);
    if (n < 15) buf_u8(t->b, (uint8_t)((n << 4) | etype));
    else { buf_u8(t->b, (uint8_t)(0xF0 | etype)); tc_varint(t->b, n); }
}
static void tc_elem_struct_begin(tc_t *t) { t->depth++; t->last[t->depth] = 0; }

/* ParquetMetadataConverter.toParquetStatistics (1.10.1). */
static void tc_statistics(tc_t *t, int16_t id, const stats_t *s)
{
    buf_t mn = {0}, mx = {0};
    int write_vals = 0;
    if (s->has) {
        if (s->phys == KPW_BYTE_ARRAY) { buf_put(&mn, s->bmin.p, s->bmin.n); buf_put(&mx, s->bmax.p, s->bmax.n); }
        else { fixed_le_bytes(s->phys, s->min, &mn); fixed_le_bytes(s->phys, s->max, &mx); }
    }
    int smaller = !s->has || s->phys != KPW_BYTE_ARRAY || (mn.n + mx.n) < 4096;
    tc_struct_begin(t, id);
    if (!stats_empty(s) && smaller) {
        write_vals = s->has;
        int same = write_vals && mn.n == mx.n && (mn.n == 0 || memcmp(mn.p, mx.p, mn.n) == 0);
        int signed_order = s->phys != KPW_BYTE_ARRAY;
        if (write_vals && (signed_order || same)) { tc_bin(t, 1, mx.p, mx.n); tc_bin(t, 2, mn.p, mn.n); }
        tc_i64(t, 3, s->nulls);
        if (write_vals) { tc_bin(t, 5, mx.p, mx.n); tc_bin(t, 6, mn.p, mn.n); }
    }
    tc_struct_end(t);
    buf_free(&mn); buf_free(&mx);
}

/* ------------------------------------------------------------------ values writers */

/* Plain{Integer,Long,Float,Double,Binary}DictionaryValuesWriter (DictionaryValuesWriter).
 * Keys: fixed types by canonical bits (fastutil equality on floatToIntBits /
 * doubleToLongBits); binary by content.  Entry ids = insertion (first-occurrence) order. */
typedef struct {
    int phys;
    uint64_t *hkeys; int32_t *hids; uint64_t hcap, hsize;
    uint64_t *ekeys;                      /* fixed entries by id */
    uint64_t *eoff; uint32_t *elen;       /* binary entries by id (into arena) */
    buf_t arena;
    int32_t nent, ecap;
    int64_t dict_byte_size;
    int32_t last_used_size, last_used_byte_size;
    int32_t *enc; int64_t nenc, enccap;   /* encodedValues */
    int32_t max_bytes;
} dictw_t;

static uint64_t mix64(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; }
static uint64_t hash_bin(const uint8_t *p, uint32_t n) { uint64_t h = 1469598103934665603ull ^ n; for (uint32_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; } return mix64(h); }

static void dict_init(dictw_t *d, int phys, int32_t max_bytes)
{
    memset(d, 0, sizeof(*d));
    d->phys = phys;
    d->max_bytes = max_bytes;
    d->hcap = 1024;
    d->hkeys = (uint64_t *)xmalloc(d->hcap * 8);
    d->hids = (int32_t *)xmalloc(d->hcap * 4);
    for (uint64_t i = 0; i < d->hcap; i++) d->hids[i] = -1;
}
static void dict_clear_content(dictw_t *d)
{
    for (uint64_t i = 0; i < d->hcap; i++) d->hids[i] = -1;
    d->hsize = 0;
    d->nent = 0;
    d->arena.n = 0;
}
static void dict_free(dictw_t *d)
{
    free(d->hkeys); free(d->hids); free(d->ekeys); free(d->eoff); free(d->elen); free(d->enc); buf_free(&d->arena);
}
static int dict_key_eq(const dictw_t *d, int32_t id, uint64_t key, const uint8_t *p, uint32_t n)
{
    if (d->phys != KPW_BYTE_ARRAY) return d->ekeys[id] == key;
    return d->elen[id] == n && (n == 0 || memcmp(d->arena.p + d->eoff[id], p, n) == 0);
}
static uint64_t dict_hash_of(const dictw_t *d, int32_t id)
{
    if (d->phys != KPW_BYTE_ARRAY) return mix64(d->ekeys[id]);
    return hash_bin(d->arena.p + d->eoff[id], d->elen[id]);
}
static void dict_grow(dictw_t *d)
{
    uint64_t ncap = d->hcap * 2;
    int32_t *nids = (int32_t *)xmalloc(ncap * 4);
    for (uint64_t i = 0; i < ncap; i++) nids[i] = -1;
    for (uint64_t i = 0; i < d->hcap; i++) {
        if (d->hids[i] < 0) continue;
        uint64_t h = dict_hash_of(d, d->hids[i]) & (ncap - 1);
        while (nids[h] >= 0) h = (h + 1) & (ncap - 1);
        nids[h] = d->hids[i];
    }
    free(d->hids); free(d->hkeys);
    d->hids = nids;
    d->hkeys = (uint64_t *)xmalloc(ncap * 8);
    d->hcap = ncap;
}
/* returns id (assigning a new one on first occurrence) */
static int32_t dict_lookup_insert(dictw_t *d, uint64_t key, const uint8_t *p, uint32_t n, int *is_new)
{
    uint64_t h = (d->phys != KPW_BYTE_ARRAY ? mix64(key) : hash_bin(p, n)) & (d->hcap - 1);
    while (d->hids[h] >= 0) {
        if (dict_key_eq(d, d->hids[h], key, p, n)) { *is_new = 0; return d->hids[h]; }
        h = (h + 1) & (d->hcap - 1);
    }
    int32_t id = d->nent++;
    if (d->nent > d->ecap) {
        d->ecap = d->ecap ? d->ecap * 2 : 256;
        d->ekeys = (uint64_t *)xrealloc(d->ekeys, (size_t)d->ecap * 8);
        d->eoff = (uint64_t *)xrealloc(d->eoff, (size_t)d->ecap * 8);
        d->elen = (uint32_t *)xrealloc(d->elen, (size_t)d->ecap * 4);
    }
    if (d->phys == KPW_BYTE_ARRAY) { d->eoff[id] = d->arena.n; d->elen[id] = n; buf_put(&d->arena, p, n); }
    else d->ekeys[id] = key;
    d->hids[h] = id;
    d->hsize++;
    if (d->hsize * 2 > d->hcap) dict_grow(d);
    *is_new = 1;
    return id;
}
static int dict_entry_size(const dictw_t *d, uint32_t n)
{
    switch (d->phys) {
    case KPW_INT32: case KPW_FLOAT: return 4;
    case KPW_INT64: case KPW_DOUBLE: return 8;
    default: return 4 + (int)n;
    }
}
static void dict_write(dictw_t *d, uint64_t key, const uint8_t *p, uint32_t n)
{
    int is_new;
    int32_t id = dict_lookup_insert(d, key, p, n, &is_new);
    if (is_new) d->dict_byte_size += dict_entry_size(d, n);
    if (d->nenc == d->enccap) { d->enccap = d->enccap ? d->enccap * 2 : 1024; d->enc = (int32_t *)xrealloc(d->enc, (size_t)d->enccap * 4); }
    d->enc[d->nenc++] = id;
}
/* DictionaryValuesWriter.getBytes */
static void dict_get_bytes(dictw_t *d, buf_t *out)
{
    int bw = width_from_max_int(d->nent - 1);
    rle_t r;
    rle_init(&r, bw);
    for (int64_t i = 0; i < d->nenc; i++) rle_write(&r, (uint32_t)d->enc[i]);
    rle_finish(&r);
    buf_u8(out, (uint8_t)bw);
    buf_put(out, r.out.p, r.out.n);
    buf_free(&r.out);
    d->last_used_size = d->nent;
    d->last_used_byte_size = (int32_t)d->dict_byte_size;
}

typedef struct { buf_t b; } plainw_t;
static void plain_fixed(plainw_t *w, int phys, uint64_t v) { fixed_le_bytes(phys, v, &w->b); }
static void plain_bin(plainw_t *w, const uint8_t *p, uint32_t n) { buf_le32(&w->b, n); buf_put(&w->b, p, n); }

static void dict_entry_to_plain(const dictw_t *d, int32_t id, plainw_t *pw)
{
    if (d->phys == KPW_BYTE_ARRAY) plain_bin(pw, d->arena.p + d->eoff[id], d->elen[id]);
    else plain_fixed(pw, d->phys, d->ekeys[id]);
}

/* BooleanPlainValuesWriter -> ByteBitPackingValuesWriter(1, LITTLE_ENDIAN) */
typedef struct { buf_t b; int64_t count; } boolw_t;
static void bool_write(boolw_t *w, int v)
{
    if ((w->count & 7) == 0) buf_u8(&w->b, 0);
    if (v) w->b.p[w->b.n - 1] |= (uint8_t)(1u << (w->count & 7));
    w->count++;
}

/* The non-dictionary writer a column uses directly (dictionary off) or falls back to.
 *   v1 DefaultV1ValuesWriterFactory: PLAIN for every type (booleans: BooleanPlainValuesWriter).
 *   v2 DefaultV2ValuesWriterFactory: INT32/INT64 -> DeltaBinaryPackingValuesWriterFor{Integer,Long},
 *      BINARY -> DeltaByteArrayWriter, FLOAT/DOUBLE -> PlainValuesWriter,
 *      BOOLEAN -> RunLengthBitPackingHybridValuesWriter(1) (no dictionary). */
enum { PW_PLAIN = 0, PW_DELTA = 1, PW_DBA = 2 };

typedef struct {
    int kind;
    int phys;
    plainw_t plain;
    deltaw_t delta;
    dbaw_t dba;
} basew_t;

static void basew_init(basew_t *b, int phys, int v2)
{
    memset(b, 0, sizeof(*b));
    b->phys = phys;
    b->kind = PW_PLAIN;
    if (v2 && (phys == KPW_INT32 || phys == KPW_INT64)) { b->kind = PW_DELTA; delta_init(&b->delta, phys == KPW_INT64); }
    else if (v2 && phys == KPW_BYTE_ARRAY) { b->kind = PW_DBA; dba_init(&b->dba); }
}
static void basew_free(basew_t *b) { buf_free(&b->plain.b); delta_free(&b->delta); dba_free(&b->dba); }
static void basew_write_fixed(basew_t *b, uint64_t key)
{
    if (b->kind == PW_DELTA) delta_write(&b->delta, key); else plain_fixed(&b->plain, b->phys, key);
}
static void basew_write_bin(basew_t *b, const uint8_t *p, uint32_t n)
{
    if (b->kind == PW_DBA) dba_write(&b->dba, p, n); else plain_bin(&b->plain, p, n);
}
static int64_t basew_buffered(const basew_t *b)
{
    switch (b->kind) {
    case PW_DELTA: return (int64_t)b->delta.out.n;
    case PW_DBA: return dba_buffered(&b->dba);
    default: return (int64_t)b->plain.b.n;
    }
}
static int basew_page(basew_t *b, buf_t *out)
{
    switch (b->kind) {
    case PW_DELTA: delta_get_bytes(&b->delta, out); return KPW_ENC_DELTA_BINARY_PACKED;
    case PW_DBA: dba_get_bytes(&b->dba, out); return KPW_ENC_DELTA_BYTE_ARRAY;
    default: buf_put(out, b->plain.b.p, b->plain.b.n); return KPW_ENC_PLAIN;
    }
}
static void basew_reset(basew_t *b)
{
    switch (b->kind) {
    case PW_DELTA: delta_reset(&b->delta); break;
    case PW_DBA: dba_reset(&b->dba); break;
    default: b->plain.b.n = 0;
    }
}

/* fallBackAllValuesTo */
static void dict_fall_back_all(dictw_t *d, basew_t *bw)
{
    for (int64_t i = 0; i < d->nenc; i++) {
        const int32_t id = d->enc[i];
        if (d->phys == KPW_BYTE_ARRAY) basew_write_bin(bw, d->arena.p + d->eoff[id], d->elen[id]);
        else basew_write_fixed(bw, d->ekeys[id]);
    }
    if (d->last_used_size == 0) {
        dict_clear_content(d);
        d->dict_byte_size = 0;
        d->nenc = 0;
    }
}

/* FallbackValuesWriter state + its wrapped writers */
enum { DW_PLAIN = 0, DW_FALLBACK = 1, DW_BOOL = 2, DW_RLEBOOL = 3 };

typedef struct {
    int kind;
    int phys;
    int v2;
    /* fallback */
    dictw_t dict;
    basew_t base;        /* the direct writer (DW_PLAIN) or the fallback writer (DW_FALLBACK) */
    int fell_back, initial_used_and_had_dict, first_page;
    int64_t raw;
    /* bool */
    boolw_t bw;
    rle_t rb;            /* v2 booleans */
} dataw_t;

static void dataw_init(dataw_t *w, int phys, const kpw_props *pr)
{
    memset(w, 0, sizeof(*w));
    w->phys = phys;
    w->v2 = pr->writer_version == 2;
    if (phys == KPW_BOOLEAN) {
        w->kind = w->v2 ? DW_RLEBOOL : DW_BOOL;
        if (w->v2) rle_init(&w->rb, 1);
        return;
    }
    basew_init(&w->base, phys, w->v2);
    if (pr->enable_dictionary) { w->kind = DW_FALLBACK; dict_init(&w->dict, phys, pr->dictionary_page_size); w->first_page = 1; }
    else w->kind = DW_PLAIN;
}
static void dataw_free(dataw_t *w)
{
    if (w->kind == DW_FALLBACK) dict_free(&w->dict);
    basew_free(&w->base);
    buf_free(&w->bw.b);
    buf_free(&w->rb.out);
}
static int64_t dataw_buffered(const dataw_t *w)
{
    switch (w->kind) {
    case DW_BOOL: return (w->bw.count + 7) / 8;
    case DW_RLEBOOL: return (int64_t)w->rb.out.n;   /* RunLengthBitPackingHybridEncoder.getBufferedSize */
    case DW_FALLBACK: return w->raw;                 /* FallbackValuesWriter: rawDataByteSize */
    default: return basew_buffered(&w->base);
    }
}
static void dataw_fall_back(dataw_t *w) { w->fell_back = 1; dict_fall_back_all(&w->dict, &w->base); }

static void dataw_write(dataw_t *w, const pval_t *v)
{
    if (w->kind == DW_BOOL) { bool_write(&w->bw, v->bits != 0); return; }
    if (w->kind == DW_RLEBOOL) { rle_write(&w->rb, v->bits != 0); return; }
    int is_bin = w->phys == KPW_BYTE_ARRAY;
    uint64_t key = is_bin ? 0 : canon_bits(w->phys, v->bits);
    if (w->kind == DW_PLAIN) {
        if (is_bin) basew_write_bin(&w->base, v->ptr, v->len); else basew_write_fixed(&w->base, key);
        return;
    }
    w->raw += is_bin ? (int64_t)v->len + 4 : (w->phys == KPW_INT32 || w->phys == KPW_FLOAT ? 4 : 8);
    if (w->fell_back) {
        if (is_bin) basew_write_bin(&w->base, v->ptr, v->len); else basew_write_fixed(&w->base, key);
    } else {
        dict_write(&w->dict, key, v->ptr, v->len);
        /* checkFallback: shouldFallBack() */
        if (w->dict.dict_byte_size > w->dict.max_bytes || w->dict.nent > INT32_MAX - 1) dataw_fall_back(w);
    }
}

/* getBytes() then getEncoding() — ColumnWriterV1/V2.writePage evaluation order. */
static int dataw_page(dataw_t *w, buf_t *out)
{
    const int dict_enc = w->v2 ? KPW_ENC_RLE_DICTIONARY : KPW_ENC_PLAIN_DICTIONARY;
    switch (w->kind) {
    case DW_BOOL:
        buf_put(out, w->bw.b.p, w->bw.b.n);
        return KPW_ENC_PLAIN;
    case DW_RLEBOOL:   /* RunLengthBitPackingHybridValuesWriter.getBytes: 4-byte LE length + RLE */
        rle_finish(&w->rb);
        buf_le32(out, (uint32_t)w->rb.out.n);
        buf_put(out, w->rb.out.p, w->rb.out.n);
        return KPW_ENC_RLE;
    case DW_PLAIN:
        return basew_page(&w->base, out);
    }
    int enc;
    if (!w->fell_back && w->first_page) {
        buf_t tmp = {0};
        dict_get_bytes(&w->dict, &tmp);
        /* isCompressionSatisfying(rawSize, encodedSize) */
        if ((int64_t)tmp.n + w->dict.dict_byte_size < w->raw) {
            buf_put(out, tmp.p, tmp.n);
            buf_free(&tmp);
            enc = dict_enc;
            goto have_enc;
        }
        buf_free(&tmp);
        dataw_fall_back(w);
    }
    if (w->fell_back) enc = basew_page(&w->base, out);
    else { dict_get_bytes(&w->dict, out); enc = dict_enc; }
have_enc:
    if (!w->fell_back && !w->initial_used_and_had_dict) w->initial_used_and_had_dict = (enc == dict_enc);
    return enc;
}
static void dataw_reset(dataw_t *w)
{
    switch (w->kind) {
    case DW_BOOL: w->bw.b.n = 0; w->bw.count = 0; break;
    case DW_RLEBOOL: rle_reset(&w->rb); break;
    case DW_PLAIN: basew_reset(&w->base); break;
    default:
        w->raw = 0;
        w->first_page = 0;
        if (w->fell_back) basew_reset(&w->base); else w->dict.nenc = 0;
    }
}
/* toDictPageAndClose: returns 1 + page bytes/num entries if a dictionary page exists */
static int dataw_dict_page(dataw_t *w, buf_t *out, int32_t *nent)
{
    if (w->kind != DW_FALLBACK || !w->initial_used_and_had_dict) return 0;
    dictw_t *d = &w->dict;
    if (d->last_used_size <= 0) return 0;
    plainw_t pw = {{0}};
    for (int32_t i = 0; i < d->last_used_size; i++) dict_entry_to_plain(d, i, &pw);
    buf_put(out, pw.b.p, pw.b.n);
    buf_free(&pw.b);
    *nent = d->last_used_size;
    return 1;
}

/* ------------------------------------------------------------------ column writer + page store */

typedef struct { uint8_t v[8]; int n; } encset_t;
static void encset_add(encset_t *s, int e) { for (int i = 0; i < s->n; i++) if (s->v[i] == e) return; s->v[s->n++] = (uint8_t)e; }
typedef struct { int enc[8]; int cnt[8]; int n; } enccount_t;
static void enccount_add(enccount_t *s, int e) { for (int i = 0; i < s->n; i++) if (s->enc[i] == e) { s->cnt[i]++; return; } s->enc[s->n] = e; s->cnt[s->n++] = 1; }

typedef struct {
    const colinfo_t *ci;
    /* ColumnWriterV1 */
    rle_t dl;            /* RunLengthBitPackingHybridValuesWriter (optional columns) */
    dataw_t data;
    stats_t pstats;
    int32_t value_count, next_check;
    /* ColumnChunkPageWriter */
    buf_t pages;         /* headers + compressed bodies */
    int64_t uncomp_len, comp_len, total_values;
    stats_t tstats; int tstats_init;
    encset_t rl_encs, dl_encs;
    int *data_encs; int ndata_encs, data_encs_cap;
    int has_dict; buf_t dict_bytes; int32_t dict_uncomp, dict_nent;
    int64_t rows_written;  /* ColumnWriterV2.rowsWrittenSoFar */
} colw_t;

/* finished column chunk metadata kept for the footer */
typedef struct {
    int phys;
    int codec;
    int v2;                /* EncodingStats.usesV2Pages */
    encset_t encs;
    enccount_t dict_stats, data_stats;
    int64_t num_values, total_uncomp, total_comp, data_page_offset;
    stats_t stats;
} chunkmeta_t;

typedef struct { int64_t rows, total_bytes; chunkmeta_t *chunks; } rgmeta_t;

struct kpwo_writer {
    int ncols;
    colinfo_t *cols;
    char *message_name, *proto_class;
    kpw_props props;
    colw_t *cw;
    pval_t *vals;
    buf_t out;                 /* the file */
    int64_t record_count, next_mem_check, next_rg_size, last_rg_end;
    int64_t num_records;
    rgmeta_t *rgs; int nrgs, rgcap;
    int closed;
    uint8_t *ctmp; uint64_t ctmp_cap;
    /* ColumnWriteStoreV2 (writer_version 2): store-level page size checks per record */
    int v2;
    int64_t v2_rows, v2_next_check;
};

static void page_compress(kpwo_writer *w, const buf_t *in, buf_t *out)
{
    if (w->props.codec == KPW_SNAPPY) {
        if (in->n == 0) return; /* SnappyCompressor emits nothing for empty input */
        uint64_t need = kpwo_snappy_max_compressed_length(in->n);
        if (need > w->ctmp_cap) { w->ctmp = (uint8_t *)xrealloc(w->ctmp, need); w->ctmp_cap = need; }
        int64_t c = kpwo_snappy_compress(in->p, in->n, w->ctmp, w->ctmp_cap);
        buf_put(out, w->ctmp, (uint64_t)c);
    } else if (w->props.codec == KPW_GZIP) {
        /* GzipCodec without native hadoop: one java.util.zip.GZIPOutputStream member per page,
         * also for an empty page (oracle_deflate.c) */
        uint64_t need = kpwo_gzip_bound(in->n);
        if (need > w->ctmp_cap) { w->ctmp = (uint8_t *)xrealloc(w->ctmp, need); w->ctmp_cap = need; }
        int64_t c = kpwo_gzip_compress(in->p, in->n, w->ctmp, w->ctmp_cap);
        buf_put(out, w->ctmp, (uint64_t)c);
    } else {
        buf_put(out, in->p, in->n);
    }
}

static void colw_init(colw_t *c, const colinfo_t *ci, const kpw_props *pr)
{
    memset(c, 0, sizeof(*c));
    c->ci = ci;
    if (ci->optional) rle_init(&c->dl, 1);
    dataw_init(&c->data, ci->phys, pr);
    stats_reset(&c->pstats, ci->phys);
    stats_reset(&c->tstats, ci->phys);
    c->next_check = 100; /* props.getMinRowCountForPageSizeCheck() */
}
static void colw_free(colw_t *c)
{
    buf_free(&c->dl.out);
    dataw_free(&c->data);
    stats_free(&c->pstats);
    stats_free(&c->tstats);
    buf_free(&c->pages);
    buf_free(&c->dict_bytes);
    free(c->data_encs);
}

/* ColumnChunkPageWriter.writePage */
static void pagestore_write_page(kpwo_writer *w, colw_t *c, const buf_t *body, int32_t nvalues,
                                 int rl_enc, int dl_enc, int data_enc)
{
    buf_t comp = {0};
    page_compress(w, body, &comp);
    buf_t hdr = {0};
    tc_t t = {&hdr, {0}, 0};
    tc_i32(&t, 1, KPW_DATA_PAGE);
    tc_i32(&t, 2, (int32_t)body->n);
    tc_i32(&t, 3, (int32_t)comp.n);
    tc_struct_begin(&t, 5);
    tc_i32(&t, 1, nvalues);
    tc_i32(&t, 2, data_enc);
    tc_i32(&t, 3, dl_enc);
    tc_i32(&t, 4, rl_enc);
    if (!stats_empty(&c->pstats)) tc_statistics(&t, 5, &c->pstats);
    tc_struct_end(&t);
    buf_u8(&hdr, 0);
    c->uncomp_len += (int64_t)body->n;
    c->comp_len += (int64_t)comp.n;
    c->total_values += nvalues;
    if (!c->tstats_init) { stats_copy(&c->tstats, &c->pstats); c->tstats_init = 1; }
    else stats_merge(&c->tstats, &c->pstats);
    buf_put(&c->pages, hdr.p, hdr.n);
    buf_put(&c->pages, comp.p, comp.n);
    encset_add(&c->rl_encs, rl_enc);
    encset_add(&c->dl_encs, dl_enc);
    if (c->ndata_encs == c->data_encs_cap) { c->data_encs_cap = c->data_encs_cap ? c->data_encs_cap * 2 : 16; c->data_encs = (int *)xrealloc(c->data_encs, (size_t)c->data_encs_cap * sizeof(int)); }
    c->data_encs[c->ndata_encs++] = data_enc;
    buf_free(&hdr);
    buf_free(&comp);
}

/* ColumnChunkPageWriter.writePageV2: rl and dl stay uncompressed in front of the
 * compressed values; ParquetMetadataConverter.writeDataPageV2Header (is_compressed is
 * never set, so it is not serialised). */
static void pagestore_write_page_v2(kpwo_writer *w, colw_t *c, int32_t rows, int32_t nulls, int32_t nvalues,
                                    const buf_t *rl, const buf_t *dl, int data_enc, const buf_t *data)
{
    buf_t comp = {0};
    page_compress(w, data, &comp);
    const int32_t lv = (int32_t)(rl->n + dl->n);
    const int32_t uncomp = (int32_t)data->n + lv, compsz = (int32_t)comp.n + lv;
    buf_t hdr = {0};
    tc_t t = {&hdr, {0}, 0};
    tc_i32(&t, 1, KPW_DATA_PAGE_V2);
    tc_i32(&t, 2, uncomp);
    tc_i32(&t, 3, compsz);
    tc_struct_begin(&t, 8);
    tc_i32(&t, 1, nvalues);
    tc_i32(&t, 2, nulls);
    tc_i32(&t, 3, rows);
    tc_i32(&t, 4, data_enc);
    tc_i32(&t, 5, (int32_t)dl->n);
    tc_i32(&t, 6, (int32_t)rl->n);
    if (!stats_empty(&c->pstats)) tc_statistics(&t, 8, &c->pstats);
    tc_struct_end(&t);
    buf_u8(&hdr, 0);
    c->uncomp_len += uncomp;
    c->comp_len += compsz;
    c->total_values += nvalues;
    if (!c->tstats_init) { stats_copy(&c->tstats, &c->pstats); c->tstats_init = 1; }
    else stats_merge(&c->tstats, &c->pstats);
    buf_put(&c->pages, hdr.p, hdr.n);
    buf_put(&c->pages, rl->p, rl->n);
    buf_put(&c->pages, dl->p, dl->n);
    buf_put(&c->pages, comp.p, comp.n);
    if (c->ndata_encs == c->data_encs_cap) { c->data_encs_cap = c->data_encs_cap ? c->data_encs_cap * 2 : 16; c->data_encs = (int *)xrealloc(c->data_encs, (size_t)c->data_encs_cap * sizeof(int)); }
    c->data_encs[c->ndata_encs++] = data_enc;
    buf_free(&hdr);
    buf_free(&comp);
}

/* RunLengthBitPackingHybridEncoder(bitWidth 0).toBytes() after n writeInt(0): the level encoder
 * parquet-mr 1.10.1's ColumnWriterV2 builds for a max level of 0 (ParquetProperties
 * .newLevelEncoder: always an RLE encoder in v2, unlike v1's DevNullValuesWriter): nothing
 * for n = 0, one bit-packed run header (0x03) for n < 8, else varint(n << 1) of one RLE run. */
static void rle0_bytes(int32_t n, buf_t *out)
{
    rle_t r;
    rle_init(&r, 0);
    for (int32_t i = 0; i < n; i++) rle_write(&r, 0);
    rle_finish(&r);
    buf_put(out, r.out.p, r.out.n);
    buf_free(&r.out);
}

/* ColumnWriterV2.writePage(rowCount): dataColumn.getBytes()/getEncoding() first, then the
 * levels; RLE levels carry no length prefix in a v2 page.  Every column is top-level and not
 * repeated: the repetition levels are a width-0 stream, and so are the definition levels of
 * REQUIRED columns (rle0_bytes). */
static void colw_write_page_v2(kpwo_writer *w, colw_t *c, int64_t row_count)
{
    const int32_t page_rows = (int32_t)(row_count - c->rows_written);
    c->rows_written = row_count;
    buf_t data = {0}, dl = {0}, rl = {0};
    const int enc = dataw_page(&c->data, &data);
    rle0_bytes(c->value_count, &rl);
    if (c->ci->optional) {
        rle_finish(&c->dl);
        buf_put(&dl, c->dl.out.p, c->dl.out.n);
    } else {
        rle0_bytes(c->value_count, &dl);
    }
    pagestore_write_page_v2(w, c, page_rows, (int32_t)c->pstats.nulls, c->value_count, &rl, &dl, enc, &data);
    buf_free(&data);
    buf_free(&dl);
    buf_free(&rl);
    if (c->ci->optional) rle_reset(&c->dl);
    dataw_reset(&c->data);
    c->value_count = 0;
    stats_reset(&c->pstats, c->ci->phys);
}

/* ColumnWriterV1.writePage */
static void colw_write_page(kpwo_writer *w, colw_t *c)
{
    buf_t body = {0};
    int dl_enc = KPW_ENC_BIT_PACKED;
    if (c->ci->optional) {
        rle_finish(&c->dl);
        buf_le32(&body, (uint32_t)c->dl.out.n);
        buf_put(&body, c->dl.out.p, c->dl.out.n);
        dl_enc = KPW_ENC_RLE;
    }
    int data_enc = dataw_page(&c->data, &body);
    pagestore_write_page(w, c, &body, c->value_count, KPW_ENC_BIT_PACKED, dl_enc, data_enc);
    buf_free(&body);
    if (c->ci->optional) rle_reset(&c->dl);
    dataw_reset(&c->data);
    c->value_count = 0;
    stats_reset(&c->pstats, c->ci->phys);
}

static int64_t colw_mem(const colw_t *c) /* rl + dl + data buffered sizes */
{
    return (c->ci->optional ? (int64_t)c->dl.out.n : 0) + dataw_buffered(&c->data);
}

/* ColumnWriterV1.accountForValueWritten (estimateNextSizeCheck = true) */
static void colw_account(kpwo_writer *w, colw_t *c)
{
    ++c->value_count;
    if (c->value_count > c->next_check) {
        int64_t mem = colw_mem(c);
        if (mem > w->props.page_size) {
            c->next_check = c->value_count / 2;
            colw_write_page(w, c);
        } else {
            float t = (float)c->value_count * (float)w->props.page_size;
            t = t / (float)mem;
            float s = (float)c->value_count + t;
            c->next_check = java_f2i(s) / 2 + 1;
        }
    }
}

static void colw_write_value(kpwo_writer *w, colw_t *c, const pval_t *v)
{
    if (v->present) {
        if (c->ci->optional) rle_write(&c->dl, 1);
        dataw_write(&c->data, v);
        if (c->ci->phys == KPW_BYTE_ARRAY) stats_update_bin(&c->pstats, v->ptr, v->len);
        else stats_update_fixed(&c->pstats, canon_bits(c->ci->phys, v->bits));
    } else {
        rle_write(&c->dl, 0);
        c->pstats.nulls++;
    }
    if (w->v2) ++c->value_count;   /* ColumnWriterV2: page checks happen per record, in the store */
    else colw_account(w, c);
}

/* ColumnWriteStoreV2.sizeCheck (1.10.1), run from endRecord when rowCount reaches
 * rowCountForNextSizeCheck.  thresholdTolerance = (long)(pageSize * 0.1f); a column whose
 * page has <= tolerance bytes left is written out; rowsToFillPage keeps parquet-mr's
 * `(long)((float)rows) / usedMem * remainingMem` (integer division first). */
static void store_size_check_v2(kpwo_writer *w)
{
    const int64_t ps = w->props.page_size;
    const int64_t tol = (int64_t)((float)ps * 0.1f);
    int64_t min_wait = INT64_MAX;
    for (int k = 0; k < w->ncols; k++) {
        colw_t *c = &w->cw[k];
        const int64_t used = colw_mem(c);
        const int64_t rows = w->v2_rows - c->rows_written;
        int64_t remaining = ps - used;
        if (remaining <= tol) {
            colw_write_page_v2(w, c, w->v2_rows);
            remaining = ps;
        }
        const int64_t fill = used == 0 ? 10000 : ((int64_t)(float)rows / used) * remaining;
        if (fill < min_wait) min_wait = fill;
    }
    if (min_wait == INT64_MAX) min_wait = 100;
    int64_t half = min_wait / 2;
    if (half < 100) half = 100;
    if (half > 10000) half = 10000;
    w->v2_next_check = w->v2_rows + half;
}

/* ColumnWriterV1.flush / ColumnWriteStoreV2.flush + ColumnWriterV2.finalizeColumnChunk */
static void colw_flush(kpwo_writer *w, colw_t *c)
{
    if (w->v2) {
        if (w->v2_rows - c->rows_written > 0) colw_write_page_v2(w, c, w->v2_rows);
    } else if (c->value_count > 0) {
        colw_write_page(w, c);
    }
    buf_t dp = {0};
    int32_t nent = 0;
    if (dataw_dict_page(&c->data, &dp, &nent)) {
        /* ColumnChunkPageWriter.writeDictionaryPage: compress now, keep separately */
        c->has_dict = 1;
        c->dict_uncomp = (int32_t)dp.n;
        c->dict_nent = nent;
        c->dict_bytes.n = 0;
        page_compress(w, &dp, &c->dict_bytes);
    }
    buf_free(&dp);
}

/* ------------------------------------------------------------------ file writer */

static void rg_push(kpwo_writer *w, rgmeta_t *rg)
{
    if (w->nrgs == w->rgcap) { w->rgcap = w->rgcap ? w->rgcap * 2 : 8; w->rgs = (rgmeta_t *)xrealloc(w->rgs, (size_t)w->rgcap * sizeof(rgmeta_t)); }
    w->rgs[w->nrgs++] = *rg;
}

/* PaddingAlignment / NoAlignment (ParquetFileWriter 1.10.1) */
static int64_t dfs_block(const kpwo_writer *w)
{
    return w->props.dfs_block_size > w->props.block_size ? w->props.dfs_block_size : w->props.block_size;
}
static void align_for_row_group(kpwo_writer *w)
{
    if (w->props.dfs_block_size <= 0 || w->props.max_padding_size <= 0) return;
    int64_t bs = dfs_block(w);
    int64_t remaining = bs - ((int64_t)w->out.n % bs);
    if (remaining <= w->props.max_padding_size) {
        buf_reserve(&w->out, (uint64_t)remaining);
        memset(w->out.p + w->out.n, 0, (size_t)remaining);
        w->out.n += (uint64_t)remaining;
    }
}
static int64_t next_row_group_size(const kpwo_writer *w)
{
    if (w->props.dfs_block_size <= 0 || w->props.max_padding_size <= 0) return w->props.block_size;
    int64_t bs = dfs_block(w);
    int64_t remaining = bs - ((int64_t)w->out.n % bs);
    if (remaining <= w->props.max_padding_size) return w->props.block_size;
    return remaining < w->props.block_size ? remaining : w->props.block_size;
}

static void store_init(kpwo_writer *w)
{
    for (int c = 0; c < w->ncols; c++) colw_init(&w->cw[c], &w->cols[c], &w->props);
    w->v2_rows = 0;
    w->v2_next_check = 100;   /* props.getMinRowCountForPageSizeCheck() */
}
static void store_free(kpwo_writer *w)
{
    for (int c = 0; c < w->ncols; c++) colw_free(&w->cw[c]);
}

/* InternalParquetRecordWriter.flushRowGroupToStore + ParquetFileWriter block/column calls */
static void flush_row_group(kpwo_writer *w)
{
    if (w->record_count > 0) {
        align_for_row_group(w); /* startBlock */
        rgmeta_t rg;
        rg.rows = w->record_count;
        rg.total_bytes = 0;
        rg.chunks = (chunkmeta_t *)xmalloc((size_t)w->ncols * sizeof(chunkmeta_t));
        for (int c = 0; c < w->ncols; c++) colw_flush(w, &w->cw[c]); /* columnStore.flush() */
        for (int c = 0; c < w->ncols; c++) {                         /* pageStore.flushToFileWriter() */
            colw_t *cc = &w->cw[c];
            chunkmeta_t *m = &rg.chunks[c];
            memset(m, 0, sizeof(*m));
            m->phys = w->cols[c].phys;
            m->codec = w->props.codec;
            m->v2 = w->v2;
            m->num_values = cc->total_values;
            m->data_page_offset = (int64_t)w->out.n; /* startColumn: currentChunkFirstDataPage */
            int64_t uncomp = 0, comp = 0;
            if (cc->has_dict) {
                /* DictionaryValuesWriter: PLAIN_DICTIONARY (v1) / PLAIN (v2) dictionary pages */
                const int denc = w->v2 ? KPW_ENC_PLAIN : KPW_ENC_PLAIN_DICTIONARY;
                buf_t hdr = {0};
                tc_t t = {&hdr, {0}, 0};
                tc_i32(&t, 1, KPW_DICTIONARY_PAGE);
                tc_i32(&t, 2, cc->dict_uncomp);
                tc_i32(&t, 3, (int32_t)cc->dict_bytes.n);
                tc_struct_begin(&t, 7);
                tc_i32(&t, 1, cc->dict_nent);
                tc_i32(&t, 2, denc);
                tc_struct_end(&t);
                buf_u8(&hdr, 0);
                uncomp += cc->dict_uncomp + (int64_t)hdr.n;
                comp += (int64_t)cc->dict_bytes.n + (int64_t)hdr.n;
                buf_put(&w->out, hdr.p, hdr.n);
                buf_put(&w->out, cc->dict_bytes.p, cc->dict_bytes.n);
                buf_free(&hdr);
                enccount_add(&m->dict_stats, denc);
                encset_add(&m->encs, denc);
            }
            int64_t headers = (int64_t)cc->pages.n - cc->comp_len;
            uncomp += cc->uncomp_len + headers;
            comp += cc->comp_len + headers;
            buf_put(&w->out, cc->pages.p, cc->pages.n);
            for (int i = 0; i < cc->ndata_encs; i++) enccount_add(&m->data_stats, cc->data_encs[i]);
            for (int i = 0; i < cc->rl_encs.n; i++) encset_add(&m->encs, cc->rl_encs.v[i]);
            for (int i = 0; i < cc->dl_encs.n; i++) encset_add(&m->encs, cc->dl_encs.v[i]);
            for (int i = 0; i < cc->ndata_encs; i++) encset_add(&m->encs, cc->data_encs[i]);
            stats_reset(&m->stats, m->phys);
            if (cc->tstats_init) stats_copy(&m->stats, &cc->tstats);
            m->total_uncomp = uncomp;
            m->total_comp = comp;
            rg.total_bytes += uncomp;
        }
        rg_push(w, &rg);
        w->record_count = 0;
        w->next_rg_size = next_row_group_size(w) < w->props.block_size ? next_row_group_size(w) : w->props.block_size;
    }
    store_free(w);
}

/* InternalParquetRecordWriter.checkBlockSizeReached */
static int64_t store_buffered(const kpwo_writer *w)
{
    int64_t s = 0;
    for (int c = 0; c < w->ncols; c++) s += colw_mem(&w->cw[c]) + (int64_t)w->cw[c].pages.n;
    return s;
}
static void check_block_size(kpwo_writer *w)
{
    if (w->record_count >= w->next_mem_check) {
        int64_t mem = store_buffered(w);
        int64_t rec_size = mem / w->record_count;
        if (mem > w->next_rg_size - 2 * rec_size) {
            flush_row_group(w);
            store_init(w);
            int64_t half = w->record_count / 2; /* record_count was reset to 0 by the flush */
            int64_t v = half > 100 ? half : 100;
            w->next_mem_check = v < 10000 ? v : 10000;
            w->last_rg_end = (int64_t)w->out.n;
        } else {
            float q = (float)w->next_rg_size / (float)rec_size;
            int64_t est = jadd64(w->record_count, java_f2l(q)) / 2;
            int64_t a = est > 100 ? est : 100;
            int64_t b = jadd64(w->record_count, 10000);
            w->next_mem_check = a < b ? a : b;
        }
    }
}

/* ------------------------------------------------------------------ footer */

static int32_t java_string_hash(const char *s)
{
    uint32_t h = 0;
    for (const unsigned char *p = (const unsigned char *)s; *p; p++) h = 31 * h + *p; /* ASCII keys */
    return (int32_t)h;
}
static uint32_t java_hashmap_spread(const char *s) { uint32_t h = (uint32_t)java_string_hash(s); return h ^ (h >> 16); }

static const char *proto_type_name(int pt)
{
    static const char *n[] = {"", "TYPE_DOUBLE", "TYPE_FLOAT", "TYPE_INT64", "TYPE_UINT64", "TYPE_INT32",
                              "TYPE_FIXED64", "TYPE_FIXED32", "TYPE_BOOL", "TYPE_STRING", "TYPE_GROUP",
                              "TYPE_MESSAGE", "TYPE_BYTES", "TYPE_UINT32", "TYPE_ENUM", "TYPE_SFIXED32",
                              "TYPE_SFIXED64", "TYPE_SINT32", "TYPE_SINT64"};
    return (pt > 0 && pt <= 18) ? n[pt] : "TYPE_UNKNOWN";
}

/* TextFormat.printToString(descriptor.toProto()) as ProtoWriteSupport.serializeDescriptor does. */
static void descriptor_text(const kpwo_writer *w, buf_t *b)
{
    char line[512];
    const char *mn = w->message_name;
    const char *dot = strrchr(mn, '.');
    snprintf(line, sizeof line, "name: \"%s\"\n", dot ? dot + 1 : mn);
    buf_put(b, line, strlen(line));
    for (int c = 0; c < w->ncols; c++) {
        const colinfo_t *ci = &w->cols[c];
        snprintf(line, sizeof line, "field {\n  name: \"%s\"\n  number: %d\n  label: %s\n  type: %s\n}\n",
                 ci->name, ci->field_number, ci->optional ? "LABEL_OPTIONAL" : "LABEL_REQUIRED",
                 proto_type_name(ci->proto_type));
        buf_put(b, line, strlen(line));
    }
}

static void write_footer(kpwo_writer *w)
{
    buf_t f = {0};
    tc_t t = {&f, {0}, 0};
    int64_t num_rows = 0;
    for (int i = 0; i < w->nrgs; i++) num_rows += w->rgs[i].rows;
    tc_i32(&t, 1, 1);
    /* schema */
    tc_list_begin(&t, 2, 12, (uint32_t)w->ncols + 1);
    tc_elem_struct_begin(&t);
    tc_bin(&t, 4, w->message_name, strlen(w->message_name));
    tc_i32(&t, 5, w->ncols);
    tc_struct_end(&t);
    for (int c = 0; c < w->ncols; c++) {
        const colinfo_t *ci = &w->cols[c];
        tc_elem_struct_begin(&t);
        tc_i32(&t, 1, ci->phys);
        tc_i32(&t, 3, ci->optional ? 1 : 0);
        tc_bin(&t, 4, ci->name, strlen(ci->name));
        if (ci->utf8) tc_i32(&t, 6, 0);
        tc_i32(&t, 9, ci->field_number);
        tc_struct_end(&t);
    }
    tc_i64(&t, 3, num_rows);
    tc_list_begin(&t, 4, 12, (uint32_t)w->nrgs);
    for (int r = 0; r < w->nrgs; r++) {
        rgmeta_t *rg = &w->rgs[r];
        tc_elem_struct_begin(&t);
        tc_list_begin(&t, 1, 12, (uint32_t)w->ncols);
        for (int c = 0; c < w->ncols; c++) {
            chunkmeta_t *m = &rg->chunks[c];
            tc_elem_struct_begin(&t);
            tc_i64(&t, 2, m->data_page_offset);          /* ColumnChunk.file_offset */
            tc_struct_begin(&t, 3);                      /* ColumnMetaData */
            tc_i32(&t, 1, m->phys);
            tc_list_begin(&t, 2, 5, (uint32_t)m->encs.n);
            for (int i = 0; i < m->encs.n; i++) tc_varint(&f, zz64(m->encs.v[i]));
            tc_list_begin(&t, 3, 8, 1);
            tc_varint(&f, strlen(w->cols[c].name));
            buf_put(&f, w->cols[c].name, strlen(w->cols[c].name));
            tc_i32(&t, 4, m->codec);
            tc_i64(&t, 5, m->num_values);
            tc_i64(&t, 6, m->total_uncomp);
            tc_i64(&t, 7, m->total_comp);
            tc_i64(&t, 9, m->data_page_offset);
            /* dictionary_page_offset: assigned as a plain field by 1.10's converter, so the
             * Thrift isset bit stays clear and it is never serialised. */
            if (!stats_empty(&m->stats)) tc_statistics(&t, 12, &m->stats);
            tc_list_begin(&t, 13, 12, (uint32_t)(m->dict_stats.n + m->data_stats.n));
            for (int i = 0; i < m->dict_stats.n; i++) {
                tc_elem_struct_begin(&t);
                tc_i32(&t, 1, KPW_DICTIONARY_PAGE); tc_i32(&t, 2, m->dict_stats.enc[i]); tc_i32(&t, 3, m->dict_stats.cnt[i]);
                tc_struct_end(&t);
            }
            for (int i = 0; i < m->data_stats.n; i++) {
                tc_elem_struct_begin(&t);
                tc_i32(&t, 1, m->v2 ? KPW_DATA_PAGE_V2 : KPW_DATA_PAGE);
                tc_i32(&t, 2, m->data_stats.enc[i]); tc_i32(&t, 3, m->data_stats.cnt[i]);
                tc_struct_end(&t);
            }
            tc_struct_end(&t);   /* ColumnMetaData */
            tc_struct_end(&t);   /* ColumnChunk */
        }
        tc_i64(&t, 2, rg->total_bytes);
        tc_i64(&t, 3, rg->rows);
        tc_struct_end(&t);
    }
    /* key_value_metadata: java.util.HashMap iteration order of
     * {parquet.proto.class, parquet.proto.descriptor, writer.model.name} (table of 4). */
    {
        const char *keys[3] = {"parquet.proto.class", "parquet.proto.descriptor", "writer.model.name"};
        buf_t desc = {0};
        descriptor_text(w, &desc);
        const char *cls = w->proto_class ? w->proto_class : w->message_name;
        const void *vals[3] = {cls, desc.p, "protobuf"};
        uint64_t lens[3] = {strlen(cls), desc.n, 8};
        /* source map (16 buckets) iteration order of the two ProtoWriteSupport keys */
        int src[2] = {0, 1};
        if ((java_hashmap_spread(keys[1]) & 15) < (java_hashmap_spread(keys[0]) & 15)) { src[0] = 1; src[1] = 0; }
        int order[3] = {src[0], src[1], 2};
        /* stable sort by bucket (h & 3): insertion order within a bucket */
        int sorted[3], ns = 0;
        for (int bkt = 0; bkt < 4; bkt++)
            for (int i = 0; i < 3; i++)
                if ((int)(java_hashmap_spread(keys[order[i]]) & 3) == bkt) sorted[ns++] = order[i];
        tc_list_begin(&t, 5, 12, 3);
        for (int i = 0; i < 3; i++) {
            int k = sorted[i];
            tc_elem_struct_begin(&t);
            tc_bin(&t, 1, keys[k], strlen(keys[k]));
            tc_bin(&t, 2, vals[k], lens[k]);
            tc_struct_end(&t);
        }
        buf_free(&desc);
    }
    static const char created_by[] = "parquet-mr version 1.10.1 (build a89df8f9932b6ef6633d06069e50c9b7970bebd1)";
    tc_bin(&t, 6, created_by, strlen(created_by));
    tc_list_begin(&t, 7, 12, (uint32_t)w->ncols);  /* column_orders: TYPE_ORDER */
    for (int c = 0; c < w->ncols; c++) {
        tc_elem_struct_begin(&t);
        tc_struct_begin(&t, 1);
        tc_struct_end(&t);
        tc_struct_end(&t);
    }
    buf_u8(&f, 0); /* FileMetaData stop */
    buf_put(&w->out, f.p, f.n);
    buf_le32(&w->out, (uint32_t)f.n);
    buf_put(&w->out, "PAR1", 4);
    buf_free(&f);
}

/* ------------------------------------------------------------------ public API */

kpwo_writer *kpwo_open(const kpw_schema *schema, const kpw_props *props, int *status)
{
    int st = KPW_OK;
    if (!schema || !props || schema->num_columns <= 0 || !schema->columns || !schema->message_name) { st = KPW_ERR_INVALID_ARG; goto fail; }
    if ((props->writer_version != 1 && props->writer_version != 2) ||
        (props->codec != KPW_UNCOMPRESSED && props->codec != KPW_SNAPPY && props->codec != KPW_GZIP) ||
        props->block_size <= 0 || props->page_size <= 0 || props->dictionary_page_size <= 0) { st = KPW_ERR_UNSUPPORTED; goto fail; }
    kpwo_writer *w = (kpwo_writer *)xmalloc(sizeof(*w));
    memset(w, 0, sizeof(*w));
    w->ncols = schema->num_columns;
    w->cols = (colinfo_t *)xmalloc((size_t)w->ncols * sizeof(colinfo_t));
    for (int c = 0; c < w->ncols; c++) {
        const kpw_column_desc *d = &schema->columns[c];
        colinfo_t *ci = &w->cols[c];
        int wt, utf8;
        int phys = proto_to_phys(d->proto_type, &wt, &utf8);
        if (phys < 0 || (d->label != KPW_LABEL_OPTIONAL && d->label != KPW_LABEL_REQUIRED) || !d->name || d->field_number <= 0) {
            for (int k = 0; k < c; k++) free(w->cols[k].name);
            free(w->cols); free(w);
            st = KPW_ERR_UNSUPPORTED;
            goto fail;
        }
        ci->name = strdup(d->name);
        ci->field_number = d->field_number;
        ci->proto_type = d->proto_type;
        ci->label = d->label;
        ci->phys = phys;
        ci->optional = d->label == KPW_LABEL_OPTIONAL;
        ci->utf8 = utf8;
        ci->wire_type = wt;
    }
    w->message_name = strdup(schema->message_name);
    w->proto_class = schema->proto_class ? strdup(schema->proto_class) : NULL;
    w->props = *props;
    w->v2 = props->writer_version == 2;
    w->cw = (colw_t *)xmalloc((size_t)w->ncols * sizeof(colw_t));
    w->vals = (pval_t *)xmalloc((size_t)w->ncols * sizeof(pval_t));
    buf_put(&w->out, "PAR1", 4);
    w->next_mem_check = 100;
    w->next_rg_size = props->block_size;
    store_init(w);
    if (status) *status = KPW_OK;
    return w;
fail:
    if (status) *status = st;
    return NULL;
}

int kpwo_write(kpwo_writer *w, const uint8_t *rec, uint64_t len)
{
    if (!w) return KPW_ERR_INVALID_ARG;
    if (w->closed) return KPW_ERR_STATE;
    if (proto_decode(w->cols, w->ncols, rec, len, w->vals)) return KPW_ERR_INVALID_PROTO;
    for (int c = 0; c < w->ncols; c++) colw_write_value(w, &w->cw[c], &w->vals[c]);
    if (w->v2) {   /* ColumnWriteStoreV2.endRecord (MessageColumnIO endMessage), before the block check */
        ++w->v2_rows;
        if (w->v2_rows >= w->v2_next_check) store_size_check_v2(w);
    }
    ++w->record_count;
    check_block_size(w);
    ++w->num_records;
    return KPW_OK;
}

int kpwo_write_batch(kpwo_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n, uint64_t *n_written)
{
    uint64_t i;
    int st = KPW_OK;
    for (i = 0; i < n; i++) {
        st = kpwo_write(w, data + offsets[i], offsets[i + 1] - offsets[i]);
        if (st) break;
    }
    if (n_written) *n_written = i;
    return st;
}

int kpwo_write_until_full(kpwo_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                          int64_t max_file_size, uint64_t *n_accepted, int *full)
{
    uint64_t i;
    int st = KPW_OK, f = 0;
    for (i = 0; i < n; i++) {
        st = kpwo_write(w, data + offsets[i], offsets[i + 1] - offsets[i]);
        if (st) break;
        if (kpwo_data_size(w) >= max_file_size) { f = 1; i++; break; }
    }
    if (n_accepted) *n_accepted = i;
    if (full) *full = f;
    return st;
}

int64_t kpwo_data_size(const kpwo_writer *w)
{
    if (!w) return -1;
    if (w->closed) return (int64_t)w->out.n;
    return w->last_rg_end + store_buffered(w);
}

int64_t kpwo_num_records(const kpwo_writer *w) { return w ? w->num_records : -1; }

int kpwo_close(kpwo_writer *w)
{
    if (!w) return KPW_ERR_INVALID_ARG;
    if (w->closed) return KPW_OK;
    flush_row_group(w);
    write_footer(w);
    w->closed = 1;
    return KPW_OK;
}

int kpwo_file_bytes(const kpwo_writer *w, const uint8_t **bytes, uint64_t *len)
{
    if (!w || !w->closed) return KPW_ERR_STATE;
    *bytes = w->out.p;
    *len = w->out.n;
    return KPW_OK;
}

int kpwo_num_row_groups(const kpwo_writer *w) { return w ? w->nrgs : -1; }

void kpwo_free(kpwo_writer *w)
{
    if (!w) return;
    if (!w->closed) store_free(w);
    for (int r = 0; r < w->nrgs; r++) {
        for (int c = 0; c < w->ncols; c++) stats_free(&w->rgs[r].chunks[c].stats);
        free(w->rgs[r].chunks);
    }
    free(w->rgs);
    for (int c = 0; c < w->ncols; c++) free(w->cols[c].name);
    free(w->cols);
    free(w->message_name);
    free(w->proto_class);
    free(w->cw);
    free(w->vals);
    free(w->ctmp);
    buf_free(&w->out);
    free(w);
}
