// k_decode.hip — K1: proto2 wire bytes -> per-column (columnar) buffers.
//
// Restates, per record, what the reference does on the worker thread before any Parquet
// encoding happens (KafkaProtoParquetWriter.java:268-277):
//   parser.parseFrom(record.value())  — protobuf-java CodedInputStream + the generated
//       proto2 parse loop (src/test/java/ir/sahab/kafka/test/proto/TestMessage.java:85-139):
//       switch on the full tag, last occurrence wins, unknown fields (including a known
//       number with a foreign wire type) skipped, groups skipped recursively, varints of at
//       most 10 bytes, missing required field -> InvalidProtocolBufferException
//       (isInitialized, TestMessage.java:263-278);
//   ProtoWriteSupport.write -> RecordConsumer.add* (parquet-protobuf 1.10.1): one value or
//       one null per column per record, doubles/floats observed through
//       doubleToLongBits/floatToIntBits (NaN canonicalised).
//
// Layout: one lane per record, 256-record blocks whose bytes are staged in LDS (coalesced
// 16-byte loads; varints decoded from 8-byte reads); each wave covers 64 consecutive records
// so presence / boolean bits are produced with one __ballot per column per wave
// (word w of a bitmask = records [64w, 64w+64)).  Fixed-width values are stored record-
// indexed (SoA, coalesced per wave), strings as (absolute offset, length) into the batch
// bytes — the bytes are never copied here; the PLAIN/dictionary kernels gather them.
#include "kpw_device.h"
#include "kpw_kernels.h"

namespace kpw {

// Byte sources: the block's record bytes staged in LDS (GSrc for blocks whose bytes do not
// fit).  Positions are absolute offsets into the batch; 8-byte reads may run past the record
// (callers mask), never past the staged range + 16 or the batch end.
// GSrc keeps a 16-byte window of the lane's record in registers (8-aligned): consecutive reads
// of a record's fields mostly fall inside it, so a wide row (C3: ~200 fields of a few bytes)
// takes about half the dependent global loads of an 8-byte load per read.
struct GSrc {
    const uint8_t *d;
    uint64_t end;   // batch end
    uint64_t wpos = ~0ull, lo = 0, hi = 0;
    __device__ __forceinline__ uint8_t b(uint64_t p) const { return d[p]; }
    __device__ __forceinline__ uint64_t w64(uint64_t p)
    {
        if (p < wpos || p - wpos > 8) {
            const uint64_t a = p & ~7ull;
            if (a + 16 > end) return ldu64(d, p, end);   // the batch's last bytes: bounded loads
            lo = *(const uint64_t *)(d + a);
            hi = *(const uint64_t *)(d + a + 8);
            wpos = a;
        }
        const uint32_t sh = (uint32_t)(p - wpos) * 8;
        return sh == 0 ? lo : sh == 64 ? hi : ((lo >> sh) | (hi << (64 - sh)));
    }
};
struct LSrc {
    const uint32_t *w;   // LDS words holding bytes [base, ...)
    uint64_t base;       // 4-aligned
    __device__ __forceinline__ uint8_t b(uint64_t p) const
    {
        const uint32_t o = (uint32_t)(p - base);
        return (uint8_t)(w[o >> 2] >> (8 * (o & 3)));
    }
    __device__ __forceinline__ uint64_t w64(uint64_t p) const
    {
        const uint32_t o = (uint32_t)(p - base), i = o >> 2, s = o & 3;
        const uint32_t a0 = w[i], a1 = w[i + 1], a2 = w[i + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, s) << 32);
    }
};

// protobuf varint: 8 bytes at once (one load, the stop byte found with ctz), byte loop only for
// 9- and 10-byte varints
template <class Src>
__device__ __forceinline__ bool rd_varint64(Src &S, uint64_t &pos, uint64_t end, uint64_t &out)
{
    if (pos >= end) return false;
    const uint64_t w = S.w64(pos);
    const uint64_t stop = ~w & 0x8080808080808080ull;
    if (stop) {
        const uint32_t len = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;
        if (len > end - pos) return false;
        uint64_t v = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) v |= ((w >> i) & (0x7full << (7 * i)));
        out = len == 8 ? v : (v & ((1ull << (7 * len)) - 1));
        pos += len;
        return true;
    }
    uint64_t r = 0;
#pragma unroll 1
    for (int i = 0; i < 10; i++) {
        if (pos >= end) return false;
        const uint8_t c = S.b(pos++);
        r |= (uint64_t)(c & 0x7f) << (7 * i);
        if (!(c & 0x80)) { out = r; return true; }
    }
    return false;
}

// Skip one unknown field whose tag has already been read. Groups are skipped
// iteratively with a bounded stack (protobuf-java recursion limit 100).
template <class Src>
__device__ bool skip_field(Src &S, uint64_t &pos, uint64_t end, uint32_t tag)
{
    uint32_t wt = tag & 7;
    uint64_t v;
    switch (wt) {
    case 0: return rd_varint64(S, pos, end, v);
    case 1: if (end - pos < 8) return false; pos += 8; return true;
    case 2:
        if (!rd_varint64(S, pos, end, v)) return false;
        if ((int32_t)(uint32_t)v < 0) return false;
        if (end - pos < (uint32_t)v) return false;
        pos += (uint32_t)v;
        return true;
    case 5: if (end - pos < 4) return false; pos += 4; return true;
    case 3: {
        uint32_t stack[100];
        int depth = 0;
        stack[depth++] = tag >> 3;
#pragma unroll 1
        while (depth > 0) {
            uint64_t t64;
            if (!rd_varint64(S, pos, end, t64)) return false;
            uint32_t t = (uint32_t)t64;
            if ((t >> 3) == 0) return false;
            uint32_t w = t & 7;
            if (w == 4) {
                if ((t >> 3) != stack[depth - 1]) return false;
                depth--;
            } else if (w == 3) {
                if (depth >= 100) return false;
                stack[depth++] = t >> 3;
            } else if (w == 0) {
                if (!rd_varint64(S, pos, end, v)) return false;
            } else if (w == 1) {
                if (end - pos < 8) return false; pos += 8;
            } else if (w == 5) {
                if (end - pos < 4) return false; pos += 4;
            } else if (w == 2) {
                if (!rd_varint64(S, pos, end, v)) return false;
                if ((int32_t)(uint32_t)v < 0) return false;
                if (end - pos < (uint32_t)v) return false;
                pos += (uint32_t)v;
            } else {
                return false;
            }
        }
        return true;
    }
    default: return false;  // END_GROUP at top level (checkLastTagWas fails) or wire type 6/7
    }
}

__device__ __forceinline__ uint64_t canon_double(uint64_t b)
{
    if ((b & 0x7ff0000000000000ull) == 0x7ff0000000000000ull && (b & 0x000fffffffffffffull)) return 0x7ff8000000000000ull;
    return b;
}
__device__ __forceinline__ uint32_t canon_float(uint32_t b)
{
    if ((b & 0x7f800000u) == 0x7f800000u && (b & 0x007fffffu)) return 0x7fc00000u;
    return b;
}

// 64-bit hash of a value's bytes (the dictionary key of BYTE_ARRAY columns; the same function
// as bytes_hash in kpw_device.h, through a byte source)
template <class Src>
__device__ __forceinline__ uint64_t src_bytes_hash(Src &S, uint64_t off, uint32_t len)
{
    uint64_t h = 0x9E3779B97F4A7C15ull ^ len;
    for (uint32_t k = 0; k < len; k += 8) {
        const uint64_t w = S.w64(off + k) & tail_mask(len - k);
        h = (h ^ w) * 0xff51afd7ed558ccdull;
        h ^= h >> 29;
    }
    return mix64(h);
}

// One value of column c (tag already consumed, wire type matches): decode, store, account.
template <class Src>
__device__ __forceinline__ bool parse_value(const DevCol *col, int c, uint32_t wt, Src &S, uint64_t &pos, uint64_t end,
                                            uint64_t r, uint64_t *seen, uint64_t *bval, uint32_t *raw)
{
    const bool again = (seen[c >> 6] >> (c & 63)) & 1;
    uint64_t v = 0;
    if (wt == 0) {
        if (!rd_varint64(S, pos, end, v)) return false;
        switch (col->proto_type) {
        case 5: case 13: v = (uint32_t)v; break;                                            // int32/uint32
        case 17: { uint32_t u = (uint32_t)v; v = (uint32_t)((u >> 1) ^ (0u - (u & 1))); break; }  // sint32
        case 18: v = (v >> 1) ^ (0ull - (v & 1)); break;                                   // sint64
        case 8: v = v != 0; break;                                                          // bool
        default: break;
        }
    } else if (wt == 1) {
        if (end - pos < 8) return false;
        v = S.w64(pos);
        pos += 8;
        if (col->phys == 5) v = canon_double(v);
    } else if (wt == 5) {
        if (end - pos < 4) return false;
        v = S.w64(pos) & 0xffffffffull;
        pos += 4;
        if (col->phys == 4) v = canon_float((uint32_t)v);
    } else {  // wt == 2
        uint64_t l;
        if (!rd_varint64(S, pos, end, l)) return false;
        if ((int32_t)(uint32_t)l < 0 || end - pos < (uint32_t)l) return false;
        if (again) *raw -= 4 + col->slen[r];
        *raw += 4 + (uint32_t)l;
        col->soff[r] = pos;
        col->slen[r] = (uint32_t)l;
        // first 16 bytes, zero padded: exact compares for short strings (stats,
        // dictionary verification) without touching the batch bytes again
        col->spfx[2 * r] = l ? S.w64(pos) & tail_mask(l) : 0ull;
        col->spfx[2 * r + 1] = l > 8 ? S.w64(pos + 8) & tail_mask(l - 8) : 0ull;
        if (col->dict) col->shash[r] = src_bytes_hash(S, pos, (uint32_t)l);
        pos += (uint32_t)l;
    }
    if (col->phys != 0 && col->phys != 6 && !again) *raw += (uint32_t)col->vsize;
    if (col->phys == 0) {
        if (v) bval[c >> 6] |= 1ull << (c & 63); else bval[c >> 6] &= ~(1ull << (c & 63));
    } else if (col->vsize == 4) {
        ((uint32_t *)col->vals)[r] = (uint32_t)v;
    } else if (col->vsize == 8) {
        ((uint64_t *)col->vals)[r] = v;
    }
    seen[c >> 6] |= 1ull << (c & 63);
    return true;
}

// Parse record r from source S.  Returns false on an invalid record.  `cols` holds every
// column (LDS copy); *raw accumulates the plain-equivalent bytes of the present values (a
// repeated field replaces its earlier occurrence: last one wins).
//
// Lockstep pass first: protobuf-java writes the known fields in field-number order, so the
// lanes of a wave walk the columns in that order (`order`) together, each taking its record's
// next field when it is that column's.  The lanes holding column c then store c's values in
// the same instruction (coalesced per wave; a free-running loop has every lane at a different
// column after the first null, and every store touches its own cache line).  Whatever the pass
// leaves (unknown fields, another order, repeats) the general loop parses from there.
template <class Src>
__device__ __forceinline__ bool parse_record(const DecodeArgs &a, const DevCol *cols, const int16_t *fmap, const uint8_t *order,
                                             Src &S, uint64_t r, uint64_t pos, uint64_t end, uint64_t *seen,
                                             uint64_t *bval, uint32_t *raw)
{
    for (int k = 0; k < a.ncols; k++) {
        if (pos >= end) break;
        const int c = order[k];
        const DevCol *col = &cols[c];
        const uint64_t w = S.w64(pos);
        // the expected tag: field number and wire type of column c, as a 1- or 2-byte varint
        const uint32_t t = ((uint32_t)col->field_number << 3) | (uint32_t)col->wire_type;
        uint32_t tl;
        if (t < 0x80) { if ((uint32_t)(w & 0xff) != t) continue; tl = 1; }
        else if (t < 0x4000) {
            if ((uint32_t)(w & 0xffff) != ((t & 0x7f) | 0x80 | ((t >> 7) << 8))) continue;
            tl = 2;
        } else break;   // longer tags: the general loop
        if (end - pos < tl) break;
        pos += tl;
        if (!parse_value(col, c, (uint32_t)col->wire_type, S, pos, end, r, seen, bval, raw)) return false;
    }
#pragma unroll 1
    while (pos < end) {
        uint64_t t64;
        if (!rd_varint64(S, pos, end, t64)) return false;
        const uint32_t tag = (uint32_t)t64;
        const uint32_t fno = tag >> 3, wt = tag & 7;
        if (fno == 0) return false;
        int c = -1;
        if (fno < FMAP_SIZE) c = fmap[fno];
        else {
            for (int k = 0; k < a.ncols; k++) if ((uint32_t)a.cols[k].field_number == fno) { c = k; break; }
        }
        const DevCol *col = c >= 0 ? &cols[c] : nullptr;
        if (c < 0 || (uint32_t)col->wire_type != wt) {
            if (!skip_field(S, pos, end, tag)) return false;
            continue;
        }
        if (!parse_value(col, c, wt, S, pos, end, r, seen, bval, raw)) return false;
    }
    return true;
}

// Tile kernel: one block = 256 consecutive records.  When the block's bytes fit K1_LDS bytes
// they are staged into LDS with coalesced 16-byte loads and every lane parses its record from
// LDS; wider records (C3-like rows of > 96 bytes) parse straight from global memory.  Every
// column descriptor is copied to LDS (dynamic: ncols * 96 bytes), so a wide schema's fields
// never wait on a global descriptor load.
constexpr uint32_t K1_LDS = 24576;

__global__ void __launch_bounds__(KPW_BLOCK) k_decode(DecodeArgs a)
{
    __shared__ int16_t fmap[FMAP_SIZE];
    __shared__ uint4 stage[K1_LDS / 16 + 2];
    __shared__ uint64_t reqm[MAX_COLS / 64];     // required (non-optional) columns
    __shared__ uint8_t order[MAX_COLS];          // columns by field number (the wire order)
    extern __shared__ DevCol cols[];             // [ncols]
    for (int i = threadIdx.x; i < FMAP_SIZE; i += blockDim.x) fmap[i] = a.fmap[i];
    for (int i = threadIdx.x; i < a.ncols; i += blockDim.x) {
        cols[i] = a.cols[i];
        const int f = a.cols[i].field_number;
        int rank = 0;   // field numbers are distinct
        for (int k = 0; k < a.ncols; k++) rank += a.cols[k].field_number < f;
        order[rank] = (uint8_t)i;
    }
    if (threadIdx.x < MAX_COLS / 64) {
        uint64_t m = 0;
        for (int k = 0; k < 64; k++) {
            const int c = (int)threadIdx.x * 64 + k;
            if (c < a.ncols && !a.cols[c].optional) m |= 1ull << k;
        }
        reqm[threadIdx.x] = m;
    }

    if (blockIdx.x == 0) {   // bitmask words past the last record's word (the waves write the rest)
        const uint64_t w0 = (a.n + 63) / 64;
        for (uint64_t i = threadIdx.x; i < (uint64_t)a.ncols * (a.nwords - w0); i += blockDim.x) {
            const DevCol &col = a.cols[i / (a.nwords - w0)];
            const uint64_t w = w0 + i % (a.nwords - w0);
            if (col.optional) col.pres[w] = 0;
            if (col.phys == 0) col.vbits[w] = 0;
        }
    }
    const uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x;
    const uint64_t r = r0 + threadIdx.x;
    const bool valid = r < a.n;
    const uint64_t data_end = a.off[a.n];
    const uint64_t rl = r0 + blockDim.x < a.n ? r0 + blockDim.x : a.n;
    const uint64_t B0 = a.off[r0], B1 = a.off[rl];
    const uint64_t S0 = B0 & ~15ull;                          // 16-aligned staging start
    const bool staged = B1 - S0 <= K1_LDS;
    if (staged) {
        // [S0, B1) + 16 bytes of read padding; nothing at or past the batch end is read (the
        // caller's buffer may end there): the 16-byte piece holding it is copied byte by byte
        const uint64_t lim = (B1 + 16 + 15) & ~15ull;
        const uint4 *src = (const uint4 *)(a.data + S0);
        const uint32_t nv = (uint32_t)((lim - S0) >> 4);
        for (uint32_t i = threadIdx.x; i < nv; i += blockDim.x) {
            const uint64_t p = S0 + 16ull * i;
            if (p + 16 <= data_end) {
                stage[i] = src[i];
            } else {
                uint32_t q[4] = {0, 0, 0, 0};
                for (uint32_t k = 0; k < 16 && p + k < data_end; k++) q[k >> 2] |= (uint32_t)a.data[p + k] << (8 * (k & 3));
                stage[i] = uint4{q[0], q[1], q[2], q[3]};
            }
        }
    }
    __syncthreads();

    uint64_t seen[4] = {0, 0, 0, 0};
    uint64_t bval[4] = {0, 0, 0, 0};   // boolean values (by column)
    bool bad = false;
    uint32_t raw = 0;

    if (valid) {
        const uint64_t pos = a.off[r], end = a.off[r + 1];
        if (staged) {
            LSrc src{(const uint32_t *)stage, S0};
            bad = !parse_record(a, cols, fmap, order, src, r, pos, end, seen, bval, &raw);
        } else {
            GSrc src{a.data, data_end};
            bad = !parse_record(a, cols, fmap, order, src, r, pos, end, seen, bval, &raw);
        }
        // a missing required field (isInitialized)
        for (int k = 0; k < MAX_COLS / 64 && !bad; k++) bad = (seen[k] & reqm[k]) != reqm[k];
        if (bad) atomicMin(a.err_min, (unsigned long long)r);
        a.raw[r] = bad ? 0 : raw;
    }

    // presence / boolean bitmasks: one ballot per column per wave (all lanes take part)
    const uint64_t word = r >> 6;
    // lane 0 of a wave lying wholly past n must not write (bitmasks hold n/64+2 words)
    const bool lane0 = (threadIdx.x & 63) == 0 && r < a.n;
    for (int c = 0; c < a.ncols; c++) {
        const DevCol *col = &cols[c];
        const bool pr = valid && !bad && ((seen[c >> 6] >> (c & 63)) & 1);
        if (col->optional) {
            uint64_t m = __ballot(pr);
            if (lane0) col->pres[word] = m;
        }
        if (col->phys == 0) {
            uint64_t m = __ballot(pr && ((bval[c >> 6] >> (c & 63)) & 1));
            if (lane0) col->vbits[word] = m;
        }
    }
}

void launch_decode(const DecodeArgs &a, hipStream_t s)
{
    if (a.n == 0) return;
    const uint64_t blocks = (a.n + KPW_BLOCK - 1) / KPW_BLOCK;
    hipLaunchKernelGGL(k_decode, dim3((unsigned)blocks), dim3(KPW_BLOCK), (size_t)a.ncols * sizeof(DevCol), s, a);
}

}  // namespace kpw
