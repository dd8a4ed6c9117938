/*
 * oracle_snappy.c — CPU ORACLE (test infrastructure only): Snappy raw-format compressor.
 *
 * What the reference runs: parquet-mr 1.10.1 SnappyCompressor.compress() buffers the whole
 * page and makes ONE snappy-java Snappy.compress(ByteBuffer, ByteBuffer) call
 * (JNI -> snappy::RawCompress).  snappy-java is a transitive dependency of
 * parquet-hadoop 1.10.1 (reference pom.xml:44-48; not vendored, not present here).
 *
 * PINNED ALGORITHM (stated because snappy's encoder output is version dependent):
 * Google Snappy 1.1.2 `Compress` / `internal::CompressFragment`:
 *   - varint32(uncompressed length), then the input in independent 64 KiB fragments;
 *   - per fragment a zeroed uint16 hash table of size max(256, next pow2 >= fragment
 *     length) capped at 1<<14, hash = (load32(p) * 0x1e35a7bd) >> (32 - log2(size));
 *   - kInputMarginBytes = 15; the literal scan probes ip, advancing by (skip++ >> 5) with
 *     skip starting at 32 (the 1.1.2 heuristic; 1.1.4+ advance by skip>>5, skip += step);
 *   - after each copy: table[hash(ip-1)] = ip-1, then test table[hash(ip)];
 *   - EmitCopy in 64-byte pieces, keeping >= 4 bytes for the last (60-byte split);
 *     COPY_1_BYTE_OFFSET when len < 12 && offset < 2048, else COPY_2_BYTE_OFFSET;
 *   - literals: tag (len-1)<<2 when len <= 60, else 60..63 with 1..4 length bytes.
 * Byte identity of this choice to the snappy-java build parquet-mr 1.10.1 resolves is
 * UNPINNED offline (no jar here); every stream is checked by pyarrow's Snappy decoder.
 *
 * ATTRIBUTION: the fragment compressor below follows the structure and names of Google
 * Snappy 1.1.2's snappy.cc (CompressFragment, EmitLiteral, EmitCopy, FindMatchLength;
 * ip_limit, next_emit, bytes_between_hash_lookups, ...).  Snappy is
 *   Copyright 2005 and onwards Google Inc.
 * distributed under the BSD 3-Clause license: redistribution in source and binary forms,
 * with or without modification, is permitted provided that the copyright notice, this list
 * of conditions and the disclaimer are retained, and that neither the name of Google Inc.
 * nor the names of its contributors are used to endorse or promote derived products
 * without specific prior written permission.  THE SOFTWARE IS PROVIDED "AS IS", WITHOUT
 * ANY EXPRESS OR IMPLIED WARRANTIES.  It is test infrastructure here: nothing in
 * libkpw_gpu.so links or includes it.
 */
#include <stdint.h>
#include <string.h>
#include "kpw_oracle.h"

#define SNAPPY_BLOCK_SIZE (1u << 16)
#define SNAPPY_MAX_HASH_TABLE (1u << 14)

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ld64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t hash_bytes(uint32_t bytes, int shift) { return (bytes * 0x1e35a7bdu) >> shift; }

static uint8_t *emit_literal(uint8_t *op, const uint8_t *lit, uint32_t len)
{
    uint32_t n = len - 1;
    if (n < 60) {
        *op++ = (uint8_t)(n << 2);
    } else {
        uint8_t *base = op++;
        int count = 0;
        while (n > 0) { *op++ = (uint8_t)(n & 0xff); n >>= 8; count++; }
        *base = (uint8_t)((59 + count) << 2);
    }
    memcpy(op, lit, len);
    return op + len;
}

static uint8_t *emit_copy_lt64(uint8_t *op, uint32_t offset, uint32_t len)
{
    if (len < 12 && offset < 2048) {
        *op++ = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
        *op++ = (uint8_t)(offset & 0xff);
    } else {
        *op++ = (uint8_t)(2 + ((len - 1) << 2));
        *op++ = (uint8_t)(offset & 0xff);
        *op++ = (uint8_t)(offset >> 8);
    }
    return op;
}

static uint8_t *emit_copy(uint8_t *op, uint32_t offset, uint32_t len)
{
    while (len >= 68) { op = emit_copy_lt64(op, offset, 64); len -= 64; }
    if (len > 64) { op = emit_copy_lt64(op, offset, 60); len -= 60; }
    return emit_copy_lt64(op, offset, len);
}

static uint32_t find_match_length(const uint8_t *s1, const uint8_t *s2, const uint8_t *s2_limit)
{
    uint32_t m = 0;
    while (s2 + m < s2_limit && s1[m] == s2[m]) m++;
    return m;
}

static int log2_floor(uint32_t n) { int l = -1; while (n) { n >>= 1; l++; } return l; }

static uint8_t *compress_fragment(const uint8_t *input, uint32_t input_size, uint8_t *op,
                                  uint16_t *table, uint32_t table_size)
{
    const uint8_t *ip = input;
    const int shift = 32 - log2_floor(table_size);
    const uint8_t *ip_end = input + input_size;
    const uint8_t *base_ip = ip;
    const uint8_t *next_emit = ip;
    const uint32_t kInputMarginBytes = 15;

    if (input_size >= kInputMarginBytes) {
        const uint8_t *ip_limit = input + input_size - kInputMarginBytes;
        uint32_t next_hash = hash_bytes(ld32(++ip), shift);
        for (;;) {
            uint32_t skip = 32;
            const uint8_t *next_ip = ip;
            const uint8_t *candidate;
            do {
                ip = next_ip;
                uint32_t hash = next_hash;
                uint32_t bytes_between_hash_lookups = skip++ >> 5;
                next_ip = ip + bytes_between_hash_lookups;
                if (next_ip > ip_limit) goto emit_remainder;
                next_hash = hash_bytes(ld32(next_ip), shift);
                candidate = base_ip + table[hash];
                table[hash] = (uint16_t)(ip - base_ip);
            } while (ld32(ip) != ld32(candidate));

            op = emit_literal(op, next_emit, (uint32_t)(ip - next_emit));

            uint64_t input_bytes;
            uint32_t candidate_bytes;
            do {
                const uint8_t *base = ip;
                uint32_t matched = 4 + find_match_length(candidate + 4, ip + 4, ip_end);
                ip += matched;
                uint32_t offset = (uint32_t)(base - candidate);
                op = emit_copy(op, offset, matched);
                const uint8_t *insert_tail = ip - 1;
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                input_bytes = ld64(insert_tail);
                uint32_t prev_hash = hash_bytes((uint32_t)input_bytes, shift);
                table[prev_hash] = (uint16_t)(ip - base_ip - 1);
                uint32_t cur_hash = hash_bytes((uint32_t)(input_bytes >> 8), shift);
                candidate = base_ip + table[cur_hash];
                candidate_bytes = ld32(candidate);
                table[cur_hash] = (uint16_t)(ip - base_ip);
            } while ((uint32_t)(input_bytes >> 8) == candidate_bytes);

            next_hash = hash_bytes((uint32_t)(input_bytes >> 16), shift);
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal(op, next_emit, (uint32_t)(ip_end - next_emit));
    return op;
}

uint64_t kpwo_snappy_max_compressed_length(uint64_t n) { return 32 + n + n / 6; }

int64_t kpwo_snappy_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap)
{
    if (cap < kpwo_snappy_max_compressed_length(n) || n > 0xffffffffull) return -1;
    uint8_t *op = out;
    uint32_t v = (uint32_t)n;
    while (v >= 0x80) { *op++ = (uint8_t)(v | 0x80); v >>= 7; }
    *op++ = (uint8_t)v;
    static __thread uint16_t table[SNAPPY_MAX_HASH_TABLE];
    uint64_t pos = 0;
    while (pos < n) {
        uint32_t frag = (uint32_t)((n - pos) < SNAPPY_BLOCK_SIZE ? (n - pos) : SNAPPY_BLOCK_SIZE);
        uint32_t ts = 256;
        while (ts < SNAPPY_MAX_HASH_TABLE && ts < frag) ts <<= 1;
        memset(table, 0, ts * sizeof(uint16_t));
        op = compress_fragment(in + pos, frag, op, table, ts);
        pos += frag;
    }
    return (int64_t)(op - out);
}
