/*
 * oracle_deflate.c — TEST INFRASTRUCTURE ONLY (the CPU oracle; never linked into the product).
 *
 * CompressionCodecName.GZIP as parquet-mr 1.10.1 writes it on Hadoop 2.7.7 without the native
 * hadoop library (the reference passes any codec through: KafkaProtoParquetWriter.java:484,
 * 690-694 -> ParquetFile.java:45):
 *   CodecFactory.HeapBytesCompressor.compress -> GzipCodec.createOutputStream(out, null)
 *   ("null compressor for non-native gzip") -> GzipCodec.GzipOutputStream ->
 *   ResetableGZIPOutputStream extends java.util.zip.GZIPOutputStream (Java 8):
 *     header 1f 8b 08 00 | 00 00 00 00 | 00 00   (MTIME 0, XFL 0, OS 0)
 *     raw deflate: java.util.zip.Deflater(DEFAULT_COMPRESSION, nowrap) = zlib
 *       deflateInit2(level 6, Z_DEFLATED, -15, memLevel 8, Z_DEFAULT_STRATEGY), Z_NO_FLUSH writes
 *       then Z_FINISH
 *     trailer CRC-32 (LE), ISIZE (LE)
 * One gzip member per page (and per dictionary page), as SnappyCompressor does per page.
 *
 * The deflate below restates zlib 1.2.11 (the version bundled with late Java 8 updates, and the
 * one Python's zlib module reports in this image) for that configuration only: deflate.c
 * (lm_init, fill_window with its window slide and high-water zeroing, deflate_slow with lazy
 * matching, longest_match with good_length 8 / max_lazy 16 / nice_length 128 / max_chain 128)
 * and trees.c (_tr_tally, _tr_flush_block with its stored / static / dynamic choice,
 * build_tree with the heap order and depth tie-break, gen_bitlen with its overflow repair,
 * gen_codes, scan_tree / send_tree, build_bl_tree, compress_block, _tr_stored_block).  It is
 * checked byte-for-byte against Python's zlib (tests/test_oracle.py).  Identity to the JVM's
 * own bundled zlib build is parity unpinned (no JVM here); zlib's level-6 output has been
 * stable across 1.2.x.  Input chunking (Java writes a page's rl / dl / values parts
 * separately) does not change zlib's output for Z_NO_FLUSH writes; the whole page is fed at once.
 *
 * ATTRIBUTION: the deflate_slow / longest_match restatement and the trees.c routines below
 * (pqdownheap, gen_bitlen, gen_codes, build_tree, scan_tree, send_tree, build_bl_tree,
 * compress_block, _tr_flush_block, _tr_stored_block) follow zlib 1.2.11's deflate.c and trees.c
 * closely, names and control flow included: byte identity with zlib needs its exact heap
 * tie-breaks and block decisions.  This is an ALTERED version of that code (restated in one
 * file for a single configuration), not the original.  zlib is
 *   Copyright (C) 1995-2017 Jean-loup Gailly and Mark Adler
 * and distributed under the zlib license:
 *   This software is provided 'as-is', without any express or implied warranty.  In no event
 *   will the authors be held liable for any damages arising from the use of this software.
 *   Permission is granted to anyone to use this software for any purpose, including commercial
 *   applications, and to alter it and redistribute it freely, subject to the following
 *   restrictions:
 *   1. The origin of this software must not be misrepresented; you must not claim that you
 *      wrote the original software.  If you use this software in a product, an acknowledgment
 *      in the product documentation would be appreciated but is not required.
 *   2. Altered source versions must be plainly marked as such, and must not be misrepresented
 *      as being the original software.
 *   3. This notice may not be removed or altered from any source distribution.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define L_CODES 286
#define D_CODES 30
#define BL_CODES 19
#define HEAP_SIZE (2 * L_CODES + 1)
#define MAX_BITS 15
#define MAX_BL_BITS 7
#define LITERALS 256
#define END_BLOCK 256
#define LENGTH_CODES 29
#define REP_3_6 16
#define REPZ_3_10 17
#define REPZ_11_138 18
#define MIN_MATCH 3
#define MAX_MATCH 258
#define MIN_LOOKAHEAD (MAX_MATCH + MIN_MATCH + 1)
#define WSIZE 32768u
#define WMASK (WSIZE - 1)
#define HASH_BITS 15
#define HASH_SIZE (1u << HASH_BITS)
#define HASH_MASK (HASH_SIZE - 1)
#define HASH_SHIFT ((HASH_BITS + MIN_MATCH - 1) / MIN_MATCH)
#define MAX_DIST (WSIZE - MIN_LOOKAHEAD)
#define TOO_FAR 4096
#define LIT_BUFSIZE 16384u   /* 1 << (memLevel 8 + 6) */
#define WIN_INIT MAX_MATCH
#define NIL 0
/* configuration_table[6] */
#define GOOD_LENGTH 8
#define MAX_LAZY 16
#define NICE_LENGTH 128
#define MAX_CHAIN 128

/* ct_data: the Freq/Code and Dad/Len unions of trees.c, kept as unions */
typedef struct { uint16_t fc, dl; } ct_data;
#define Freq fc
#define Code fc
#define Dad dl
#define Len dl

static const int extra_lbits[LENGTH_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const int extra_dbits[D_CODES] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const int extra_blbits[BL_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
static const uint8_t bl_order[BL_CODES] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static ct_data static_ltree[L_CODES + 2];
static ct_data static_dtree[D_CODES];
static uint8_t dist_code_tab[512];
static uint8_t length_code_tab[MAX_MATCH - MIN_MATCH + 1];
static int base_length[LENGTH_CODES];
static int base_dist[D_CODES];
static int static_ready;

typedef struct {
    const ct_data *static_tree;
    const int *extra_bits;
    int extra_base, elems, max_length;
} static_tree_desc;
static static_tree_desc static_l_desc = {static_ltree, extra_lbits, LITERALS + 1, L_CODES, MAX_BITS};
static static_tree_desc static_d_desc = {static_dtree, extra_dbits, 0, D_CODES, MAX_BITS};
static static_tree_desc static_bl_desc = {NULL, extra_blbits, 0, BL_CODES, MAX_BL_BITS};

typedef struct {
    ct_data *dyn_tree;
    int max_code;
    const static_tree_desc *stat_desc;
} tree_desc;

typedef struct {
    /* input */
    const uint8_t *next_in;
    uint64_t avail_in;
    /* window and hash chains */
    uint8_t window[2 * WSIZE];
    uint16_t prev[WSIZE];
    uint16_t head[HASH_SIZE];
    uint64_t window_size, high_water;
    unsigned ins_h, strstart, match_start, lookahead, prev_length, match_length, prev_match, insert;
    int match_available;
    long block_start;
    /* trees */
    ct_data dyn_ltree[HEAP_SIZE], dyn_dtree[2 * D_CODES + 1], bl_tree[2 * BL_CODES + 1];
    tree_desc l_desc, d_desc, bl_desc;
    uint16_t bl_count[MAX_BITS + 1];
    int heap[2 * L_CODES + 1];
    int heap_len, heap_max;
    uint8_t depth[2 * L_CODES + 1];
    uint8_t l_buf[LIT_BUFSIZE];
    uint16_t d_buf[LIT_BUFSIZE];
    unsigned last_lit, matches;
    uint64_t opt_len, static_len;
    /* output: LSB-first bit writer (zlib's 16-bit bi_buf emits the same byte stream) */
    uint8_t *out;
    uint64_t op, cap;
    uint64_t bi_buf;
    int bi_valid;
    int overflow;
} DState;

static unsigned bi_reverse(unsigned code, int len)
{
    unsigned res = 0;
    do { res |= code & 1; code >>= 1, res <<= 1; } while (--len > 0);
    return res >> 1;
}

static void put_byte(DState *s, uint8_t b)
{
    if (s->op < s->cap) s->out[s->op] = b; else s->overflow = 1;
    s->op++;
}

static void send_bits(DState *s, unsigned value, int length)
{
    s->bi_buf |= (uint64_t)value << s->bi_valid;
    s->bi_valid += length;
    while (s->bi_valid >= 16) {
        put_byte(s, (uint8_t)s->bi_buf);
        put_byte(s, (uint8_t)(s->bi_buf >> 8));
        s->bi_buf >>= 16;
        s->bi_valid -= 16;
    }
}

static void bi_windup(DState *s)
{
    if (s->bi_valid > 8) { put_byte(s, (uint8_t)s->bi_buf); put_byte(s, (uint8_t)(s->bi_buf >> 8)); }
    else if (s->bi_valid > 0) put_byte(s, (uint8_t)s->bi_buf);
    s->bi_buf = 0;
    s->bi_valid = 0;
}

static void gen_codes(ct_data *tree, int max_code, const uint16_t *bl_count)
{
    uint16_t next_code[MAX_BITS + 1];
    unsigned code = 0;
    for (int bits = 1; bits <= MAX_BITS; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; n++) {
        int len = tree[n].Len;
        if (len == 0) continue;
        tree[n].Code = (uint16_t)bi_reverse(next_code[len]++, len);
    }
}

/* tr_static_init */
static void static_init(void)
{
    if (static_ready) return;
    int n, code, length = 0, dist = 0;
    uint16_t bl_count[MAX_BITS + 1];
    for (code = 0; code < LENGTH_CODES - 1; code++) {
        base_length[code] = length;
        for (n = 0; n < (1 << extra_lbits[code]); n++) length_code_tab[length++] = (uint8_t)code;
    }
    length_code_tab[length - 1] = (uint8_t)code;
    for (code = 0; code < 16; code++) {
        base_dist[code] = dist;
        for (n = 0; n < (1 << extra_dbits[code]); n++) dist_code_tab[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < D_CODES; code++) {
        base_dist[code] = dist << 7;
        for (n = 0; n < (1 << (extra_dbits[code] - 7)); n++) dist_code_tab[256 + dist++] = (uint8_t)code;
    }
    for (n = 0; n <= MAX_BITS; n++) bl_count[n] = 0;
    n = 0;
    while (n <= 143) static_ltree[n++].Len = 8, bl_count[8]++;
    while (n <= 255) static_ltree[n++].Len = 9, bl_count[9]++;
    while (n <= 279) static_ltree[n++].Len = 7, bl_count[7]++;
    while (n <= 287) static_ltree[n++].Len = 8, bl_count[8]++;
    gen_codes(static_ltree, L_CODES + 1, bl_count);
    for (n = 0; n < D_CODES; n++) {
        static_dtree[n].Len = 5;
        static_dtree[n].Code = (uint16_t)bi_reverse((unsigned)n, 5);
    }
    static_ready = 1;
}

static unsigned d_code(unsigned dist) { return dist < 256 ? dist_code_tab[dist] : dist_code_tab[256 + (dist >> 7)]; }

static void init_block(DState *s)
{
    for (int n = 0; n < L_CODES; n++) s->dyn_ltree[n].Freq = 0;
    for (int n = 0; n < D_CODES; n++) s->dyn_dtree[n].Freq = 0;
    for (int n = 0; n < BL_CODES; n++) s->bl_tree[n].Freq = 0;
    s->dyn_ltree[END_BLOCK].Freq = 1;
    s->opt_len = s->static_len = 0;
    s->last_lit = s->matches = 0;
}

#define SMALLEST 1
static int smaller(const ct_data *tree, int n, int m, const uint8_t *depth)
{
    return tree[n].Freq < tree[m].Freq || (tree[n].Freq == tree[m].Freq && depth[n] <= depth[m]);
}

static void pqdownheap(DState *s, ct_data *tree, int k)
{
    int v = s->heap[k];
    int j = k << 1;
    while (j <= s->heap_len) {
        if (j < s->heap_len && smaller(tree, s->heap[j + 1], s->heap[j], s->depth)) j++;
        if (smaller(tree, v, s->heap[j], s->depth)) break;
        s->heap[k] = s->heap[j];
        k = j;
        j <<= 1;
    }
    s->heap[k] = v;
}

static void gen_bitlen(DState *s, tree_desc *desc)
{
    ct_data *tree = desc->dyn_tree;
    int max_code = desc->max_code;
    const ct_data *stree = desc->stat_desc->static_tree;
    const int *extra = desc->stat_desc->extra_bits;
    int base = desc->stat_desc->extra_base;
    int max_length = desc->stat_desc->max_length;
    int h, n, m, bits, xbits, overflow = 0;
    uint16_t f;
    for (bits = 0; bits <= MAX_BITS; bits++) s->bl_count[bits] = 0;
    tree[s->heap[s->heap_max]].Len = 0;
    for (h = s->heap_max + 1; h < HEAP_SIZE; h++) {
        n = s->heap[h];
        bits = tree[tree[n].Dad].Len + 1;
        if (bits > max_length) bits = max_length, overflow++;
        tree[n].Len = (uint16_t)bits;
        if (n > max_code) continue;
        s->bl_count[bits]++;
        xbits = 0;
        if (n >= base) xbits = extra[n - base];
        f = tree[n].Freq;
        s->opt_len += (uint64_t)f * (unsigned)(bits + xbits);
        if (stree) s->static_len += (uint64_t)f * (unsigned)(stree[n].Len + xbits);
    }
    if (overflow == 0) return;
    do {
        bits = max_length - 1;
        while (s->bl_count[bits] == 0) bits--;
        s->bl_count[bits]--;
        s->bl_count[bits + 1] += 2;
        s->bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = max_length; bits != 0; bits--) {
        n = s->bl_count[bits];
        while (n != 0) {
            m = s->heap[--h];
            if (m > max_code) continue;
            if ((unsigned)tree[m].Len != (unsigned)bits) {
                s->opt_len += ((uint64_t)bits - tree[m].Len) * tree[m].Freq;
                tree[m].Len = (uint16_t)bits;
            }
            n--;
        }
    }
}

static void build_tree(DState *s, tree_desc *desc)
{
    ct_data *tree = desc->dyn_tree;
    const ct_data *stree = desc->stat_desc->static_tree;
    int elems = desc->stat_desc->elems;
    int n, m, max_code = -1, node;
    s->heap_len = 0, s->heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (tree[n].Freq != 0) {
            s->heap[++(s->heap_len)] = max_code = n;
            s->depth[n] = 0;
        } else {
            tree[n].Len = 0;
        }
    }
    while (s->heap_len < 2) {
        node = s->heap[++(s->heap_len)] = (max_code < 2 ? ++max_code : 0);
        tree[node].Freq = 1;
        s->depth[node] = 0;
        s->opt_len--;
        if (stree) s->static_len -= stree[node].Len;
    }
    desc->max_code = max_code;
    for (n = s->heap_len / 2; n >= 1; n--) pqdownheap(s, tree, n);
    node = elems;
    do {
        n = s->heap[SMALLEST];
        s->heap[SMALLEST] = s->heap[s->heap_len--];
        pqdownheap(s, tree, SMALLEST);
        m = s->heap[SMALLEST];
        s->heap[--(s->heap_max)] = n;
        s->heap[--(s->heap_max)] = m;
        tree[node].Freq = (uint16_t)(tree[n].Freq + tree[m].Freq);
        s->depth[node] = (uint8_t)((s->depth[n] >= s->depth[m] ? s->depth[n] : s->depth[m]) + 1);
        tree[n].Dad = tree[m].Dad = (uint16_t)node;
        s->heap[SMALLEST] = node++;
        pqdownheap(s, tree, SMALLEST);
    } while (s->heap_len >= 2);
    s->heap[--(s->heap_max)] = s->heap[SMALLEST];
    gen_bitlen(s, desc);
    gen_codes(tree, max_code, s->bl_count);
}

static void scan_tree(DState *s, ct_data *tree, int max_code)
{
    int n, prevlen = -1, curlen, nextlen = tree[0].Len, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    tree[max_code + 1].Len = (uint16_t)0xffff;
    for (n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].Len;
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) s->bl_tree[curlen].Freq += (uint16_t)count;
        else if (curlen != 0) {
            if (curlen != prevlen) s->bl_tree[curlen].Freq++;
            s->bl_tree[REP_3_6].Freq++;
        } else if (count <= 10) s->bl_tree[REPZ_3_10].Freq++;
        else s->bl_tree[REPZ_11_138].Freq++;
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

#define send_code(s, c, tree) send_bits(s, (tree)[c].Code, (tree)[c].Len)

static void send_tree(DState *s, ct_data *tree, int max_code)
{
    int n, prevlen = -1, curlen, nextlen = tree[0].Len, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].Len;
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) {
            do { send_code(s, curlen, s->bl_tree); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) { send_code(s, curlen, s->bl_tree); count--; }
            send_code(s, REP_3_6, s->bl_tree);
            send_bits(s, (unsigned)count - 3, 2);
        } else if (count <= 10) {
            send_code(s, REPZ_3_10, s->bl_tree);
            send_bits(s, (unsigned)count - 3, 3);
        } else {
            send_code(s, REPZ_11_138, s->bl_tree);
            send_bits(s, (unsigned)count - 11, 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

static int build_bl_tree(DState *s)
{
    int max_blindex;
    scan_tree(s, s->dyn_ltree, s->l_desc.max_code);
    scan_tree(s, s->dyn_dtree, s->d_desc.max_code);
    build_tree(s, &s->bl_desc);
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (s->bl_tree[bl_order[max_blindex]].Len != 0) break;
    s->opt_len += 3 * ((uint64_t)max_blindex + 1) + 5 + 5 + 4;
    return max_blindex;
}

static void send_all_trees(DState *s, int lcodes, int dcodes, int blcodes)
{
    send_bits(s, (unsigned)lcodes - 257, 5);
    send_bits(s, (unsigned)dcodes - 1, 5);
    send_bits(s, (unsigned)blcodes - 4, 4);
    for (int rank = 0; rank < blcodes; rank++) send_bits(s, s->bl_tree[bl_order[rank]].Len, 3);
    send_tree(s, s->dyn_ltree, lcodes - 1);
    send_tree(s, s->dyn_dtree, dcodes - 1);
}

static void compress_block(DState *s, const ct_data *ltree, const ct_data *dtree)
{
    unsigned lx = 0, dist, code;
    int lc, extra;
    if (s->last_lit != 0) do {
        dist = s->d_buf[lx];
        lc = s->l_buf[lx++];
        if (dist == 0) {
            send_code(s, lc, ltree);
        } else {
            code = length_code_tab[lc];
            send_code(s, code + LITERALS + 1, ltree);
            extra = extra_lbits[code];
            if (extra != 0) { lc -= base_length[code]; send_bits(s, (unsigned)lc, extra); }
            dist--;
            code = d_code(dist);
            send_code(s, code, dtree);
            extra = extra_dbits[code];
            if (extra != 0) { dist -= (unsigned)base_dist[code]; send_bits(s, dist, extra); }
        }
    } while (lx < s->last_lit);
    send_code(s, END_BLOCK, ltree);
}

static void tr_stored_block(DState *s, const uint8_t *buf, uint64_t stored_len, int last)
{
    send_bits(s, (0u << 1) + (unsigned)last, 3);   /* STORED_BLOCK */
    bi_windup(s);
    put_byte(s, (uint8_t)stored_len);
    put_byte(s, (uint8_t)(stored_len >> 8));
    put_byte(s, (uint8_t)~stored_len);
    put_byte(s, (uint8_t)(~stored_len >> 8));
    for (uint64_t i = 0; i < stored_len; i++) put_byte(s, buf[i]);
}

static void tr_flush_block(DState *s, const uint8_t *buf, uint64_t stored_len, int last)
{
    uint64_t opt_lenb, static_lenb;
    int max_blindex;
    build_tree(s, &s->l_desc);
    build_tree(s, &s->d_desc);
    max_blindex = build_bl_tree(s);
    opt_lenb = (s->opt_len + 3 + 7) >> 3;
    static_lenb = (s->static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if (stored_len + 4 <= opt_lenb && buf != NULL) {
        tr_stored_block(s, buf, stored_len, last);
    } else if (static_lenb == opt_lenb) {
        send_bits(s, (1u << 1) + (unsigned)last, 3);   /* STATIC_TREES */
        compress_block(s, static_ltree, static_dtree);
    } else {
        send_bits(s, (2u << 1) + (unsigned)last, 3);   /* DYN_TREES */
        send_all_trees(s, s->l_desc.max_code + 1, s->d_desc.max_code + 1, max_blindex + 1);
        compress_block(s, s->dyn_ltree, s->dyn_dtree);
    }
    init_block(s);
    if (last) bi_windup(s);
}

/* _tr_tally: 1 when the symbol buffer is full (last_lit == lit_bufsize - 1) */
static int tr_tally_lit(DState *s, uint8_t c)
{
    s->d_buf[s->last_lit] = 0;
    s->l_buf[s->last_lit++] = c;
    s->dyn_ltree[c].Freq++;
    return s->last_lit == LIT_BUFSIZE - 1;
}
static int tr_tally_dist(DState *s, unsigned dist, unsigned len)
{
    s->d_buf[s->last_lit] = (uint16_t)dist;
    s->l_buf[s->last_lit++] = (uint8_t)len;
    dist--;
    s->dyn_ltree[length_code_tab[len] + LITERALS + 1].Freq++;
    s->dyn_dtree[d_code(dist)].Freq++;
    return s->last_lit == LIT_BUFSIZE - 1;
}

#define UPDATE_HASH(h, c) (h = (((h) << HASH_SHIFT) ^ (c)) & HASH_MASK)
#define INSERT_STRING(s, str, match_head)                                              \
    (UPDATE_HASH(s->ins_h, s->window[(str) + (MIN_MATCH - 1)]),                        \
     match_head = s->prev[(str) & WMASK] = s->head[s->ins_h], s->head[s->ins_h] = (uint16_t)(str))

static void fill_window(DState *s)
{
    unsigned n, more;
    do {
        more = (unsigned)(s->window_size - (uint64_t)s->lookahead - (uint64_t)s->strstart);
        if (s->strstart >= WSIZE + MAX_DIST) {
            memcpy(s->window, s->window + WSIZE, WSIZE);
            s->match_start -= WSIZE;
            s->strstart -= WSIZE;
            s->block_start -= (long)WSIZE;
            for (n = 0; n < HASH_SIZE; n++) { unsigned m = s->head[n]; s->head[n] = (uint16_t)(m >= WSIZE ? m - WSIZE : NIL); }
            for (n = 0; n < WSIZE; n++) { unsigned m = s->prev[n]; s->prev[n] = (uint16_t)(m >= WSIZE ? m - WSIZE : NIL); }
            more += WSIZE;
        }
        if (s->avail_in == 0) break;
        n = (unsigned)(s->avail_in < more ? s->avail_in : more);
        memcpy(s->window + s->strstart + s->lookahead, s->next_in, n);
        s->next_in += n;
        s->avail_in -= n;
        s->lookahead += n;
        if (s->lookahead + s->insert >= MIN_MATCH) {
            unsigned str = s->strstart - s->insert;
            s->ins_h = s->window[str];
            UPDATE_HASH(s->ins_h, s->window[str + 1]);
            while (s->insert) {
                UPDATE_HASH(s->ins_h, s->window[str + MIN_MATCH - 1]);
                s->prev[str & WMASK] = s->head[s->ins_h];
                s->head[s->ins_h] = (uint16_t)str;
                str++;
                s->insert--;
                if (s->lookahead + s->insert < MIN_MATCH) break;
            }
        }
    } while (s->lookahead < MIN_LOOKAHEAD && s->avail_in != 0);
    if (s->high_water < s->window_size) {
        uint64_t curr = s->strstart + (uint64_t)s->lookahead, init;
        if (s->high_water < curr) {
            init = s->window_size - curr;
            if (init > WIN_INIT) init = WIN_INIT;
            memset(s->window + curr, 0, (size_t)init);
            s->high_water = curr + init;
        } else if (s->high_water < curr + WIN_INIT) {
            init = curr + WIN_INIT - s->high_water;
            if (init > s->window_size - s->high_water) init = s->window_size - s->high_water;
            memset(s->window + s->high_water, 0, (size_t)init);
            s->high_water += init;
        }
    }
}

static unsigned longest_match(DState *s, unsigned cur_match)
{
    unsigned chain_length = MAX_CHAIN;
    const uint8_t *scan = s->window + s->strstart;
    const uint8_t *match;
    int len;
    int best_len = (int)s->prev_length;
    int nice_match = NICE_LENGTH;
    unsigned limit = s->strstart > MAX_DIST ? s->strstart - MAX_DIST : NIL;
    const uint8_t *strend = s->window + s->strstart + MAX_MATCH;
    uint8_t scan_end1 = scan[best_len - 1];
    uint8_t scan_end = scan[best_len];
    if (s->prev_length >= GOOD_LENGTH) chain_length >>= 2;
    if ((unsigned)nice_match > s->lookahead) nice_match = (int)s->lookahead;
    do {
        match = s->window + cur_match;
        if (match[best_len] != scan_end || match[best_len - 1] != scan_end1 || *match != *scan || *++match != scan[1])
            continue;
        scan += 2, match++;
        do {
        } while (*++scan == *++match && *++scan == *++match && *++scan == *++match && *++scan == *++match &&
                 *++scan == *++match && *++scan == *++match && *++scan == *++match && *++scan == *++match && scan < strend);
        len = MAX_MATCH - (int)(strend - scan);
        scan = strend - MAX_MATCH;
        if (len > best_len) {
            s->match_start = cur_match;
            best_len = len;
            if (len >= nice_match) break;
            scan_end1 = scan[best_len - 1];
            scan_end = scan[best_len];
        }
    } while ((cur_match = s->prev[cur_match & WMASK]) > limit && --chain_length != 0);
    if ((unsigned)best_len <= s->lookahead) return (unsigned)best_len;
    return s->lookahead;
}

#define FLUSH_BLOCK(s, last)                                                                                  \
    do {                                                                                                      \
        tr_flush_block(s, (s)->block_start >= 0L ? (s)->window + (unsigned)(s)->block_start : NULL,           \
                       (uint64_t)((long)(s)->strstart - (s)->block_start), (last));                          \
        (s)->block_start = (long)(s)->strstart;                                                               \
    } while (0)

/* deflate_slow, driven with Z_FINISH over the whole input (the same decisions as Java's
 * Z_NO_FLUSH writes followed by Z_FINISH: fill_window only ever waits for more input) */
static void deflate_slow_finish(DState *s)
{
    unsigned hash_head;
    int bflush;
    for (;;) {
        if (s->lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (s->lookahead == 0) break;
        }
        hash_head = NIL;
        if (s->lookahead >= MIN_MATCH) INSERT_STRING(s, s->strstart, hash_head);
        s->prev_length = s->match_length, s->prev_match = s->match_start;
        s->match_length = MIN_MATCH - 1;
        if (hash_head != NIL && s->prev_length < MAX_LAZY && s->strstart - hash_head <= MAX_DIST) {
            s->match_length = longest_match(s, hash_head);
            if (s->match_length <= 5 && s->match_length == MIN_MATCH && s->strstart - s->match_start > TOO_FAR)
                s->match_length = MIN_MATCH - 1;
        }
        if (s->prev_length >= MIN_MATCH && s->match_length <= s->prev_length) {
            unsigned max_insert = s->strstart + s->lookahead - MIN_MATCH;
            bflush = tr_tally_dist(s, s->strstart - 1 - s->prev_match, s->prev_length - MIN_MATCH);
            s->lookahead -= s->prev_length - 1;
            s->prev_length -= 2;
            do {
                if (++s->strstart <= max_insert) INSERT_STRING(s, s->strstart, hash_head);
            } while (--s->prev_length != 0);
            s->match_available = 0;
            s->match_length = MIN_MATCH - 1;
            s->strstart++;
            if (bflush) FLUSH_BLOCK(s, 0);
        } else if (s->match_available) {
            bflush = tr_tally_lit(s, s->window[s->strstart - 1]);
            if (bflush) FLUSH_BLOCK(s, 0);
            s->strstart++;
            s->lookahead--;
        } else {
            s->match_available = 1;
            s->strstart++;
            s->lookahead--;
        }
    }
    if (s->match_available) {
        (void)tr_tally_lit(s, s->window[s->strstart - 1]);
        s->match_available = 0;
    }
    s->insert = s->strstart < MIN_MATCH - 1 ? s->strstart : MIN_MATCH - 1;
    FLUSH_BLOCK(s, 1);
}

/* raw deflate (zlib 1.2.11, level 6, windowBits -15, memLevel 8, default strategy) of in[0, n)
 * into out; returns its length, or -1 if it does not fit `cap` */
int64_t kpwo_deflate_raw(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap)
{
    static_init();
    DState *s = (DState *)calloc(1, sizeof(DState));
    if (!s) return -1;
    s->next_in = in;
    s->avail_in = n;
    s->window_size = 2ull * WSIZE;
    s->out = out;
    s->cap = cap;
    s->l_desc.dyn_tree = s->dyn_ltree; s->l_desc.stat_desc = &static_l_desc;
    s->d_desc.dyn_tree = s->dyn_dtree; s->d_desc.stat_desc = &static_d_desc;
    s->bl_desc.dyn_tree = s->bl_tree; s->bl_desc.stat_desc = &static_bl_desc;
    init_block(s);
    s->match_length = s->prev_length = MIN_MATCH - 1;
    deflate_slow_finish(s);
    const int64_t r = s->overflow ? -1 : (int64_t)s->op;
    free(s);
    return r;
}

/* CRC-32 (IEEE, reflected 0xEDB88320), as java.util.zip.CRC32 */
uint32_t kpwo_crc32(uint32_t crc, const uint8_t *p, uint64_t n)
{
    static uint32_t T[256];
    static int ready;
    if (!ready) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            T[i] = c;
        }
        ready = 1;
    }
    crc = ~crc;
    for (uint64_t i = 0; i < n; i++) crc = T[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    return ~crc;
}

/* one gzip member as java.util.zip.GZIPOutputStream (Java 8) writes it: the page's
 * CodecFactory.compress output for CompressionCodecName.GZIP */
int64_t kpwo_gzip_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap)
{
    static const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0};
    if (cap < 18) return -1;
    memcpy(out, hdr, 10);
    const int64_t d = kpwo_deflate_raw(in, n, out + 10, cap - 18);
    if (d < 0) return -1;
    const uint32_t crc = kpwo_crc32(0, in, n), isz = (uint32_t)n;
    uint8_t *t = out + 10 + d;
    for (int i = 0; i < 4; i++) t[i] = (uint8_t)(crc >> (8 * i));
    for (int i = 0; i < 4; i++) t[4 + i] = (uint8_t)(isz >> (8 * i));
    return 10 + d + 8;
}

/* worst case of kpwo_gzip_compress (zlib deflateBound for these parameters + the framing) */
uint64_t kpwo_gzip_bound(uint64_t n) { return n + (n >> 12) + (n >> 14) + (n >> 25) + 13 + 18 + 64; }
