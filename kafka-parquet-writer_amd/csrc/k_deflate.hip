// k_deflate.hip — K7 for CompressionCodecName.GZIP: one gzip member per page, byte-identical to
// what parquet-mr 1.10.1 writes through Hadoop 2.7.7's GzipCodec without the native hadoop
// library (java.util.zip.GZIPOutputStream over zlib's level-6 raw deflate; the restatement and
// its pinning: oracle/oracle_deflate.c).  Reference seam: ParquetFile.java:45 (the codec passed
// through from KafkaProtoParquetWriter.java:484,690-694).
//
// zlib's deflate_slow is a sequential parse, but at level 6 its expensive part is not: every
// position p <= n - 3 is inserted into the hash chains whatever the parse does (the lazy
// evaluation and the insert loop after a match both insert every position), so a position's
// chain = the earlier positions with the same 3-byte hash, and longest_match(p) depends only on
// p and on whether the previous match was >= good_length (chain 128 or 32 candidates); the
// previous match length only filters the result (a candidate counts iff it beats it).  So:
//   k_dfl_prev   per 32 KiB tile of a page, one wave: the previous position with the same hash
//                (64 positions per step: hash peers by ballots, a 32 K-entry head table in LDS);
//   k_dfl_match  per position, in parallel: the chain walk of longest_match for 128 and for 32
//                candidates (first longest, nice_length 128 stops) -> (length, distance);
//   k_dfl_page   per page, one wave: the lazy parse itself (window slides tracked for the
//                stored-block rule), trees.c's block decisions and Huffman trees per 16383
//                symbols, the bit stream, CRC-32 and the gzip framing;
//   k_dfl_sizes / k_dfl_copy   compressed page sizes and offsets, pages packed in order.
#include "kpw_chunk.h"
#include "kpw_device.h"

namespace kpw {

namespace {

constexpr uint32_t D_WSIZE = 32768;
constexpr uint32_t D_MIN_MATCH = 3, D_MAX_MATCH = 258;
constexpr uint32_t D_MIN_LOOKAHEAD = D_MAX_MATCH + D_MIN_MATCH + 1;
constexpr uint32_t D_MAX_DIST = D_WSIZE - D_MIN_LOOKAHEAD;   // 32506
constexpr uint32_t D_TOO_FAR = 4096;
constexpr uint32_t D_GOOD = 8, D_LAZY = 16, D_NICE = 128, D_CHAIN = 128;
constexpr uint32_t D_LIT_BUFSIZE = 16384;
constexpr int L_CODES = 286, D_CODES = 30, BL_CODES = 19, HEAP_SIZE = 2 * L_CODES + 1, MAX_BITS = 15, MAX_BL_BITS = 7;
constexpr int LITERALS = 256, END_BLOCK = 256, LENGTH_CODES = 29;
constexpr int REP_3_6 = 16, REPZ_3_10 = 17, REPZ_11_138 = 18;

__device__ __forceinline__ uint32_t hash3(const uint8_t *b) { return (((uint32_t)b[0] << 10) ^ ((uint32_t)b[1] << 5) ^ b[2]) & 0x7fffu; }

}  // namespace

// ------------------------------------------------------------------ k_dfl_prev
// One wave per (page, 32 KiB tile).  The window [ws, te) runs from MAX_DIST before the tile to
// its end; positions are visited in order 64 at a time.  pdist[q] = q - (the previous position
// with the same hash), 0 when there is none within MAX_DIST or it is position 0 (zlib's NIL).
__global__ void __launch_bounds__(64) k_dfl_prev(DflArgs a)
{
    __shared__ uint16_t head[D_WSIZE];
    const DflTile T = a.tiles[blockIdx.x];
    const DflPage P = a.pages[T.page];
    const uint32_t lane = threadIdx.x;
    const uint8_t *in = a.in + P.off;
    const uint64_t ts = (uint64_t)T.tile * D_WSIZE, te = ts + D_WSIZE < P.len ? ts + D_WSIZE : P.len;
    const uint64_t ws = ts > D_MAX_DIST ? ts - D_MAX_DIST : 0;
    for (uint32_t i = lane; i < D_WSIZE; i += 64) head[i] = 0xffffu;
    __syncthreads();
    const uint64_t last = P.len >= 3 ? P.len - 3 : 0;   // positions <= last are inserted
    const uint64_t lt = (1ull << lane) - 1, gt = lane == 63 ? 0ull : ~((2ull << lane) - 1);
    for (uint64_t q0 = ws; q0 < te; q0 += 64) {
        const uint64_t q = q0 + lane;
        const bool v = P.len >= 3 && q < te && q <= last;
        const uint32_t h = v ? hash3(in + q) : 0;
        uint64_t peers = __ballot(v);
#pragma unroll
        for (int b = 0; b < 15; b++) {
            const bool bit = (h >> b) & 1;
            const uint64_t m = __ballot(v && bit);
            peers &= bit ? m : ~m;
        }
        if (!v) peers = 0;
        const uint64_t lower = peers & lt;
        uint64_t prevq = ~0ull;
        if (v) {
            if (lower) prevq = q0 + (63 - __clzll(lower));
            else {
                const uint32_t e = head[h];
                if (e != 0xffffu) prevq = ws + e;
            }
        }
        __syncthreads();   // every head read of this step before its writes
        if (v && !(peers & gt)) head[h] = (uint16_t)(q - ws);
        if (q >= ts && q < te)
            a.pdist[P.off + q] = (uint16_t)((prevq != ~0ull && prevq != 0 && q - prevq <= D_MAX_DIST) ? q - prevq : 0);
        __syncthreads();
    }
}

// ------------------------------------------------------------------ k_dfl_match
// longest_match for every position p <= n - 3 with a chain head within MAX_DIST: the
// candidates in chain order (newest first, later ones only above limit = p - MAX_DIST), each
// compared over min(258, n - p) bytes; the first longest one wins and one of >= nice_length
// (128, or n - p near the end) stops the walk.  m128 / m32 = length | distance << 9 for chain
// lengths 128 and 32 (the latter after a previous match >= good_length), 0 = no candidate
// longer than MIN_MATCH - 1.
__device__ __forceinline__ uint32_t dfl_len(const uint8_t *in, uint64_t c, uint64_t p, uint32_t maxlen)
{
    uint32_t l = 0;
    while (l + 8 <= maxlen) {
        uint64_t x = 0, y = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) { x |= (uint64_t)in[c + l + k] << (8 * k); y |= (uint64_t)in[p + l + k] << (8 * k); }
        const uint64_t d = x ^ y;
        if (d) return l + ((uint32_t)__builtin_ctzll(d) >> 3);
        l += 8;
    }
    while (l < maxlen && in[c + l] == in[p + l]) l++;
    return l;
}

__global__ void __launch_bounds__(256) k_dfl_match(DflArgs a)
{
    const DflTile T = a.tiles[blockIdx.x / (D_WSIZE / 256)];
    const DflPage P = a.pages[T.page];
    const uint64_t p = (uint64_t)T.tile * D_WSIZE + (blockIdx.x % (D_WSIZE / 256)) * 256 + threadIdx.x;
    if (p >= P.len) return;
    const uint8_t *in = a.in + P.off;
    uint32_t r128 = 0, r32 = 0;
    const uint32_t d0 = (P.len >= 3 && p + 3 <= P.len) ? a.pdist[P.off + p] : 0u;
    if (d0) {
        const uint64_t rem = P.len - p;
        const uint32_t maxlen = rem < D_MAX_MATCH ? (uint32_t)rem : D_MAX_MATCH;
        const uint32_t nice = rem < D_NICE ? (uint32_t)rem : D_NICE;
        const uint64_t limit = p > D_MAX_DIST ? p - D_MAX_DIST : 0;
        uint64_t c = p - d0;
        uint32_t best = D_MIN_MATCH - 1, bdist = 0;
        uint32_t k = 0;
        bool snap = false;
        for (;;) {
            k++;
            const uint32_t l = dfl_len(in, c, p, maxlen);
            if (l > best) {
                best = l;
                bdist = (uint32_t)(p - c);
                if (l >= nice) break;
            }
            if (k == 32) { r32 = best > D_MIN_MATCH - 1 ? best | (bdist << 9) : 0; snap = true; }
            if (k == D_CHAIN) break;
            const uint32_t d = a.pdist[P.off + c];
            if (!d) break;
            c -= d;
            if (c <= limit) break;
        }
        r128 = best > D_MIN_MATCH - 1 ? best | (bdist << 9) : 0;
        if (!snap) r32 = r128;
    }
    a.m128[P.off + p] = r128;
    a.m32[P.off + p] = r32;
}

// ------------------------------------------------------------------ k_dfl_page
// trees.c state of one page (LDS); the tables tr_static_init builds are built per workgroup
struct CtData { uint16_t fc, dl; };   // Freq/Code, Dad/Len unions

struct DflTrees {
    CtData dyn_ltree[HEAP_SIZE], dyn_dtree[2 * D_CODES + 1], bl_tree[2 * BL_CODES + 1];
    CtData static_ltree[L_CODES + 2], static_dtree[D_CODES];
    uint16_t bl_count[MAX_BITS + 1];
    int16_t heap[2 * L_CODES + 1];
    uint8_t depth[2 * L_CODES + 1];
    uint8_t dist_code[512], length_code[256];
    int16_t base_length[LENGTH_CODES], base_dist[D_CODES];
    int heap_len, heap_max;
    int l_max, d_max, bl_max;
    uint64_t opt_len, static_len;
    // bit writer
    uint64_t bi_buf;
    int bi_valid;
    uint64_t op;          // output bytes written (from the page's deflate start)
    uint32_t last_lit;
};

__constant__ int8_t c_extra_lbits[LENGTH_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ int8_t c_extra_dbits[D_CODES] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ int8_t c_extra_blbits[BL_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
__constant__ uint8_t c_bl_order[BL_CODES] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

namespace {

__device__ uint32_t bi_reverse(uint32_t code, int len)
{
    uint32_t res = 0;
    do { res |= code & 1; code >>= 1, res <<= 1; } while (--len > 0);
    return res >> 1;
}

__device__ void gen_codes(CtData *tree, int max_code, const uint16_t *bl_count)
{
    uint16_t next_code[MAX_BITS + 1];
    uint32_t code = 0;
    for (int bits = 1; bits <= MAX_BITS; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; n++) {
        const int len = tree[n].dl;
        if (len == 0) continue;
        tree[n].fc = (uint16_t)bi_reverse(next_code[len]++, len);
    }
}

__device__ void static_init(DflTrees &S)
{
    int n, code, length = 0, dist = 0;
    uint16_t blc[MAX_BITS + 1];
    for (code = 0; code < LENGTH_CODES - 1; code++) {
        S.base_length[code] = (int16_t)length;
        for (n = 0; n < (1 << c_extra_lbits[code]); n++) S.length_code[length++] = (uint8_t)code;
    }
    S.length_code[length - 1] = (uint8_t)code;
    for (code = 0; code < 16; code++) {
        S.base_dist[code] = (int16_t)dist;
        for (n = 0; n < (1 << c_extra_dbits[code]); n++) S.dist_code[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < D_CODES; code++) {
        S.base_dist[code] = (int16_t)(dist << 7);
        for (n = 0; n < (1 << (c_extra_dbits[code] - 7)); n++) S.dist_code[256 + dist++] = (uint8_t)code;
    }
    for (n = 0; n <= MAX_BITS; n++) blc[n] = 0;
    n = 0;
    while (n <= 143) S.static_ltree[n++].dl = 8, blc[8]++;
    while (n <= 255) S.static_ltree[n++].dl = 9, blc[9]++;
    while (n <= 279) S.static_ltree[n++].dl = 7, blc[7]++;
    while (n <= 287) S.static_ltree[n++].dl = 8, blc[8]++;
    gen_codes(S.static_ltree, L_CODES + 1, blc);
    for (n = 0; n < D_CODES; n++) {
        S.static_dtree[n].dl = 5;
        S.static_dtree[n].fc = (uint16_t)bi_reverse((uint32_t)n, 5);
    }
}

__device__ __forceinline__ uint32_t d_code(const DflTrees &S, uint32_t dist) { return dist < 256 ? S.dist_code[dist] : S.dist_code[256 + (dist >> 7)]; }

__device__ void init_block(DflTrees &S)
{
    for (int n = 0; n < L_CODES; n++) S.dyn_ltree[n].fc = 0;
    for (int n = 0; n < D_CODES; n++) S.dyn_dtree[n].fc = 0;
    for (int n = 0; n < BL_CODES; n++) S.bl_tree[n].fc = 0;
    S.dyn_ltree[END_BLOCK].fc = 1;
    S.opt_len = S.static_len = 0;
    S.last_lit = 0;
}

__device__ __forceinline__ bool smaller(const CtData *tree, int n, int m, const uint8_t *depth)
{
    return tree[n].fc < tree[m].fc || (tree[n].fc == tree[m].fc && depth[n] <= depth[m]);
}

__device__ void pqdownheap(DflTrees &S, const CtData *tree, int k)
{
    const int v = S.heap[k];
    int j = k << 1;
    while (j <= S.heap_len) {
        if (j < S.heap_len && smaller(tree, S.heap[j + 1], S.heap[j], S.depth)) j++;
        if (smaller(tree, v, S.heap[j], S.depth)) break;
        S.heap[k] = S.heap[j];
        k = j;
        j <<= 1;
    }
    S.heap[k] = (int16_t)v;
}

// which: 0 literal/length, 1 distance, 2 bit-length tree
__device__ void gen_bitlen(DflTrees &S, CtData *tree, int max_code, int which)
{
    const CtData *stree = which == 0 ? S.static_ltree : which == 1 ? S.static_dtree : nullptr;
    const int8_t *extra = which == 0 ? c_extra_lbits : which == 1 ? c_extra_dbits : c_extra_blbits;
    const int base = which == 0 ? LITERALS + 1 : 0;
    const int max_length = which == 2 ? MAX_BL_BITS : MAX_BITS;
    int h, n, m, bits, xbits, overflow = 0;
    for (bits = 0; bits <= MAX_BITS; bits++) S.bl_count[bits] = 0;
    tree[S.heap[S.heap_max]].dl = 0;
    for (h = S.heap_max + 1; h < HEAP_SIZE; h++) {
        n = S.heap[h];
        bits = tree[tree[n].dl].dl + 1;
        if (bits > max_length) bits = max_length, overflow++;
        tree[n].dl = (uint16_t)bits;
        if (n > max_code) continue;
        S.bl_count[bits]++;
        xbits = 0;
        if (n >= base) xbits = extra[n - base];
        const uint16_t f = tree[n].fc;
        S.opt_len += (uint64_t)f * (uint32_t)(bits + xbits);
        if (stree) S.static_len += (uint64_t)f * (uint32_t)(stree[n].dl + xbits);
    }
    if (overflow == 0) return;
    do {
        bits = max_length - 1;
        while (S.bl_count[bits] == 0) bits--;
        S.bl_count[bits]--;
        S.bl_count[bits + 1] += 2;
        S.bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = max_length; bits != 0; bits--) {
        n = S.bl_count[bits];
        while (n != 0) {
            m = S.heap[--h];
            if (m > max_code) continue;
            if ((uint32_t)tree[m].dl != (uint32_t)bits) {
                S.opt_len += ((uint64_t)bits - tree[m].dl) * tree[m].fc;
                tree[m].dl = (uint16_t)bits;
            }
            n--;
        }
    }
}

__device__ int build_tree(DflTrees &S, CtData *tree, int which)
{
    const CtData *stree = which == 0 ? S.static_ltree : which == 1 ? S.static_dtree : nullptr;
    const int elems = which == 0 ? L_CODES : which == 1 ? D_CODES : BL_CODES;
    int n, m, max_code = -1, node;
    S.heap_len = 0, S.heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (tree[n].fc != 0) {
            S.heap[++(S.heap_len)] = (int16_t)(max_code = n);
            S.depth[n] = 0;
        } else {
            tree[n].dl = 0;
        }
    }
    while (S.heap_len < 2) {
        node = max_code < 2 ? ++max_code : 0;
        S.heap[++(S.heap_len)] = (int16_t)node;
        tree[node].fc = 1;
        S.depth[node] = 0;
        S.opt_len--;
        if (stree) S.static_len -= stree[node].dl;
    }
    for (n = S.heap_len / 2; n >= 1; n--) pqdownheap(S, tree, n);
    node = elems;
    do {
        n = S.heap[1];
        S.heap[1] = S.heap[S.heap_len--];
        pqdownheap(S, tree, 1);
        m = S.heap[1];
        S.heap[--(S.heap_max)] = (int16_t)n;
        S.heap[--(S.heap_max)] = (int16_t)m;
        tree[node].fc = (uint16_t)(tree[n].fc + tree[m].fc);
        S.depth[node] = (uint8_t)((S.depth[n] >= S.depth[m] ? S.depth[n] : S.depth[m]) + 1);
        tree[n].dl = tree[m].dl = (uint16_t)node;
        S.heap[1] = (int16_t)(node++);
        pqdownheap(S, tree, 1);
    } while (S.heap_len >= 2);
    S.heap[--(S.heap_max)] = S.heap[1];
    gen_bitlen(S, tree, max_code, which);
    gen_codes(tree, max_code, S.bl_count);
    return max_code;
}

__device__ void scan_tree(DflTrees &S, CtData *tree, int max_code)
{
    int n, prevlen = -1, curlen, nextlen = tree[0].dl, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    tree[max_code + 1].dl = (uint16_t)0xffff;
    for (n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].dl;
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) S.bl_tree[curlen].fc += (uint16_t)count;
        else if (curlen != 0) {
            if (curlen != prevlen) S.bl_tree[curlen].fc++;
            S.bl_tree[REP_3_6].fc++;
        } else if (count <= 10) S.bl_tree[REPZ_3_10].fc++;
        else S.bl_tree[REPZ_11_138].fc++;
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

__device__ __forceinline__ void put_byte(DflTrees &S, uint8_t *out, uint64_t cap, uint8_t b)
{
    if (S.op < cap) out[S.op] = b;
    S.op++;
}
__device__ __forceinline__ void send_bits(DflTrees &S, uint8_t *out, uint64_t cap, uint32_t value, int length)
{
    S.bi_buf |= (uint64_t)value << S.bi_valid;
    S.bi_valid += length;
    while (S.bi_valid >= 16) {
        put_byte(S, out, cap, (uint8_t)S.bi_buf);
        put_byte(S, out, cap, (uint8_t)(S.bi_buf >> 8));
        S.bi_buf >>= 16;
        S.bi_valid -= 16;
    }
}
__device__ void bi_windup(DflTrees &S, uint8_t *out, uint64_t cap)
{
    if (S.bi_valid > 8) { put_byte(S, out, cap, (uint8_t)S.bi_buf); put_byte(S, out, cap, (uint8_t)(S.bi_buf >> 8)); }
    else if (S.bi_valid > 0) put_byte(S, out, cap, (uint8_t)S.bi_buf);
    S.bi_buf = 0;
    S.bi_valid = 0;
}

__device__ void send_tree(DflTrees &S, uint8_t *out, uint64_t cap, const CtData *tree, int max_code)
{
    int n, prevlen = -1, curlen, nextlen = tree[0].dl, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[n + 1].dl;
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) {
            do { send_bits(S, out, cap, S.bl_tree[curlen].fc, S.bl_tree[curlen].dl); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) { send_bits(S, out, cap, S.bl_tree[curlen].fc, S.bl_tree[curlen].dl); count--; }
            send_bits(S, out, cap, S.bl_tree[REP_3_6].fc, S.bl_tree[REP_3_6].dl);
            send_bits(S, out, cap, (uint32_t)count - 3, 2);
        } else if (count <= 10) {
            send_bits(S, out, cap, S.bl_tree[REPZ_3_10].fc, S.bl_tree[REPZ_3_10].dl);
            send_bits(S, out, cap, (uint32_t)count - 3, 3);
        } else {
            send_bits(S, out, cap, S.bl_tree[REPZ_11_138].fc, S.bl_tree[REPZ_11_138].dl);
            send_bits(S, out, cap, (uint32_t)count - 11, 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

// symbols of the current block: lit (dist 0) or (length - 3, distance) packed lc | dist << 8
__device__ void compress_block(DflTrees &S, uint8_t *out, uint64_t cap, const uint32_t *sym, const CtData *ltree,
                               const CtData *dtree)
{
    for (uint32_t lx = 0; lx < S.last_lit; lx++) {
        const uint32_t sv = sym[lx];
        uint32_t dist = sv >> 8;
        int lc = (int)(sv & 0xff);
        if (dist == 0) {
            send_bits(S, out, cap, ltree[lc].fc, ltree[lc].dl);
        } else {
            uint32_t code = S.length_code[lc];
            send_bits(S, out, cap, ltree[code + LITERALS + 1].fc, ltree[code + LITERALS + 1].dl);
            int extra = c_extra_lbits[code];
            if (extra != 0) { lc -= S.base_length[code]; send_bits(S, out, cap, (uint32_t)lc, extra); }
            dist--;
            code = d_code(S, dist);
            send_bits(S, out, cap, dtree[code].fc, dtree[code].dl);
            extra = c_extra_dbits[code];
            if (extra != 0) { dist -= (uint32_t)S.base_dist[code]; send_bits(S, out, cap, dist, extra); }
        }
    }
    send_bits(S, out, cap, ltree[END_BLOCK].fc, ltree[END_BLOCK].dl);
}

// _tr_flush_block (zlib 1.2.11, level > 0); buf: the block's bytes when they are still in
// zlib's window (block_start >= 0), else nullptr
__device__ void flush_block(DflTrees &S, uint8_t *out, uint64_t cap, const uint32_t *sym, const uint8_t *buf,
                            uint64_t stored_len, int last)
{
    S.l_max = build_tree(S, S.dyn_ltree, 0);
    S.d_max = build_tree(S, S.dyn_dtree, 1);
    scan_tree(S, S.dyn_ltree, S.l_max);
    scan_tree(S, S.dyn_dtree, S.d_max);
    S.bl_max = build_tree(S, S.bl_tree, 2);
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (S.bl_tree[c_bl_order[max_blindex]].dl != 0) break;
    S.opt_len += 3 * ((uint64_t)max_blindex + 1) + 5 + 5 + 4;
    uint64_t opt_lenb = (S.opt_len + 3 + 7) >> 3;
    const uint64_t static_lenb = (S.static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if (stored_len + 4 <= opt_lenb && buf) {
        send_bits(S, out, cap, (0u << 1) + (uint32_t)last, 3);
        bi_windup(S, out, cap);
        put_byte(S, out, cap, (uint8_t)stored_len);
        put_byte(S, out, cap, (uint8_t)(stored_len >> 8));
        put_byte(S, out, cap, (uint8_t)~stored_len);
        put_byte(S, out, cap, (uint8_t)(~stored_len >> 8));
        for (uint64_t i = 0; i < stored_len; i++) put_byte(S, out, cap, buf[i]);
    } else if (static_lenb == opt_lenb) {
        send_bits(S, out, cap, (1u << 1) + (uint32_t)last, 3);
        compress_block(S, out, cap, sym, S.static_ltree, S.static_dtree);
    } else {
        send_bits(S, out, cap, (2u << 1) + (uint32_t)last, 3);
        const int lcodes = S.l_max + 1, dcodes = S.d_max + 1, blcodes = max_blindex + 1;
        send_bits(S, out, cap, (uint32_t)lcodes - 257, 5);
        send_bits(S, out, cap, (uint32_t)dcodes - 1, 5);
        send_bits(S, out, cap, (uint32_t)blcodes - 4, 4);
        for (int rank = 0; rank < blcodes; rank++) send_bits(S, out, cap, S.bl_tree[c_bl_order[rank]].dl, 3);
        send_tree(S, out, cap, S.dyn_ltree, lcodes - 1);
        send_tree(S, out, cap, S.dyn_dtree, dcodes - 1);
        compress_block(S, out, cap, sym, S.dyn_ltree, S.dyn_dtree);
    }
    init_block(S);
    if (last) bi_windup(S, out, cap);
}

// CRC-32 (IEEE reflected), java.util.zip.CRC32; zlib's crc32_combine for the lanes' pieces
__device__ uint32_t gf2_times(const uint32_t *mat, uint32_t vec)
{
    uint32_t sum = 0;
    while (vec) {
        if (vec & 1) sum ^= *mat;
        vec >>= 1;
        mat++;
    }
    return sum;
}
__device__ void gf2_square(uint32_t *square, const uint32_t *mat)
{
    for (int n = 0; n < 32; n++) square[n] = gf2_times(mat, mat[n]);
}
__device__ uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2)
{
    uint32_t even[32], odd[32];
    if (len2 == 0) return crc1;
    odd[0] = 0xedb88320u;
    uint32_t row = 1;
    for (int n = 1; n < 32; n++) { odd[n] = row; row <<= 1; }
    gf2_square(even, odd);
    gf2_square(odd, even);
    do {
        gf2_square(even, odd);
        if (len2 & 1) crc1 = gf2_times(even, crc1);
        len2 >>= 1;
        if (len2 == 0) break;
        gf2_square(odd, even);
        if (len2 & 1) crc1 = gf2_times(odd, crc1);
        len2 >>= 1;
    } while (len2 != 0);
    return crc1 ^ crc2;
}

}  // namespace

// One wave per page.  Thread 0 runs deflate_slow over the precomputed matches (the symbols of
// the open block in the page's symbol slots), trees.c per block and the bit stream; then the
// wave computes the CRC-32 in 64 pieces and writes the framing.  Output: the page's gzip member
// at a.gz + P.slot (capacity P.cap), its length in a.glen[page index].
__global__ void __launch_bounds__(64) k_dfl_page(DflArgs a)
{
    __shared__ DflTrees S;
    __shared__ uint32_t crc_t[256];
    __shared__ uint32_t lcrc[64];
    const DflPage P = a.pages[blockIdx.x];
    const uint32_t lane = threadIdx.x;
    const uint8_t *in = a.in + P.off;
    uint8_t *gz = a.gz + P.slot;
    for (uint32_t i = lane; i < 256; i += 64) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_t[i] = c;
    }
    if (lane == 0) {
        static_init(S);
        init_block(S);
        S.bi_buf = 0;
        S.bi_valid = 0;
        S.op = 0;
        const uint64_t n = P.len, cap = P.cap - 18;
        uint8_t *out = gz + 10;
        uint32_t *sym = a.sym + P.off;   // a block's symbols: at most one per input byte
        uint64_t p = 0, base = 0, block_start = 0;
        uint32_t prev_length, match_length = D_MIN_MATCH - 1, prev_match = 0, match_start = 0;
        bool match_available = false;
        auto tally = [&](uint32_t v, uint32_t lc, uint32_t dist) -> bool {
            sym[S.last_lit++] = lc | (dist << 8);
            if (dist == 0) S.dyn_ltree[lc].fc++;
            else {
                S.dyn_ltree[S.length_code[lc] + LITERALS + 1].fc++;
                S.dyn_dtree[d_code(S, dist - 1)].fc++;
            }
            (void)v;
            return S.last_lit == D_LIT_BUFSIZE - 1;
        };
        auto flush = [&](int last) {
            const bool in_window = block_start >= base;   // zlib: block_start >= 0 after the slides
            flush_block(S, out, cap, sym, in_window ? in + block_start : nullptr, p - block_start, last);
            block_start = p;
        };
        for (;;) {
            uint64_t wend = base + 2 * D_WSIZE < n ? base + 2 * D_WSIZE : n;
            uint64_t lookahead = wend - p;
            if (lookahead < D_MIN_LOOKAHEAD) {   // fill_window: slide once the window is nearly full
                if (p - base >= D_WSIZE + D_MAX_DIST) base += D_WSIZE;
                wend = base + 2 * D_WSIZE < n ? base + 2 * D_WSIZE : n;
                lookahead = wend - p;
                if (lookahead == 0) break;
            }
            uint64_t hash_head = 0;   // NIL
            if (lookahead >= D_MIN_MATCH) {
                const uint32_t d = a.pdist[P.off + p];
                if (d) hash_head = p - d;
            }
            prev_length = match_length, prev_match = match_start;
            match_length = D_MIN_MATCH - 1;
            if (hash_head != 0 && prev_length < D_LAZY && p - hash_head <= D_MAX_DIST) {
                const uint32_t r = prev_length >= D_GOOD ? a.m32[P.off + p] : a.m128[P.off + p];
                const uint32_t rl = r & 0x1ff;
                if (r && rl > prev_length) {
                    match_length = rl;
                    match_start = (uint32_t)(p - (r >> 9));
                } else {
                    match_length = prev_length;   // longest_match returns best_len unchanged
                }
                if (match_length == D_MIN_MATCH && p - match_start > D_TOO_FAR) match_length = D_MIN_MATCH - 1;
            }
            if (prev_length >= D_MIN_MATCH && match_length <= prev_length) {
                const bool bf = tally(0, prev_length - D_MIN_MATCH, (uint32_t)(p - 1 - prev_match));
                p += prev_length - 1;
                match_available = false;
                match_length = D_MIN_MATCH - 1;
                if (bf) flush(0);
            } else if (match_available) {
                const bool bf = tally(0, in[p - 1], 0);
                if (bf) flush(0);
                p++;
            } else {
                match_available = true;
                p++;
            }
        }
        if (match_available) (void)tally(0, in[p - 1], 0);
        flush(1);
        a.glen[blockIdx.x] = S.op <= cap ? S.op : ~0ull;
    }
    __syncthreads();
    // CRC-32 of the page: 64 contiguous pieces, combined in order
    const uint64_t per = (P.len + 63) / 64, b0 = lane * per < P.len ? lane * per : P.len;
    const uint64_t b1 = b0 + per < P.len ? b0 + per : P.len;
    uint32_t c = 0xffffffffu;
    for (uint64_t i = b0; i < b1; i++) c = crc_t[(c ^ in[i]) & 0xff] ^ (c >> 8);
    lcrc[lane] = ~c;
    __syncthreads();
    if (lane == 0) {
        uint32_t crc = 0;
        for (uint32_t k = 0; k < 64; k++) {
            const uint64_t s0 = k * per < P.len ? k * per : P.len;
            const uint64_t s1 = s0 + per < P.len ? s0 + per : P.len;
            crc = crc32_combine(crc, lcrc[k], s1 - s0);
        }
        const uint64_t dl = a.glen[blockIdx.x];
        if (dl != ~0ull) {
            const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0};
            for (int i = 0; i < 10; i++) gz[i] = hdr[i];
            uint8_t *t = gz + 10 + dl;
            const uint32_t isz = (uint32_t)P.len;
            for (int i = 0; i < 4; i++) t[i] = (uint8_t)(crc >> (8 * i));
            for (int i = 0; i < 4; i++) t[4 + i] = (uint8_t)(isz >> (8 * i));
            a.glen[blockIdx.x] = dl + 18;
        }
    }
}

// page slot p: clen = [v2 level prefix] + its gzip member (pages not listed: the prefix only);
// exclusive offsets, total in tot[0]; an overflowing member sets *overflow = 1
__global__ void __launch_bounds__(KPW_BLOCK) k_dfl_sizes(DflArgs a)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    uint64_t carry = 0;
    bool bad = false;
    for (uint32_t b = 0; b < a.nslots; b += KPW_BLOCK) {
        const uint32_t p = b + threadIdx.x;
        uint64_t c = 0;
        if (p < a.nslots) {
            c = a.page_pre ? a.page_pre[p] : 0;
            const int32_t k = a.slot_page[p];
            if (k >= 0) {
                const uint64_t g = a.glen[k];
                if (g == ~0ull) bad = true; else c += g;
            }
            a.page_clen[p] = c;
        }
        uint64_t tot;
        const uint64_t ex = block_scan_excl<uint64_t, OpSum64>(c, lds, &tot) + carry;
        if (p < a.nslots) a.page_coff[p] = ex;
        carry += tot;
    }
    if (bad) *a.overflow = 1;   // (benign race: every writer stores 1)
    __syncthreads();
    if (threadIdx.x == 0) a.tot[0] = carry;
}

__global__ void __launch_bounds__(KPW_BLOCK) k_dfl_copy(DflArgs a)
{
    const uint32_t p = blockIdx.x;
    const uint64_t pre = a.page_pre ? a.page_pre[p] : 0;
    uint8_t *dst = a.out + a.page_coff[p];
    if (pre) block_copy(dst, a.in + a.page_off[p] - pre, (uint32_t)pre, threadIdx.x, KPW_BLOCK);
    const int32_t k = a.slot_page[p];
    if (k < 0 || a.glen[k] == ~0ull) return;
    const uint64_t g = a.glen[k];
    const uint8_t *src = a.gz + a.pages[k].slot;
    for (uint64_t o = 0; o < g; o += 1u << 20) {
        const uint32_t m = (uint32_t)(g - o < (1u << 20) ? g - o : (1u << 20));
        block_copy(dst + pre + o, src + o, m, threadIdx.x, KPW_BLOCK);
    }
}

void launch_deflate(const DflArgs &a, uint32_t npages_listed, uint32_t ntiles, hipStream_t s)
{
    if (ntiles) {
        hipLaunchKernelGGL(k_dfl_prev, dim3(ntiles), dim3(64), 0, s, a);
        hipLaunchKernelGGL(k_dfl_match, dim3(ntiles * (D_WSIZE / 256)), dim3(256), 0, s, a);
    }
    if (npages_listed) hipLaunchKernelGGL(k_dfl_page, dim3(npages_listed), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_dfl_sizes, dim3(1), dim3(KPW_BLOCK), 0, s, a);
    if (a.nslots) hipLaunchKernelGGL(k_dfl_copy, dim3(a.nslots), dim3(KPW_BLOCK), 0, s, a);
}

}  // namespace kpw
