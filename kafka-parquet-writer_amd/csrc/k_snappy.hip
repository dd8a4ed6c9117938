// k_snappy.hip — K7: Snappy raw-format page compression, byte-identical to the CPU
// oracle's pinned algorithm (oracle/oracle_snappy.c header: Google Snappy 1.1.2
// CompressFragment).  parquet-mr 1.10.1 SnappyCompressor makes one Snappy.compress call per
// page (data pages and the dictionary page); snappy compresses independent 64 KiB
// fragments with a fresh hash table each, so fragments are the unit of parallelism: one
// wave per fragment; the fragment's uint16 hash table (<= 32 KiB) in LDS, input from L1/L2.
// The wave runs the sequential match loop in lock-step (every lane holds the same scalar
// state); literal copies and match-length extension use all 64 lanes.
#include "kpw_device.h"
#include "kpw_chunk.h"

namespace kpw {

constexpr int SNAPPY_MAX_TABLE = 1 << 14;

// Input bytes are read straight from the page buffer in global memory (L1/L2 resident while
// the wave scans its fragment); only the uint16 hash table (<= 32 KiB) lives in LDS, so five
// fragments run per CU.  `src` is the fragment start; reads never go semantically beyond
// the fragment (positions <= ip_limit+7 or < ip_end), and the page buffer is padded.
struct Src {
    const uint8_t *p;
    __device__ __forceinline__ uint32_t ld32(uint32_t i) const
    {
        const uintptr_t a = (uintptr_t)(p + i);
        const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3) * 8;
        const uint32_t lo = w[0];
        return sh ? ((lo >> sh) | (w[1] << (32 - sh))) : lo;
    }
    __device__ __forceinline__ uint8_t ld8(uint32_t i) const { return p[i]; }
};

__device__ __forceinline__ uint32_t sn_hash(uint32_t bytes, int shift) { return (bytes * 0x1e35a7bdu) >> shift; }

__device__ __forceinline__ uint32_t emit_literal(uint8_t *out, uint32_t op, const Src &in, uint32_t lit, uint32_t len, int lane)
{
    uint32_t n = len - 1;
    if (n < 60) {
        if (lane == 0) out[op] = (uint8_t)(n << 2);
        op += 1;
    } else {
        uint32_t base = op++;
        int count = 0;
        uint32_t nn = n;
        while (nn > 0) { if (lane == 0) out[op] = (uint8_t)(nn & 0xff); op++; nn >>= 8; count++; }
        if (lane == 0) out[base] = (uint8_t)((59 + count) << 2);
    }
    for (uint32_t i = lane; i < len; i += 64) out[op + i] = in.ld8(lit + i);
    return op + len;
}

__device__ __forceinline__ uint32_t emit_copy_lt64(uint8_t *out, uint32_t op, uint32_t offset, uint32_t len, int lane)
{
    if (len < 12 && offset < 2048) {
        if (lane == 0) {
            out[op] = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 8) << 5));
            out[op + 1] = (uint8_t)(offset & 0xff);
        }
        return op + 2;
    }
    if (lane == 0) {
        out[op] = (uint8_t)(2 + ((len - 1) << 2));
        out[op + 1] = (uint8_t)(offset & 0xff);
        out[op + 2] = (uint8_t)(offset >> 8);
    }
    return op + 3;
}

__device__ __forceinline__ uint32_t emit_copy(uint8_t *out, uint32_t op, uint32_t offset, uint32_t len, int lane)
{
    while (len >= 68) { op = emit_copy_lt64(out, op, offset, 64, lane); len -= 64; }
    if (len > 64) { op = emit_copy_lt64(out, op, offset, 60, lane); len -= 60; }
    return emit_copy_lt64(out, op, offset, len, lane);
}

// matching bytes of [s1..) vs [s2..s2_limit): a scalar 4-byte check first (most matches
// are short), then 64 lanes compare 64 bytes per step
__device__ __forceinline__ uint32_t find_match_length(const Src &in, uint32_t s1, uint32_t s2, uint32_t s2_limit, int lane)
{
    if (s2 + 4 <= s2_limit) {
        const uint32_t x = in.ld32(s1) ^ in.ld32(s2);
        if (x) return (uint32_t)(__ffs((int)x) - 1) >> 3;
    }
    uint32_t m = 0;
    for (;;) {
        const uint32_t p2 = s2 + m + lane;
        const bool ok = p2 < s2_limit && in.ld8(s1 + m + lane) == in.ld8(p2);
        const uint64_t bad = __ballot(!ok);
        if (bad) return m + (uint32_t)(__ffsll((long long)bad) - 1);
        m += 64;
    }
}

__global__ void __launch_bounds__(64) k_snappy_frag(SnappyArgs a)
{
    __shared__ uint16_t table[SNAPPY_MAX_TABLE];
    const int lane = threadIdx.x;
    const uint32_t f = blockIdx.x;
    const uint32_t pg = a.frag_page[f];
    const uint32_t fi = a.frag_idx[f];
    const uint64_t plen = a.page_len[pg];
    const uint64_t fstart = (uint64_t)fi * SNAPPY_FRAG;
    const uint32_t n = (uint32_t)((plen - fstart) < SNAPPY_FRAG ? (plen - fstart) : SNAPPY_FRAG);
    const Src in{a.in + a.page_off[pg] + fstart};
    uint32_t tsize = 256;
    while (tsize < SNAPPY_MAX_TABLE && tsize < n) tsize <<= 1;
    for (uint32_t i = lane; i < tsize; i += 64) table[i] = 0;
    __syncthreads();

    uint8_t *out = a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP;
    uint32_t op = 0;
    int shift = 32;
    for (uint32_t t = tsize; t > 1; t >>= 1) shift--;
    const uint32_t ip_end = n;
    uint32_t next_emit = 0;
    uint32_t ip = 0;
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        ip = 1;
        uint32_t next_hash = sn_hash(in.ld32(ip), shift);
        for (;;) {
            uint32_t skip = 32;
            uint32_t next_ip = ip;
            uint32_t candidate;
            for (;;) {
                ip = next_ip;
                const uint32_t hash = next_hash;
                const uint32_t step = skip++ >> 5;
                next_ip = ip + step;
                if (next_ip > ip_limit) goto emit_remainder;
                next_hash = sn_hash(in.ld32(next_ip), shift);
                candidate = table[hash];
                if (lane == 0) table[hash] = (uint16_t)ip;
                if (in.ld32(ip) == in.ld32(candidate)) break;
            }
            op = emit_literal(out, op, in, next_emit, ip - next_emit, lane);
            uint32_t input_lo, input_hi;
            for (;;) {
                const uint32_t base = ip;
                const uint32_t matched = 4 + find_match_length(in, candidate + 4, ip + 4, ip_end, lane);
                ip += matched;
                op = emit_copy(out, op, base - candidate, matched, lane);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                input_lo = in.ld32(ip - 1);         // bytes [ip-1, ip+3)
                input_hi = in.ld32(ip + 3);         // bytes [ip+3, ip+7)
                const uint32_t b1 = (input_lo >> 8) | (input_hi << 24);
                if (lane == 0) table[sn_hash(input_lo, shift)] = (uint16_t)(ip - 1);
                const uint32_t cur_hash = sn_hash(b1, shift);
                candidate = table[cur_hash];
                const uint32_t candidate_bytes = in.ld32(candidate);
                if (lane == 0) table[cur_hash] = (uint16_t)ip;
                if (b1 != candidate_bytes) break;
            }
            next_hash = sn_hash((input_lo >> 16) | (input_hi << 16), shift);
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal(out, op, in, next_emit, ip_end - next_emit, lane);
    if (lane == 0) a.frag_len[f] = op;
}

// per page: compressed size = varint(len) + sum of its fragments
__global__ void __launch_bounds__(KPW_BLOCK) k_snappy_page_sizes(SnappyArgs a, const uint32_t *page_frag0)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    uint64_t carry = 0;
    for (uint32_t b = 0; b < a.npages; b += KPW_BLOCK) {
        const uint32_t p = b + threadIdx.x;
        uint64_t c = 0;
        if (p < a.npages) {
            const uint64_t len = a.page_len[p];
            if (len) {
                uint32_t v = (uint32_t)len;
                c = varint_len32(v);
                const uint32_t nf = (uint32_t)((len + SNAPPY_FRAG - 1) / SNAPPY_FRAG);
                uint64_t fo = c;
                for (uint32_t k = 0; k < nf; k++) {
                    a.frag_coff[page_frag0[p] + k] = fo;
                    fo += a.frag_len[page_frag0[p] + k];
                }
                c = fo;
            }
            a.page_clen[p] = c;
        }
        uint64_t tot;
        const uint64_t ex = block_scan_excl<uint64_t, OpSum64>(c, lds, &tot) + carry;
        if (p < a.npages) a.page_coff[p] = ex;
        carry += tot;
    }
    if (threadIdx.x == 0) a.tot[0] = carry;
}

__global__ void __launch_bounds__(KPW_BLOCK) k_snappy_copy(SnappyArgs a)
{
    const uint32_t f = blockIdx.x;
    const uint32_t pg = a.frag_page[f];
    uint8_t *dst = a.out + a.page_coff[pg];
    if (a.frag_idx[f] == 0 && threadIdx.x == 0) {
        uint32_t v = (uint32_t)a.page_len[pg];
        uint32_t i = 0;
        while (v >= 0x80u) { dst[i++] = (uint8_t)(v | 0x80u); v >>= 7; }
        dst[i] = (uint8_t)v;
    }
    const uint8_t *s = a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP;
    uint8_t *d = dst + a.frag_coff[f];
    const uint32_t n = a.frag_len[f];
    for (uint32_t i = threadIdx.x; i < n; i += KPW_BLOCK) d[i] = s[i];
}

void launch_snappy(const SnappyArgs &a, hipStream_t s)
{
    if (!a.nfrags) return;
    hipLaunchKernelGGL(k_snappy_frag, dim3(a.nfrags), dim3(64), 0, s, a);
}

void launch_snappy_finish(const SnappyArgs &a, const uint32_t *page_frag0, hipStream_t s)
{
    hipLaunchKernelGGL(k_snappy_page_sizes, dim3(1), dim3(KPW_BLOCK), 0, s, a, page_frag0);
    if (a.nfrags) hipLaunchKernelGGL(k_snappy_copy, dim3(a.nfrags), dim3(KPW_BLOCK), 0, s, a);
}

}  // namespace kpw
