// k_snappy.hip — K7: Snappy raw-format page compression, byte-identical to the CPU
// oracle's pinned algorithm (oracle/oracle_snappy.c header: Google Snappy 1.1.2
// CompressFragment).  parquet-mr 1.10.1 SnappyCompressor makes one Snappy.compress call per
// page (data pages and the dictionary page); snappy compresses independent 64 KiB
// fragments with a fresh hash table each, so fragments are the unit of parallelism: one
// wave per fragment; the fragment's uint16 hash table (<= 32 KiB) in LDS, input from L1/L2.
// The wave runs the sequential match loop in lock-step (every lane holds the same scalar
// state); literal copies and match-length extension use all 64 lanes.  The literal search
// is batched: the positions it probes before the next match do not depend on the data
// (ip += skip++ >> 5), so lane k probes the k-th next position; candidates come from the
// table as it was before the batch, or from the nearest earlier probe with the same hash
// (detected by a write/read-back on the table), and only probes up to the first hit are
// committed to the table — the same table states and output as the sequential loop.
#include <cstdlib>
#include <cstring>
#include "kpw_device.h"
#include "kpw_chunk.h"

namespace kpw {

constexpr int SNAPPY_MAX_TABLE = 1 << 14;
#ifndef SNAPPY_SEQ_PROBES
#define SNAPPY_SEQ_PROBES 2     // sequential probes after each match before batching (tests/microbench/snappy_bench.hip)
#endif

// Input bytes are read straight from the page buffer in global memory (L1/L2 resident while
// the wave scans its fragment); only the uint16 hash table (<= 32 KiB) lives in LDS, so five
// fragments run per CU.  `src` is the fragment start; reads never go semantically beyond
// the fragment (positions <= ip_limit+7 or < ip_end), and the page buffer is padded.
typedef const __attribute__((address_space(1))) uint8_t g_u8;
typedef const __attribute__((address_space(1))) uint32_t g_u32;
struct Src {
    g_u8 *p;
    __device__ __forceinline__ uint32_t ld32(uint32_t i) const
    {
        const uintptr_t a = (uintptr_t)(p + i);
        g_u32 *w = (g_u32 *)(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3) * 8;
        const uint32_t lo = w[0];
        return sh ? ((lo >> sh) | (w[1] << (32 - sh))) : lo;
    }
    __device__ __forceinline__ uint8_t ld8(uint32_t i) const { return p[i]; }
};

__device__ __forceinline__ uint32_t sn_hash(uint32_t bytes, int shift) { return (bytes * 0x1e35a7bdu) >> shift; }

__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }

// sum_{x < v} floor(x / 32): the search loop's position after probes with skip values
// s, s+1, ..., s+k-1 is ip + skip_sum(s+k) - skip_sum(s) (snappy: ip += skip++ >> 5)
__device__ __forceinline__ uint32_t skip_sum(uint32_t v)
{
    const uint32_t q = v >> 5, r = v & 31;
    return 16u * q * (q - 1u) + r * q;   // 32 * q(q-1)/2 for the whole blocks of 32, r * q for the rest
}

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
    uint32_t i = lane;
    for (; i + 192 < len; i += 256) {
        const uint8_t b0 = in.ld8(lit + i), b1 = in.ld8(lit + i + 64), b2 = in.ld8(lit + i + 128), b3 = in.ld8(lit + i + 192);
        out[op + i] = b0; out[op + i + 64] = b1; out[op + i + 128] = b2; out[op + i + 192] = b3;
    }
    for (; i < len; i += 64) out[op + i] = in.ld8(lit + i);
    return op + len;
}

// emit_literal for the LDS-table kernel (k_snappy_s / k_snappy_s_rest, the fragments the
// register kernels hand on: mostly incompressible, i.e. one 64 KiB literal)
__device__ __forceinline__ uint32_t emit_literal_wide(uint8_t *out, uint32_t op, const Src &in, uint32_t lit, uint32_t len, int lane)
{
    if (len < 512) return emit_literal(out, op, in, lit, len, lane);
    {
        uint32_t n = len - 1;
        uint32_t base = op++;
        int count = 0;
        while (n > 0) { if (lane == 0) out[op] = (uint8_t)(n & 0xff); op++; n >>= 8; count++; }
        if (lane == 0) out[base] = (uint8_t)((59 + count) << 2);
    }
    {
        // long literal (incompressible stretches): aligned 16-byte loads, 1 KiB per wave step and
        // four steps in flight, bytes stored to their output positions.  Reads stay inside the
        // 16-byte blocks that overlap [lit, lit + len): the page buffer starts 256-aligned and is
        // padded past its last page.
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(1))) v4u g_u4;
        const uintptr_t src0 = (uintptr_t)(in.p + lit), end = src0 + len;
        uint8_t *dst = out + op;
        for (uintptr_t a = (src0 & ~(uintptr_t)15) + 16 * (uintptr_t)lane; a < end; a += 4096) {
            v4u v[4];
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (a + 1024 * u < end) v[u] = *(g_u4 *)(a + 1024 * u);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uintptr_t b0 = a + 1024 * u;
                if (b0 >= end) break;
                const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                if (b0 >= src0 && b0 + 16 <= end) {
#pragma unroll
                    for (int j = 0; j < 16; j++) dst[b0 - src0 + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
                } else {
#pragma unroll
                    for (int j = 0; j < 16; j++)
                        if (b0 + j >= src0 && b0 + j < end) dst[b0 + j - src0] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
                }
            }
        }
        return op + len;
    }
}

// ------------------------------------------------------------------ scalar variant
// All match-loop state is wave-uniform, so it lives in SGPRs: input bytes come through the
// scalar cache (s_load, lgkmcnt) and output bytes leave as lane-parallel byte stores of a
// uniform 64-bit word.  The hot path never waits on vmcnt, so output stores never sit on
// its critical path.  Long matches, long literals and the batched search keep vector code.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16 bytes at 4-aligned wave-uniform addresses a0 and a1 (SMEM; inputs are never written by
// this kernel, and the page buffer is padded past its last page)
__device__ __forceinline__ void sload2(uint64_t a0, uint64_t a1, u32x4 &x, u32x4 &y)
{
    asm volatile("s_load_dwordx4 %0, %2, 0x0\n\t"
                 "s_load_dwordx4 %1, %3, 0x0\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(x), "=&s"(y)
                 : "s"(a0), "s"(a1));
}
__device__ __forceinline__ void sload1(uint64_t a0, u32x4 &x)
{
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(x)
                 : "s"(a0));
}
// 8 bytes starting (addr & 3) bytes into the 16 loaded at addr & ~3
__device__ __forceinline__ uint64_t pick64(const u32x4 &v, uint32_t sh8)
{
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x;
    const uint64_t hi = ((uint64_t)v.w << 32) | v.z;
    return sh8 ? (lo >> sh8) | (hi << (64 - sh8)) : lo;
}

struct SIn {
    uint64_t base;   // absolute address of fragment byte 0
    __device__ __forceinline__ uint64_t ld64(uint32_t p) const
    {
        const uint64_t a = base + p;
        u32x4 v;
        sload1(a & ~3ull, v);
        return pick64(v, (uint32_t)(a & 3) * 8);
    }
    __device__ __forceinline__ void ld64x2(uint32_t p, uint32_t q, uint64_t &vp, uint64_t &vq) const
    {
        const uint64_t a = base + p, b = base + q;
        u32x4 x, y;
        sload2(a & ~3ull, b & ~3ull, x, y);
        vp = pick64(x, (uint32_t)(a & 3) * 8);
        vq = pick64(y, (uint32_t)(b & 3) * 8);
    }
    __device__ __forceinline__ uint32_t ld32(uint32_t p) const { return (uint32_t)ld64(p); }
};

__device__ __forceinline__ uint32_t ufl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// out[op .. op+c) = bytes of the uniform word w (c <= 8), one lane per byte
__device__ __forceinline__ void st_word(uint8_t *out, uint32_t op, uint64_t w, uint32_t c, int lane)
{
    if ((uint32_t)lane < c) out[op + lane] = (uint8_t)(w >> (8 * lane));
}

__device__ __forceinline__ uint32_t emit_copy_lt64_s(uint8_t *out, uint32_t op, uint32_t offset, uint32_t len, int lane)
{
    if (len < 12 && offset < 2048) {
        st_word(out, op, (1 + ((len - 4) << 2) + ((offset >> 8) << 5)) | ((offset & 0xff) << 8), 2, lane);
        return op + 2;
    }
    st_word(out, op, (2 + ((len - 1) << 2)) | ((offset & 0xff) << 8) | ((offset >> 8) << 16), 3, lane);
    return op + 3;
}

__device__ __forceinline__ uint32_t emit_copy_s(uint8_t *out, uint32_t op, uint32_t offset, uint32_t len, int lane)
{
    while (len >= 68) { op = emit_copy_lt64_s(out, op, offset, 64, lane); len -= 64; }
    if (len > 64) { op = emit_copy_lt64_s(out, op, offset, 60, lane); len -= 60; }
    return emit_copy_lt64_s(out, op, offset, len, lane);
}

__device__ __forceinline__ uint32_t emit_literal_s(uint8_t *out, uint32_t op, const SIn &si, const Src &g, uint32_t lit,
                                                   uint32_t len, int lane)
{
    if (len <= 7) {   // tag + bytes in one word
        const uint64_t b = si.ld64(lit) & ((1ull << (8 * len)) - 1);
        st_word(out, op, ((uint64_t)((len - 1) << 2)) | (b << 8), 1 + len, lane);
        return op + 1 + len;
    }
    return emit_literal_wide(out, op, g, lit, len, lane);
}

// matching bytes of [s1..) vs [s2..s2_limit): 8 bytes per scalar step for up to 64 bytes,
// then 64 lanes compare 64 bytes per step (long matches and the fragment tail)
__device__ __forceinline__ uint32_t find_match_length_s(const SIn &si, const Src &g, uint32_t s1, uint32_t s2,
                                                        uint32_t s2_limit, int lane)
{
    uint32_t m = 0;
    while (m < 64 && s2 + m + 8 <= s2_limit) {
        uint64_t a, b;
        si.ld64x2(s1 + m, s2 + m, a, b);
        const uint64_t x = a ^ b;
        if (x) return m + ((uint32_t)__builtin_ctzll(x) >> 3);
        m += 8;
    }
    for (;;) {
        const uint32_t p2 = s2 + m + lane;
        const bool ok = p2 < s2_limit && g.ld8(s1 + m + lane) == g.ld8(p2);
        const uint64_t bad = __ballot(!ok);
        if (bad) return m + (uint32_t)(__ffsll((long long)bad) - 1);
        m += 64;
    }
}

template <int SEQ>
__device__ __forceinline__ void k_snappy_s_body(const SnappyArgs &a)
{
    __shared__ uint16_t table[SNAPPY_MAX_TABLE];
    const int lane = threadIdx.x;
    const uint32_t f = blockIdx.x;
    const uint32_t pg = a.frag_page[f];
    const uint32_t fi = a.frag_idx[f];
    const uint64_t plen = a.page_len[pg];
    const uint64_t fstart = (uint64_t)fi * SNAPPY_FRAG;
    const uint32_t n = (uint32_t)((plen - fstart) < SNAPPY_FRAG ? (plen - fstart) : SNAPPY_FRAG);
    const uint8_t *fbase = a.in + a.page_off[pg] + fstart;
    const Src g{(g_u8 *)fbase};
    const SIn si{(uint64_t)(uintptr_t)fbase};
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
    uint32_t budget = a.s_budget ? a.s_budget : 0xffffffffu;   // search batches + copies before handing over to k_snappy_seg
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        ip = 1;
        for (;;) {
            uint32_t skip = 32;
            uint32_t candidate;
            int nseq = 0;
            if (!--budget) goto handed_on;
            for (;;) {
                if (nseq < SEQ) {
                    nseq++;
                    const uint32_t next_ip = ip + (skip++ >> 5);
                    if (next_ip > ip_limit) goto emit_remainder;
                    const uint32_t cur_s = si.ld32(ip);
                    const uint32_t h = sn_hash(cur_s, shift);
                    candidate = ufl(table[h]);
                    table[h] = (uint16_t)ip;
                    if (cur_s == si.ld32(candidate)) break;
                    ip = next_ip;
                    continue;
                }
                const uint32_t base_f = skip_sum(skip);
                const uint32_t ipk = ip + skip_sum(skip + lane) - base_f;
                const uint32_t ipk1 = ip + skip_sum(skip + lane + 1) - base_f;
                const bool valid = ipk1 <= ip_limit;
                const uint64_t vmask = __ballot(valid);
                const uint32_t cur = valid ? g.ld32(ipk) : 0u;
                const uint32_t h = sn_hash(cur, shift);
                uint32_t old = 0;
                if (valid) old = table[h];
                if (valid) table[h] = (uint16_t)ipk;
                cbar();
                uint32_t chk = ipk;
                if (valid) chk = table[h];
                const uint64_t losers = __ballot(valid && (uint16_t)chk != (uint16_t)ipk);
                uint32_t cand = old;
                uint64_t grp = 0;
                if (losers) {
                    uint64_t L = losers;
                    while (L) {
                        const int leader = __ffsll((long long)L) - 1;
                        const uint32_t hv = __builtin_amdgcn_readlane(h, leader);
                        const uint64_t gm = __ballot(valid && h == hv);
                        if ((gm >> lane) & 1) grp = gm;
                        L &= ~gm;
                    }
                    const uint64_t below = grp & ((1ull << lane) - 1);
                    const int pred = below ? 63 - __clzll((long long)below) : lane;
                    const uint32_t ipp = __shfl(ipk, pred, 64);
                    if (below) cand = ipp;
                }
                const uint64_t hit = __ballot(valid && g.ld32(cand) == cur);
                if (hit) {
                    const int m = __ffsll((long long)hit) - 1;
                    if (valid && lane > m) table[h] = (uint16_t)old;
                    if (losers) {
                        cbar();
                        const uint64_t upto = m == 63 ? ~0ull : ((2ull << m) - 1);
                        if (lane <= m && ((grp & upto) >> lane) <= 1) table[h] = (uint16_t)ipk;
                    }
                    ip = __builtin_amdgcn_readlane(ipk, m);
                    candidate = __builtin_amdgcn_readlane(cand, m);
                    break;
                }
                if (vmask != ~0ull) goto emit_remainder;
                if (!--budget) goto handed_on;
                if (losers && (grp >> lane) <= 1) table[h] = (uint16_t)ipk;
                ip = ip + skip_sum(skip + 64) - base_f;
                skip += 64;
            }
            op = emit_literal_s(out, op, si, g, next_emit, ip - next_emit, lane);
            for (;;) {
                const uint32_t base = ip;
                const uint32_t matched = 4 + find_match_length_s(si, g, candidate + 4, ip + 4, ip_end, lane);
                ip += matched;
                op = emit_copy_s(out, op, base - candidate, matched, lane);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                const uint64_t in8 = si.ld64(ip - 1);   // bytes [ip-1, ip+7)
                const uint32_t input_lo = (uint32_t)in8;
                const uint32_t b1 = (uint32_t)(in8 >> 8);
                table[sn_hash(input_lo, shift)] = (uint16_t)(ip - 1);
                const uint32_t cur_hash = sn_hash(b1, shift);
                candidate = ufl(table[cur_hash]);
                table[cur_hash] = (uint16_t)ip;
                if (b1 != si.ld32(candidate)) break;
            }
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal_wide(out, op, g, next_emit, ip_end - next_emit, lane);
    if (lane == 0) a.frag_len[f] = op;
    return;
handed_on:   // past the budget: k_snappy_seg compresses the fragment (from its start)
    if (lane == 0) a.frag_len[f] = SEG_TODO;
}

// ------------------------------------------------------------------ register-table variant
// The LDS table above caps residency at 5 fragments per CU (32 KiB each) and puts an LDS
// round trip on every probe.  Here the 16384-entry uint16 table lives in 128 VGPRs of the
// wave (4 vectors of 32 dwords; entry h -> register h>>7, lane (h>>1)&63, half h&1), read
// with one indexed v_movrels + v_readlane and written with v_movreld of a lane-selected
// value; the input comes through a 256-byte VGPR window (InWin).  No LDS: occupancy is
// bound by registers only.  The literal search is sequential, so a fragment whose literal
// search runs past VT_ABORT probes (incompressible data) stops and is left to k_snappy_s
// (frag_len = VT_ABORTED), which has the 64-probe batched search.  Same algorithm, same
// output bytes.
constexpr uint32_t VT_ABORTED = 0xffffffffu;
#ifndef VT_ABORT
#define VT_ABORT 128
#endif

// The table is pinned to v128..v255: k_snappy_v is compiled with amdgpu_num_vgpr(128), so
// the register allocator only uses v0..v127, and one asm statement that clobbers
// v128..v255 makes the kernel descriptor allocate all 256 (checked: .vgpr_count 256, no
// scratch; tests/microbench/vtab_probe.hip).  A compiler-visible vector table does not
// work: ext_vector element stores with a runtime index go to scratch, and vector SSA values
// are copied whole at every control-flow merge.  Rows are read/written through VGPR index
// mode (s_set_gpr_idx_on, index = row < 128); volatile asm statements keep program order.
#define VT_CLOBBERS \
    "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", \
    "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", \
    "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", \
    "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", \
    "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", \
    "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", \
    "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", \
    "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", \
    "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", \
    "v254", "v255"

// (gfx950 has no v_movrels/v_movreld: VGPR index mode is the only runtime register index).
// s_set_gpr_idx_on writes M0, hence the M0 clobber (the compiler warns it reserves M0; nothing
// in k_snappy_v keeps a value in M0 across these statements).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ uint32_t vt_row(uint32_t r)
{
    uint32_t x;
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_mov_b32 %0, v128\n\ts_set_gpr_idx_off" : "=v"(x) : "s"(r & 127u) : "m0");
    return x;
}
__device__ __forceinline__ void vt_set_row(uint32_t r, uint32_t v)
{
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(DST)\n\tv_mov_b32 v128, %0\n\ts_set_gpr_idx_off" : : "v"(v), "s"(r & 127u) : "m0");
}
#pragma clang diagnostic pop

// entry h (< 16384) -> row h>>7, lane (h>>1)&63, half h&1
struct VTab {
    uint32_t lane;
    __device__ __forceinline__ void clear() const
    {
        asm volatile("; k_snappy_v: v128..v255 hold the hash table" ::: VT_CLOBBERS);
        for (uint32_t r = 0; r < 128; r++) vt_set_row(r, 0);
    }
    __device__ __forceinline__ uint32_t get(uint32_t h) const
    {
        const uint32_t x = __builtin_amdgcn_readlane(vt_row(h >> 7), (h >> 1) & 63);
        return (h & 1) ? (x >> 16) : (x & 0xffffu);
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const
    {
        const uint32_t r = h >> 7;
        const uint32_t old = vt_row(r);
        const uint32_t sh = (h & 1) * 16;
        const uint32_t nv = (old & ~(0xffffu << sh)) | ((v & 0xffffu) << sh);
        vt_set_row(r, lane == ((h >> 1) & 63) ? nv : old);
    }
    // candidate = table[h]; table[h] = v  (one row read)
    __device__ __forceinline__ uint32_t swap(uint32_t h, uint32_t v) const
    {
        const uint32_t r = h >> 7, L = (h >> 1) & 63, sh = (h & 1) * 16;
        const uint32_t old = vt_row(r);
        const uint32_t x = __builtin_amdgcn_readlane(old, L);
        const uint32_t nv = (old & ~(0xffffu << sh)) | ((v & 0xffffu) << sh);
        vt_set_row(r, lane == L ? nv : old);
        return (x >> sh) & 0xffffu;
    }
};

// 256-byte input window in one VGPR (lane i = dword i), all bookkeeping in 32-bit scalars
// relative to abs0 = (fragment start & ~3); a refill waits for its load right away so no
// later read of the window waits on vmcnt (which the output byte stores share).
struct VWin {
    const uint8_t *abs0;
    uint32_t off0;    // fragment byte 0 = abs0 + off0
    uint32_t A;       // window start (multiple of 4, relative to abs0)
    uint32_t w;
    int lane;
    __device__ __forceinline__ void refill(uint32_t q)
    {
        A = q >= 64 ? ((q - 64) & ~3u) : 0u;
        w = ((const __attribute__((address_space(1))) uint32_t *)(abs0 + A))[lane];
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    }
    // 4 / 8 bytes at fragment position p; `advance` may move the window forward, reads behind
    // it (old candidates) take one scalar load
    __device__ __forceinline__ uint32_t ld32(uint32_t p, const SIn &si, bool advance)
    {
        const uint32_t q = p + off0;
        uint32_t d = q - A;
        if (d > 248) {
            if (!advance || q < A) return si.ld32(p);
            refill(q);
            d = q - A;
        }
        const uint32_t l0 = d >> 2, sh = (d & 3) * 8;
        const uint32_t x = __builtin_amdgcn_readlane(w, l0);
        const uint32_t y = __builtin_amdgcn_readlane(w, l0 + 1);
        return sh ? (x >> sh) | (y << (32 - sh)) : x;
    }
    __device__ __forceinline__ uint64_t ld64(uint32_t p, const SIn &si, bool advance)
    {
        const uint32_t q = p + off0;
        uint32_t d = q - A;
        if (d > 244) {
            if (!advance || q < A) return si.ld64(p);
            refill(q);
            d = q - A;
        }
        const uint32_t l0 = d >> 2, sh = (d & 3) * 8;
        const uint32_t x = __builtin_amdgcn_readlane(w, l0);
        const uint32_t y = __builtin_amdgcn_readlane(w, l0 + 1);
        const uint32_t z = __builtin_amdgcn_readlane(w, l0 + 2);
        const uint64_t lo = ((uint64_t)y << 32) | x;
        return sh ? (lo >> sh) | ((uint64_t)z << (64 - sh)) : lo;
    }
};

__device__ __forceinline__ uint32_t find_match_length_v(VWin &in, const SIn &si, const Src &g, uint32_t s1, uint32_t s2,
                                                        uint32_t s2_limit, int lane)
{
    uint32_t m = 0;
    while (m < 64 && s2 + m + 8 <= s2_limit) {
        const uint64_t b = in.ld64(s2 + m, si, true);
        const uint64_t a = in.ld64(s1 + m, si, false);
        const uint64_t x = a ^ b;
        if (x) return m + ((uint32_t)__builtin_ctzll(x) >> 3);
        m += 8;
    }
    for (;;) {
        const uint32_t p2 = s2 + m + lane;
        const bool ok = p2 < s2_limit && g.ld8(s1 + m + lane) == g.ld8(p2);
        const uint64_t bad = __ballot(!ok);
        if (bad) return m + (uint32_t)(__ffsll((long long)bad) - 1);
        m += 64;
    }
}

__global__ void __launch_bounds__(64, 2) __attribute__((amdgpu_num_vgpr(128))) k_snappy_v(SnappyArgs a)
{
    const int lane = threadIdx.x;
    const uint32_t f = a.order ? a.order[blockIdx.x] : blockIdx.x;
    if (a.v_only_handed_on && a.frag_len[f] != SEG_ABORTED) return;
    if (a.ftime && lane == 0) a.ftime[2 * f] = wall_clock64();
    const uint32_t pg = a.frag_page[f];
    const uint32_t fi = a.frag_idx[f];
    const uint64_t plen = a.page_len[pg];
    const uint64_t fstart = (uint64_t)fi * SNAPPY_FRAG;
    const uint32_t n = (uint32_t)((plen - fstart) < SNAPPY_FRAG ? (plen - fstart) : SNAPPY_FRAG);
    const uint8_t *fbase = a.in + a.page_off[pg] + fstart;
    const Src g{(g_u8 *)fbase};
    const SIn si{(uint64_t)(uintptr_t)fbase};
    VWin in;
    in.abs0 = (const uint8_t *)((uintptr_t)fbase & ~(uintptr_t)3);
    in.off0 = (uint32_t)((uintptr_t)fbase & 3);
    in.lane = lane;
    in.refill(0);
    VTab T;
    T.lane = (uint32_t)lane;
    T.clear();
    uint32_t tsize = 256;
    while (tsize < SNAPPY_MAX_TABLE && tsize < n) tsize <<= 1;

    uint8_t *out = a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP;
    uint32_t op = 0;
    int shift = 32;
    for (uint32_t t = tsize; t > 1; t >>= 1) shift--;
    const uint32_t ip_end = n;
    uint32_t next_emit = 0;
    uint32_t ip = 0;
    uint32_t budget = a.v_budget ? a.v_budget : 0xffffffffu;   // decisions before handing over to k_snappy_seg
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        ip = 1;
        for (;;) {
            uint32_t skip = 32;
            uint32_t candidate;
            for (;;) {
                const uint32_t next_ip = ip + (skip++ >> 5);
                if (next_ip > ip_limit) goto emit_remainder;
                if (!--budget) {
                    if (lane == 0) { a.frag_len[f] = SEG_TODO; if (a.ftime) a.ftime[2 * f + 1] = wall_clock64() | (1ull << 63); }
                    return;
                }
                if (skip > 32 + VT_ABORT) {
                    if (lane == 0) { a.frag_len[f] = VT_ABORTED; if (a.ftime) a.ftime[2 * f + 1] = wall_clock64() | (1ull << 63); }
                    return;
                }
                const uint32_t cur_s = in.ld32(ip, si, true);
                candidate = T.swap(sn_hash(cur_s, shift), ip);
                if (cur_s == in.ld32(candidate, si, false)) break;
                ip = next_ip;
            }
            {
                const uint32_t len = ip - next_emit;
                if (len <= 7) {
                    const uint64_t b = in.ld64(next_emit, si, false) & ((1ull << (8 * len)) - 1);
                    st_word(out, op, ((uint64_t)((len - 1) << 2)) | (b << 8), 1 + len, lane);
                    op += 1 + len;
                } else {
                    op = emit_literal(out, op, g, next_emit, len, lane);
                }
            }
            for (;;) {
                if (!--budget) {
                    if (lane == 0) { a.frag_len[f] = SEG_TODO; if (a.ftime) a.ftime[2 * f + 1] = wall_clock64() | (1ull << 63); }
                    return;
                }
                const uint32_t base = ip;
                const uint32_t matched = 4 + find_match_length_v(in, si, g, candidate + 4, ip + 4, ip_end, lane);
                ip += matched;
                op = emit_copy_s(out, op, base - candidate, matched, lane);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                const uint64_t in8 = in.ld64(ip - 1, si, true);   // bytes [ip-1, ip+7)
                const uint32_t input_lo = (uint32_t)in8;
                const uint32_t b1 = (uint32_t)(in8 >> 8);
                T.put(sn_hash(input_lo, shift), ip - 1);
                candidate = T.swap(sn_hash(b1, shift), ip);
                if (b1 != in.ld32(candidate, si, false)) break;
            }
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal(out, op, g, next_emit, ip_end - next_emit, lane);
    if (lane == 0) { a.frag_len[f] = op; if (a.ftime) a.ftime[2 * f + 1] = wall_clock64(); }
}
// k_snappy_s restricted to the fragments k_snappy_v gave up on
__global__ void __launch_bounds__(64) k_snappy_s_rest(SnappyArgs a)
{
    if (a.frag_len[blockIdx.x] != VT_ABORTED) return;
    k_snappy_s_body<SNAPPY_SEQ_PROBES>(a);
}

// per page: compressed size = [uncompressed level prefix (v2)] + varint(len) + its fragments
// (SnappyCompressor emits nothing for an empty input)
__global__ void __launch_bounds__(KPW_BLOCK) k_snappy_page_sizes(SnappyArgs a, const uint32_t *page_frag0)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    uint64_t carry = 0;
    for (uint32_t b = 0; b < a.npages; b += KPW_BLOCK) {
        const uint32_t p = b + threadIdx.x;
        uint64_t c = 0;
        if (p < a.npages) {
            const uint64_t len = a.page_len[p];
            const uint64_t pre = a.page_pre ? a.page_pre[p] : 0;
            c = pre;
            if (len) {
                uint32_t v = (uint32_t)len;
                uint64_t fo = pre + varint_len32(v);
                // the page's fragments as listed (a page-size probe lists only the pages it
                // needs: the others have none, and their sizes here are not used)
                const uint32_t nf = (p + 1 < a.npages ? page_frag0[p + 1] : a.nfrags) - page_frag0[p];
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
    uint8_t *dst = a.out + a.page_coff[pg] + (a.page_pre ? a.page_pre[pg] : 0);
    if (a.frag_idx[f] == 0 && threadIdx.x == 0) {
        uint32_t v = (uint32_t)a.page_len[pg];
        uint32_t i = 0;
        while (v >= 0x80u) { dst[i++] = (uint8_t)(v | 0x80u); v >>= 7; }
        dst[i] = (uint8_t)v;
    }
    const uint8_t *s = a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP;
    uint8_t *d = a.out + a.page_coff[pg] + a.frag_coff[f];
    block_copy(d, s, a.frag_len[f], threadIdx.x, KPW_BLOCK);
}

// v2: the level bytes that sit in front of a page's values, copied verbatim ahead of its
// compressed stream (ColumnChunkPageWriter.writePageV2: header | rl | dl | compressed data)
__global__ void __launch_bounds__(KPW_BLOCK) k_snappy_prefix(SnappyArgs a)
{
    const uint32_t p = blockIdx.x;
    const uint64_t pre = a.page_pre[p];
    if (!pre) return;
    const uint8_t *src = a.in + a.page_off[p] - pre;
    uint8_t *dst = a.out + a.page_coff[p];
    for (uint64_t i = threadIdx.x; i < pre; i += KPW_BLOCK) dst[i] = src[i];
}

__global__ void k_snappy_seg(SnappyArgs a);

// K7: the segment-parallel kernel (k_snappy_seg.hip) on every fragment, the register-table
// kernel (8 waves/CU, no LDS) on the fragments it hands on, then the batched LDS kernel on the
// fragments that one gives up on (incompressible data: long literal searches).  Without
// seg_scratch the register-table kernel takes every fragment.  Other variants measured against
// these live in tests/microbench/snappy_variants.hip.
void launch_snappy(const SnappyArgs &a, hipStream_t s)
{
    if (!a.nfrags) return;
    if (a.seg_scratch) {
        // register-table kernel with a decision budget, then the batched LDS kernel on the ones it
        // gives up on (incompressible) with a budget of search batches; the fragments that run
        // past either budget (long chains of short matches, or of rare matches between literal
        // stretches: sequential per-match latency) go to the segment-parallel kernel; the ones
        // that hands back (rounds, long copies) to k_snappy_v, then k_snappy_s_rest, unbudgeted
        static const uint32_t vbudget = [] { const char *e = getenv("KPW_SNAPPY_VBUDGET"); return e ? (uint32_t)atoi(e) : 256u; }();
        static const uint32_t sbudget = [] { const char *e = getenv("KPW_SNAPPY_SBUDGET"); return e ? (uint32_t)atoi(e) : 128u; }();
        // A launch of few fragments (a page-size probe's cut pages) is latency-bound: one wave
        // per fragment takes ~40 us per 64 KiB where a segment-parallel workgroup takes ~10, so
        // they all go to the segment kernel first (the same bytes either way)
        static const uint32_t few_max = [] { const char *e = getenv("KPW_SNAPPY_FEW"); return e ? (uint32_t)atoi(e) : 64u; }();
        const bool few = a.nfrags <= few_max;
        SnappyArgs v = a;
        v.v_budget = vbudget;
        if (!few) hipLaunchKernelGGL(k_snappy_v, dim3(a.nfrags), dim3(64), 0, s, v);
        if (!few && vbudget && sbudget) {   // the batched LDS kernel on the incompressible ones, also with a budget
            SnappyArgs r = a;
            r.s_budget = sbudget;
            hipLaunchKernelGGL(k_snappy_s_rest, dim3(a.nfrags), dim3(64), 0, s, r);
        }
        SnappyArgs g = a;   // (the fragment counter is 0: zeroed once, left at 0 by every launch)
        g.order = nullptr;
        g.seg_only_marked = (vbudget && !few) ? 1 : 0;
        hipLaunchKernelGGL(k_snappy_seg, dim3(a.seg_grid), dim3(1024), 0, s, g);
        SnappyArgs b = a;
        b.order = nullptr;
        b.v_only_handed_on = 1;
        hipLaunchKernelGGL(k_snappy_v, dim3(a.nfrags), dim3(64), 0, s, b);
    } else {
        hipLaunchKernelGGL(k_snappy_v, dim3(a.nfrags), dim3(64), 0, s, a);
    }
    hipLaunchKernelGGL(k_snappy_s_rest, dim3(a.nfrags), dim3(64), 0, s, a);
}

void launch_snappy_finish(const SnappyArgs &a, const uint32_t *page_frag0, hipStream_t s)
{
    hipLaunchKernelGGL(k_snappy_page_sizes, dim3(1), dim3(KPW_BLOCK), 0, s, a, page_frag0);
    if (a.nfrags) hipLaunchKernelGGL(k_snappy_copy, dim3(a.nfrags), dim3(KPW_BLOCK), 0, s, a);
    if (a.page_pre && a.npages) hipLaunchKernelGGL(k_snappy_prefix, dim3(a.npages), dim3(KPW_BLOCK), 0, s, a);
}

}  // namespace kpw
