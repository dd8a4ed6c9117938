// snappy_variants.hip — K7 kernel variants kept for A/B measurement (test infrastructure,
// NOT part of libkpw_gpu.so).  Included by snappy_bench.hip after the production
// kafka-parquet-writer_amd/csrc/k_snappy.hip, whose helpers (Src, SIn, emit_*, VTab, ...)
// they share.  Every variant produces the same bytes as the production kernels (the
// pinned Snappy 1.1.2 algorithm); the bench checks each against the CPU oracle.
namespace kpw {

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

template <int SEQ>
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
    const Src in{(g_u8 *)(a.in + a.page_off[pg] + fstart)};
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
        for (;;) {
            // ---- literal search: the first SEQ probes one at a time (short literals between
            // nearby matches are the common case on compressible pages), then 64 probe
            // positions per step (see header comment)
            uint32_t skip = 32;
            uint32_t candidate;
            int nseq = 0;
            uint32_t cur_s = SEQ > 0 ? in.ld32(ip) : 0u;
            for (;;) {
                if (nseq < SEQ) {
                    nseq++;
                    const uint32_t h = sn_hash(cur_s, shift);
                    const uint32_t next_ip = ip + (skip++ >> 5);
                    if (next_ip > ip_limit) goto emit_remainder;
                    const uint32_t nxt = in.ld32(next_ip);   // issued before the dependent table/candidate loads
                    candidate = table[h];
                    table[h] = (uint16_t)ip;
                    if (cur_s == in.ld32(candidate)) break;
                    ip = next_ip;
                    cur_s = nxt;
                    continue;
                }
                const uint32_t base_f = skip_sum(skip);
                const uint32_t ipk = ip + skip_sum(skip + lane) - base_f;         // lane k's probe position
                const uint32_t ipk1 = ip + skip_sum(skip + lane + 1) - base_f;    // its next_ip
                const bool valid = ipk1 <= ip_limit;
                const uint64_t vmask = __ballot(valid);
                const uint32_t cur = valid ? in.ld32(ipk) : 0u;
                const uint32_t h = sn_hash(cur, shift);
                // compiler barriers (cbar): the read-back must really be issued after every
                // lane's store (no store-to-load forwarding), and the lane-ordered store loops
                // below must not be merged into one store whose same-address winner would be
                // unspecified.  LDS operations of one wave execute in program order.
                uint32_t old = 0;
                if (valid) old = table[h];
                if (valid) table[h] = (uint16_t)ipk;
                cbar();
                uint32_t chk = ipk;
                if (valid) chk = table[h];
                const uint64_t losers = __ballot(valid && (uint16_t)chk != (uint16_t)ipk);
                uint32_t cand = old;
                uint64_t grp = 0;   // lanes sharing my hash (only when some hash repeats)
                if (losers) {
                    // several probes share a hash: group them (one ballot per repeated hash);
                    // a probe's candidate is then the nearest earlier probe of its group
                    uint64_t L = losers;
                    while (L) {
                        const int leader = __ffsll((long long)L) - 1;
                        const uint32_t hv = __builtin_amdgcn_readlane(h, leader);
                        const uint64_t g = __ballot(valid && h == hv);
                        if ((g >> lane) & 1) grp = g;
                        L &= ~g;
                    }
                    const uint64_t below = grp & ((1ull << lane) - 1);
                    const int pred = below ? 63 - __clzll((long long)below) : lane;
                    const uint32_t ipp = __shfl(ipk, pred, 64);
                    if (below) cand = ipp;
                }
                const uint64_t hit = __ballot(valid && in.ld32(cand) == cur);
                if (hit) {
                    const int m = __ffsll((long long)hit) - 1;
                    // probes after the hit never ran: put their slots back; among the probes
                    // up to the hit, the last of each hash group holds the slot
                    if (valid && lane > m) table[h] = (uint16_t)old;
                    if (losers) {
                        cbar();
                        const uint64_t upto = m == 63 ? ~0ull : ((2ull << m) - 1);
                        if (lane <= m && ((grp & upto) >> lane) <= 1) table[h] = (uint16_t)ipk;
                    }
                    ip = __shfl(ipk, m, 64);
                    candidate = __shfl(cand, m, 64);
                    break;
                }
                if (vmask != ~0ull) goto emit_remainder;   // the first invalid probe ends the fragment
                if (losers && (grp >> lane) <= 1) table[h] = (uint16_t)ipk;   // last of each group wins
                ip = ip + skip_sum(skip + 64) - base_f;
                skip += 64;
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
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal(out, op, in, next_emit, ip_end - next_emit, lane);
    if (lane == 0) a.frag_len[f] = op;
}

// ------------------------------------------------------------------ register-window variant
// The match loop above pays a global-memory round trip (plus the wait for earlier byte
// stores, which share vmcnt) for nearly every step.  Here the 64 lanes hold a 256-byte
// window of the fragment input, one dword each: reads near ip (and the usual nearby match
// candidate) are two v_readlane; the window is refilled with one coalesced load when ip
// moves past it.  Output bytes accumulate in a second 256-byte register window flushed with
// one coalesced dword store.  The algorithm (and so every output byte) is unchanged.
typedef __attribute__((address_space(1))) uint32_t g_u32w;

__device__ __forceinline__ uint32_t funnel(uint32_t x, uint32_t y, uint32_t sh) { return sh ? (x >> sh) | (y << (32 - sh)) : x; }

struct InWin {
    uintptr_t base;   // absolute address of fragment byte 0
    uintptr_t lo;     // lowest address read (base & ~3: inside the page buffer)
    uintptr_t A;      // 4-aligned absolute address of the window start
    uint32_t w;       // bytes [A + 4 lane, A + 4 lane + 4)
    int lane;
    // called with all 64 lanes active (wave-uniform control flow only)
    __device__ __forceinline__ void refill(uintptr_t abs)
    {
        A = abs >= lo + 64 ? ((abs - 64) & ~(uintptr_t)3) : lo;
        w = *(g_u32 *)(A + 4 * (uintptr_t)lane);
    }
    __device__ __forceinline__ uint32_t gld32(uintptr_t abs) const
    {
        const uintptr_t a = abs & ~(uintptr_t)3;
        const uint32_t x = a >= lo ? *(g_u32 *)a : 0u;
        const uint32_t y = *(g_u32 *)(a + 4);
        return funnel(x, y, (uint32_t)(abs & 3) * 8);
    }
    // 4 bytes at fragment position p (wave-uniform p)
    __device__ __forceinline__ uint32_t ld32(uint32_t p)
    {
        const uintptr_t abs = base + p;
        uintptr_t d = abs - A;
        if (d > 248) {
            if (abs < A) return gld32(abs);   // behind the window: one global read
            refill(abs);
            d = abs - A;
        }
        const uint32_t l0 = (uint32_t)d >> 2;
        const uint32_t x = __builtin_amdgcn_readlane(w, l0);
        const uint32_t y = __builtin_amdgcn_readlane(w, l0 + 1);
        return funnel(x, y, ((uint32_t)d & 3) * 8);
    }
};

struct OutWin {
    g_u32w *out;
    uint32_t ob;      // output position of the window start (multiple of 256)
    uint32_t w;
    int lane;
    __device__ __forceinline__ void flush() { out[(ob >> 2) + lane] = w; w = 0; ob += 256; }
    __device__ __forceinline__ void put8(uint32_t op, uint32_t b)
    {
        if (op - ob >= 256) flush();
        const uint32_t d = op - ob;
        if ((uint32_t)lane == (d >> 2)) w |= (b & 0xffu) << ((d & 3) * 8);
    }
};

// output [op, op+len) = input [lit, lit+len)
__device__ __forceinline__ void copy_lit(OutWin &ow, InWin &in, uint32_t op, uint32_t lit, uint32_t len)
{
    const int lane = ow.lane;
    uint32_t done = 0;
    while (done < len) {
        const uint32_t opc = op + done;
        if (opc - ow.ob >= 256) ow.flush();
        const uint32_t room = ow.ob + 256 - opc;
        const uint32_t c = (len - done) < room ? (len - done) : room;
        const int32_t q0 = (int32_t)(ow.ob + 4 * lane);
        const bool touch = q0 + 4 > (int32_t)opc && q0 < (int32_t)(opc + c);
        const intptr_t src = (intptr_t)lit + (intptr_t)done + (intptr_t)q0 - (intptr_t)opc;   // >= -3
        const uintptr_t sabs = in.base + src;
        const uintptr_t d = sabs - in.A;
        const uint64_t need = __ballot(touch);
        const uint64_t ok = __ballot(touch && d <= 248);
        uint32_t v = 0;
        if (ok == need) {
            const uint32_t l0 = touch ? (uint32_t)d >> 2 : 0u;
            const uint32_t x = __shfl(in.w, (int)l0, 64);
            const uint32_t y = __shfl(in.w, (int)l0 + 1 < 64 ? (int)l0 + 1 : 63, 64);
            v = funnel(x, y, ((uint32_t)d & 3) * 8);
        } else if (touch) {
            v = in.gld32(sabs);
        }
        if (touch) {
            const int lo_k = (int32_t)opc > q0 ? (int32_t)opc - q0 : 0;
            const int hi_k = (int32_t)(opc + c) - q0 < 4 ? (int32_t)(opc + c) - q0 : 4;
            const uint32_t mhi = hi_k >= 4 ? 0xffffffffu : ((1u << (8 * hi_k)) - 1);
            const uint32_t mlo = (0xffffffffu << (8 * lo_k));
            ow.w |= v & mhi & mlo;
        }
        done += c;
    }
}

__device__ __forceinline__ uint32_t emit_literal_w(OutWin &ow, InWin &in, uint32_t op, uint32_t lit, uint32_t len)
{
    const uint32_t n = len - 1;
    if (n < 60) {
        ow.put8(op++, n << 2);
    } else {
        int count = 0;
        for (uint32_t nn = n; nn > 0; nn >>= 8) count++;
        ow.put8(op++, (uint32_t)(59 + count) << 2);
        for (uint32_t nn = n; nn > 0; nn >>= 8) ow.put8(op++, nn & 0xff);
    }
    copy_lit(ow, in, op, lit, len);
    return op + len;
}

__device__ __forceinline__ uint32_t emit_copy_lt64_w(OutWin &ow, uint32_t op, uint32_t offset, uint32_t len)
{
    if (len < 12 && offset < 2048) {
        ow.put8(op, 1 + ((len - 4) << 2) + ((offset >> 8) << 5));
        ow.put8(op + 1, offset & 0xff);
        return op + 2;
    }
    ow.put8(op, 2 + ((len - 1) << 2));
    ow.put8(op + 1, offset & 0xff);
    ow.put8(op + 2, offset >> 8);
    return op + 3;
}

__device__ __forceinline__ uint32_t emit_copy_w(OutWin &ow, uint32_t op, uint32_t offset, uint32_t len)
{
    while (len >= 68) { op = emit_copy_lt64_w(ow, op, offset, 64); len -= 64; }
    if (len > 64) { op = emit_copy_lt64_w(ow, op, offset, 60); len -= 60; }
    return emit_copy_lt64_w(ow, op, offset, len);
}

// matching bytes of [s1..) vs [s2..s2_limit): up to 16 bytes through the window, then 64
// lanes compare 64 bytes per step from global memory (long matches only)
__device__ __forceinline__ uint32_t find_match_length_w(InWin &in, const Src &g, uint32_t s1, uint32_t s2, uint32_t s2_limit, int lane)
{
    uint32_t m = 0;
#pragma unroll 1
    for (int k = 0; k < 4 && s2 + m + 4 <= s2_limit; k++) {
        const uint32_t a = in.ld32(s1 + m);
        const uint32_t b = in.ld32(s2 + m);
        const uint32_t x = a ^ b;
        if (x) return m + ((uint32_t)(__ffs((int)x) - 1) >> 3);
        m += 4;
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
__global__ void __launch_bounds__(64) k_snappy_win(SnappyArgs a)
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
    InWin in;
    in.base = (uintptr_t)fbase;
    in.lo = in.base & ~(uintptr_t)3;
    in.lane = lane;
    in.refill(in.base);
    OutWin ow;
    ow.out = (g_u32w *)(a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP);
    ow.ob = 0;
    ow.w = 0;
    ow.lane = lane;
    uint32_t tsize = 256;
    while (tsize < SNAPPY_MAX_TABLE && tsize < n) tsize <<= 1;
    for (uint32_t i = lane; i < tsize; i += 64) table[i] = 0;
    __syncthreads();

    uint32_t op = 0;
    int shift = 32;
    for (uint32_t t = tsize; t > 1; t >>= 1) shift--;
    const uint32_t ip_end = n;
    uint32_t next_emit = 0;
    uint32_t ip = 0;
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        ip = 1;
        for (;;) {
            uint32_t skip = 32;
            uint32_t candidate;
            int nseq = 0;
            uint32_t cur_s = SEQ > 0 ? in.ld32(ip) : 0u;
            for (;;) {
                if (nseq < SEQ) {
                    nseq++;
                    const uint32_t h = sn_hash(cur_s, shift);
                    const uint32_t next_ip = ip + (skip++ >> 5);
                    if (next_ip > ip_limit) goto emit_remainder;
                    candidate = table[h];
                    table[h] = (uint16_t)ip;
                    const uint32_t cb = in.ld32(candidate);
                    if (cur_s == cb) break;
                    ip = next_ip;
                    cur_s = in.ld32(ip);
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
                    ip = __shfl(ipk, m, 64);
                    candidate = __shfl(cand, m, 64);
                    break;
                }
                if (vmask != ~0ull) goto emit_remainder;
                if (losers && (grp >> lane) <= 1) table[h] = (uint16_t)ipk;
                ip = ip + skip_sum(skip + 64) - base_f;
                skip += 64;
            }
            ip = __builtin_amdgcn_readfirstlane(ip);
            candidate = __builtin_amdgcn_readfirstlane(candidate);
            op = emit_literal_w(ow, in, op, next_emit, ip - next_emit);
            uint32_t input_lo, input_hi;
            for (;;) {
                const uint32_t base = ip;
                const uint32_t matched = 4 + find_match_length_w(in, g, candidate + 4, ip + 4, ip_end, lane);
                ip += matched;
                op = emit_copy_w(ow, op, base - candidate, matched);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                input_lo = in.ld32(ip - 1);
                input_hi = in.ld32(ip + 3);
                const uint32_t b1 = (input_lo >> 8) | (input_hi << 24);
                table[sn_hash(input_lo, shift)] = (uint16_t)(ip - 1);
                const uint32_t cur_hash = sn_hash(b1, shift);
                candidate = __builtin_amdgcn_readfirstlane((uint32_t)table[cur_hash]);
                table[cur_hash] = (uint16_t)ip;
                const uint32_t candidate_bytes = in.ld32(candidate);
                if (b1 != candidate_bytes) break;
            }
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal_w(ow, in, op, next_emit, ip_end - next_emit);
    if (op > ow.ob) ow.out[(ow.ob >> 2) + lane] = ow.w;
    if (lane == 0) a.frag_len[f] = op;
}

template <int SEQ>
__global__ void __launch_bounds__(64) k_snappy_s(SnappyArgs a)
{
    k_snappy_s_body<SEQ>(a);
}

// ------------------------------------------------------------------ scalar + SGPR window
// k_snappy_s plus a 64-byte window of the input around ip held in SGPRs (one
// s_load_dwordx16): on typical pages the match candidate is a few bytes behind ip (the
// previous record), so the match-length compare, the post-match reads, the candidate check
// and the literal bytes all come from the window; it is reloaded when ip moves past it, and
// reads outside it (far candidates) take one direct scalar load.
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

struct SWin {
    uint64_t base;    // absolute address of fragment byte 0
    uint64_t lo;      // lowest address read (base & ~3)
    uint64_t A;       // 4-aligned absolute address of the window start
    u32x16 w;
    __device__ __forceinline__ void load(uint32_t p)
    {
        const uint64_t a = base + p;
        A = a >= lo + 16 ? ((a - 16) & ~3ull) : lo;
        asm volatile("s_load_dwordx16 %0, %1, 0x0\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&s"(w)
                     : "s"(A));
    }
    // 8 bytes at fragment position p when they lie inside the window (o <= 52)
    __device__ __forceinline__ bool has(uint32_t p) const { return base + p - A <= 52; }
    __device__ __forceinline__ uint64_t rd(uint32_t p) const
    {
        const uint32_t o = (uint32_t)(base + p - A);
        const uint32_t d = o >> 2, sh = (o & 3) * 8;
        const uint64_t x = ((uint64_t)w[d + 1] << 32) | w[d];
        const uint64_t y = w[d + 2];
        return sh ? (x >> sh) | (y << (64 - sh)) : x;
    }
    // 8 bytes at p: window, else reload when ahead, else one scalar load
    __device__ __forceinline__ uint64_t ld64(uint32_t p, const SIn &si)
    {
        if (has(p)) return rd(p);
        if (base + p >= A) { load(p); return rd(p); }
        return si.ld64(p);
    }
    // 8 bytes at p without moving the window (candidates behind ip)
    __device__ __forceinline__ uint64_t peek64(uint32_t p, const SIn &si) const { return has(p) ? rd(p) : si.ld64(p); }
};

__device__ __forceinline__ uint32_t find_match_length_w(SWin &W, const SIn &si, const Src &g, uint32_t s1, uint32_t s2,
                                                        uint32_t s2_limit, int lane)
{
    uint32_t m = 0;
    while (m < 64 && s2 + m + 8 <= s2_limit) {
        const uint64_t a = W.peek64(s1 + m, si);
        const uint64_t b = W.ld64(s2 + m, si);
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
__global__ void __launch_bounds__(64) k_snappy_w(SnappyArgs a)
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
    SWin W;
    W.base = (uint64_t)(uintptr_t)fbase;
    W.lo = W.base & ~3ull;
    W.load(0);
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
        for (;;) {
            uint32_t skip = 32;
            uint32_t candidate;
            int nseq = 0;
            for (;;) {
                if (nseq < SEQ) {
                    nseq++;
                    const uint32_t next_ip = ip + (skip++ >> 5);
                    if (next_ip > ip_limit) goto emit_remainder;
                    const uint32_t cur_s = (uint32_t)W.ld64(ip, si);
                    const uint32_t h = sn_hash(cur_s, shift);
                    candidate = ufl(table[h]);
                    table[h] = (uint16_t)ip;
                    if (cur_s == (uint32_t)W.peek64(candidate, si)) break;
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
                if (losers && (grp >> lane) <= 1) table[h] = (uint16_t)ipk;
                ip = ip + skip_sum(skip + 64) - base_f;
                skip += 64;
            }
            {
                const uint32_t len = ip - next_emit;
                if (len <= 7) {
                    const uint64_t b = W.peek64(next_emit, si) & ((1ull << (8 * len)) - 1);
                    st_word(out, op, ((uint64_t)((len - 1) << 2)) | (b << 8), 1 + len, lane);
                    op += 1 + len;
                } else {
                    op = emit_literal(out, op, g, next_emit, len, lane);
                }
            }
            for (;;) {
                const uint32_t base = ip;
                const uint32_t matched = 4 + find_match_length_w(W, si, g, candidate + 4, ip + 4, ip_end, lane);
                ip += matched;
                op = emit_copy_s(out, op, base - candidate, matched, lane);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                const uint64_t in8 = W.ld64(ip - 1, si);   // bytes [ip-1, ip+7)
                const uint32_t input_lo = (uint32_t)in8;
                const uint32_t b1 = (uint32_t)(in8 >> 8);
                table[sn_hash(input_lo, shift)] = (uint16_t)(ip - 1);
                const uint32_t cur_hash = sn_hash(b1, shift);
                candidate = ufl(table[cur_hash]);
                table[cur_hash] = (uint16_t)ip;
                if (b1 != (uint32_t)W.peek64(candidate, si)) break;
            }
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal(out, op, g, next_emit, ip_end - next_emit, lane);
    if (lane == 0) a.frag_len[f] = op;
}

// ------------------------------------------------------------------ register-resident variant
// k_snappy_v still reads the input through memory: every match candidate outside its 256-byte
// window (a third of them on timestamp-like pages) is a scalar load from L2, and those round
// trips (~2000 cycles per match-loop step measured on C2's INT64 page) are the whole cost.
// Here the wave holds the entire 64 KiB fragment in its 256 AGPRs (dword d of the fragment
// at a[d >> 6], lane d & 63) next to the 128-VGPR hash table, so the match loop touches no
// memory except output stores (which nothing waits on).  512 registers per lane: one wave
// per SIMD, four fragments per CU.  AGPR rows are read/written through the same VGPR index
// mode as the table (checked on gfx950: tests/microbench/agpr_probe.hip).  Same algorithm,
// same output bytes; long literals and matches beyond 64 bytes still use lane-parallel
// global reads, and fragments with long literal searches still go to k_snappy_s_rest.
#define RA_CLOBBERS \
    "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", \
    "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", \
    "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", \
    "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", \
    "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", \
    "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", \
    "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", \
    "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", \
    "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", \
    "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", \
    "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", \
    "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", \
    "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", \
    "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207", "a208", "a209", "a210", "a211", "a212", "a213", \
    "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223", "a224", "a225", "a226", "a227", \
    "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239", "a240", "a241", \
    "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255"

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ uint32_t ra_row(uint32_t r)
{
    uint32_t x;
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_accvgpr_read_b32 %0, a0\n\ts_set_gpr_idx_off" : "=v"(x) : "s"(r & 255u) : "m0");
    return x;
}
__device__ __forceinline__ void ra_set_row(uint32_t r, uint32_t v)
{
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(DST)\n\tv_accvgpr_write_b32 a0, %0\n\ts_set_gpr_idx_off" : : "v"(v), "s"(r & 255u) : "m0");
}
#pragma clang diagnostic pop

// the fragment, register-resident: byte p at row p >> 8, lane (p >> 2) & 63, byte p & 3
struct RIn {
    // fragment bytes [0, n) from global memory (fbase need not be aligned; the page buffer
    // is padded past its end), 16 rows per batch of loads
    __device__ __forceinline__ void load(const uint8_t *fbase, uint32_t n, int lane) const
    {
        const uintptr_t fb = (uintptr_t)fbase;
        g_u32 *w = (g_u32 *)(fb & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(fb & 3) * 8;
        const uint32_t rows = (n + 255) >> 8;
        for (uint32_t r0 = 0; r0 < rows; r0 += 16) {
            uint32_t lo[16], hi[16];
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint32_t i = (r0 + j) * 64 + lane;
                lo[j] = r0 + j < rows ? w[i] : 0u;
                hi[j] = r0 + j < rows ? w[i + 1] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (r0 + j < rows) ra_set_row(r0 + j, sh ? (lo[j] >> sh) | (hi[j] << (32 - sh)) : lo[j]);
        }
    }
    __device__ __forceinline__ uint32_t ld32(uint32_t p) const
    {
        const uint32_t d = p >> 2, l = d & 63, sh = (p & 3) * 8;
        const uint32_t row = ra_row(d >> 6);
        const uint32_t x = __builtin_amdgcn_readlane(row, l);
        if (!sh) return x;
        const uint32_t y = l < 63 ? __builtin_amdgcn_readlane(row, l + 1) : __builtin_amdgcn_readlane(ra_row((d >> 6) + 1), 0);
        return (x >> sh) | (y << (32 - sh));
    }
    __device__ __forceinline__ uint64_t ld64(uint32_t p) const
    {
        const uint32_t d = p >> 2, l = d & 63, sh = (p & 3) * 8;
        const uint32_t row = ra_row(d >> 6);
        uint32_t x, y, z;
        if (l < 62) {
            x = __builtin_amdgcn_readlane(row, l);
            y = __builtin_amdgcn_readlane(row, l + 1);
            z = __builtin_amdgcn_readlane(row, l + 2);
        } else {
            const uint32_t row2 = ra_row((d >> 6) + 1);
            x = __builtin_amdgcn_readlane(row, l);
            y = l == 62 ? __builtin_amdgcn_readlane(row, 63) : __builtin_amdgcn_readlane(row2, 0);
            z = __builtin_amdgcn_readlane(row2, l == 62 ? 0 : 1);
        }
        const uint64_t lo = ((uint64_t)y << 32) | x;
        return sh ? (lo >> sh) | ((uint64_t)z << (64 - sh)) : lo;
    }
};

__device__ __forceinline__ uint32_t find_match_length_r(const RIn &in, const Src &g, uint32_t s1, uint32_t s2, uint32_t s2_limit,
                                                        int lane)
{
    uint32_t m = 0;
    while (m < 64 && s2 + m + 8 <= s2_limit) {
        const uint64_t x = in.ld64(s1 + m) ^ in.ld64(s2 + m);
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

__global__ void __launch_bounds__(64, 1) __attribute__((amdgpu_num_vgpr(128))) k_snappy_r(SnappyArgs a)
{
    const int lane = threadIdx.x;
    const uint32_t f = blockIdx.x;
    const uint32_t pg = a.frag_page[f];
    const uint32_t fi = a.frag_idx[f];
    const uint64_t plen = a.page_len[pg];
    const uint64_t fstart = (uint64_t)fi * SNAPPY_FRAG;
    const uint32_t n = (uint32_t)((plen - fstart) < SNAPPY_FRAG ? (plen - fstart) : SNAPPY_FRAG);
    const uint8_t *fbase = a.in + a.page_off[pg] + fstart;
    const Src g{(g_u8 *)fbase};
    asm volatile("; k_snappy_r: a0..a255 hold the fragment" ::: RA_CLOBBERS);
    RIn in;
    in.load(fbase, n, lane);
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
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        ip = 1;
        for (;;) {
            uint32_t skip = 32;
            uint32_t candidate;
            for (;;) {
                const uint32_t next_ip = ip + (skip++ >> 5);
                if (next_ip > ip_limit) goto emit_remainder;
                if (skip > 32 + VT_ABORT) {
                    if (lane == 0) a.frag_len[f] = VT_ABORTED;
                    return;
                }
                const uint32_t cur_s = in.ld32(ip);
                candidate = T.swap(sn_hash(cur_s, shift), ip);
                if (cur_s == in.ld32(candidate)) break;
                ip = next_ip;
            }
            {
                const uint32_t len = ip - next_emit;
                if (len <= 7) {
                    const uint64_t b = in.ld64(next_emit) & ((1ull << (8 * len)) - 1);
                    st_word(out, op, ((uint64_t)((len - 1) << 2)) | (b << 8), 1 + len, lane);
                    op += 1 + len;
                } else {
                    op = emit_literal(out, op, g, next_emit, len, lane);
                }
            }
            for (;;) {
                const uint32_t base = ip;
                const uint32_t matched = 4 + find_match_length_r(in, g, candidate + 4, ip + 4, ip_end, lane);
                ip += matched;
                op = emit_copy_s(out, op, base - candidate, matched, lane);
                next_emit = ip;
                if (ip >= ip_limit) goto emit_remainder;
                const uint64_t in8 = in.ld64(ip - 1);   // bytes [ip-1, ip+7)
                const uint32_t input_lo = (uint32_t)in8;
                const uint32_t b1 = (uint32_t)(in8 >> 8);
                T.put(sn_hash(input_lo, shift), ip - 1);
                candidate = T.swap(sn_hash(b1, shift), ip);
                if (b1 != in.ld32(candidate)) break;
            }
            ++ip;
        }
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal(out, op, g, next_emit, ip_end - next_emit, lane);
    if (lane == 0) a.frag_len[f] = op;
}

// ------------------------------------------------------------------ register-resident, scheduled
// k_snappy_r measured ~1400 cycles per match-loop step for a lone wave: hipcc's structurized
// control flow and branchy byte extraction cost ~150-300 instructions per step.  The common
// steps (probe, short literal, match of < 64 bytes, continuation check) are written here as
// one scheduled scalar program (about 40-60 instructions per step); the rare ones (long
// literal, long match / fragment end, remainder, abort) leave the program and run in C++.
// Scratch registers are fixed and clobbered: s56..s91, v100..v105.  Wait states: a VGPR
// written by a VALU is read by v_readlane only after s_nop 1 (the string is not padded by
// hipcc); every SGPR a VALU writes (v_readlane) is read by SALU only; the string ends with
// s_nop 4 so no compiler VMEM reads an SGPR a readlane just wrote.
enum : uint32_t { RA_SEARCH = 0, RA_COPY = 1, RA_REMAINDER = 2, RA_ABORT = 3, RA_LITERAL = 4, RA_LONGMATCH = 5 };

// s60 = 4 bytes at fragment position P (register P; s63..s65 scratch)
#define RA_LD32(P, L)                                                        \
    "s_lshr_b32 s63, " P ", 8\n\t"                                          \
    "s_bfe_u32 s64, " P ", 0x60002\n\t"                                     \
    "s_set_gpr_idx_on s63, gpr_idx(SRC0)\n\t"                                \
    "v_accvgpr_read_b32 v100, a0\n\t"                                        \
    "s_set_gpr_idx_off\n\t"                                                  \
    "s_nop 1\n\t"                                                            \
    "v_readlane_b32 s60, v100, s64\n\t"                                      \
    "s_cmp_eq_u32 s64, 63\n\t"                                               \
    "s_cbranch_scc1 ld32w_" L "%=\n\t"                                       \
    "s_add_u32 s64, s64, 1\n\t"                                              \
    "v_readlane_b32 s61, v100, s64\n\t"                                      \
    "s_branch ld32d_" L "%=\n"                                               \
    "ld32w_" L "%=:\n\t"                                                     \
    "s_add_u32 s63, s63, 1\n\t"                                              \
    "s_and_b32 s63, s63, 255\n\t"                                            \
    "s_set_gpr_idx_on s63, gpr_idx(SRC0)\n\t"                                \
    "v_accvgpr_read_b32 v100, a0\n\t"                                        \
    "s_set_gpr_idx_off\n\t"                                                  \
    "s_nop 1\n\t"                                                            \
    "v_readlane_b32 s61, v100, 0\n"                                          \
    "ld32d_" L "%=:\n\t"                                                     \
    "s_and_b32 s65, " P ", 3\n\t"                                            \
    "s_lshl_b32 s65, s65, 3\n\t"                                             \
    "s_lshr_b64 s[60:61], s[60:61], s65\n\t"

// s[60:61] = 8 bytes at fragment position P (s58, s59, s62..s65 scratch; v100, v105)
#define RA_LD64(P, L)                                                        \
    "s_lshr_b32 s63, " P ", 8\n\t"                                          \
    "s_bfe_u32 s64, " P ", 0x60002\n\t"                                     \
    "s_set_gpr_idx_on s63, gpr_idx(SRC0)\n\t"                                \
    "v_accvgpr_read_b32 v100, a0\n\t"                                        \
    "s_set_gpr_idx_off\n\t"                                                  \
    "s_cmp_gt_u32 s64, 61\n\t"                                               \
    "s_cbranch_scc1 ld64w_" L "%=\n\t"                                       \
    "s_nop 1\n\t"                                                            \
    "v_readlane_b32 s60, v100, s64\n\t"                                      \
    "s_add_u32 s64, s64, 1\n\t"                                              \
    "v_readlane_b32 s61, v100, s64\n\t"                                      \
    "s_add_u32 s64, s64, 1\n\t"                                              \
    "v_readlane_b32 s62, v100, s64\n\t"                                      \
    "s_branch ld64d_" L "%=\n"                                               \
    "ld64w_" L "%=:\n\t"                                                     \
    "s_add_u32 s63, s63, 1\n\t"                                              \
    "s_and_b32 s63, s63, 255\n\t"                                            \
    "s_set_gpr_idx_on s63, gpr_idx(SRC0)\n\t"                                \
    "v_accvgpr_read_b32 v105, a0\n\t"                                        \
    "s_set_gpr_idx_off\n\t"                                                  \
    "s_nop 1\n\t"                                                            \
    "v_readlane_b32 s60, v100, s64\n\t"                                      \
    "s_cmp_eq_u32 s64, 63\n\t"                                               \
    "s_cbranch_scc1 ld64x_" L "%=\n\t"                                       \
    "v_readlane_b32 s61, v100, 63\n\t"                                       \
    "v_readlane_b32 s62, v105, 0\n\t"                                        \
    "s_branch ld64d_" L "%=\n"                                               \
    "ld64x_" L "%=:\n\t"                                                     \
    "v_readlane_b32 s61, v105, 0\n\t"                                        \
    "v_readlane_b32 s62, v105, 1\n"                                          \
    "ld64d_" L "%=:\n\t"                                                     \
    "s_and_b32 s65, " P ", 3\n\t"                                            \
    "s_lshl_b32 s65, s65, 3\n\t"                                             \
    "s_mov_b32 s58, s61\n\t"                                                 \
    "s_mov_b32 s59, s62\n\t"                                                 \
    "s_lshr_b64 s[60:61], s[60:61], s65\n\t"                                 \
    "s_lshr_b64 s[58:59], s[58:59], s65\n\t"                                 \
    "s_mov_b32 s61, s58\n\t"

// s66 = hash(X) (X a register)
#define RA_HASH(X)                                                           \
    "s_mul_i32 s66, " X ", 0x1e35a7bd\n\t"                                  \
    "s_lshr_b32 s66, s66, %[shift]\n\t"

// table[s66] = V (register); if CAND is non-empty, CAND = the old entry.  Entry h: VGPR row
// v128 + (h >> 7), lane (h >> 1) & 63, half h & 1 (s67..s71 scratch, v101)
#define RA_TSET(V, CAND_INSNS)                                               \
    "s_lshr_b32 s67, s66, 7\n\t"                                             \
    "s_bfe_u32 s68, s66, 0x60001\n\t"                                       \
    "s_and_b32 s69, s66, 1\n\t"                                              \
    "s_lshl_b32 s69, s69, 4\n\t"                                             \
    "s_set_gpr_idx_on s67, gpr_idx(SRC0)\n\t"                                \
    "v_mov_b32 v101, v128\n\t"                                               \
    "s_set_gpr_idx_off\n\t"                                                  \
    "s_nop 1\n\t"                                                            \
    "v_readlane_b32 s70, v101, s68\n\t"                                      \
    CAND_INSNS                                                               \
    "s_lshl_b32 s71, 0xffff, s69\n\t"                                        \
    "s_andn2_b32 s70, s70, s71\n\t"                                          \
    "s_lshl_b32 s71, " V ", s69\n\t"                                         \
    "s_or_b32 s70, s70, s71\n\t"                                             \
    "s_mov_b32 m0, s68\n\t"                                                 \
    "v_writelane_b32 v101, s70, m0\n\t"                                     \
    "s_set_gpr_idx_on s67, gpr_idx(DST)\n\t"                                 \
    "v_mov_b32 v128, v101\n\t"                                               \
    "s_set_gpr_idx_off\n\t"
#define RA_CAND_OUT                                                          \
    "s_lshr_b32 %[cand], s70, s69\n\t"                                       \
    "s_and_b32 %[cand], %[cand], 0xffff\n\t"

#ifdef RA_NOSTORE   // microbenchmark only: time the match loop without its output stores
#define RA_STORE_INSN ""
#else
#define RA_STORE_INSN "global_store_byte v104, v102, %[outp]\n\t"
#endif
// out[op .. op + s74) = bytes of s[72:73], one lane per byte; op += s74
#define RA_STORE                                                             \
    "v_mov_b32 v102, s72\n\t"                                                \
    "v_mov_b32 v103, s73\n\t"                                                \
    "v_lshrrev_b64 v[102:103], %[vl8], v[102:103]\n\t"                       \
    "v_add_u32 v104, %[op], %[vlane]\n\t"                                    \
    "s_bfm_b64 s[76:77], s74, 0\n\t"                                         \
    "s_mov_b64 exec, s[76:77]\n\t"                                           \
    RA_STORE_INSN                                                            \
    "s_mov_b64 exec, -1\n\t"                                                 \
    "s_add_u32 %[op], %[op], s74\n\t"

__device__ __forceinline__ void ra_run(uint32_t &mode, uint32_t &ip, uint32_t &next_emit, uint32_t &op, uint32_t &cand,
                                       uint32_t ip_limit, uint32_t n, uint32_t shift, uint32_t abt, uint8_t *out, int lane)
{
    const uint32_t vl8 = (uint32_t)lane * 8;
    asm volatile(
        "s_cmp_eq_u32 %[mode], 1\n\t"
        "s_cbranch_scc1 copy_%=\n"
        // ---- literal search from ip (skip = 32)
        "search0_%=:\n\t"
        "s_mov_b32 s86, 32\n"
        "search_%=:\n\t"
        "s_lshr_b32 s85, s86, 5\n\t"
        "s_add_u32 s85, %[ip], s85\n\t"            // next_ip
        "s_add_u32 s86, s86, 1\n\t"                // skip++
        "s_cmp_gt_u32 s85, %[ipl]\n\t"
        "s_cbranch_scc1 rem_%=\n\t"
        "s_cmp_gt_u32 s86, %[abt]\n\t"
        "s_cbranch_scc1 abort_%=\n\t"
        RA_LD32("%[ip]", "a")
        "s_mov_b32 s84, s60\n\t"                   // cur
        RA_HASH("s84")
        RA_TSET("%[ip]", RA_CAND_OUT)
        RA_LD32("%[cand]", "b")
        "s_cmp_eq_u32 s60, s84\n\t"
        "s_cbranch_scc1 hit_%=\n\t"
        "s_mov_b32 %[ip], s85\n\t"
        "s_branch search_%=\n"
        // ---- hit: literal [next_emit, ip)
        "hit_%=:\n\t"
        "s_sub_u32 s80, %[ip], %[ne]\n\t"
        "s_cmp_gt_u32 s80, 7\n\t"
        "s_cbranch_scc1 lit_%=\n\t"
        RA_LD64("%[ne]", "c")
        "s_lshl_b32 s81, s80, 3\n\t"
        "s_bfm_b64 s[88:89], s81, 0\n\t"
        "s_and_b64 s[72:73], s[60:61], s[88:89]\n\t"
        "s_lshl_b64 s[72:73], s[72:73], 8\n\t"
        "s_sub_u32 s81, s80, 1\n\t"
        "s_lshl_b32 s81, s81, 2\n\t"
        "s_or_b32 s72, s72, s81\n\t"
        "s_add_u32 s74, s80, 1\n\t"
        RA_STORE
        // ---- copy at ip from cand: match length over at most 64 bytes after the first 4
        "copy_%=:\n\t"
        "s_add_u32 s87, %[cand], 4\n\t"            // s1
        "s_add_u32 s83, %[ip], 4\n\t"              // s2
        "s_mov_b32 s82, 0\n"                       // m
        "mloop_%=:\n\t"
        "s_add_u32 s81, s83, 8\n\t"
        "s_cmp_gt_u32 s81, %[n]\n\t"
        "s_cbranch_scc1 long_%=\n\t"
        RA_LD64("s87", "d")
        "s_mov_b32 s90, s60\n\t"
        "s_mov_b32 s91, s61\n\t"
        RA_LD64("s83", "e")
        "s_xor_b64 s[60:61], s[60:61], s[90:91]\n\t"
        "s_cmp_lg_u64 s[60:61], 0\n\t"
        "s_cbranch_scc1 mfound_%=\n\t"
        "s_add_u32 s82, s82, 8\n\t"
        "s_add_u32 s87, s87, 8\n\t"
        "s_add_u32 s83, s83, 8\n\t"
        "s_cmp_lt_u32 s82, 64\n\t"
        "s_cbranch_scc1 mloop_%=\n\t"
        "s_branch long_%=\n"
        "mfound_%=:\n\t"
        "s_ff1_i32_b64 s81, s[60:61]\n\t"
        "s_lshr_b32 s81, s81, 3\n\t"
        "s_add_u32 s80, s82, s81\n\t"
        "s_add_u32 s80, s80, 4\n\t"                // matched (<= 67)
        "s_sub_u32 s81, %[ip], %[cand]\n\t"        // offset
        "s_mov_b32 s73, 0\n\t"
        "s_add_u32 %[ip], %[ip], s80\n\t"
        "s_cmp_gt_u32 s80, 64\n\t"
        "s_cbranch_scc0 one_%=\n\t"
        // 60-byte piece (COPY_2_BYTE_OFFSET tag 2 + (59 << 2))
        "s_lshl_b32 s72, s81, 8\n\t"
        "s_or_b32 s72, s72, 238\n\t"
        "s_mov_b32 s74, 3\n\t"
        RA_STORE
        "s_sub_u32 s80, s80, 60\n"
        "one_%=:\n\t"
        "s_cmp_lt_u32 s80, 12\n\t"
        "s_cbranch_scc0 three_%=\n\t"
        "s_cmp_lt_u32 s81, 2048\n\t"
        "s_cbranch_scc0 three_%=\n\t"
        // COPY_1_BYTE_OFFSET: 1 + ((len - 4) << 2) + ((offset >> 8) << 5), offset & 0xff
        "s_sub_u32 s72, s80, 4\n\t"
        "s_lshl_b32 s72, s72, 2\n\t"
        "s_lshr_b32 s88, s81, 8\n\t"
        "s_lshl_b32 s88, s88, 5\n\t"
        "s_add_u32 s72, s72, s88\n\t"
        "s_add_u32 s72, s72, 1\n\t"
        "s_and_b32 s88, s81, 0xff\n\t"
        "s_lshl_b32 s88, s88, 8\n\t"
        "s_or_b32 s72, s72, s88\n\t"
        "s_mov_b32 s74, 2\n\t"
        "s_branch emit_%=\n"
        "three_%=:\n\t"
        // COPY_2_BYTE_OFFSET: 2 + ((len - 1) << 2), offset (2 bytes LE)
        "s_sub_u32 s72, s80, 1\n\t"
        "s_lshl_b32 s72, s72, 2\n\t"
        "s_add_u32 s72, s72, 2\n\t"
        "s_lshl_b32 s88, s81, 8\n\t"
        "s_or_b32 s72, s72, s88\n\t"
        "s_mov_b32 s74, 3\n"
        "emit_%=:\n\t"
        RA_STORE
        "s_mov_b32 %[ne], %[ip]\n\t"
        "s_cmp_ge_u32 %[ip], %[ipl]\n\t"
        "s_cbranch_scc1 rem_%=\n\t"
        // table[hash(ip-1)] = ip-1; cand = table[hash(ip)]; table[...] = ip
        "s_sub_u32 s87, %[ip], 1\n\t"
        RA_LD64("s87", "f")
        RA_HASH("s60")
        RA_TSET("s87", "")
        "s_lshr_b64 s[60:61], s[60:61], 8\n\t"
        "s_mov_b32 s84, s60\n\t"                   // bytes [ip, ip+4)
        RA_HASH("s84")
        RA_TSET("%[ip]", RA_CAND_OUT)
        RA_LD32("%[cand]", "g")
        "s_cmp_eq_u32 s60, s84\n\t"
        "s_cbranch_scc1 copy_%=\n\t"
        "s_add_u32 %[ip], %[ip], 1\n\t"
        "s_branch search0_%=\n"
        // ---- exits
        "rem_%=:\n\t"
        "s_mov_b32 %[mode], 2\n\t"
        "s_branch done_%=\n"
        "abort_%=:\n\t"
        "s_mov_b32 %[mode], 3\n\t"
        "s_branch done_%=\n"
        "lit_%=:\n\t"
        "s_mov_b32 %[mode], 4\n\t"
        "s_branch done_%=\n"
        "long_%=:\n\t"
        "s_mov_b32 %[mode], 5\n"
        "done_%=:\n\t"
        "s_nop 4\n\t"
        : [mode] "+s"(mode), [ip] "+s"(ip), [ne] "+s"(next_emit), [op] "+s"(op), [cand] "+s"(cand)
        : [ipl] "s"(ip_limit), [n] "s"(n), [shift] "s"(shift), [abt] "s"(abt), [outp] "s"(out), [vl8] "v"(vl8),
          [vlane] "v"(lane)
        : "memory", "scc", "m0", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69",
          "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85",
          "s86", "s87", "s88", "s89", "s90", "s91", "v100", "v101", "v102", "v103", "v104", "v105");
}

__global__ void __launch_bounds__(64, 1) __attribute__((amdgpu_num_vgpr(128))) k_snappy_ra(SnappyArgs a)
{
    const int lane = threadIdx.x;
    const uint32_t f = blockIdx.x;
    const uint32_t pg = a.frag_page[f];
    const uint32_t fi = a.frag_idx[f];
    const uint64_t plen = a.page_len[pg];
    const uint64_t fstart = (uint64_t)fi * SNAPPY_FRAG;
    const uint32_t n = (uint32_t)((plen - fstart) < SNAPPY_FRAG ? (plen - fstart) : SNAPPY_FRAG);
    const uint8_t *fbase = a.in + a.page_off[pg] + fstart;
    const Src g{(g_u8 *)fbase};
    asm volatile("; k_snappy_ra: a0..a255 hold the fragment" ::: RA_CLOBBERS);
    RIn in;
    in.load(fbase, n, lane);
    VTab T;
    T.lane = (uint32_t)lane;
    T.clear();
    uint32_t tsize = 256;
    while (tsize < SNAPPY_MAX_TABLE && tsize < n) tsize <<= 1;

    uint8_t *out = a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP;
    uint32_t op = 0;
    uint32_t shift = 32;
    for (uint32_t t = tsize; t > 1; t >>= 1) shift--;
    const uint32_t ip_end = n;
    uint32_t next_emit = 0;
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        uint32_t ip = 1, cand = 0, mode = RA_SEARCH;
        for (;;) {
            ip = ufl(ip); next_emit = ufl(next_emit); op = ufl(op); cand = ufl(cand); mode = ufl(mode);
            ra_run(mode, ip, next_emit, op, cand, ip_limit, n, shift, 32 + VT_ABORT, out, lane);
            mode = __builtin_amdgcn_readfirstlane(mode);
            if (mode == RA_REMAINDER) break;
            if (mode == RA_ABORT) {
                if (lane == 0) a.frag_len[f] = VT_ABORTED;
                return;
            }
            if (mode == RA_LITERAL) {
                op = emit_literal(out, op, g, next_emit, ip - next_emit, lane);
                mode = RA_COPY;
                continue;
            }
            // RA_LONGMATCH: the whole copy step with an unbounded match length
            const uint32_t base = ip;
            const uint32_t matched = 4 + find_match_length_r(in, g, cand + 4, ip + 4, ip_end, lane);
            ip += matched;
            op = emit_copy_s(out, op, base - cand, matched, lane);
            next_emit = ip;
            if (ip >= ip_limit) break;
            const uint64_t in8 = in.ld64(ip - 1);
            const uint32_t b1 = (uint32_t)(in8 >> 8);
            T.put(sn_hash((uint32_t)in8, shift), ip - 1);
            cand = T.swap(sn_hash(b1, shift), ip);
            if (b1 == in.ld32(cand)) {
                mode = RA_COPY;
            } else {
                ++ip;
                mode = RA_SEARCH;
            }
        }
    }
    if (next_emit < ip_end) op = emit_literal(out, op, g, next_emit, ip_end - next_emit, lane);
    if (lane == 0) a.frag_len[f] = op;
}

// ------------------------------------------------------------------ windowed variant
// k_snappy_ra still spends ~140 instructions (~1000 cycles) per match-loop step, nearly all
// of it plumbing around ONE position at a time: pull 4 unaligned bytes out of the register
// rows, hash them, read-modify-write a 16-bit half of a table register.  Here the wave keeps
// a 64-position window W..W+63 in three VGPRs, built in one batch (lane i: the 4 bytes at
// W+i, their hash, and table[hash] as of the build):
//   - the table lives in LDS (32 KiB; four waves per CU, as register-bound anyway) and every
//     insert goes to it at once (one ds_write_b16), so a rebuild sees all of them;
//   - a probe at W+i reads its bytes and hash with two v_readlane; its candidate is the
//     highest lane below i with the same hash inserted since the build (one v_cmp ballot and
//     the insert mask M), else lane i's snapshot: exactly what the live table holds then,
//     since inserts only ever store larger positions;
//   - bytes outside the window (far candidates) come from the AGPR rows as in k_snappy_ra.
// The window is rebuilt when the parse position reaches W+60.  Same algorithm, same output
// bytes; the rare steps leave the program as in k_snappy_ra, and since the C++ long-match
// step inserts into the table itself, it invalidates the window (W = RW_NOWIN).
constexpr uint32_t RW_NOWIN = 0xffff0000u;

// rebuild the window at %[W]: v96 = bytes, v97 = hash, v98 = table snapshot; M = 0.
// Scratch s56..s59, v99..v110, vcc.
#define RW_BUILD(L)                                                          \
    "s_lshr_b32 s56, %[W], 2\n\t"                                            \
    "s_lshr_b32 s57, s56, 6\n\t"                                             \
    "s_and_b32 s57, s57, 255\n\t"                                            \
    "s_set_gpr_idx_on s57, gpr_idx(SRC0)\n\t"                                \
    "v_accvgpr_read_b32 v99, a0\n\t"                                         \
    "s_set_gpr_idx_off\n\t"                                                  \
    "s_add_u32 s58, s57, 1\n\t"                                              \
    "s_and_b32 s58, s58, 255\n\t"                                            \
    "s_set_gpr_idx_on s58, gpr_idx(SRC0)\n\t"                                \
    "v_accvgpr_read_b32 v100, a0\n\t"                                        \
    "s_set_gpr_idx_off\n\t"                                                  \
    "s_and_b32 s59, %[W], 3\n\t"                                             \
    "v_add_u32 v101, s59, %[vlane]\n\t"                                      \
    "v_lshrrev_b32 v102, 2, v101\n\t"                                        \
    "v_add_u32 v102, s56, v102\n\t"                                          \
    "v_add_u32 v103, 1, v102\n\t"                                            \
    "v_and_b32 v104, 63, v102\n\t"                                           \
    "v_lshlrev_b32 v104, 2, v104\n\t"                                        \
    "v_and_b32 v105, 63, v103\n\t"                                           \
    "v_lshlrev_b32 v105, 2, v105\n\t"                                        \
    "s_nop 1\n\t"                                                            \
    "ds_bpermute_b32 v106, v104, v99\n\t"                                    \
    "ds_bpermute_b32 v107, v104, v100\n\t"                                   \
    "ds_bpermute_b32 v108, v105, v99\n\t"                                    \
    "ds_bpermute_b32 v109, v105, v100\n\t"                                   \
    "v_and_b32 v101, 3, v101\n\t"                                            \
    "v_lshlrev_b32 v101, 3, v101\n\t"                                        \
    "v_lshrrev_b32 v102, 6, v102\n\t"                                        \
    "v_and_b32 v102, 255, v102\n\t"                                          \
    "v_lshrrev_b32 v103, 6, v103\n\t"                                        \
    "v_and_b32 v103, 255, v103\n\t"                                          \
    "s_mov_b32 s58, 0x1e35a7bd\n\t"                                          \
    "s_waitcnt lgkmcnt(0)\n\t"                                               \
    "v_cmp_eq_u32_e32 vcc, s57, v102\n\t"                                    \
    "v_cndmask_b32_e32 v106, v107, v106, vcc\n\t"                            \
    "v_cmp_eq_u32_e32 vcc, s57, v103\n\t"                                    \
    "v_cndmask_b32_e32 v108, v109, v108, vcc\n\t"                            \
    "v_alignbit_b32 v96, v108, v106, v101\n\t"                               \
    "v_mul_lo_u32 v97, s58, v96\n\t"                                         \
    "v_lshrrev_b32 v97, %[shift], v97\n\t"                                   \
    "v_lshlrev_b32 v110, 1, v97\n\t"                                         \
    "v_add_u32 v110, %[tab], v110\n\t"                                       \
    "ds_read_u16 v98, v110\n\t"                                              \
    "s_mov_b64 %[M], 0\n\t"                                                  \
    "s_waitcnt lgkmcnt(0)\n\t"

// parse-side position P (register): s67 = P - W (rebuilding the window at P - 4 when P is
// not below W + 60), DST = its 4 bytes, s66 = their hash
#define RW_IPGET(P, DST, L)                                                  \
    "s_sub_u32 s67, " P ", %[W]\n\t"                                         \
    "s_cmp_lt_u32 s67, 60\n\t"                                               \
    "s_cbranch_scc1 ipok_" L "%=\n\t"                                        \
    "s_max_u32 s67, " P ", 4\n\t"                                            \
    "s_sub_u32 %[W], s67, 4\n\t"                                             \
    RW_BUILD(L)                                                              \
    "s_sub_u32 s67, " P ", %[W]\n"                                           \
    "ipok_" L "%=:\n\t"                                                      \
    "v_readlane_b32 " DST ", v96, s67\n\t"                                   \
    "v_readlane_b32 s66, v97, s67\n\t"                                       \
    "s_nop 1\n\t"

// %[cand] = table[s66] as the sequential loop would read it at window lane s67
#define RW_RESOLVE(L)                                                        \
    "v_cmp_eq_u32_e64 s[60:61], s66, v97\n\t"                                \
    "s_bfm_b64 s[62:63], s67, 0\n\t"                                         \
    "s_and_b64 s[60:61], s[60:61], s[62:63]\n\t"                             \
    "s_and_b64 s[60:61], s[60:61], %[M]\n\t"                                 \
    "s_cmp_lg_u64 s[60:61], 0\n\t"                                           \
    "s_cbranch_scc1 rin_" L "%=\n\t"                                         \
    "v_readlane_b32 %[cand], v98, s67\n\t"                                   \
    "s_branch rdone_" L "%=\n"                                               \
    "rin_" L "%=:\n\t"                                                       \
    "s_flbit_i32_b64 s62, s[60:61]\n\t"                                      \
    "s_sub_u32 s62, 63, s62\n\t"                                             \
    "s_add_u32 %[cand], %[W], s62\n"                                         \
    "rdone_" L "%=:\n\t"

// table[s66] = P; window lane s67 marked inserted
#define RW_INSERT(P)                                                         \
    "s_lshl_b32 s64, s66, 1\n\t"                                             \
    "s_add_u32 s64, s64, %[tab]\n\t"                                         \
    "v_mov_b32 v110, s64\n\t"                                                \
    "v_mov_b32 v111, " P "\n\t"                                              \
    "s_mov_b64 exec, 1\n\t"                                                  \
    "ds_write_b16 v110, v111\n\t"                                            \
    "s_mov_b64 exec, -1\n\t"                                                 \
    "s_bitset1_b64 %[M], s67\n\t"

// DST = 4 bytes at any position P (window lane, else the AGPR rows)
#define RW_CUR(P, DST, L)                                                    \
    "s_sub_u32 s63, " P ", %[W]\n\t"                                         \
    "s_cmp_lt_u32 s63, 64\n\t"                                               \
    "s_cbranch_scc0 cfar_" L "%=\n\t"                                        \
    "v_readlane_b32 " DST ", v96, s63\n\t"                                   \
    "s_branch cdone_" L "%=\n"                                               \
    "cfar_" L "%=:\n\t"                                                      \
    RA_LD32(P, L)                                                            \
    "s_mov_b32 " DST ", s60\n"                                               \
    "cdone_" L "%=:\n\t"

__device__ __forceinline__ void rw_run(uint32_t &mode, uint32_t &ip, uint32_t &next_emit, uint32_t &op, uint32_t &cand,
                                       uint32_t &W, uint64_t &M, uint32_t ip_limit, uint32_t n, uint32_t shift, uint32_t abt,
                                       uint8_t *out, uint32_t tab, int lane)
{
    const uint32_t vl8 = (uint32_t)lane * 8;
    asm volatile(
        "s_cmp_eq_u32 %[mode], 1\n\t"
        "s_cbranch_scc1 copy_%=\n"
        // ---- literal search from ip (skip = 32)
        "search0_%=:\n\t"
        "s_mov_b32 s86, 32\n"
        "search_%=:\n\t"
        "s_lshr_b32 s85, s86, 5\n\t"
        "s_add_u32 s85, %[ip], s85\n\t"            // next_ip
        "s_add_u32 s86, s86, 1\n\t"                // skip++
        "s_cmp_gt_u32 s85, %[ipl]\n\t"
        "s_cbranch_scc1 rem_%=\n\t"
        "s_cmp_gt_u32 s86, %[abt]\n\t"
        "s_cbranch_scc1 abort_%=\n\t"
        RW_IPGET("%[ip]", "s84", "a")
        RW_RESOLVE("a")
        RW_INSERT("%[ip]")
        RW_CUR("%[cand]", "s88", "b")
        "s_cmp_eq_u32 s88, s84\n\t"
        "s_cbranch_scc1 hit_%=\n\t"
        "s_mov_b32 %[ip], s85\n\t"
        "s_branch search_%=\n"
        // ---- hit: literal [next_emit, ip)
        "hit_%=:\n\t"
        "s_sub_u32 s80, %[ip], %[ne]\n\t"
        "s_cmp_gt_u32 s80, 7\n\t"
        "s_cbranch_scc1 lit_%=\n\t"
        RW_CUR("%[ne]", "s90", "c")
        "s_add_u32 s89, %[ne], 4\n\t"
        RW_CUR("s89", "s91", "c2")
        "s_lshl_b32 s81, s80, 3\n\t"
        "s_bfm_b64 s[88:89], s81, 0\n\t"
        "s_and_b64 s[72:73], s[90:91], s[88:89]\n\t"
        "s_lshl_b64 s[72:73], s[72:73], 8\n\t"
        "s_sub_u32 s81, s80, 1\n\t"
        "s_lshl_b32 s81, s81, 2\n\t"
        "s_or_b32 s72, s72, s81\n\t"
        "s_add_u32 s74, s80, 1\n\t"
        RA_STORE
        // ---- copy at ip from cand: match length over at most 64 bytes after the first 4
        "copy_%=:\n\t"
        "s_add_u32 s87, %[cand], 4\n\t"            // s1
        "s_add_u32 s83, %[ip], 4\n\t"              // s2
        "s_mov_b32 s82, 0\n"                       // m
        "mloop_%=:\n\t"
        "s_add_u32 s81, s83, 4\n\t"
        "s_cmp_gt_u32 s81, %[n]\n\t"
        "s_cbranch_scc1 long_%=\n\t"
        RW_CUR("s87", "s90", "d")
        RW_CUR("s83", "s91", "e")
        "s_xor_b32 s90, s90, s91\n\t"
        "s_cmp_lg_u32 s90, 0\n\t"
        "s_cbranch_scc1 mfound_%=\n\t"
        "s_add_u32 s82, s82, 4\n\t"
        "s_add_u32 s87, s87, 4\n\t"
        "s_add_u32 s83, s83, 4\n\t"
        "s_cmp_lt_u32 s82, 64\n\t"
        "s_cbranch_scc1 mloop_%=\n\t"
        "s_branch long_%=\n"
        "mfound_%=:\n\t"
        "s_ff1_i32_b32 s81, s90\n\t"
        "s_lshr_b32 s81, s81, 3\n\t"
        "s_add_u32 s80, s82, s81\n\t"
        "s_add_u32 s80, s80, 4\n\t"                // matched (<= 67)
        "s_sub_u32 s81, %[ip], %[cand]\n\t"        // offset
        "s_mov_b32 s73, 0\n\t"
        "s_add_u32 %[ip], %[ip], s80\n\t"
        "s_cmp_gt_u32 s80, 64\n\t"
        "s_cbranch_scc0 one_%=\n\t"
        "s_lshl_b32 s72, s81, 8\n\t"               // 60-byte piece: tag 2 + (59 << 2)
        "s_or_b32 s72, s72, 238\n\t"
        "s_mov_b32 s74, 3\n\t"
        RA_STORE
        "s_sub_u32 s80, s80, 60\n"
        "one_%=:\n\t"
        "s_cmp_lt_u32 s80, 12\n\t"
        "s_cbranch_scc0 three_%=\n\t"
        "s_cmp_lt_u32 s81, 2048\n\t"
        "s_cbranch_scc0 three_%=\n\t"
        "s_sub_u32 s72, s80, 4\n\t"                // COPY_1_BYTE_OFFSET
        "s_lshl_b32 s72, s72, 2\n\t"
        "s_lshr_b32 s88, s81, 8\n\t"
        "s_lshl_b32 s88, s88, 5\n\t"
        "s_add_u32 s72, s72, s88\n\t"
        "s_add_u32 s72, s72, 1\n\t"
        "s_and_b32 s88, s81, 0xff\n\t"
        "s_lshl_b32 s88, s88, 8\n\t"
        "s_or_b32 s72, s72, s88\n\t"
        "s_mov_b32 s74, 2\n\t"
        "s_branch emit_%=\n"
        "three_%=:\n\t"
        "s_sub_u32 s72, s80, 1\n\t"                // COPY_2_BYTE_OFFSET
        "s_lshl_b32 s72, s72, 2\n\t"
        "s_add_u32 s72, s72, 2\n\t"
        "s_lshl_b32 s88, s81, 8\n\t"
        "s_or_b32 s72, s72, s88\n\t"
        "s_mov_b32 s74, 3\n"
        "emit_%=:\n\t"
        RA_STORE
        "s_mov_b32 %[ne], %[ip]\n\t"
        "s_cmp_ge_u32 %[ip], %[ipl]\n\t"
        "s_cbranch_scc1 rem_%=\n\t"
        // table[hash(ip-1)] = ip-1; cand = table[hash(ip)]; table[...] = ip
        "s_sub_u32 s87, %[ip], 1\n\t"
        RW_IPGET("s87", "s89", "f")
        RW_INSERT("s87")
        RW_IPGET("%[ip]", "s84", "g")
        RW_RESOLVE("g")
        RW_INSERT("%[ip]")
        RW_CUR("%[cand]", "s88", "h")
        "s_cmp_eq_u32 s88, s84\n\t"
        "s_cbranch_scc1 copy_%=\n\t"
        "s_add_u32 %[ip], %[ip], 1\n\t"
        "s_branch search0_%=\n"
        // ---- exits
        "rem_%=:\n\t"
        "s_mov_b32 %[mode], 2\n\t"
        "s_branch done_%=\n"
        "abort_%=:\n\t"
        "s_mov_b32 %[mode], 3\n\t"
        "s_branch done_%=\n"
        "lit_%=:\n\t"
        "s_mov_b32 %[mode], 4\n\t"
        "s_branch done_%=\n"
        "long_%=:\n\t"
        "s_mov_b32 %[mode], 5\n"
        "done_%=:\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_nop 4\n\t"
        : [mode] "+s"(mode), [ip] "+s"(ip), [ne] "+s"(next_emit), [op] "+s"(op), [cand] "+s"(cand), [W] "+s"(W), [M] "+s"(M)
        : [ipl] "s"(ip_limit), [n] "s"(n), [shift] "s"(shift), [abt] "s"(abt), [outp] "s"(out), [tab] "s"(tab),
          [vl8] "v"(vl8), [vlane] "v"(lane)
        : "memory", "scc", "vcc", "m0", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67",
          "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83",
          "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103",
          "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111");
}

#define RW_RESERVE \
    "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111"

__global__ void __launch_bounds__(64, 1) __attribute__((amdgpu_num_vgpr(96))) k_snappy_w2(SnappyArgs a)
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
    asm volatile("; k_snappy_w2: a0..a255 hold the fragment" ::: RA_CLOBBERS);
    asm volatile("; k_snappy_w2: v96..v111 window + scratch" ::: RW_RESERVE);
    RIn in;
    in.load(fbase, n, lane);
    uint32_t tsize = 256;
    while (tsize < SNAPPY_MAX_TABLE && tsize < n) tsize <<= 1;
    for (uint32_t i = lane; i < tsize; i += 64) table[i] = 0;
    __syncthreads();
    const uint32_t tab = (uint32_t)(uintptr_t)table;

    uint8_t *out = a.frag_out + (uint64_t)f * SNAPPY_FRAG_CAP;
    uint32_t op = 0;
    uint32_t shift = 32;
    for (uint32_t t = tsize; t > 1; t >>= 1) shift--;
    const uint32_t ip_end = n;
    uint32_t next_emit = 0;
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        uint32_t ip = 1, cand = 0, mode = RA_SEARCH, W = RW_NOWIN;
        uint64_t M = 0;
        for (;;) {
            ip = ufl(ip); next_emit = ufl(next_emit); op = ufl(op); cand = ufl(cand); mode = ufl(mode); W = ufl(W);
            M = ((uint64_t)ufl((uint32_t)(M >> 32)) << 32) | ufl((uint32_t)M);
            rw_run(mode, ip, next_emit, op, cand, W, M, ip_limit, n, shift, 32 + VT_ABORT, out, tab, lane);
            mode = ufl(mode);
            if (mode == RA_REMAINDER) break;
            if (mode == RA_ABORT) {
                if (lane == 0) a.frag_len[f] = VT_ABORTED;
                return;
            }
            if (mode == RA_LITERAL) {
                op = emit_literal(out, op, g, next_emit, ip - next_emit, lane);
                mode = RA_COPY;
                continue;
            }
            // RA_LONGMATCH: the whole copy step with an unbounded match length
            W = RW_NOWIN;
            const uint32_t base = ip;
            const uint32_t matched = 4 + find_match_length_r(in, g, cand + 4, ip + 4, ip_end, lane);
            ip += matched;
            op = emit_copy_s(out, op, base - cand, matched, lane);
            next_emit = ip;
            if (ip >= ip_limit) break;
            const uint64_t in8 = in.ld64(ip - 1);
            const uint32_t b1 = (uint32_t)(in8 >> 8);
            table[sn_hash((uint32_t)in8, shift)] = (uint16_t)(ip - 1);
            const uint32_t h1 = sn_hash(b1, shift);
            cand = ufl(table[h1]);
            table[h1] = (uint16_t)ip;
            if (b1 == in.ld32(cand)) {
                mode = RA_COPY;
            } else {
                ++ip;
                mode = RA_SEARCH;
            }
        }
    }
    if (next_emit < ip_end) op = emit_literal(out, op, g, next_emit, ip_end - next_emit, lane);
    if (lane == 0) a.frag_len[f] = op;
}

// ------------------------------------------------------------------ experiment: k_snappy_v without output stores
// Timing only (its output is not Snappy): how much of the per-match latency of the serial
// parse is the emission (per-lane byte stores, which share vmcnt with the window refills).
__global__ void __launch_bounds__(64, 2) __attribute__((amdgpu_num_vgpr(128))) k_snappy_vns(SnappyArgs a)
{
    const int lane = threadIdx.x;
    const uint32_t f = a.order ? a.order[blockIdx.x] : blockIdx.x;
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
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        ip = 1;
        for (;;) {
            uint32_t skip = 32;
            uint32_t candidate;
            for (;;) {
                const uint32_t next_ip = ip + (skip++ >> 5);
                if (next_ip > ip_limit) goto emit_remainder;
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
                    (void)b;
                    op += 1 + len;
                } else {
                    op += len + 1 + (len > 60) + (len > 256);
                }
            }
            for (;;) {
                const uint32_t base = ip;
                const uint32_t matched = 4 + find_match_length_v(in, si, g, candidate + 4, ip + 4, ip_end, lane);
                ip += matched;
                op += 2 + (matched > 11) + 2 * (matched / 64);
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
    if (next_emit < ip_end) op += ip_end - next_emit + 3;
    if (lane == 0) { a.frag_len[f] = op; if (a.ftime) a.ftime[2 * f + 1] = wall_clock64(); }
}

}  // namespace kpw
