// kpw_lookback.h — single-pass chained scans (decoupled look-back), shared by the scan and
// RLE kernels.
//
// Every tile publishes its aggregate as soon as its own elements are reduced, then its
// inclusive prefix once its look-back (one wave, 64 predecessors per step) has found a
// predecessor whose inclusive prefix is out.  One launch per scan instead of reduce / carry /
// apply, and a kernel can chain several scans (status words of scan k at k * ntiles).
//
// Status word of tile i (u64, written and read as one agent-scope atomic, so value and state
// arrive together): value << 17 | epoch << 2 | state (1: aggregate, 2: inclusive prefix).
// The epoch changes every launch on the scratch, so stale words read as "not yet" without a
// clear; values fit 47 bits (byte counts and positions of one encode, < 2^40).
//
// Tile index = blockIdx.x.  A tile waits only on lower-numbered tiles, and each XCD dispatches
// its workgroups in index order, so with the kernel alone on the chip the lowest unfinished
// tile always runs.  That fails with concurrent look-back kernels on other hardware queues:
// kernel A's waiting tiles can fill XCD x while A's lowest unfinished tile is queued on XCD y,
// full of kernel B's waiting tiles whose own lowest is queued on x (r05au: C5 with 8 and 16
// hardware queues, eight writers, waited out a 2^25-spin bound).  A ticket counter avoids that
// but one atomic per tile on a single address serialised the launch (r04: 0.7 ms where the
// multi-launch scans took 0.1 over ~50 k tiles).  So the wait is bounded and then falls back
// (decoupled fallback): the waiting lane recomputes the missing tile's own contribution from
// the tile's inputs (every look-back kernel passes that function, `fb`), publishes it and goes
// on.  Results stay exact; only the rare slow path pays, and progress no longer depends on
// dispatch order.  Fallbacks are counted in *fails (traced by the engine).
#pragma once
#include "kpw_device.h"

namespace kpw {

struct LbView {
    uint64_t *w;      // status words from w[8]
    uint32_t epoch;
    uint32_t *fails;  // fallbacks taken (SegScratch::fails)
    uint32_t spin;    // polls of a predecessor's status word before the fallback (KPW_LB_SPIN)
};
constexpr uint32_t LB_ST_AGG = 1, LB_ST_INC = 2;

// status word idx (= scan * ntiles + tile)
__device__ __forceinline__ void lb_publish(const LbView &L, uint32_t idx, uint64_t enc, uint32_t st)
{
    __hip_atomic_store(&L.w[8 + idx], (enc << 17) | ((uint64_t)L.epoch << 2) | st, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0: the combination (in order) of tiles [first, tile) of scan `sbase` (= scan * ntiles)
// that enters `tile`, where `first` is the first tile of its run (the job); the look-back also
// ends at any tile that published its inclusive value.  Values travel encoded (Enc).
// fb(q, &v, &inc): tile q's status recomputed from its inputs (lane-local: no cross-lane ops),
// v its aggregate, or its inclusive value when inc (what tile q itself would publish).
template <typename T, typename Op, typename Enc, typename FB>
__device__ __forceinline__ T lb_lookback(const LbView &L, uint32_t sbase, uint32_t tile, uint32_t first, const FB &fb)
{
    const uint32_t lane = threadIdx.x & 63;
    T acc = Op::id();
    int64_t base = (int64_t)tile - 1;
    for (;;) {
        const int64_t q = base - (int64_t)lane;
        const bool valid = q >= (int64_t)first;
        uint64_t wv = 0;
        if (valid) {
            bool ok = false;
            for (uint32_t spin = 0;; spin++) {
                wv = __hip_atomic_load(&L.w[8 + sbase + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)((wv >> 2) & 0x7fff) == L.epoch && (wv & 3) != 0) { ok = true; break; }
                if (spin >= L.spin) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) {
                T v;
                bool inc;
                fb((uint32_t)q, v, inc);
                // An in-place scan (in == out) overwrites tile q's inputs once q has published:
                // so the recomputation stands only if q had still published nothing after its
                // loads completed (the fence waits for them); otherwise q's own word is used.
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
                const uint64_t w2 = __hip_atomic_load(&L.w[8 + sbase + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)((w2 >> 2) & 0x7fff) == L.epoch && (w2 & 3) != 0) {
                    wv = w2;
                } else {
                    wv = (Enc::enc(v) << 17) | ((uint64_t)L.epoch << 2) | (inc ? LB_ST_INC : LB_ST_AGG);
                    // (if tile q publishes too, both words are right: an AGG landing after its
                    // INC only lengthens later look-backs)
                    __hip_atomic_store(&L.w[8 + sbase + q], wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    atomicAdd(L.fails, 1u);
                }
            }
        }
        const bool term = !valid || (wv & 3) == LB_ST_INC;
        const uint64_t tm = __ballot(term);
        const uint32_t stop = tm ? (uint32_t)__builtin_ctzll(tm) : 64u;   // nearest terminal lane
        T v = (valid && lane <= stop) ? Enc::dec(wv >> 17) : Op::id();
        // ordered reduction: higher lanes are earlier tiles
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const T o = __shfl_down(v, d, 64);
            if (lane + d < 64) v = Op::op(o, v);
        }
        v = __shfl(v, 0, 64);
        acc = Op::op(v, acc);
        if (tm) return acc;
        base -= 64;
    }
}

// Tile q's published status read once, recomputed by fb when it is not out (the sequential
// prefix a fallback of a chained scan needs).
template <typename T, typename Enc, typename FB>
__device__ __forceinline__ void lb_peek(const LbView &L, uint32_t idx, uint32_t q, const FB &fb, T &v, bool &inc)
{
    const uint64_t wv = __hip_atomic_load(&L.w[8 + idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)((wv >> 2) & 0x7fff) == L.epoch && (wv & 3) != 0) {
        v = Enc::dec(wv >> 17);
        inc = (wv & 3) == LB_ST_INC;
    } else {
        fb(q, v, inc);
    }
}

struct EncU64 {
    __device__ static uint64_t enc(uint64_t v) { return v; }
    __device__ static uint64_t dec(uint64_t e) { return e; }
};
struct EncU32 {
    __device__ static uint64_t enc(uint32_t v) { return v; }
    __device__ static uint32_t dec(uint64_t e) { return (uint32_t)e; }
};
struct EncI64 {   // max-scan values are >= -1 (OpMaxI64's identity)
    __device__ static uint64_t enc(int64_t v) { return (uint64_t)(v + 1); }
    __device__ static int64_t dec(uint64_t e) { return (int64_t)e - 1; }
};
template <typename T> struct EncOf;
template <> struct EncOf<uint64_t> { using E = EncU64; };
template <> struct EncOf<uint32_t> { using E = EncU32; };
template <> struct EncOf<int64_t> { using E = EncI64; };

// One scan's tile (exclusive prefix within its run returned to every thread; `agg` = the
// tile's own aggregate, valid in thread 0).  `inc_now`: the tile's inclusive value does not
// depend on earlier tiles (first of its run, or a segment head inside it), so it is published
// at once; `need`: the tile needs its carry-in.  Returns Op::id() when !need.
template <typename T, typename Op, typename FB>
__device__ __forceinline__ T lb_tile(const LbView &L, uint32_t sbase, uint32_t tile, uint32_t first, T agg, bool inc_now,
                                     bool need, T *slot, const FB &fb)
{
    using Enc = typename EncOf<T>::E;
    if (threadIdx.x == 0) {
        *slot = Op::id();
        lb_publish(L, sbase + tile, Enc::enc(agg), inc_now ? LB_ST_INC : LB_ST_AGG);
    }
    if (need && threadIdx.x < 64) {
        const T c = lb_lookback<T, Op, Enc>(L, sbase, tile, first, fb);
        if (threadIdx.x == 0) {
            *slot = c;
            if (!inc_now) lb_publish(L, sbase + tile, Enc::enc(Op::op(c, agg)), LB_ST_INC);
        }
    }
    // Published before overwritten: an in-place scan's tile stores its outputs over its inputs
    // after this barrier, and a fallback that recomputes this tile (lb_lookback) trusts its
    // inputs only while it still sees no status word.  The status word is an agent-scope atomic
    // store (written through to the coherence point), so thread 0 waits for it to complete
    // (s_waitcnt 0) before the barrier: every output store of the tile is issued after the
    // publish is visible device-wide.  (An agent-scope release fence does the same plus an L2
    // write-back of every prior plain store, which no reader needs here: it made the K3
    // phase / size passes 2.7-4x slower, r06n against r05 profiles.)
    if (threadIdx.x == 0) __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const T c = *slot;
    __syncthreads();
    return c;
}

}  // namespace kpw
