// k_chunk.hip — per column-chunk kernels (one chunk = one column of one row group = one
// data page in the single-page regime):
//   K6 statistics   (Int/Long/Float/Double/Boolean/BinaryStatistics, parquet-mr 1.10.1
//                    PrimitiveComparator order; null_count)
//   K2 dictionary   (Plain*DictionaryValuesWriter: ids in first-occurrence order over the
//                    chunk, dictionaryByteSize += 4/8/4+len per new entry, fallback when it
//                    exceeds dictPageSize; FallbackValuesWriter.isCompressionSatisfying on the
//                    (first and only) page)
//   K4 PLAIN        (PlainValuesWriter little-endian values / 4-byte-length binaries,
//                    BooleanPlainValuesWriter LSB-first bits)
//   page layout     (ColumnWriterV1.writePage: rl(empty) | dl(4-byte length + RLE) | values;
//                    dictionary page first in the chunk, ColumnChunkPageWriter order)
//
// Chunks are processed through "chunk tiles" (2048 records of one chunk per 256-thread
// block, 8 consecutive records per thread) so ranks of non-null values follow record
// order: rank = popcount prefix of the presence bits (pcnt + in-word popcount).
#include "kpw_device.h"
#include "kpw_kernels.h"
#include "kpw_chunk.h"

namespace kpw {

__device__ __forceinline__ bool present_at(const DevCol &c, uint64_t r)
{
    return !c.optional || ((c.pres[r >> 6] >> (r & 63)) & 1ull);
}
__device__ __forceinline__ uint64_t rank_base(const DevCol &c, uint64_t s, uint64_t x)
{
    if (!c.optional) return x - s;
    auto pc = [&](uint64_t y) -> uint64_t {
        const uint64_t wi = y >> 6;
        const uint64_t m = (y & 63) ? (c.pres[wi] & ((1ull << (y & 63)) - 1)) : 0ull;
        return (uint64_t)c.pcnt[wi] + (uint64_t)__popcll(m);
    };
    return pc(x) - pc(s);
}

// Coalesced chunk-tile layout: thread t of tile T handles records T0 + k*KPW_BLOCK + t,
// k = 0..7 (one fully used line per wave and k), and gets each record's rank (index among
// the chunk's non-null values) from the presence popcount prefix instead of a running
// count.  Used by every per-record kernel whose result does not depend on a thread's
// records being contiguous.
__device__ __forceinline__ uint64_t pres_rank(const DevCol &c, uint64_t y)
{
    const uint64_t wi = y >> 6;
    const uint64_t m = (y & 63) ? (c.pres[wi] & ((1ull << (y & 63)) - 1)) : 0ull;
    return (uint64_t)c.pcnt[wi] + (uint64_t)__popcll(m);
}
struct TileRecs {
    uint64_t t0, e;       // first record of the tile, chunk end
    uint64_t rank0;       // rank base of the chunk (pres_rank(C.s) or C.s)
    __device__ __forceinline__ uint64_t rec(int k) const { return t0 + (uint64_t)k * KPW_BLOCK + threadIdx.x; }
    __device__ __forceinline__ uint64_t rank(const DevCol &c, uint64_t r) const
    {
        return (c.optional ? pres_rank(c, r) : r) - rank0;
    }
};
__device__ __forceinline__ TileRecs tile_recs(const ChunkDesc &C, const DevCol &col, uint32_t t, const uint32_t *ctile_first, uint32_t ci)
{
    TileRecs T;
    T.t0 = (uint64_t)C.s + C.tile_skip + (uint64_t)(t - ctile_first[ci]) * KPW_TILE_P;
    T.e = (uint64_t)C.e;
    T.rank0 = col.optional ? pres_rank(col, (uint64_t)C.s) : (uint64_t)C.s;
    return T;
}

__device__ __forceinline__ uint64_t fixed_val(const DevCol &c, uint64_t r)
{
    return c.vsize == 4 ? (uint64_t)((const uint32_t *)c.vals)[r] : ((const uint64_t *)c.vals)[r];
}

// order-preserving key for the Java comparators
__device__ __forceinline__ uint64_t order_key(int phys, uint64_t v)
{
    switch (phys) {
    case 1: return (uint64_t)((uint32_t)v ^ 0x80000000u);
    case 2: return v ^ 0x8000000000000000ull;
    case 4: { uint32_t b = (uint32_t)v; return (uint64_t)((b >> 31) ? ~b : (b | 0x80000000u)); }
    case 5: return (v >> 63) ? ~v : (v | 0x8000000000000000ull);
    default: return v;  // boolean 0/1
    }
}

// ------------------------------------------------------------------ K6 stats + sizes

// BYTE_ARRAY compare / equality of records a and b through the 16-byte prefix arrays; the
// batch bytes are read only when both values are longer than 16 bytes with equal prefixes.
// Unsigned lexicographic order, shorter first on a common prefix (BinaryStatistics).
__device__ __forceinline__ int str_cmp(const DevCol &col, const uint8_t *data, uint64_t a, uint64_t b, uint64_t data_end)
{
    const uint64_t a0 = col.spfx[2 * a], b0 = col.spfx[2 * b];
    if (a0 != b0) return __builtin_bswap64(a0) < __builtin_bswap64(b0) ? -1 : 1;
    const uint64_t a1 = col.spfx[2 * a + 1], b1 = col.spfx[2 * b + 1];
    if (a1 != b1) return __builtin_bswap64(a1) < __builtin_bswap64(b1) ? -1 : 1;
    const uint32_t la = col.slen[a], lb = col.slen[b];
    if (la <= 16 || lb <= 16) return la == lb ? 0 : (la < lb ? -1 : 1);
    return bytes_cmp(data, col.soff[a] + 16, la - 16, col.soff[b] + 16, lb - 16, data_end);
}
__device__ __forceinline__ bool str_eq(const DevCol &col, const uint8_t *data, uint64_t a, uint64_t b, uint64_t data_end)
{
    const uint32_t la = col.slen[a];
    if (la != col.slen[b] || col.spfx[2 * a] != col.spfx[2 * b] || col.spfx[2 * a + 1] != col.spfx[2 * b + 1]) return false;
    return la <= 16 || bytes_cmp(data, col.soff[a] + 16, la - 16, col.soff[b] + 16, la - 16, data_end) == 0;
}

__global__ void __launch_bounds__(KPW_BLOCK) k_chunk_stats(ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                           const uint32_t *ctile_chunk, const uint32_t *ctile_first,
                                                           uint64_t *tile_raw, uint64_t *tile_smin, uint64_t *tile_smax,
                                                           const uint64_t *data_end_p, uint4 *ht_clear, uint64_t ht_clear_n,
                                                           uint64_t *flags_clear)
{
    if (flags_clear && blockIdx.x == 0 && threadIdx.x == 0) *flags_clear = 0;   // set by the dictionary kernels after
    for (uint64_t i = (uint64_t)blockIdx.x * KPW_BLOCK + threadIdx.x; i < ht_clear_n; i += (uint64_t)gridDim.x * KPW_BLOCK)
        ht_clear[i] = make_uint4(~0u, ~0u, ~0u, ~0u);   // empty dictionary slots for the phase after
    const uint64_t data_end = *data_end_p;
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    ChunkDesc &C = ch[ci];
    const DevCol col = cols[C.col];   // by value: loaded once, not after every store
    const TileRecs T = tile_recs(C, col, t, ctile_first, ci);
    uint64_t nn = 0, raw = 0;
    uint64_t kmin = ~0ull, kmax = 0;
    bool ok[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t r = T.rec(k);
        ok[k] = r < T.e && present_at(col, r);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t r = T.rec(k);
        if (!ok[k]) continue;
        nn++;
        if (col.phys == 6) {
            raw += 4 + col.slen[r];   // min/max: k_str_minmax, after the dictionary phase
        } else if (col.phys == 0) {
            const uint64_t v = (col.vbits[r >> 6] >> (r & 63)) & 1ull;
            kmin = v < kmin ? v : kmin;
            kmax = v > kmax ? v : kmax;
        } else {
            raw += (uint64_t)col.vsize;
            const uint64_t key = order_key(col.phys, fixed_val(col, r));
            kmin = key < kmin ? key : kmin;
            kmax = key > kmax ? key : kmax;
        }
    }
    const uint64_t snn = block_reduce<uint64_t, OpSum64>(nn, lds);
    const uint64_t sraw = block_reduce<uint64_t, OpSum64>(raw, lds);
    if (col.phys == 6) {
        if (threadIdx.x == 0) tile_raw[t] = sraw;
    } else {
        if (snn) {
            // wave-level min/max then one atomic per wave
            for (int o = 32; o > 0; o >>= 1) {
                const uint64_t a = __shfl_xor(kmin, o, 64), b = __shfl_xor(kmax, o, 64);
                kmin = a < kmin ? a : kmin;
                kmax = b > kmax ? b : kmax;
            }
            if ((threadIdx.x & 63) == 0) {
                if (kmin != ~0ull) atomicMin((unsigned long long *)&C.smin, (unsigned long long)kmin);
                atomicMax((unsigned long long *)&C.smax, (unsigned long long)kmax);
            }
        }
        if (threadIdx.x == 0) tile_raw[t] = sraw;
    }
    if (threadIdx.x == 0) {
        atomicAdd(&C.nn, (uint32_t)snn);
        atomicAdd((unsigned long long *)&C.raw_bytes, (unsigned long long)sraw);
    }
}

// (null_count = records - nn and has_minmax = nn > 0 are derived by the host from the read-back
// descriptors, chunk_stats_derive)

// BYTE_ARRAY min/max, after the dictionary phase: a complete dictionary holds every
// distinct value of its chunk, so its entries stand in for the values (one entry per
// distinct string instead of one compare per value); other chunks reduce their values.
// One block per chunk tile: tile k covers entries [2048k, 2048k+2048) or its records.
__global__ void __launch_bounds__(KPW_BLOCK) k_str_minmax(const ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                          const uint32_t *ctile_chunk, const uint32_t *ctile_first,
                                                          const uint64_t *ent_rec, uint64_t *tile_smin, uint64_t *tile_smax,
                                                          const uint64_t *data_end_p, int mp)
{
    __shared__ uint64_t li[KPW_BLOCK], la[KPW_BLOCK];
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    const DevCol col = cols[C.col];   // by value: not reloaded after stores
    if (col.phys != 6) return;
    const uint64_t data_end = *data_end_p;
    // a page of a multi-page chunk is only part of what its dictionary covers: use its values
    const bool ents = !mp && C.is_dict && !C.fallback;
    const uint64_t q0 = (uint64_t)(t - ctile_first[ci]) * KPW_TILE_P + threadIdx.x;   // coalesced (equal strings tie harmlessly)
    uint64_t a = ~0ull, b = ~0ull;
    for (int k = 0; k < 8; k++) {
        const uint64_t q = q0 + (uint64_t)k * KPW_BLOCK;
        uint64_t r;
        if (ents) {
            if (q >= C.dict_n) break;
            r = ent_rec[C.ent_off + q];
        } else {
            r = (uint64_t)C.s + q;
            if (r >= (uint64_t)C.e) break;
            if (!present_at(col, r)) continue;
        }
        if (a == ~0ull || str_cmp(col, data, r, a, data_end) < 0) a = r;
        if (b == ~0ull || str_cmp(col, data, r, b, data_end) > 0) b = r;
    }
    li[threadIdx.x] = a;
    la[threadIdx.x] = b;
    __syncthreads();
    for (int d = KPW_BLOCK / 2; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d) {
            const uint64_t x = li[threadIdx.x], y = li[threadIdx.x + d];
            if (y != ~0ull && (x == ~0ull || str_cmp(col, data, y, x, data_end) < 0)) li[threadIdx.x] = y;
            const uint64_t u = la[threadIdx.x], v = la[threadIdx.x + d];
            if (v != ~0ull && (u == ~0ull || str_cmp(col, data, v, u, data_end) > 0)) la[threadIdx.x] = v;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { tile_smin[t] = li[0]; tile_smax[t] = la[0]; }
}

// per BYTE_ARRAY chunk: reduce its tiles' candidates
__global__ void __launch_bounds__(KPW_BLOCK) k_str_final(ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                         const uint32_t *ctile_first, const uint32_t *ctile_count,
                                                         const uint64_t *tile_smin, const uint64_t *tile_smax,
                                                         const uint64_t *data_end_p)
{
    __shared__ uint64_t li[KPW_BLOCK], la[KPW_BLOCK];
    const int ci = blockIdx.x;
    ChunkDesc &C = ch[ci];
    const DevCol col = cols[C.col];   // by value: not reloaded after stores
    if (col.phys != 6 || !C.nn) return;
    const uint64_t data_end = *data_end_p;
    uint64_t a = ~0ull, b = ~0ull;
    for (uint32_t k = threadIdx.x; k < ctile_count[ci]; k += KPW_BLOCK) {
        const uint64_t x = tile_smin[ctile_first[ci] + k], y = tile_smax[ctile_first[ci] + k];
        if (x != ~0ull && (a == ~0ull || str_cmp(col, data, x, a, data_end) < 0)) a = x;
        if (y != ~0ull && (b == ~0ull || str_cmp(col, data, y, b, data_end) > 0)) b = y;
    }
    li[threadIdx.x] = a;
    la[threadIdx.x] = b;
    __syncthreads();
    for (int d = KPW_BLOCK / 2; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d) {
            const uint64_t x = li[threadIdx.x], y = li[threadIdx.x + d];
            if (y != ~0ull && (x == ~0ull || str_cmp(col, data, y, x, data_end) < 0)) li[threadIdx.x] = y;
            const uint64_t u = la[threadIdx.x], v = la[threadIdx.x + d];
            if (v != ~0ull && (u == ~0ull || str_cmp(col, data, v, u, data_end) > 0)) la[threadIdx.x] = v;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { C.smin = li[0]; C.smax = la[0]; }
}

// ------------------------------------------------------------------ K2 dictionary

constexpr uint64_t HT_EMPTY = ~0ull;

// Insert one key into the chunk's global open-addressing table; returns the slot or -1 when
// the table is full / the chunk already fell back.  Plain loads are used where a stale
// value is harmless: keys only go EMPTY -> key (a stale EMPTY just leads to a CAS that
// returns the real key), and recorded ranks only decrease.
__device__ __forceinline__ int64_t global_insert(ChunkDesc &C, HtSlot *tab, uint32_t cap, uint64_t key,
                                                 uint64_t h, uint32_t rank, uint32_t esize, uint32_t max_dict_bytes,
                                                 bool is_bin, const DevCol &col, const uint8_t *data, uint64_t r,
                                                 uint64_t data_end, uint32_t *acc_n = nullptr,
                                                 unsigned long long *acc_b = nullptr)
{
    if (!is_bin && key == HT_EMPTY) {
        const uint32_t slot = cap;  // reserved slot for the sentinel value
        if (atomicCAS((unsigned long long *)&tab[slot].key, (unsigned long long)HT_EMPTY, 0ull) == HT_EMPTY) {
            const unsigned long long nb = atomicAdd((unsigned long long *)&C.dict_bytes, (unsigned long long)esize) + esize;
            atomicAdd(&C.dict_n, 1u);
            if (nb > max_dict_bytes) __hip_atomic_store(&C.fallback, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tab[slot].min > rank) atomicMin(&tab[slot].min, rank);
        return slot;
    }
    uint32_t i = (uint32_t)(h & (cap - 1));
    const uint32_t plim = C.ht_plim ? C.ht_plim : cap;   // hint-sized table: a long chain flags a retry
    for (uint32_t probe = 0; probe < plim; probe++) {
        uint64_t cur = tab[i].key;
        if (cur == HT_EMPTY) {
            const unsigned long long old = atomicCAS((unsigned long long *)&tab[i].key, (unsigned long long)HT_EMPTY, (unsigned long long)key);
            if (old == HT_EMPTY) {
                if (acc_n) {   // block-local totals, added to the chunk once per tile
                    atomicAdd(acc_n, 1u);
                    atomicAdd(acc_b, (unsigned long long)esize);
                } else {
                    const unsigned long long nb = atomicAdd((unsigned long long *)&C.dict_bytes, (unsigned long long)esize) + esize;
                    atomicAdd(&C.dict_n, 1u);
                    if (nb > max_dict_bytes) __hip_atomic_store(&C.fallback, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                atomicMin(&tab[i].min, rank);
                return i;
            }
            cur = old;
        }
        const bool eq = is_bin ? str_eq(col, data, cur, r, data_end) : cur == key;
        if (eq) {
            if (tab[i].min > rank) atomicMin(&tab[i].min, rank);
            return i;
        }
        i = (i + 1) & (cap - 1);
        if ((probe & 15) == 15 && __hip_atomic_load(&C.fallback, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return -1;
    }
    return -1;
}

// One block per chunk tile (2048 records).  Keys are first deduplicated in an LDS table
// (first rank per key within the tile); each distinct key then goes to the chunk's global
// table once, so low-cardinality columns do not serialise on a few hot global slots.
constexpr uint32_t LDS_T = 2048;
constexpr uint32_t LDS_PROBES = 32;

// BT threads per tile (KPW_BLOCK, or 1024 for a page-size probe: its few tiles are a chain of
// dependent global atomics per thread, 2048 / BT of them)
template <int BT>
__global__ void __launch_bounds__(BT) k_dict_insert(ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                    const uint32_t *order, const uint32_t *ctile_chunk, const uint32_t *ctile_first,
                                                    HtSlot *ht, uint32_t *slotof, uint32_t max_dict_bytes,
                                                    int exact, const uint64_t *data_end_p)
{
    constexpr int NK = KPW_TILE_P / BT;   // records per thread
    static_assert(NK * BT == KPW_TILE_P && KPW_TILE_P <= LDS_T, "tile / block shape");
    __shared__ uint64_t lkey[LDS_T];
    __shared__ uint32_t lmin[LDS_T];   // phase 1: first rank per key; phase 2 on: its global slot
    __shared__ uint16_t lrec[LDS_T];   // first record of the key, relative to the tile (28 KiB per block in all)
    __shared__ uint32_t acc_n;
    __shared__ unsigned long long acc_b;
    const uint64_t data_end = *data_end_p;
    const uint32_t t = order[blockIdx.x];
    const uint32_t ci = ctile_chunk[t];
    ChunkDesc &C = ch[ci];
    __shared__ uint32_t skip;
    if (!C.is_dict) return;
    // block-uniform: another block may set `fallback` while this one reads it
    if (threadIdx.x == 0) skip = __hip_atomic_load(&C.fallback, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (skip) return;
    if (C.stop_tile && t - ctile_first[ci] >= C.stop_tile) return;   // multi-page: past dictPageSize
    const DevCol col = cols[C.col];   // by value: not reloaded after stores
    const TileRecs T = tile_recs(C, col, t, ctile_first, ci);
    if (T.t0 >= T.e) return;   // past the chunk's records (a probe round's fixed tile count)
    const uint32_t cap = C.ht_cap;
    HtSlot *tab = ht + C.ht_off;
    // BYTE_ARRAY keys: the 64-bit hash computed by K1 (verified byte-for-byte afterwards in
    // k_dict_ids); `exact` re-runs with byte comparisons after a detected hash collision
    // (then the LDS stage is skipped: every value goes straight to the global table).
    const bool is_bin = col.phys == 6 && exact;
    for (uint32_t i = threadIdx.x; i < LDS_T; i += BT) { lkey[i] = HT_EMPTY; lmin[i] = 0xffffffffu; }
    if (threadIdx.x == 0) { acc_n = 0; acc_b = 0; }
    __syncthreads();
    int32_t li[NK];
    uint64_t keyv[NK];
    uint32_t rk[NK];
    // phase 1: LDS dedup
    for (int k = 0; k < NK; k++) {
        li[k] = -2;  // not present
        const uint64_t r = (T.t0 + (uint64_t)k * BT + threadIdx.x);
        if (r >= T.e) continue;
        if (!present_at(col, r)) continue;
        uint64_t key;
        if (is_bin) key = r;
        else if (col.phys == 6) key = col.shash[r];
        else key = fixed_val(col, r);
        keyv[k] = key;
        rk[k] = (uint32_t)T.rank(col, r);
        li[k] = -1;  // global path
        if (is_bin || key == HT_EMPTY) continue;
        uint32_t i = (uint32_t)(mix64(key) >> 40) & (LDS_T - 1);
        for (uint32_t probe = 0; probe < LDS_PROBES; probe++) {
            uint64_t cur = lkey[i];
            if (cur == HT_EMPTY) {
                const unsigned long long old = atomicCAS((unsigned long long *)&lkey[i], (unsigned long long)HT_EMPTY,
                                                         (unsigned long long)key);
                cur = old == HT_EMPTY ? key : old;
                if (old == HT_EMPTY) lrec[i] = (uint16_t)(r - T.t0);
            }
            if (cur == key) {
                atomicMin(&lmin[i], rk[k]);
                li[k] = (int32_t)i;
                break;
            }
            i = (i + 1) & (LDS_T - 1);
        }
    }
    __syncthreads();
    // phase 2: one global insert per distinct key of the tile
    for (uint32_t i = threadIdx.x; i < LDS_T; i += BT) {
        const uint64_t key = lkey[i];
        if (key == HT_EMPTY) continue;
        const uint64_t r = T.t0 + lrec[i];
        const uint32_t esize = col.phys == 6 ? 4 + col.slen[r] : (uint32_t)col.vsize;
        const int64_t g = global_insert(C, tab, cap, key, mix64(key), lmin[i], esize, max_dict_bytes, false, col, data, r,
                                        data_end, &acc_n, &acc_b);
        lmin[i] = g < 0 ? 0xffffffffu : (uint32_t)g;   // this thread owns slot i in phase 2
        if (g < 0 && !__hip_atomic_load(&C.fallback, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            atomicOr(&C.overflow, 1u);
            __hip_atomic_store(&C.fallback, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    // the tile's new entries: two chunk-wide atomics per tile instead of two per entry (a
    // high-cardinality tile would otherwise serialise 4096 atomics on one address)
    if (threadIdx.x == 0 && acc_n) {
        const unsigned long long nb = atomicAdd((unsigned long long *)&C.dict_bytes, acc_b) + acc_b;
        atomicAdd(&C.dict_n, acc_n);
        if (nb > max_dict_bytes) __hip_atomic_store(&C.fallback, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // phase 3: slots for every value (LDS hit or direct global insert)
    for (int k = 0; k < NK; k++) {
        if (li[k] == -2) continue;
        const uint64_t r = (T.t0 + (uint64_t)k * BT + threadIdx.x);
        int64_t g;
        if (li[k] >= 0) {
            g = lmin[li[k]] == 0xffffffffu ? -1 : (int64_t)lmin[li[k]];
        } else {
            if (__hip_atomic_load(&C.fallback, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
            uint64_t h;
            uint32_t esize;
            if (is_bin) { h = bytes_hash(data, col.soff[r], col.slen[r], data_end); esize = 4 + col.slen[r]; }
            else { h = mix64(keyv[k]); esize = col.phys == 6 ? 4 + col.slen[r] : (uint32_t)col.vsize; }
            g = global_insert(C, tab, cap, keyv[k], h, rk[k], esize, max_dict_bytes, is_bin, col, data, r, data_end);
            if (g < 0 && !__hip_atomic_load(&C.fallback, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                atomicOr(&C.overflow, 1u);
                __hip_atomic_store(&C.fallback, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (g < 0) return;
        slotof[C.ids_off + rk[k]] = (uint32_t)g;
    }
}

// count (write=0) / assign (write=1) first occurrences in record order.  In the coalesced
// tile layout record order is (k, wave, lane); the write pass ranks a thread's first
// occurrences with one ballot + one wave scan per k and 32 (k, wave) totals in LDS.
// per dictionary chunk after the insert pass: fallback, id width and id-job length
__device__ void dict_jobs(ChunkDesc &C, RleJob *jobs, uint32_t max_dict_bytes, uint32_t *retry)
{
    if (!C.is_dict) return;
    if (C.overflow && C.ht_plim) atomicOr(retry, 1u);   // hint-sized table too small: the host redoes the phase
    if (C.dict_bytes > max_dict_bytes || C.overflow) C.fallback = 1;
    if (C.id_job < 0) return;   // multi-page dictionary descriptor: pages carry the id jobs
    RleJob &J = jobs[C.id_job];
    if (C.fallback) { J.len = 0; J.bw = 0; return; }
    // DictionaryValuesWriter.getBytes: bitWidth = getWidthFromMaxInt(dictSize - 1)
    const uint32_t m = C.dict_n - 1;
    C.bw = m ? 32 - __clz(m) : (C.dict_n ? 0 : 32);
    J.len = C.nn;
    J.bw = C.bw;
}

__global__ void __launch_bounds__(KPW_BLOCK) k_dict_firsts(ChunkDesc *ch, const DevCol *cols, const uint32_t *ctile_chunk,
                                                           const uint32_t *ctile_first, HtSlot *ht,
                                                           const uint32_t *slotof, uint32_t *tile_cnt, uint64_t *tile_sz,
                                                           const uint32_t *tile_cnt_off, const uint64_t *tile_sz_off,
                                                           uint64_t *ent_rec, uint64_t *ent_boff, int write, RleJob *jobs,
                                                           uint32_t max_dict_bytes, uint32_t *retry, uint8_t *fmask)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    __shared__ uint32_t ldu[KPW_BLOCK];
    __shared__ uint32_t wcnt[8][KPW_BLOCK / 64];
    __shared__ uint64_t wsz[8][KPW_BLOCK / 64];
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    ChunkDesc &C = ch[ci];
    // the dictionary outcome (dict_jobs, stored by the chunk's first tile) from the insert pass, so no tile
    // depends on whether that store has happened yet
    const bool fb = C.fallback || C.dict_bytes > max_dict_bytes || C.overflow;
    if (!write && t == ctile_first[ci] && threadIdx.x == 0) dict_jobs(C, jobs, max_dict_bytes, retry);
    const bool active = C.is_dict && !fb && !(C.stop_tile && t - ctile_first[ci] >= C.stop_tile);
    const DevCol col = cols[C.col];   // by value: not reloaded after stores
    const TileRecs T = tile_recs(C, col, t, ctile_first, ci);
    uint32_t cnt = 0;
    uint64_t sz = 0;
    uint32_t firsts = 0;  // bitmask over the 8 records
    uint32_t esz[8];
    if (!write) {
        // the count pass finds the first occurrences (a slot and a table load per value) and keeps
        // them per thread in fmask, so the write pass loads nothing per value but that byte
        if (active) {
            for (int k = 0; k < 8; k++) {
                const uint64_t r = T.rec(k);
                if (r >= T.e) break;
                if (!present_at(col, r)) continue;
                const uint64_t rank = T.rank(col, r);
                const uint32_t slot = slotof[C.ids_off + rank];
                if (ht[C.ht_off + slot].min == (uint32_t)rank) {
                    firsts |= 1u << k;
                    cnt++;
                    sz += col.phys == 6 ? 4 + col.slen[r] : (uint32_t)col.vsize;
                }
            }
        }
        fmask[(uint64_t)t * KPW_BLOCK + threadIdx.x] = (uint8_t)firsts;
        const uint32_t sc = block_reduce<uint32_t, OpSum32>(cnt, ldu);
        const uint64_t ss = block_reduce<uint64_t, OpSum64>(sz, lds);
        if (threadIdx.x == 0) { tile_cnt[t] = sc; tile_sz[t] = ss; }
        return;
    }
    if (!active) return;   // block-uniform
    firsts = fmask[(uint64_t)t * KPW_BLOCK + threadIdx.x];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        esz[k] = 0;
        if ((firsts >> k) & 1) esz[k] = col.phys == 6 ? 4 + col.slen[T.rec(k)] : (uint32_t)col.vsize;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t lpre[8];
    uint64_t spre[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const bool f = (firsts >> k) & 1;
        const uint64_t m = __ballot(f);
        lpre[k] = (uint32_t)__popcll(m & lt);
        uint64_t x = f ? esz[k] : 0, inc = x;   // inclusive wave scan of entry sizes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        spre[k] = inc - x;
        if (lane == 63) { wcnt[k][w] = (uint32_t)__popcll(m); wsz[k][w] = inc; }
    }
    __syncthreads();
    if (!firsts) return;
    uint32_t ebase = tile_cnt_off[t] + C.ent_base;   // (a probe continuation numbers after the kept entries)
    uint64_t bbase = tile_sz_off[t] + C.boff_base;
    const int klast = 31 - __clz(firsts);
    for (int k = 0; k <= klast; k++) {
        for (int w2 = 0; w2 < KPW_BLOCK / 64; w2++) {
            if (((firsts >> k) & 1) && w2 == w) {   // my segment (k, w): emit, then keep counting
                const uint64_t r = T.rec(k);
                const uint64_t rank = T.rank(col, r);
                const uint32_t eid = ebase + lpre[k];
                const uint32_t slot = slotof[C.ids_off + rank];
                ht[C.ht_off + slot].id = eid;
                ent_rec[C.ent_off + eid] = r;
                ent_boff[C.ent_off + eid] = bbase + spre[k];
            }
            ebase += wcnt[k][w2];
            bbase += wsz[k][w2];
        }
    }
}

// slot -> id for every value (overwrites slotof in place); sets id-job width/length
__global__ void __launch_bounds__(KPW_BLOCK) k_dict_ids(const ChunkDesc *ch, const DevCol *cols, const uint32_t *ctile_chunk,
                                                        const uint32_t *ctile_first, const HtSlot *ht, uint32_t *ids,
                                                        const uint8_t *data, const uint64_t *ent_rec, const uint64_t *data_end_p,
                                                        uint32_t *collision)
{
    const uint64_t data_end = *data_end_p;
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    if (!C.is_dict || C.fallback) return;
    if (C.stop_tile && t - ctile_first[ci] >= C.stop_tile) return;   // multi-page: those pages are PLAIN
    // by value: the stores to ids[] below may not alias them, so their loads are not repeated
    const DevCol col = cols[C.col];
    const uint64_t ids_off = C.ids_off, ht_off = C.ht_off, ent_off = C.ent_off;
    const TileRecs T = tile_recs(C, col, t, ctile_first, ci);
    // three independent passes over the 8 records (positions, slots, ids) so each pass's
    // loads are in flight together instead of one dependent chain per record
    uint64_t o[8];
    bool ok[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t r = T.rec(k);
        ok[k] = r < T.e && present_at(col, r);
        o[k] = ok[k] ? ids_off + T.rank(col, r) : 0;
    }
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = ok[k] ? ids[o[k]] : 0;
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = ok[k] ? ht[ht_off + v[k]].id : 0;
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (ok[k]) ids[o[k]] = v[k];
    if (col.phys == 6) {   // verify the hash-keyed dictionary byte-for-byte
        bool bad = false;
        for (int k = 0; k < 8; k++)
            if (ok[k]) bad |= !str_eq(col, data, ent_rec[ent_off + v[k]], T.rec(k), data_end);
        if (bad) atomicOr(collision, 1u);
    }
}


// ------------------------------------------------------------------ layout (one block, all chunks)

// v2 level streams of max level 0: ColumnWriterV2's RunLengthBitPackingHybridEncoder of width 0
// after n writeInt(0) (parquet-mr 1.10.1 ParquetProperties.newLevelEncoder; v1 uses
// DevNullValuesWriter instead): nothing for n = 0, one bit-packed run header for n < 8 (0x03),
// else one RLE run header varint(n << 1) (the width-0 value takes no bytes).
__device__ __forceinline__ uint32_t rle0_len(uint64_t n) { return n == 0 ? 0u : n < 8 ? 1u : varint_len32((uint32_t)(n << 1)); }
__device__ __forceinline__ void rle0_put(uint8_t *p, uint64_t n)
{
    if (n == 0) return;
    if (n < 8) { p[0] = 3; return; }
    uint32_t v = (uint32_t)(n << 1);
    while (v >= 0x80u) { *p++ = (uint8_t)(v | 0x80u); v >>= 7; }
    *p = (uint8_t)v;
}

// Page bodies of every chunk, back to back: [dictionary page][data page].
//   v1 data page (ColumnWriterV1.writePage): dl = 4-byte length + RLE (optional) | values
//   v2 data page (ColumnWriterV2.writePage / writePageV2): dl = RLE without length (optional,
//      stays uncompressed: page_pre) | values (the compressed part); values = 1-byte bit
//      width + RLE ids (RLE_DICTIONARY), DELTA streams (INT32/INT64/BYTE_ARRAY fallback),
//      PLAIN (FLOAT/DOUBLE fallback) or 4-byte length + RLE (BOOLEAN)
__global__ void __launch_bounds__(KPW_BLOCK) k_layout(ChunkDesc *ch, int nchunks, const DevCol *cols, RleJob *jobs, uint64_t *page_off,
                                                      uint64_t *page_len, uint64_t *tot, int v2, DeltaJob *djobs,
                                                      const uint64_t *chunk_sfx, uint64_t *page_pre, int mp)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    uint64_t carry = 0;
    for (int b = 0; b < nchunks; b += KPW_BLOCK) {
        const int ci = b + threadIdx.x;
        uint64_t body = 0;
        if (ci < nchunks) {
            ChunkDesc &C = ch[ci];
            const DevCol &col = cols[C.col];
            C.dl_len = col.optional ? jobs[C.dl_job].total_bytes : 0;
            C.rl0_len = 0;
            if (v2) {   // every page: width-0 repetition levels; REQUIRED columns: width-0 definition levels
                C.rl0_len = (int32_t)rle0_len((uint64_t)(C.e - C.s));
                if (!col.optional) C.dl_len = C.rl0_len;
            }
            uint64_t val = 0, dictp = 0;
            if (C.is_dict && !C.fallback) {
                val = 1 + jobs[C.id_job].total_bytes;
                // FallbackValuesWriter.getBytes on the first page: isCompressionSatisfying
                // (multi-page: decided per chunk by k_mp_satisfy, dictionary page preset)
                if (mp) dictp = C.dictpage_len;
                else if (!(val + C.dict_bytes < C.raw_bytes)) C.fallback = 1;
                else dictp = C.dict_bytes;
            }
            if (!C.is_dict || C.fallback) {
                if (v2 && col.phys == 0) val = 4 + jobs[C.bool_job].total_bytes;
                else if (v2 && C.dj0 >= 0 && col.phys == 6) val = djobs[C.dj0].total + djobs[C.dj0 + 1].total + chunk_sfx[ci];
                else if (v2 && C.dj0 >= 0) val = djobs[C.dj0].total;
                else val = col.phys == 0 ? (uint64_t)(C.nn + 7) / 8 : C.raw_bytes;
                dictp = mp ? C.dictpage_len : 0;
                if (C.is_dict) {  // do not write ids
                    RleJob &J = jobs[C.id_job];
                    J.n_rle = 0; J.total_groups = 0; J.final_gap_groups = 0; J.total_bytes = 0;
                }
            }
            C.val_len = val;
            C.dictpage_len = dictp;
            const uint64_t lv = v2 ? (uint64_t)C.rl0_len + C.dl_len : col.optional ? 4 + C.dl_len : 0;
            body = dictp + lv + val;
        }
        uint64_t t2;
        const uint64_t ex = block_scan_excl<uint64_t, OpSum64>(body, lds, &t2) + carry;
        if (ci < nchunks) {
            ChunkDesc &C = ch[ci];
            const DevCol &col = cols[C.col];
            C.body_off = ex;
            const uint64_t dpage = ex + C.dictpage_len;
            const uint64_t lv = v2 ? (uint64_t)C.rl0_len + C.dl_len : col.optional ? 4 + C.dl_len : 0;
            C.val_off = dpage + lv;
            if (col.optional) jobs[C.dl_job].out_off = dpage + (v2 ? (uint64_t)C.rl0_len : 4);
            if (C.is_dict) jobs[C.id_job].out_off = C.val_off + 1;
            if (v2 && C.bool_job >= 0) jobs[C.bool_job].out_off = C.val_off + 4;
            if (v2 && C.dj0 >= 0 && C.fallback) {
                djobs[C.dj0].out_off = C.val_off;
                if (col.phys == 6) djobs[C.dj0 + 1].out_off = C.val_off + djobs[C.dj0].total;
            }
            page_off[2 * ci] = ex;
            page_len[2 * ci] = C.dictpage_len;
            if (v2) {   // the codec sees only the values; the levels go in front uncompressed
                page_off[2 * ci + 1] = C.val_off;
                page_len[2 * ci + 1] = C.val_len;
                page_pre[2 * ci] = 0;
                page_pre[2 * ci + 1] = lv;
            } else {
                page_off[2 * ci + 1] = dpage;
                page_len[2 * ci + 1] = body - C.dictpage_len;
            }
        }
        carry += t2;
    }
    if (threadIdx.x == 0) tot[0] = carry;
}

// ------------------------------------------------------------------ writers

__device__ __forceinline__ void chunk_header(const ChunkDesc *ch, int nchunks, const DevCol *cols, uint8_t *out, int v2,
                                             const RleJob *jobs, int ci)
{
    if (ci >= nchunks) return;
    const ChunkDesc &C = ch[ci];
    const DevCol col = cols[C.col];   // by value: not reloaded after stores
    if (col.optional && !v2) {   // v1: 4-byte length in front of the definition levels
        uint8_t *p = out + C.body_off + C.dictpage_len;
        const uint32_t l = (uint32_t)C.dl_len;
        p[0] = (uint8_t)l; p[1] = (uint8_t)(l >> 8); p[2] = (uint8_t)(l >> 16); p[3] = (uint8_t)(l >> 24);
    }
    if (v2) {   // width-0 repetition levels (+ definition levels of a REQUIRED column)
        uint8_t *p = out + C.body_off + C.dictpage_len;
        const uint64_t n = (uint64_t)(C.e - C.s);
        rle0_put(p, n);
        if (!col.optional) rle0_put(p + C.rl0_len, n);
    }
    uint8_t *p = out + C.val_off;
    if (C.is_dict && !C.fallback) p[0] = (uint8_t)C.bw;
    if (v2 && C.bool_job >= 0) {   // RunLengthBitPackingHybridValuesWriter.getBytes: 4-byte length
        const uint32_t l = (uint32_t)jobs[C.bool_job].total_bytes;
        p[0] = (uint8_t)l; p[1] = (uint8_t)(l >> 8); p[2] = (uint8_t)(l >> 16); p[3] = (uint8_t)(l >> 24);
    }
}

// String bytes to their page position: 32 independent byte loads per round trip (the bytes go
// to registers before any store, so the loads are not serialised behind the char-aliasing
// stores).
__device__ __forceinline__ void copy_bytes32(uint8_t *d, const uint8_t *src, uint32_t l)
{
    uint32_t i = 0;
    for (; i + 32 <= l; i += 32) {
        uint8_t b[32];
#pragma unroll
        for (int j = 0; j < 32; j++) b[j] = src[i + j];
#pragma unroll
        for (int j = 0; j < 32; j++) d[i + j] = b[j];
    }
    if (i < l) {
        uint8_t b[32];
#pragma unroll
        for (int j = 0; j < 32; j++) b[j] = i + j < l ? src[i + j] : 0;
#pragma unroll
        for (int j = 0; j < 32; j++)
            if (i + j < l) d[i + j] = b[j];
    }
}

__global__ void __launch_bounds__(KPW_BLOCK) k_dict_page(const ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                         const uint32_t *ctile_chunk, const uint32_t *ctile_first,
                                                         const uint64_t *ent_rec, const uint64_t *ent_boff, uint8_t *out)
{
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    if (!C.is_dict || C.fallback) return;
    const DevCol col = cols[C.col];   // by value: not reloaded after stores
    const uint64_t e0 = (uint64_t)(t - ctile_first[ci]) * KPW_TILE_P + threadIdx.x * 8;
    uint8_t *page = out + C.body_off;
    for (int k = 0; k < 8; k++) {
        const uint64_t e = e0 + k;
        if (e >= C.dict_n) break;
        const uint64_t r = ent_rec[C.ent_off + e];
        uint8_t *o = page + ent_boff[C.ent_off + e];
        if (col.phys == 6) {
            const uint32_t l = col.slen[r];
            o[0] = (uint8_t)l; o[1] = (uint8_t)(l >> 8); o[2] = (uint8_t)(l >> 16); o[3] = (uint8_t)(l >> 24);
            const uint8_t *src = data + col.soff[r];
            copy_bytes32(o + 4, src, l);
        } else {
            const uint64_t v = fixed_val(col, r);
            for (int i = 0; i < col.vsize; i++) o[i] = (uint8_t)(v >> (8 * i));
        }
    }
}

// PLAIN values (fixed / binary) for chunks without dictionary encoding
__global__ void __launch_bounds__(KPW_BLOCK) k_plain(const ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                     const uint32_t *ctile_chunk, const uint32_t *ctile_first,
                                                     const uint64_t *tile_raw_off, uint8_t *out)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    const DevCol col = cols[C.col];   // by value: not reloaded after stores
    if ((C.is_dict && !C.fallback) || col.phys == 0 || C.dj0 >= 0) return;   // dj0: v2 DELTA fallback instead
    const uint64_t p0 = (uint64_t)C.s + (uint64_t)(t - ctile_first[ci]) * KPW_TILE_P + threadIdx.x * 8;
    uint8_t *vout = out + C.val_off;
    if (col.phys == 6) {
        uint64_t sz = 0;
        for (int k = 0; k < 8; k++) {
            const uint64_t r = p0 + k;
            if (r >= (uint64_t)C.e) break;
            if (present_at(col, r)) sz += 4 + col.slen[r];
        }
        uint64_t tot;
        uint64_t o = block_scan_excl<uint64_t, OpSum64>(sz, lds, &tot) + tile_raw_off[t];
        for (int k = 0; k < 8; k++) {
            const uint64_t r = p0 + k;
            if (r >= (uint64_t)C.e) break;
            if (!present_at(col, r)) continue;
            const uint32_t l = col.slen[r];
            uint8_t *d = vout + o;
            d[0] = (uint8_t)l; d[1] = (uint8_t)(l >> 8); d[2] = (uint8_t)(l >> 16); d[3] = (uint8_t)(l >> 24);
            const uint8_t *src = data + col.soff[r];
            copy_bytes32(d + 4, src, l);
            o += 4 + l;
        }
    } else {
        const TileRecs T = tile_recs(C, col, t, ctile_first, ci);
        for (int k = 0; k < 8; k++) {
            const uint64_t r = T.rec(k);
            if (r >= T.e) break;
            if (!present_at(col, r)) continue;
            const uint64_t v = fixed_val(col, r);
            uint8_t *d = vout + T.rank(col, r) * col.vsize;
            if (col.vsize == 8) {
                if (((uintptr_t)d & 7) == 0) { *(uint64_t *)d = v; continue; }
            } else if (col.vsize == 4) {
                if (((uintptr_t)d & 3) == 0) { *(uint32_t *)d = (uint32_t)v; continue; }
            }
            for (int i = 0; i < col.vsize; i++) d[i] = (uint8_t)(v >> (8 * i));
        }
    }
}

// BooleanPlainValuesWriter: compacted value bits, LSB first (output pre-zeroed)
// position of the j-th (0-based) set bit of m (m has more than j set bits)
__device__ __forceinline__ uint32_t select_bit(uint64_t m, uint32_t j)
{
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t w = 32; w >= 1; w >>= 1) {
        const uint64_t low = m & ((1ull << w) - 1);
        const uint32_t c = (uint32_t)__popcll(low);
        if (j >= c) { j -= c; m >>= w; pos += w; }
        else m = low;
    }
    return pos;
}

// PLAIN booleans (BooleanPlainValuesWriter: LSB-first bit packing).  Each wave packs its 64
// records per step with ballots: the values of the present records, in rank order, become one
// 64-bit word (lane j picks the j-th present lane), and lane 0 ORs it into the output at the
// slice's first rank (at most three 32-bit atomics per 64 records instead of one per true value).
__global__ void __launch_bounds__(KPW_BLOCK) k_plain_bool(const ChunkDesc *ch, const DevCol *cols, const uint32_t *ctile_chunk,
                                                          const uint32_t *ctile_first, uint8_t *out)
{
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    const DevCol col = cols[C.col];
    if (col.phys != 0 || C.bool_job >= 0) return;   // bool_job: v2 RLE booleans instead
    const TileRecs T = tile_recs(C, col, t, ctile_first, ci);
    const uint64_t base_bit = C.val_off * 8;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t *o32 = (uint32_t *)out;
    for (int k = 0; k < 8; k++) {
        const uint64_t r = T.rec(k);
        const uint64_t r0 = r - lane;   // the wave's first record of this step
        if (r0 >= T.e) break;           // wave-uniform
        const bool pres = r < T.e && present_at(col, r);
        const bool val = pres && ((col.vbits[r >> 6] >> (r & 63)) & 1ull);
        const uint64_t pm = __ballot(pres), tm = __ballot(val);
        const uint32_t cnt = (uint32_t)__popcll(pm);
        const bool bit = lane < cnt && ((tm >> select_bit(pm, lane)) & 1ull);
        const uint64_t P = __ballot(bit);
        if (lane == 0 && P) {
            const uint64_t B = base_bit + T.rank(col, r0);
            const uint64_t w = B >> 5;
            const uint32_t sh = (uint32_t)(B & 31);
            const uint64_t lo = P << sh;
            const uint32_t hi = sh ? (uint32_t)(P >> (64 - sh)) : 0u;
            if ((uint32_t)lo) atomicOr(&o32[w], (uint32_t)lo);
            if ((uint32_t)(lo >> 32)) atomicOr(&o32[w + 1], (uint32_t)(lo >> 32));
            if (hi) atomicOr(&o32[w + 2], hi);
        }
    }
}

// Zero the values part of the PLAIN boolean pages before k_plain_bool ORs its words in (the rest
// of the page body is written in full by its kernels, so the body is not cleared as a whole).
// 16 blocks per chunk: the dwords inside the range with dword stores, the edge bytes with byte stores.
constexpr uint32_t ZB_BLOCKS = 16;
__device__ __forceinline__ void zero_bool(const ChunkDesc *ch, const DevCol *cols, uint8_t *out, uint32_t chunk, uint32_t y)
{
    const ChunkDesc &C = ch[chunk];
    const DevCol col = cols[C.col];
    if (col.phys != 0 || C.bool_job >= 0 || C.val_len == 0) return;
    const uint64_t b = C.val_off, e = C.val_off + C.val_len;
    const uint64_t wb = (b + 3) & ~3ull, we = e & ~3ull;
    const uint64_t tid = (uint64_t)y * KPW_BLOCK + threadIdx.x, nth = (uint64_t)ZB_BLOCKS * KPW_BLOCK;
    if (wb >= we) {
        for (uint64_t i = b + tid; i < e; i += nth) out[i] = 0;
        return;
    }
    uint32_t *o32 = (uint32_t *)out;
    for (uint64_t w = (wb >> 2) + tid; w < (we >> 2); w += nth) o32[w] = 0u;
    if (tid < wb - b) out[b + tid] = 0;
    if (tid < e - we) out[we + tid] = 0;
}

// One launch before the page writers: blocks [0, hb) the chunks' level-stream headers (a thread
// per chunk), then ZB_BLOCKS per chunk zeroing the PLAIN boolean ranges, then one block clearing
// the 512 bytes at tail_off (the body's end) that K7's read windows may reach past the last page.
__global__ void __launch_bounds__(KPW_BLOCK) k_chunk_prep(const ChunkDesc *ch, int nchunks, const DevCol *cols, uint8_t *out, int v2,
                                                          const RleJob *jobs, uint32_t hb, uint64_t tail_off)
{
    if (blockIdx.x < hb) { chunk_header(ch, nchunks, cols, out, v2, jobs, (int)(blockIdx.x * KPW_BLOCK + threadIdx.x)); return; }
    const uint32_t b = blockIdx.x - hb;
    if (b < (uint32_t)nchunks * ZB_BLOCKS) { zero_bool(ch, cols, out, b / ZB_BLOCKS, b % ZB_BLOCKS); return; }
    out[tail_off + threadIdx.x] = 0;
    out[tail_off + KPW_BLOCK + threadIdx.x] = 0;
}

// Binary statistics: meta[4c..4c+3] = (min offset, min len, max offset | eq << 63, max len) of
// chunk c, eq = the min and max values are the same bytes (pass 1, blob == nullptr: what a
// page-size probe needs for the header sizes); pass 2 copies the bytes into blob at the running
// offset.
__global__ void __launch_bounds__(KPW_BLOCK) k_stats_gather(const ChunkDesc *ch, int nchunks, const DevCol *cols,
                                                            const uint8_t *data, uint64_t *meta, uint8_t *blob)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    uint64_t carry = 0;
    for (int b = 0; b < nchunks; b += KPW_BLOCK) {
        const int ci = b + threadIdx.x;
        uint64_t len = 0;
        bool bin = false;
        if (ci < nchunks) {
            const ChunkDesc &C = ch[ci];
            const DevCol &col = cols[C.col];
            bin = col.phys == 6 && C.nn > 0;   // has_minmax
            if (!blob) {
                if (bin) {
                    const uint64_t o1 = col.soff[C.smin], o2 = col.soff[C.smax];
                    const uint32_t l1 = col.slen[C.smin], l2 = col.slen[C.smax];
                    bool eq = l1 == l2;
                    for (uint32_t i = 0; eq && i < l1; i++) eq = data[o1 + i] == data[o2 + i];
                    meta[4 * ci] = o1; meta[4 * ci + 1] = l1;
                    meta[4 * ci + 2] = o2 | ((uint64_t)eq << 63); meta[4 * ci + 3] = l2;
                } else {
                    meta[4 * ci] = meta[4 * ci + 1] = meta[4 * ci + 2] = meta[4 * ci + 3] = 0;
                }
            } else if (bin) {
                len = meta[4 * ci + 1] + meta[4 * ci + 3];
            }
        }
        if (!blob) continue;
        uint64_t tot;
        const uint64_t o = block_scan_excl<uint64_t, OpSum64>(len, lds, &tot) + carry;
        if (ci < nchunks && bin) {
            const uint64_t l1 = meta[4 * ci + 1], l2 = meta[4 * ci + 3];
            for (uint64_t i = 0; i < l1; i++) blob[o + i] = data[meta[4 * ci] + i];
            const uint64_t o2 = meta[4 * ci + 2] & ~(1ull << 63);
            for (uint64_t i = 0; i < l2; i++) blob[o + l1 + i] = data[o2 + i];
        }
        carry += tot;
    }
}

void launch_stats_gather(const ChunkDesc *ch, int nchunks, const DevCol *cols, const uint8_t *data, uint64_t *meta,
                         uint8_t *blob, hipStream_t s)
{
    hipLaunchKernelGGL(k_stats_gather, dim3(1), dim3(KPW_BLOCK), 0, s, ch, nchunks, cols, data, meta, blob);
}

// ------------------------------------------------------------------ host launchers

void launch_chunk_stats(const ChunkArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(k_chunk_stats, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_chunk, a.ctile_first,
                       a.tile_raw, a.tile_smin, a.tile_smax, a.data_end, (uint4 *)a.ht_clear, a.ht_clear_n,
                       a.flags_clear);
}

// multi-page dictionary rounds: a chunk whose dictionary passed dictPageSize with the tiles of
// the rounds so far skips its later tiles (their values fall in the fallback page or after it,
// so they need no ids); stop is decided between rounds, so no earlier tile is ever skipped
__global__ void k_mp_dict_stop(ChunkDesc *ch, int nchunks, uint32_t round_end, uint32_t limit)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    ChunkDesc &C = ch[c];
    if (C.is_dict && !C.stop_tile && C.dict_bytes > limit) C.stop_tile = round_end;
}

void launch_dict(const ChunkArgs &a, RleJob *jobs, hipStream_t s)
{
    if (a.ndict_tiles && a.mp_nrounds) {
        // dict_order is round-major (tile k of every chunk before tile k + 1): a round is a slice
        uint32_t o = 0;
        for (uint32_t j = 0; j < a.mp_nrounds; j++) {
            const uint32_t cnt = a.mp_round_len[j];
            if (j)
                hipLaunchKernelGGL(k_mp_dict_stop, dim3((a.nchunks + 63) / 64), dim3(64), 0, s, a.ch, a.nchunks,
                                   a.mp_round_end[j - 1], a.mp_dict_limit);
            if (cnt && a.dict_wide)
                hipLaunchKernelGGL(k_dict_insert<1024>, dim3(cnt), dim3(1024), 0, s, a.ch, a.cols, a.data, a.dict_order + o,
                                   a.ctile_chunk, a.ctile_first, a.ht, a.ids, a.max_dict_bytes, a.exact_strings, a.data_end);
            else if (cnt)
                hipLaunchKernelGGL(k_dict_insert<KPW_BLOCK>, dim3(cnt), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.dict_order + o,
                                   a.ctile_chunk, a.ctile_first, a.ht, a.ids, a.max_dict_bytes, a.exact_strings, a.data_end);
            o += cnt;
        }
    } else if (a.ndict_tiles) {
        hipLaunchKernelGGL(k_dict_insert<KPW_BLOCK>, dim3(a.ndict_tiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.dict_order,
                           a.ctile_chunk, a.ctile_first, a.ht, a.ids, a.max_dict_bytes, a.exact_strings, a.data_end);
    }
    hipLaunchKernelGGL(k_dict_firsts, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.ctile_chunk, a.ctile_first,
                       a.ht, a.ids, a.tile_cnt, a.tile_sz, a.tile_cnt, a.tile_sz, a.ent_rec, a.ent_boff, 0, jobs, a.max_dict_bytes,
                       a.collision + 1, a.fmask);
    seg_tile_scan_u32(a.tile_cnt, a.tile_cnt, a.ctile_chunk, a.nctiles, a.seg, s);
    seg_tile_scan_u64(a.tile_sz, a.tile_sz, a.ctile_chunk, a.nctiles, a.seg, s);
    hipLaunchKernelGGL(k_dict_firsts, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.ctile_chunk, a.ctile_first,
                       a.ht, a.ids, a.tile_cnt, a.tile_sz, a.tile_cnt, a.tile_sz, a.ent_rec, a.ent_boff, 1, jobs, a.max_dict_bytes,
                       a.collision + 1, a.fmask);
    hipLaunchKernelGGL(k_dict_ids, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.ctile_chunk, a.ctile_first, a.ht, a.ids,
                       a.data, a.ent_rec, a.data_end, a.collision);
    // BYTE_ARRAY statistics need the dictionary outcome (entries stand in for the values);
    // multi-page dictionary descriptors have no statistics (their pages do)
    if (a.mp) return;
    hipLaunchKernelGGL(k_str_minmax, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_chunk, a.ctile_first,
                       a.ent_rec, a.tile_smin, a.tile_smax, a.data_end, 0);
    hipLaunchKernelGGL(k_str_final, dim3(a.nchunks), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_first, a.ctile_count,
                       a.tile_smin, a.tile_smax, a.data_end);
}

void launch_page_str_stats(const ChunkArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(k_str_minmax, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_chunk, a.ctile_first,
                       a.ent_rec, a.tile_smin, a.tile_smax, a.data_end, 1);
    hipLaunchKernelGGL(k_str_final, dim3(a.nchunks), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_first, a.ctile_count,
                       a.tile_smin, a.tile_smax, a.data_end);
}

void launch_layout(const ChunkArgs &a, RleJob *jobs, uint64_t *page_off, uint64_t *page_len, uint64_t *tot, hipStream_t s)
{
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(KPW_BLOCK), 0, s, a.ch, a.nchunks, a.cols, jobs, page_off, page_len, tot, a.v2,
                       a.djobs_w, a.chunk_sfx, a.page_pre, a.mp);
}

void launch_chunk_write(const ChunkArgs &a, const RleJob *jobs, uint8_t *out, hipStream_t s)
{
    const uint32_t hb = (uint32_t)((a.nchunks + KPW_BLOCK - 1) / KPW_BLOCK);
    hipLaunchKernelGGL(k_chunk_prep, dim3(hb + (uint32_t)a.nchunks * ZB_BLOCKS + 1), dim3(KPW_BLOCK), 0, s, a.ch, a.nchunks, a.cols, out,
                       a.v2, jobs, hb, a.body_tail);
    if (!a.mp)   // multi-page: the dictionary page is written from the dictionary descriptors
        hipLaunchKernelGGL(k_dict_page, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_chunk, a.ctile_first,
                           a.ent_rec, a.ent_boff, out);
    seg_tile_scan_u64(a.tile_raw, a.tile_raw_off, a.ctile_chunk, a.nctiles, a.seg, s);
    hipLaunchKernelGGL(k_plain, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_chunk, a.ctile_first,
                       a.tile_raw_off, out);
    hipLaunchKernelGGL(k_plain_bool, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.ctile_chunk, a.ctile_first, out);
}

// ------------------------------------------------------------------ multi-page (v1) dictionary decisions
//
// A column chunk's dictionary (first-occurrence ids over the whole chunk) is built on its
// dictionary descriptor with no size limit; the pages then take parquet-mr's decisions:
//  * FallbackValuesWriter.checkFallback: the first entry whose dictionaryByteSize pushes the
//    total past dictPageSize lands in page F; pages before F keep ids, F and later are PLAIN
//    (fallBackAllValuesTo rewrites F's values);
//  * DictionaryValuesWriter.getBytes: bit width of page p = width(entries seen by p's end - 1);
//  * isCompressionSatisfying on the first page only (all pages PLAIN when it fails);
//  * toDictPageAndClose: entries [0, lastUsedDictionarySize) of the last dictionary page.
__global__ void k_mp_pages_init(ChunkDesc *pg, int npg, const ChunkDesc *dch, const DevCol *cols, RleJob *jobs)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npg) return;
    ChunkDesc &C = pg[p];
    const ChunkDesc &D = dch[C.owner];
    const DevCol &col = cols[C.col];
    const uint64_t r0 = col.optional ? pres_rank(col, (uint64_t)D.s) : (uint64_t)D.s;
    const uint64_t rp = col.optional ? pres_rank(col, (uint64_t)C.s) : (uint64_t)C.s;
    C.ids_off = D.ids_off + (rp - r0);
    C.ent_off = D.ent_off;
    if (C.id_job >= 0) jobs[C.id_job].src.base = C.ids_off;
}

// bytes of the first k entries (dictionaryByteSize after k insertions)
__device__ __forceinline__ uint64_t ent_cum(const DevCol &col, const ChunkDesc &D, const uint64_t *ent_rec, const uint64_t *ent_boff,
                                            uint32_t k)
{
    if (!k) return 0;
    const uint64_t r = ent_rec[D.ent_off + k - 1];
    return ent_boff[D.ent_off + k - 1] + (col.phys == 6 ? 4u + col.slen[r] : (uint32_t)col.vsize);
}

__global__ void k_mp_dict_decide(ChunkDesc *pg, int npg, const ChunkDesc *dch, const DevCol *cols, const uint64_t *ent_rec,
                                 const uint64_t *ent_boff, uint32_t max_dict_bytes, RleJob *jobs)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npg) return;
    ChunkDesc &C = pg[p];
    if (!C.is_dict) return;
    const ChunkDesc &D = dch[C.owner];
    const DevCol &col = cols[C.col];
    const uint32_t dn = D.dict_n;
    // fallback record: smallest k with cum(k) > max -> entry k-1 first occurs at ent_rec[k-1]
    int64_t xf = -1;
    if (ent_cum(col, D, ent_rec, ent_boff, dn) > max_dict_bytes) {
        uint32_t lo = 1, hi = dn;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (ent_cum(col, D, ent_rec, ent_boff, mid) > max_dict_bytes) hi = mid; else lo = mid + 1;
        }
        xf = (int64_t)ent_rec[D.ent_off + lo - 1];
    }
    // entries first seen before the page end (ent_rec increases with the id)
    uint32_t lo = 0, hi = dn;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if ((int64_t)ent_rec[D.ent_off + mid] < C.e) lo = mid + 1; else hi = mid;
    }
    C.dict_n = lo;
    C.dict_bytes = ent_cum(col, D, ent_rec, ent_boff, lo);
    C.fallback = (xf >= 0 && xf < C.e) ? 1u : 0u;
    const uint32_t m = lo - 1;
    C.bw = lo ? (m ? 32 - __clz(m) : 0) : 32;
    RleJob &J = jobs[C.id_job];
    J.len = C.fallback ? 0 : C.nn;
    J.bw = C.fallback ? 0 : C.bw;
}

// per chunk (one block each, threads over its pages), after the RLE structure of the pages' id streams
__global__ void __launch_bounds__(KPW_BLOCK) k_mp_satisfy(ChunkDesc *pg, ChunkDesc *dch, int ndch, const DevCol *cols,
                                                           const uint64_t *ent_rec, const uint64_t *ent_boff, const RleJob *jobs)
{
    __shared__ int32_t lds[KPW_BLOCK];
    __shared__ int all_plain;
    const int d = blockIdx.x;
    ChunkDesc &D = dch[d];
    if (!D.is_dict) return;   // block-uniform
    const DevCol &col = cols[D.col];
    ChunkDesc &P0 = pg[D.first_page];
    const int p0 = D.first_page, p1 = D.first_page + D.npages;
    if (threadIdx.x == 0) {
        D.dict_all = D.dict_n;
        // tail_mode 2: the kept pages are PLAIN, so is the chunk's last page; 0: isCompressionSatisfying
        // on the chunk's first page (1: the kept first page passed it)
        int ap = D.tail_mode == 2;
        if (D.tail_mode == 0 && !P0.fallback) {
            const uint64_t val = 1 + jobs[P0.id_job].total_bytes;
            if (!(val + P0.dict_bytes < P0.raw_bytes)) ap = 1;
        }
        all_plain = ap;
    }
    __syncthreads();
    if (all_plain) {
        for (int p = p0 + (int)threadIdx.x; p < p1; p += KPW_BLOCK) pg[p].fallback = 1;
        if (threadIdx.x == 0) { D.fallback = 1; P0.dictpage_len = 0; }
        return;
    }
    // the last dictionary-encoded page (the fallback pages are a suffix)
    int last = -1;
    for (int p = p0 + (int)threadIdx.x; p < p1; p += KPW_BLOCK) if (!pg[p].fallback) last = p;
    lds[threadIdx.x] = last;
    __syncthreads();
    for (int o = KPW_BLOCK / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) lds[threadIdx.x] = max(lds[threadIdx.x], lds[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x) return;
    last = lds[0];
    const uint32_t dn = last >= 0 ? pg[last].dict_n : (D.tail_mode == 1 ? D.tail_dict_n : 0u);
    if (dn > 0) {
        D.dict_n = dn;
        D.fallback = 0;
        P0.dictpage_len = ent_cum(col, D, ent_rec, ent_boff, dn);
    } else {
        D.fallback = 1;
        P0.dictpage_len = 0;
    }
}

__global__ void k_mp_dictpage_off(const ChunkDesc *pg, ChunkDesc *dch, int ndch)
{
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ndch || dch[d].npages <= 0) return;   // (a probe's columns outside its subset have no pages)
    dch[d].body_off = pg[dch[d].first_page].body_off;
}

void launch_mp_pages_init(ChunkDesc *pg, int npg, const ChunkDesc *dch, const DevCol *cols, RleJob *jobs, hipStream_t s)
{
    hipLaunchKernelGGL(k_mp_pages_init, dim3((npg + 255) / 256), dim3(256), 0, s, pg, npg, dch, cols, jobs);
}
void launch_dict_page(const ChunkArgs &a, uint8_t *out, hipStream_t s)
{
    hipLaunchKernelGGL(k_dict_page, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, a.ch, a.cols, a.data, a.ctile_chunk, a.ctile_first,
                       a.ent_rec, a.ent_boff, out);
}
void launch_mp_dict_decide(ChunkDesc *pg, int npg, const ChunkDesc *dch, const DevCol *cols, const uint64_t *ent_rec,
                           const uint64_t *ent_boff, uint32_t max_dict_bytes, RleJob *jobs, hipStream_t s)
{
    hipLaunchKernelGGL(k_mp_dict_decide, dim3((npg + 255) / 256), dim3(256), 0, s, pg, npg, dch, cols, ent_rec, ent_boff,
                       max_dict_bytes, jobs);
}
void launch_mp_satisfy(ChunkDesc *pg, ChunkDesc *dch, int ndch, const DevCol *cols, const uint64_t *ent_rec,
                       const uint64_t *ent_boff, const RleJob *jobs, hipStream_t s)
{
    if (ndch) hipLaunchKernelGGL(k_mp_satisfy, dim3(ndch), dim3(KPW_BLOCK), 0, s, pg, dch, ndch, cols, ent_rec, ent_boff, jobs);
}
void launch_mp_dictpage_off(const ChunkDesc *pg, ChunkDesc *dch, int ndch, hipStream_t s)
{
    hipLaunchKernelGGL(k_mp_dictpage_off, dim3((ndch + 255) / 256), dim3(256), 0, s, pg, dch, ndch);
}

}  // namespace kpw
