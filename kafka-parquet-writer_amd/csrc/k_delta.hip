// k_delta.hip — A10, the PARQUET_2_0 fallback writers, byte-identical to parquet-mr 1.10.1
// (restated value by value in oracle/oracle_core.c delta_* / dba_*):
//   DeltaBinaryPackingValuesWriterForInteger / ForLong   INT32 / INT64 fallback pages
//   DeltaByteArrayWriter                                 BYTE_ARRAY fallback pages
//     = prefix lengths (DELTA_BINARY_PACKED) | suffix lengths (DELTA_BINARY_PACKED) | suffixes
// plus the v2 per-chunk decisions and the v2 boolean value streams (RLE, bit width 1).
//
// A stream of n values = header (varint 128, varint 4, varint n, zigzag first value) +
// ceil((n-1)/128) blocks of 128 deltas: zigzag min delta, 4 miniblock widths, then each
// present miniblock packed LSB-first (32 values x width bits).  Blocks are independent but
// for parquet-mr's never-cleared buffers: a partial last block writes block b-1's widths
// for the miniblocks it lacks and packs block b-1's min-reduced deltas into the padding of
// its last miniblock (zeros for block 0).  One wave per block; block sizes -> segmented
// scan per stream -> write (the header by the stream's first block tile).
#include "kpw_device.h"
#include "kpw_kernels.h"
#include "kpw_chunk.h"

namespace kpw {

__device__ __forceinline__ uint64_t dj_val(const DeltaJob &J, uint64_t i)
{
    if (J.flags & DJ_U32_SRC) return ((const uint32_t *)J.vals)[J.base + i];
    return ((const uint64_t *)J.vals)[J.base + i];
}
// delta i = v[i+1] - v[i] in the stream's arithmetic width (Java int / long wrapping)
__device__ __forceinline__ uint64_t dj_delta(const DeltaJob &J, uint64_t i)
{
    const uint64_t d = dj_val(J, i + 1) - dj_val(J, i);
    return (J.flags & DJ_LONG) ? d : (uint64_t)(uint32_t)d;
}
__device__ __forceinline__ int64_t dj_signed(const DeltaJob &J, uint64_t d)
{
    return (J.flags & DJ_LONG) ? (int64_t)d : (int64_t)(int32_t)(uint32_t)d;
}
// zigzag of a value in the stream's width (writeZigZagVarInt / writeZigZagVarLong)
__device__ __forceinline__ uint64_t dj_zigzag(const DeltaJob &J, uint64_t bits)
{
    if (J.flags & DJ_LONG) { const int64_t v = (int64_t)bits; return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }
    const int32_t w = (int32_t)(uint32_t)bits;
    return (uint64_t)(((uint32_t)w << 1) ^ (uint32_t)(w >> 31));
}
__device__ __forceinline__ uint32_t varint_len64(uint64_t v)
{
    uint32_t n = 1;
    while (v >= 0x80u) { v >>= 7; n++; }
    return n;
}
__device__ __forceinline__ uint8_t *put_varint64(uint8_t *o, uint64_t v)
{
    while (v >= 0x80u) { *o++ = (uint8_t)(v | 0x80u); v >>= 7; }
    *o++ = (uint8_t)v;
    return o;
}
__device__ __forceinline__ uint32_t bitlen64(uint64_t x) { return x ? 64u - (uint32_t)__clzll((long long)x) : 0u; }

__device__ __forceinline__ int64_t wave_min_i64(int64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t x = __shfl_xor(v, o, 64);
        v = x < v ? x : v;
    }
    return v;
}
// OR over each 32-lane half (lanes 0-31, 32-63)
__device__ __forceinline__ uint64_t half_or_u64(uint64_t v)
{
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ uint64_t rank_of(const DevCol &c, uint64_t y)
{
    const uint64_t wi = y >> 6;
    const uint64_t mm = (y & 63) ? (c.pres[wi] & ((1ull << (y & 63)) - 1)) : 0ull;
    return (uint64_t)c.pcnt[wi] + (uint64_t)__popcll(mm);
}

struct DBlock {
    uint32_t nd;       // deltas in this block (0: inactive)
    uint64_t d0;       // index of its first delta
};
__device__ __forceinline__ DBlock dj_block(const DeltaJob &J, uint32_t k)
{
    DBlock B;
    const uint64_t nd_all = J.n > 1 ? (uint64_t)J.n - 1 : 0;
    B.d0 = (uint64_t)k * 128;
    B.nd = B.d0 < nd_all ? (uint32_t)((nd_all - B.d0) < 128 ? (nd_all - B.d0) : 128) : 0;
    return B;
}

// per block: min delta, widths of the present miniblocks (w0 | w1<<8 | w2<<16 | w3<<24),
// encoded size
__global__ void __launch_bounds__(64) k_delta_blocks(const DeltaJob *jobs, const uint32_t *blk_job, uint64_t *blk_min,
                                                     uint32_t *blk_w, uint64_t *blk_sz)
{
    const uint32_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const DeltaJob &J = jobs[blk_job[b]];
    const DBlock B = dj_block(J, b - J.blk0);
    if (!B.nd || (J.flags & DJ_INACTIVE)) {
        if (lane == 0) { blk_min[b] = 0; blk_w[b] = 0; blk_sz[b] = 0; }
        return;
    }
    const bool v0 = (uint32_t)lane < B.nd, v1 = (uint32_t)lane + 64 < B.nd;
    const uint64_t x0 = v0 ? dj_delta(J, B.d0 + lane) : 0, x1 = v1 ? dj_delta(J, B.d0 + lane + 64) : 0;
    int64_t m = INT64_MAX;
    if (v0) m = dj_signed(J, x0);
    if (v1) { const int64_t s1 = dj_signed(J, x1); m = s1 < m ? s1 : m; }
    m = wave_min_i64(m);
    const uint64_t wmask = (J.flags & DJ_LONG) ? ~0ull : 0xffffffffull;
    const uint64_t o0 = half_or_u64(v0 ? ((x0 - (uint64_t)m) & wmask) : 0);
    const uint64_t o1 = half_or_u64(v1 ? ((x1 - (uint64_t)m) & wmask) : 0);
    const uint32_t w0 = bitlen64(__shfl(o0, 0, 64)), w1 = bitlen64(__shfl(o0, 32, 64));
    const uint32_t w2 = bitlen64(__shfl(o1, 0, 64)), w3 = bitlen64(__shfl(o1, 32, 64));
    if (lane == 0) {
        const uint32_t nmb = (B.nd + 31) / 32;
        const uint32_t w[4] = {w0, nmb > 1 ? w1 : 0u, nmb > 2 ? w2 : 0u, nmb > 3 ? w3 : 0u};
        uint64_t sz = varint_len64(dj_zigzag(J, (uint64_t)m)) + 4;
        for (uint32_t q = 0; q < nmb; q++) sz += 4ull * w[q];
        blk_min[b] = (uint64_t)m;
        blk_w[b] = w[0] | (w[1] << 8) | (w[2] << 16) | (w[3] << 24);
        blk_sz[b] = sz;
    }
}

// per stream: header size and total (block sizes summed per stream into btot[job])
__global__ void k_delta_totals(DeltaJob *jobs, int njobs, const uint64_t *btot)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= njobs) return;
    DeltaJob &J = jobs[j];
    if (J.flags & DJ_INACTIVE) { J.hdr = 0; J.total = 0; return; }
    const uint64_t first = J.n ? dj_val(J, 0) : 0;
    J.hdr = 2 + 1 + varint_len64(J.n) + varint_len64(dj_zigzag(J, first));
    J.total = J.hdr + btot[j];
}

// DeltaBinaryPackingValuesWriter.reset() clears neither deltaBlockBuffer nor bitWidths, and the
// fallback writer lives on across a column chunk's pages (multi-page regime): a page whose first
// block is partial writes the widths / padding slots the streams of the previous pages left.
// Slot p (min-reduced delta) / width q as left before the stream whose predecessor is pj (an
// inactive predecessor is a page that kept its dictionary: the fallback writer was fresh).
__device__ uint64_t dj_stale_slot(const DeltaJob *jobs, int32_t pj, uint32_t p, const uint64_t *blk_min, uint64_t wmask)
{
    while (pj >= 0) {
        const DeltaJob &P = jobs[pj];
        if (P.flags & DJ_INACTIVE) return 0;
        const uint64_t nd = P.n > 1 ? (uint64_t)P.n - 1 : 0;
        if (nd) {
            const uint32_t kl = (uint32_t)((nd - 1) / 128);
            const DBlock L = dj_block(P, kl);
            if (p < L.nd) return (dj_delta(P, L.d0 + p) - blk_min[P.blk0 + kl]) & wmask;
            if (kl) return (dj_delta(P, L.d0 - 128 + p) - blk_min[P.blk0 + kl - 1]) & wmask;   // a full block
        }
        pj = P.prev;
    }
    return 0;
}
__device__ uint32_t dj_stale_width(const DeltaJob *jobs, int32_t pj, uint32_t q, const uint32_t *blk_w)
{
    while (pj >= 0) {
        const DeltaJob &P = jobs[pj];
        if (P.flags & DJ_INACTIVE) return 0;
        const uint64_t nd = P.n > 1 ? (uint64_t)P.n - 1 : 0;
        if (nd) {
            const uint32_t kl = (uint32_t)((nd - 1) / 128);
            const uint32_t nmb = (dj_block(P, kl).nd + 31) / 32;
            if (q < nmb) return (blk_w[P.blk0 + kl] >> (8 * q)) & 0xffu;
            if (kl) return (blk_w[P.blk0 + kl - 1] >> (8 * q)) & 0xffu;
        }
        pj = P.prev;
    }
    return 0;
}

__global__ void __launch_bounds__(64) k_delta_write(const DeltaJob *jobs, const uint32_t *blk_job, const uint64_t *blk_min,
                                                    const uint32_t *blk_w, const uint64_t *blk_off, uint8_t *out)
{
    __shared__ uint32_t bits[4][64];   // 4 miniblocks x 32 values x <= 64 bits
    const uint32_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const DeltaJob &J = jobs[blk_job[b]];
    if (J.flags & DJ_INACTIVE) return;
    const uint32_t k = b - J.blk0;
    uint8_t *base = out + J.out_off;
    if (k == 0 && lane == 0) {   // getBytes: config.toBytesInput, totalValueCount, firstValue
        uint8_t *o = base;
        *o++ = 0x80; *o++ = 0x01; *o++ = 0x04;
        o = put_varint64(o, J.n);
        put_varint64(o, dj_zigzag(J, J.n ? dj_val(J, 0) : 0));
    }
    const DBlock B = dj_block(J, k);
    if (!B.nd) return;
    const uint64_t wmask = (J.flags & DJ_LONG) ? ~0ull : 0xffffffffull;
    const uint64_t m = blk_min[b];
    const uint32_t nmb = (B.nd + 31) / 32;
    const uint32_t wc = blk_w[b], wp = k ? blk_w[b - 1] : 0u;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; q++)
        w[q] = (uint32_t)q < nmb ? (wc >> (8 * q)) & 0xffu
             : k ? (wp >> (8 * q)) & 0xffu : dj_stale_width(jobs, J.prev, (uint32_t)q, blk_w);
    uint8_t *o = base + J.hdr + blk_off[b];
    const uint64_t zm = dj_zigzag(J, m);
    const uint32_t mlen = varint_len64(zm);
    if (lane == 0) {
        uint8_t *p = put_varint64(o, zm);
        p[0] = (uint8_t)w[0]; p[1] = (uint8_t)w[1]; p[2] = (uint8_t)w[2]; p[3] = (uint8_t)w[3];
    }
    for (int i = lane; i < 4 * 64; i += 64) bits[i >> 6][i & 63] = 0;
    __syncthreads();
    const uint64_t mprev = k ? blk_min[b - 1] : 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t p = (uint32_t)lane + 64u * h;   // slot within the block
        const uint32_t q = p >> 5;
        if (q >= nmb) continue;
        const uint32_t wq = w[q];
        if (!wq) continue;
        uint64_t x;
        if (p < B.nd) x = (dj_delta(J, B.d0 + p) - m) & wmask;
        else x = k ? ((dj_delta(J, B.d0 - 128 + p) - mprev) & wmask)   // stale deltaBlockBuffer slot
                   : dj_stale_slot(jobs, J.prev, p, blk_min, wmask);
        if (wq < 64) x &= (1ull << wq) - 1;
        const uint32_t bit = (p & 31) * wq;
        const uint32_t wi = bit >> 5, sh = bit & 31;
        const uint64_t lo = x << sh;
        atomicOr(&bits[q][wi], (uint32_t)lo);
        if (sh + wq > 32) atomicOr(&bits[q][wi + 1], (uint32_t)(lo >> 32));
        if (sh + wq > 64) atomicOr(&bits[q][wi + 2], (uint32_t)(x >> (64 - sh)));
    }
    __syncthreads();
    uint32_t moff = mlen + 4;
    for (uint32_t q = 0; q < nmb; q++) {
        const uint32_t nb = 4 * w[q];
        for (uint32_t i = lane; i < nb; i += 64) o[moff + i] = (uint8_t)(bits[q][i >> 2] >> (8 * (i & 3)));
        moff += nb;
    }
}

// ------------------------------------------------------------------ dense inputs per chunk

// INT32/INT64 fallback chunks: dense[ids_off + rank] = value; BYTE_ARRAY: = record index
__global__ void __launch_bounds__(KPW_BLOCK) k_delta_dense(const ChunkDesc *ch, const DevCol *cols, const uint32_t *ctile_chunk,
                                                          const uint32_t *ctile_first, uint64_t *dense)
{
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    if (C.dj0 < 0 || !C.fallback) return;
    const DevCol &col = cols[C.col];
    // coalesced tile layout: thread x handles records t0 + x, t0 + x + 256, ...
    const uint64_t t0 = (uint64_t)C.s + (uint64_t)(t - ctile_first[ci]) * KPW_TILE_P + threadIdx.x;
    const uint64_t rank0 = col.optional ? rank_of(col, (uint64_t)C.s) : (uint64_t)C.s;
    for (int k = 0; k < 8; k++) {
        const uint64_t r = t0 + (uint64_t)k * KPW_BLOCK;
        if (r >= (uint64_t)C.e) break;
        if (col.optional && !((col.pres[r >> 6] >> (r & 63)) & 1ull)) continue;
        uint64_t v;
        if (col.phys == 6) v = r;
        else v = col.vsize == 4 ? (uint64_t)((const uint32_t *)col.vals)[r] : ((const uint64_t *)col.vals)[r];
        dense[C.ids_off + (col.optional ? rank_of(col, r) : r) - rank0] = v;
    }
}

// common leading bytes of BYTE_ARRAY values a and b (the 16-byte prefix words first)
__device__ __forceinline__ uint32_t common_prefix(const DevCol &col, const uint8_t *data, uint64_t a, uint64_t b)
{
    const uint32_t la = col.slen[a], lb = col.slen[b];
    const uint32_t m = la < lb ? la : lb;
    uint32_t i = 0;
    for (int w = 0; w < 2 && i < m; w++) {
        const uint64_t x = col.spfx[2 * a + w] ^ col.spfx[2 * b + w];
        if (x) { const uint32_t c = i + ((uint32_t)__builtin_ctzll(x) >> 3); return c < m ? c : m; }
        i += 8;
    }
    if (i >= m) return m;
    const uint8_t *pa = data + col.soff[a], *pb = data + col.soff[b];
    while (i < m && pa[i] == pb[i]) i++;
    return i;
}

// DeltaByteArrayWriter.writeBytes for every value of a BYTE_ARRAY fallback chunk: prefix
// length with the previous value (pre), suffix length (sfx); per chunk tile the suffix bytes
__global__ void __launch_bounds__(KPW_BLOCK) k_dba_lengths(const ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                          const uint32_t *ctile_chunk, const uint32_t *ctile_first,
                                                          const uint64_t *dense, uint32_t *pre, uint32_t *sfx, uint64_t *tile_sfx)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    const DevCol &col = cols[C.col];
    uint64_t sum = 0;
    const bool active = C.dj0 >= 0 && C.fallback && col.phys == 6;
    if (active) {   // coalesced tile layout (the per-tile suffix total is order-independent)
        const uint64_t t0 = (uint64_t)C.s + (uint64_t)(t - ctile_first[ci]) * KPW_TILE_P + threadIdx.x;
        const uint64_t rank0 = col.optional ? rank_of(col, (uint64_t)C.s) : (uint64_t)C.s;
        for (int k = 0; k < 8; k++) {
            const uint64_t r = t0 + (uint64_t)k * KPW_BLOCK;
            if (r >= (uint64_t)C.e) break;
            if (col.optional && !((col.pres[r >> 6] >> (r & 63)) & 1ull)) continue;
            const uint64_t rank = (col.optional ? rank_of(col, r) : r) - rank0;
            const uint32_t p = rank ? common_prefix(col, data, dense[C.ids_off + rank - 1], r) : 0u;
            const uint32_t s = col.slen[r] - p;
            pre[C.ids_off + rank] = p;
            sfx[C.ids_off + rank] = s;
            sum += s;
        }
    }
    sum = block_reduce<uint64_t, OpSum64>(sum, lds);
    if (threadIdx.x == 0) tile_sfx[t] = sum;
}

// suffix bytes (the DeltaLengthByteArray body) after the two length streams
__global__ void __launch_bounds__(KPW_BLOCK) k_dba_suffixes(const ChunkDesc *ch, const DevCol *cols, const uint8_t *data,
                                                           const uint32_t *ctile_chunk, const uint32_t *ctile_first,
                                                           const uint32_t *pre, const DeltaJob *djobs, const uint64_t *tile_sfx_off,
                                                           uint8_t *out)
{
    __shared__ uint64_t lds[KPW_BLOCK];
    const uint32_t t = blockIdx.x;
    const uint32_t ci = ctile_chunk[t];
    const ChunkDesc &C = ch[ci];
    const DevCol &col = cols[C.col];
    const bool active = C.dj0 >= 0 && C.fallback && col.phys == 6;
    const uint64_t p0 = (uint64_t)C.s + (uint64_t)(t - ctile_first[ci]) * KPW_TILE_P + threadIdx.x * 8;
    const bool mine = active && p0 < (uint64_t)C.e;
    uint64_t rank0 = 0, sz = 0;
    if (mine) {
        rank0 = col.optional ? rank_of(col, p0) - rank_of(col, (uint64_t)C.s) : p0 - (uint64_t)C.s;
        uint64_t rank = rank0;
        for (int k = 0; k < 8; k++) {
            const uint64_t r = p0 + k;
            if (r >= (uint64_t)C.e) break;
            if (col.optional && !((col.pres[r >> 6] >> (r & 63)) & 1ull)) continue;
            sz += col.slen[r] - pre[C.ids_off + rank];
            rank++;
        }
    }
    uint64_t tot;
    uint64_t off = block_scan_excl<uint64_t, OpSum64>(sz, lds, &tot);
    if (!mine) return;
    off += tile_sfx_off[t];
    uint8_t *dst = out + C.val_off + djobs[C.dj0].total + djobs[C.dj0 + 1].total;
    uint64_t rank = rank0;
    for (int k = 0; k < 8; k++) {
        const uint64_t r = p0 + k;
        if (r >= (uint64_t)C.e) break;
        if (col.optional && !((col.pres[r >> 6] >> (r & 63)) & 1ull)) continue;
        const uint32_t p = pre[C.ids_off + rank];
        const uint32_t l = col.slen[r] - p;
        const uint8_t *src = data + col.soff[r] + p;
        for (uint32_t i = 0; i < l; i++) dst[off + i] = src[i];
        off += l;
        rank++;
    }
}

// ------------------------------------------------------------------ per-chunk decisions

// FallbackValuesWriter.getBytes on the (single) page: isCompressionSatisfying, decided before
// the fallback writers run (the v2 layout needs their sizes)
__global__ void k_v2_decide(ChunkDesc *ch, int nchunks, const RleJob *jobs)
{
    const int ci = blockIdx.x * blockDim.x + threadIdx.x;
    if (ci >= nchunks) return;
    ChunkDesc &C = ch[ci];
    if (!C.is_dict || C.fallback) return;
    const uint64_t val = 1 + jobs[C.id_job].total_bytes;
    if (!(val + C.dict_bytes < C.raw_bytes)) C.fallback = 1;
}

// activate the DELTA streams of chunks that fell back (n = non-null values), deactivate the rest
__global__ void k_v2_delta_jobs(const ChunkDesc *ch, int nchunks, const DevCol *cols, DeltaJob *dj)
{
    const int ci = blockIdx.x * blockDim.x + threadIdx.x;
    if (ci >= nchunks) return;
    const ChunkDesc &C = ch[ci];
    if (C.dj0 < 0) return;
    const int nj = cols[C.col].phys == 6 ? 2 : 1;
    for (int k = 0; k < nj; k++) {
        DeltaJob &J = dj[C.dj0 + k];
        J.base = C.ids_off;   // multi-page: a page's rank offset inside its chunk (device-set)
        if (C.fallback) { J.n = C.nn; J.flags &= ~DJ_INACTIVE; }
        else { J.n = 0; J.flags |= DJ_INACTIVE; }
    }
}

// v2 boolean value streams of optional columns: compacted bits (bit k = k-th present value)
__global__ void __launch_bounds__(KPW_BLOCK) k_bool_compact(const DevCol *cols, const uint32_t *bool_cols, uint64_t n,
                                                           uint64_t *const *cbits)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k = blockIdx.y;
    if (r >= n) return;
    const DevCol &c = cols[bool_cols[k]];
    if (!c.optional) return;
    if (!((c.pres[r >> 6] >> (r & 63)) & 1ull)) return;
    if (!((c.vbits[r >> 6] >> (r & 63)) & 1ull)) return;
    const uint64_t rank = rank_of(c, r);
    atomicOr((unsigned long long *)&cbits[k][rank >> 6], 1ull << (rank & 63));
}

// value-stream length of each boolean column (planning RLE jobs and planner streams)
__global__ void k_bool_stream_lens(const DevCol *cols, const uint32_t *bool_cols, uint32_t nbool, uint64_t n, RleJob *jobs,
                                   uint32_t job0, PlanStream *streams, uint32_t stream0)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nbool) return;
    const DevCol &c = cols[bool_cols[k]];
    const uint64_t len = c.optional ? rank_of(c, n) : n;
    jobs[job0 + k].len = (uint32_t)len;
    streams[stream0 + k].len = len;
}

// v2 per-chunk boolean RLE jobs of optional columns: stream base (rank of the chunk start)
// and length (non-null values)
__global__ void k_v2_bool_jobs(const ChunkDesc *ch, int nchunks, const DevCol *cols, RleJob *jobs)
{
    const int ci = blockIdx.x * blockDim.x + threadIdx.x;
    if (ci >= nchunks) return;
    const ChunkDesc &C = ch[ci];
    if (C.bool_job < 0) return;
    const DevCol &c = cols[C.col];
    if (!c.optional) return;
    RleJob &J = jobs[C.bool_job];
    J.src.base = rank_of(c, (uint64_t)C.s);
    J.len = C.nn;
}

// ------------------------------------------------------------------ host launchers

void launch_delta_structure(const DeltaArgs &d, hipStream_t s)
{
    if (!d.nblk) return;
    hipLaunchKernelGGL(k_delta_blocks, dim3(d.nblk), dim3(64), 0, s, (const DeltaJob *)d.jobs, d.blk_job, d.blk_min, d.blk_w,
                       d.blk_sz);
    seg_tile_scan<uint64_t, OpSum64>(d.blk_sz, d.blk_off, d.blk_job, d.nblk, d.btot, d.seg, s);
    hipLaunchKernelGGL(k_delta_totals, dim3((d.njobs + 255) / 256), dim3(256), 0, s, d.jobs, (int)d.njobs, (const uint64_t *)d.btot);
}

void launch_delta_write(const DeltaArgs &d, uint8_t *out, hipStream_t s)
{
    if (!d.nblk) return;
    hipLaunchKernelGGL(k_delta_write, dim3(d.nblk), dim3(64), 0, s, (const DeltaJob *)d.jobs, d.blk_job, (const uint64_t *)d.blk_min,
                       (const uint32_t *)d.blk_w, (const uint64_t *)d.blk_off, out);
}

void launch_v2_decide(const ChunkArgs &a, const RleJob *jobs, DeltaJob *djobs, hipStream_t s)
{
    const dim3 g((a.nchunks + 255) / 256);
    hipLaunchKernelGGL(k_v2_decide, g, dim3(256), 0, s, a.ch, a.nchunks, jobs);
    hipLaunchKernelGGL(k_v2_delta_jobs, g, dim3(256), 0, s, (const ChunkDesc *)a.ch, a.nchunks, a.cols, djobs);
}

// multi-page: fallback decided per page (k_mp_dict_decide / k_mp_satisfy)
void launch_v2_delta_jobs(const ChunkArgs &a, DeltaJob *djobs, hipStream_t s)
{
    hipLaunchKernelGGL(k_v2_delta_jobs, dim3((a.nchunks + 255) / 256), dim3(256), 0, s, (const ChunkDesc *)a.ch, a.nchunks, a.cols,
                       djobs);
}

void launch_v2_dense(const ChunkArgs &a, uint64_t *dense, uint32_t *pre, uint32_t *sfx, uint64_t *tile_sfx, uint64_t *tile_sfx_off,
                     uint64_t *chunk_sfx, hipStream_t s)
{
    hipLaunchKernelGGL(k_delta_dense, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, (const ChunkDesc *)a.ch, a.cols, a.ctile_chunk,
                       a.ctile_first, dense);
    hipLaunchKernelGGL(k_dba_lengths, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, (const ChunkDesc *)a.ch, a.cols, a.data,
                       a.ctile_chunk, a.ctile_first, (const uint64_t *)dense, pre, sfx, tile_sfx);
    seg_tile_scan<uint64_t, OpSum64>(tile_sfx, tile_sfx_off, a.ctile_chunk, a.nctiles, chunk_sfx, a.seg, s);
}

void launch_dba_suffixes(const ChunkArgs &a, const uint32_t *pre, const DeltaJob *djobs, const uint64_t *tile_sfx_off, uint8_t *out,
                         hipStream_t s)
{
    hipLaunchKernelGGL(k_dba_suffixes, dim3(a.nctiles), dim3(KPW_BLOCK), 0, s, (const ChunkDesc *)a.ch, a.cols, a.data, a.ctile_chunk,
                       a.ctile_first, pre, djobs, tile_sfx_off, out);
}

void launch_v2_bool_jobs(const ChunkArgs &a, RleJob *jobs, hipStream_t s)
{
    hipLaunchKernelGGL(k_v2_bool_jobs, dim3((a.nchunks + 255) / 256), dim3(256), 0, s, (const ChunkDesc *)a.ch, a.nchunks, a.cols, jobs);
}

void launch_bool_streams(const DevCol *cols, const uint32_t *bool_cols, uint32_t nbool, uint64_t n, uint64_t *const *cbits,
                         RleJob *jobs, uint32_t job0, PlanStream *streams, uint32_t stream0, hipStream_t s)
{
    if (!nbool || !n) return;
    hipLaunchKernelGGL(k_bool_compact, dim3((unsigned)((n + KPW_BLOCK - 1) / KPW_BLOCK), nbool), dim3(KPW_BLOCK), 0, s, cols, bool_cols,
                       n, cbits);
    hipLaunchKernelGGL(k_bool_stream_lens, dim3((nbool + 63) / 64), dim3(64), 0, s, cols, bool_cols, nbool, n, jobs, job0, streams,
                       stream0);
}

}  // namespace kpw
