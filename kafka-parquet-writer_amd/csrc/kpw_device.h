// kpw_device.h — device helpers shared by the CDNA4 kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KPW_BLOCK 256           // threads per block for the streaming kernels (4 waves)
#define KPW_TILE_P 2048         // positions per position-tile (256 threads x 8)
#define KPW_TILE_E 256          // elements per element-tile (1 per thread)
#define KPW_TILE_L 16384        // positions per long-run tile (256 threads x 64: one break mask each)

namespace kpw {

struct OpSum64 { __device__ static uint64_t id() { return 0; } __device__ static uint64_t op(uint64_t a, uint64_t b) { return a + b; } };
struct OpSum32 { __device__ static uint32_t id() { return 0; } __device__ static uint32_t op(uint32_t a, uint32_t b) { return a + b; } };
struct OpMaxI64 { __device__ static int64_t id() { return -1; } __device__ static int64_t op(int64_t a, int64_t b) { return a > b ? a : b; } };

// 8-state phase map: out[phi] in 3 bits each (24 bits).  compose(f, g) = "f then g".
__device__ __forceinline__ uint32_t pm_get(uint32_t m, uint32_t phi) { return (m >> (3 * phi)) & 7u; }
struct OpMapCompose {
    __device__ static uint32_t id() { return 0xFAC688u; }  // identity: phi -> phi (0,1,..,7 packed)
    __device__ static uint32_t op(uint32_t f, uint32_t g) {
        uint32_t h = 0;
#pragma unroll
        for (uint32_t p = 0; p < 8; p++) h |= pm_get(g, pm_get(f, p)) << (3 * p);
        return h;
    }
};

// Inclusive block scan over KPW_BLOCK threads (order preserving, any associative Op).
template <typename T, typename Op>
__device__ __forceinline__ T block_scan_incl(T v, T *lds)
{
    const int t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    for (int d = 1; d < KPW_BLOCK; d <<= 1) {
        T x = (t >= d) ? lds[t - d] : Op::id();
        __syncthreads();
        if (t >= d) lds[t] = Op::op(x, lds[t]);
        __syncthreads();
    }
    T r = lds[t];
    __syncthreads();
    return r;
}

// Exclusive scan; *total receives the block aggregate.
template <typename T, typename Op>
__device__ __forceinline__ T block_scan_excl(T v, T *lds, T *total)
{
    T inc = block_scan_incl<T, Op>(v, lds);
    lds[threadIdx.x] = inc;
    __syncthreads();
    T ex = threadIdx.x ? lds[threadIdx.x - 1] : Op::id();
    *total = lds[KPW_BLOCK - 1];
    __syncthreads();
    return ex;
}

template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T v, T *lds)
{
    T tot;
    (void)block_scan_excl<T, Op>(v, lds, &tot);
    return tot;
}

// Value source for the RLE/bit-packing hybrid: either a bitmask (definition levels,
// bit i of the stream = bit (base+i)) or a u32 array (dictionary ids).
struct ValSrc {
    uint32_t kind;   // 0 = bits, 1 = u32
    uint32_t pad;
    const void *ptr;
    uint64_t base;
};
__device__ __forceinline__ uint32_t src_get(const ValSrc &s, uint64_t i)
{
    if (s.kind == 0) {
        uint64_t b = s.base + i;
        return (uint32_t)((((const uint64_t *)s.ptr)[b >> 6] >> (b & 63)) & 1ull);
    }
    return ((const uint32_t *)s.ptr)[s.base + i];
}

__device__ __forceinline__ uint32_t varint_len32(uint32_t v)
{
    uint32_t n = 1;
    while (v >= 0x80u) { v >>= 7; n++; }
    return n;
}

// 64-bit hash (splitmix finaliser) for dictionary keys.
__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

// 8 bytes at base[off..off+8) (base 8-byte aligned), zero beyond `end`; two aligned loads
// + funnel shift instead of 8 byte loads.
__device__ __forceinline__ uint64_t ldu64(const uint8_t *base, uint64_t off, uint64_t end)
{
    if (off + 16 <= end) {
        const uint64_t a = off & ~7ull;
        const uint64_t lo = *(const uint64_t *)(base + a), hi = *(const uint64_t *)(base + a + 8);
        const uint32_t sh = (uint32_t)(off & 7) * 8;
        return sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
    }
    uint64_t v = 0;
    for (int i = 0; i < 8; i++)
        if (off + i < end) v |= (uint64_t)base[off + i] << (8 * i);
    return v;
}
__device__ __forceinline__ uint64_t tail_mask(uint64_t rem) { return rem >= 8 ? ~0ull : ((1ull << (8 * rem)) - 1); }

// 64-bit hash of a byte string (dictionary keys of BYTE_ARRAY columns).
__device__ __forceinline__ uint64_t bytes_hash(const uint8_t *base, uint64_t off, uint32_t len, uint64_t end)
{
    uint64_t h = 0x9E3779B97F4A7C15ull ^ len;
    for (uint32_t k = 0; k < len; k += 8) {
        const uint64_t w = ldu64(base, off + k, end) & tail_mask(len - k);
        h = (h ^ w) * 0xff51afd7ed558ccdull;
        h ^= h >> 29;
    }
    return mix64(h);
}

// unsigned lexicographic compare (BinaryStatistics / UNSIGNED_LEXICOGRAPHICAL comparator)
__device__ __forceinline__ int bytes_cmp(const uint8_t *base, uint64_t oa, uint32_t la, uint64_t ob, uint32_t lb, uint64_t end)
{
    const uint32_t m = la < lb ? la : lb;
    for (uint32_t k = 0; k < m; k += 8) {
        const uint64_t msk = tail_mask(m - k);
        const uint64_t x = ldu64(base, oa + k, end) & msk, y = ldu64(base, ob + k, end) & msk;
        if (x != y) {
            const uint64_t bx = __builtin_bswap64(x), by = __builtin_bswap64(y);
            return bx < by ? -1 : 1;
        }
    }
    return la == lb ? 0 : (la < lb ? -1 : 1);
}

__device__ __forceinline__ uint64_t bits_window(const uint64_t *w, uint64_t bit)
{
    // 64 bits starting at absolute bit index `bit` (words are padded by one extra word)
    uint64_t lo = w[bit >> 6];
    uint32_t sh = (uint32_t)(bit & 63);
    if (!sh) return lo;
    return (lo >> sh) | (w[(bit >> 6) + 1] << (64 - sh));
}

// A workgroup copies n bytes between arbitrary byte addresses: 16-byte aligned stores for the
// body (each built from aligned dword loads of the source shifted with alignbyte), single bytes
// for the unaligned head and the tail.  Reads never end past src + n (a chunk whose last source
// dword would is copied bytewise); they may start up to 3 bytes before src + head, inside the
// same aligned dword, so they never touch another page.
__device__ __forceinline__ void block_copy(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t tid, uint32_t nth)
{
    uint32_t head = (uint32_t)((16u - ((uintptr_t)dst & 15u)) & 15u);
    if (head > n) head = n;
    const uint32_t chunks = (n - head) / 16u;
    const uint32_t tail0 = head + chunks * 16u;
    if (tid < head) dst[tid] = src[tid];
    for (uint32_t i = tail0 + tid; i < n; i += nth) dst[i] = src[i];
    const uintptr_t sa = (uintptr_t)(src + head);
    const uint32_t sh = (uint32_t)(sa & 3u);
    const uint32_t *sw = (const uint32_t *)(sa & ~(uintptr_t)3);
    uint4 *dw = (uint4 *)(dst + head);
    for (uint32_t k = tid; k < chunks; k += nth) {
        const uint32_t *w = sw + 4u * k;
        if (sh && head + 16u * k + 20u - sh > n) {   // the fifth dword would read past the source
            for (uint32_t i = 0; i < 16u; i++) dst[head + 16u * k + i] = src[head + 16u * k + i];
            continue;
        }
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = sh ? w[4] : 0u;
        uint4 v;
        v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
        v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
        v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
        v.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
        dw[k] = v;
    }
}

}  // namespace kpw
