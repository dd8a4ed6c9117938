// k_maps.hip — tile -> job maps and the dictionary insertion order, built on the device.
//
// Every tiled pass (K3's position / element tiles, K6/K2's chunk tiles, the DELTA block tiles)
// finds its job through a map with one word per tile.  The host used to expand these maps and
// upload them with the job tables: on C3 (200 columns, ~2000 chunks per job) that was ~2.5 MB of
// pageable copies per job, each a PCIe-bound blit of ~1 ms (profiles/r05e_c3_copies.md).  The
// job tables already hold (first tile, tile count) per job, so the maps are expanded here from
// the uploaded tables instead: one wave per job, lanes write its tile range.
#include "kpw_device.h"
#include "kpw_kernels.h"

namespace kpw {

__global__ void __launch_bounds__(256) k_tile_maps(TileMapArgs a)
{
    const TileMapSpec M = a.m[blockIdx.y];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6); j < M.n; j += nw) {
        const uint32_t f = M.first[(uint64_t)j * M.stride], c = M.count[(uint64_t)j * M.stride];
        for (uint32_t i = lane; i < c; i += 64) M.map[f + i] = j;
    }
}

// Round k (one block): tile k of every listed chunk with more than k tiles, in list order, at
// round_off[k] (the host's counts of such chunks per round, prefix-summed).
__global__ void __launch_bounds__(256) k_dict_order(const uint32_t *list, uint32_t nl, const uint32_t *first,
                                                    const uint32_t *count, const uint32_t *round_off, uint32_t *out)
{
    __shared__ uint32_t wsum[4];
    const uint32_t k = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t base = round_off[k];
    for (uint32_t i0 = 0; i0 < nl; i0 += 256) {
        const uint32_t i = i0 + threadIdx.x;
        const uint32_t ci = i < nl ? list[i] : 0u;
        const bool on = i < nl && count[ci] > k;
        const uint64_t m = __ballot(on);
        if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t at = base;
        for (uint32_t q = 0; q < w; q++) at += wsum[q];
        at += (uint32_t)__popcll(m & ((1ull << lane) - 1));
        if (on) out[at] = first[ci] + k;
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

void launch_tile_maps(const TileMapArgs &a, hipStream_t s)
{
    uint32_t nmax = 0;
    for (uint32_t i = 0; i < a.nm; i++) nmax = a.m[i].n > nmax ? a.m[i].n : nmax;
    if (!a.nm || !nmax) return;
    const uint32_t gx = (nmax + 3) / 4 < 2048 ? (nmax + 3) / 4 : 2048;
    hipLaunchKernelGGL(k_tile_maps, dim3(gx, a.nm), dim3(256), 0, s, a);
}

void launch_dict_order(const uint32_t *list, uint32_t nl, const uint32_t *first, const uint32_t *count,
                       const uint32_t *round_off, uint32_t nrounds, uint32_t *out, hipStream_t s)
{
    if (!nl || !nrounds) return;
    hipLaunchKernelGGL(k_dict_order, dim3(nrounds), dim3(256), 0, s, list, nl, first, count, round_off, out);
}

}  // namespace kpw
