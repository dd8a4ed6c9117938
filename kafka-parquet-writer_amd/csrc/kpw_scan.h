// kpw_scan.h — scan launchers (k_scan.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kpw_kernels.h"
#include "kpw_lookback.h"

namespace kpw {

struct OpSum64;
struct OpSum32;
struct OpMaxI64;
struct OpMapCompose;

// Multi-job scans (reduce -> scan -> apply, k_scan.hip); `sc` holds their tile sums.  If the
// scratch cannot grow, the scan is skipped and sc->failed is set: the caller must fail the
// encode.
void launch_pcnt_scan(const DevCol *cols_d, const uint32_t *opt_d, uint32_t nopt, uint64_t nwords, SegScratch *sc, hipStream_t s);
// per stream j: E8[j * (ev_stride / 8 + 1) + g] = event bytes of positions [0, 8g) (ev_stride: bytes
// per stream in ev, a multiple of 8)
// the planner's prefixes over groups of 8 positions (k_scan.hip PlanPrefixF): E8 of nev event
// streams, P8 of the raw record sizes, Q8 of the folded sizes when val != null
void launch_plan_prefix(const uint8_t *ev, uint32_t *E8, uint32_t nev, uint64_t ev_stride, const uint32_t *raw, const uint32_t *val,
                        uint64_t n, uint64_t *P8, uint64_t *Q8, SegScratch *sc, hipStream_t s);

// Status words for one single-pass launch over `nwords` tiles x scans (w == nullptr: the
// scratch could not grow, sc->failed set; the caller skips the launch).
LbView lb_prepare(SegScratch *sc, uint64_t nwords, hipStream_t s);
// look-back fallbacks counted on this scratch since the previous call, which it clears
// (kpw_lookback.h: a tile that waited past the spin bound recomputed its predecessor's status;
// the scans' results stay exact, the count is a health figure), -1 if unreadable.
// Synchronises `s` (the stream the scans ran on).
int lb_failures(SegScratch *sc, hipStream_t s);

// Exclusive segmented scan over tile aggregates (same scratch contract).
template <typename T, typename Op>
void seg_tile_scan(const T *in, T *out, const uint32_t *seg, uint32_t n, T *tot, SegScratch *sc, hipStream_t s);
void seg_scratch_free(SegScratch &sc);

}  // namespace kpw
