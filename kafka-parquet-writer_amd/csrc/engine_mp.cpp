// engine_mp.cpp — the multi-page regime: PARQUET_1_0 with pageSize < blockSize, and PARQUET_2_0.
//
// parquet-mr 1.10.1 cuts a column's page inside a row group (ColumnWriterV1
// .accountForValueWritten per column; v2: ColumnWriteStoreV2.sizeCheck per store, once a
// column's page is within 10% of pageSize), and from then on the row-group size check
// (InternalParquetRecordWriter.checkBlockSizeReached) counts the flushed pages by their
// header + compressed bytes (ColumnChunkPageWriter.getMemSize) instead of their raw size.  A
// row-group boundary therefore depends on the encoded and compressed sizes of the pages
// before it, so row groups are planned one at a time:
//
//   1. k_page_cuts   page cuts of every column from the row-group start s to a horizon h
//                    (they depend only on s and the values);
//   2. mp_pipeline   encode [s, h) as pages (statistics, dictionary per column chunk with
//                    per-page fallback / bit width, RLE, PLAIN, Snappy) -> page bytes;
//   3. k_plan_mp     the row-group check walk with those page bytes -> end r (or none: h
//                    doubles and 1-3 repeat);
//   4. mp_pipeline   encode [s, r) exactly (the last page of every column ends at r) and
//                    append it to the batch output.
//
// The single-page regime (pageSize >= blockSize, the reference default) stays in engine.cpp
// and plans every row group of a batch in one pass.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "engine.h"
#include "filewriter.h"
#include "kpw_chunk.h"
#include "kpw_scan.h"
#include "memcache.h"

namespace kpw {

void launch_snappy_finish(const SnappyArgs &a, const uint32_t *page_frag0, hipStream_t s);
void launch_stats_gather(const ChunkDesc *ch, int nchunks, const DevCol *cols, const uint8_t *data, uint64_t *meta,
                         uint8_t *blob, hipStream_t s);

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return fail(KPW_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define ENS(buf, bytes) do { if ((buf).ensure(bytes)) return fail(KPW_ERR_NOMEM, "device allocation failed: " #buf); } while (0)

// mp_pipeline: a continuation probe found a string hash collision (probe_mp restarts exact)
constexpr int kPdRetry = -77;

// KPW_PROBE_CONT=0: every probe re-inserts the open row group's prefix (A/B of the continuation)
static bool pd_enabled()
{
    static const bool on = [] { const char *e = getenv("KPW_PROBE_CONT"); return !(e && e[0] == '0'); }();
    return on;
}

// multi-page dictionary insertion round: tiles (of KPW_TILE_P_H records) per chunk and round
constexpr uint32_t kMpRoundTiles = 64;

static inline uint64_t next_pow2_mp(uint64_t x)
{
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Grow `b` to hold `bytes`, keeping its first `keep` bytes.
int Engine::grow_keep(DevBuf &b, size_t bytes, size_t keep)
{
    if (bytes <= b.cap && b.p) return KPW_OK;
    const size_t c = bytes + bytes / 2 + 256;
    void *np = dev_alloc(c);
    if (!np) return fail(KPW_ERR_NOMEM, "device allocation failed: multi-page output");
    if (keep && b.p) CK(hipMemcpyAsync(np, b.p, keep, hipMemcpyDeviceToDevice, stream));
    CK(xsync(stream));
    dev_free(b.p);
    b.p = np;
    b.cap = c;
    return KPW_OK;
}

// Page cuts of every column over [s, h).
int Engine::mp_cuts(PageCutArgs &a, int64_t s, int64_t h, std::vector<std::vector<int64_t>> &cuts)
{
    const int nc = (int)cols.size();
    a.s = s;
    a.h = h;
    a.cap = (uint32_t)std::min<uint64_t>((uint64_t)(h - s) / 2 + 2, 0xFFFFFFF0ull);
    ENS(mp_ncuts, nc * 4); ENS(mp_cutpos, (uint64_t)nc * a.cap * 8); ENS(mp_flag, 64);
    a.ncuts = mp_ncuts.as<uint32_t>();
    a.cuts = mp_cutpos.as<int64_t>();
    a.overflow = mp_flag.as<int32_t>();
    a.out = mp_flag.as<int64_t>() + 1;
    CK(hipMemsetAsync(mp_flag.p, 0, 64, stream));
    launch_page_cuts(a, stream);
    CK(hipGetLastError());
    std::vector<uint32_t> nct(nc);
    int32_t ovf = 0;
    CK(xd2h(nct.data(), mp_ncuts.p, nc * 4, stream));
    CK(xd2h(&ovf, mp_flag.p, 4, stream));
    CK(xsync(stream));
    if (ovf) return fail(KPW_ERR_DEVICE, "page cut table overflow");
    cuts.assign(nc, {});
    for (int c = 0; c < nc; c++) {
        cuts[c].resize(nct[c]);
        if (nct[c]) CK(hipMemcpyAsync(cuts[c].data(), mp_cutpos.as<int64_t>() + (uint64_t)c * a.cap, nct[c] * 8ull,
                                      hipMemcpyDeviceToHost, stream));
    }
    CK(xsync(stream));
    return KPW_OK;
}

// Encode the column chunks [s, e) split at `cuts` (page ends <= e).  Result pages are in
// pages_dev_ (PageOut offsets), grouped per column: optional dictionary page, data pages.
int Engine::mp_pipeline(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, const std::vector<DevCol> &hc, int64_t s,
                        int64_t e, const std::vector<std::vector<int64_t>> &cuts, MpRun &run, const std::vector<char> *mask,
                        const std::vector<uint32_t> *k7_from, const MpRun *spec)
{
    if (spec && (v2_ || mask || k7_from)) return fail(KPW_ERR_STATE, "multi-page splice: v1 bulk passes only");
    hipStream_t st = stream;
    const int nc = (int)cols.size();
    run.cols.assign(nc, {});
    std::vector<ChunkDesc> dch(nc), pg;
    std::vector<RleJob> ej;
    std::vector<DeltaJob> dj;          // v2: DELTA streams of the pages (INT32/INT64: 1, BYTE_ARRAY: 2)
    std::vector<uint32_t> dblk_job;    // v2: job of each DELTA block tile
    std::vector<int> bool_pos(nc, -1);
    for (size_t i = 0; i < bool_idx_.size(); i++) bool_pos[bool_idx_[i]] = (int)i;
    uint64_t ht_off = 0, ids_off = 0;
    std::vector<uint32_t> dfirst(nc), dcount(nc), pfirst, pcount;
    std::vector<uint8_t> ddict(nc);
    uint32_t npt = 0, ndt = 0;
    std::vector<char> k7_on;           // per page: its data page is compressed (k7_from)
    // dictionary insertion rounds of at least ~1024 tiles over all dictionary chunks: a probe of
    // one column inserts its prefix in 4x fewer launches (each a latency-bound ~50 us), a bulk
    // row group of 8 columns in the same rounds as before
    uint32_t ndict = 0;
    for (int c = 0; c < nc; c++) ndict += (cols[c].dict && (!mask || (*mask)[c])) ? 1 : 0;
    // (a continuation probe inserts in fixed rounds of kMpRoundTiles: its kept table is sized for one)
    const uint32_t round_tiles = pd_on_ ? kMpRoundTiles
                                        : std::min<uint32_t>(4 * kMpRoundTiles, std::max<uint32_t>(kMpRoundTiles, 1024 / std::max<uint32_t>(1, ndict)));
    // rounds double up to round_grow x round_tiles: the stop matters near a chunk's crossing, which
    // the high-cardinality chunks reach in the first rounds; the later, larger rounds cost fewer
    // latency-bound launches (a bulk row group: 23 -> 8 rounds).  The table holds one round more.
    static const uint32_t round_grow = [] { const char *e = getenv("KPW_MP_ROUND_GROW"); const int v = e ? atoi(e) : 4; return (uint32_t)(v > 0 ? v : 1); }();
    const uint32_t round_max = pd_on_ ? round_tiles : round_tiles * round_grow;
    for (int c = 0; c < nc; c++) {
        ChunkDesc &D = dch[c];
        memset(&D, 0, sizeof(D));
        const uint64_t len = (uint64_t)(e - s);
        D.s = s; D.e = e; D.col = c; D.rg = 0;
        bool on = !mask || (*mask)[c];   // a probe of a column subset: the others get no pages
        if (on && k7_from && !v2_ && (size_t)(*k7_from)[c] >= cuts[c].size()) on = false;   // (nothing new cut)
        D.is_dict = cols[c].dict && on ? 1 : 0;
        D.smin = ~0ull; D.smax = 0;
        D.ids_off = ids_off; D.ent_off = ids_off;
        if (on && !spec) ids_off += len;
        if (D.is_dict && pd_on_) {
            // continuation probe: the column's table, ids and entries of [0, done) are kept in the
            // pd_ buffers; only [done, e) is inserted (a dictionary past dictPageSize inserts no more)
            const ProbeDict &Q = pd_[c];
            const uint64_t k = (uint64_t)pd_slot_[c];
            D.ht_cap = (uint32_t)pd_ht_cap_; D.ht_off = k * (pd_ht_cap_ + 1);
            D.ids_off = k * pd_ids_cap_; D.ent_off = k * pd_ent_cap_;
            D.dict_n = Q.n; D.dict_bytes = Q.bytes; D.ent_base = Q.n; D.boff_base = Q.bytes;
            D.tile_skip = Q.stopped ? len : (uint64_t)std::min<int64_t>(Q.done, (int64_t)len);
        } else if (D.is_dict && spec) {
            // the speculative pass's dictionary (ids, entries, tables) stays where it is; the
            // chunk's pages before its last cut are spec's pages, decided as they were there
            const ChunkDesc &S = spec->dch[c];
            D.ht_off = S.ht_off; D.ht_cap = S.ht_cap; D.ht_plim = S.ht_plim;
            D.ids_off = S.ids_off; D.ent_off = S.ent_off;
            D.dict_n = S.dict_all;
            const size_t kept = cuts[c].size();
            if (kept) {
                const ChunkDesc &P0 = spec->pg[S.first_page];
                D.tail_mode = P0.fallback ? 2u : 1u;
                for (size_t i = 0; i < kept; i++)
                    if (!spec->pg[S.first_page + i].fallback) D.tail_dict_n = spec->pg[S.first_page + i].dict_n;
            }
        } else if (D.is_dict) {
            // Insertion runs in rounds of round_tiles tiles per chunk and a chunk stops after
            // the round in which its dictionary passed dictPageSize (pages before the fallback
            // page keep their ids: every value before the crossing is inserted).  So a table
            // holds at most dictPageSize / (smallest entry) + 1 entries plus one round's values.
            const uint64_t esz = (cols[c].phys == KPW_INT64 || cols[c].phys == KPW_DOUBLE) ? 8 : 4;
            const uint64_t maxent = (uint64_t)props.dictionary_page_size / esz + 1 + (uint64_t)round_max * KPW_TILE_P_H;
            D.ht_cap = (uint32_t)next_pow2_mp(std::max<uint64_t>(16, 2 * std::min<uint64_t>(len, maxent)));
            D.ht_off = ht_off;
            ht_off += D.ht_cap + 1;
        }
        D.dl_job = D.id_job = D.bool_job = D.dj0 = -1;
        D.owner = -1;
        D.first_page = (int32_t)pg.size();
        // a probe (k7_from) encodes only the pages cut since its previous probe of the open row
        // group: the pages before are cached, the open page after the last cut is not flushed yet
        // (ColumnChunkPageWriter.getMemSize counts written pages only).  Without the chunk's first
        // page, its isCompressionSatisfying outcome comes from the probe that encoded it
        // (probe_mode_: 1 satisfied, 2 every page PLAIN), as in the splice's tail mode.
        // (v2 encodes every page: a DELTA stream inherits the previous page's stale bit widths)
        const bool newonly = k7_from && !v2_;
        const size_t p_from = newonly ? (size_t)(*k7_from)[c] : 0;
        if (on && newonly && p_from >= cuts[c].size()) on = false;   // nothing new cut in this column
        if (on && newonly && p_from > 0) {
            D.tail_mode = probe_mode_.size() > (size_t)c ? probe_mode_[c] : 0u;
            if (D.tail_mode == 0) return fail(KPW_ERR_STATE, "probe: first page outcome of a cached column unknown");
        }
        const uint64_t tlen = len - D.tile_skip;   // (a continuation's tiles start at its kept records)
        const uint32_t nt = on ? (uint32_t)std::max<uint64_t>(1, (tlen + KPW_TILE_P_H - 1) / KPW_TILE_P_H) : 0u;
        dfirst[c] = ndt;
        dcount[c] = nt;
        ddict[c] = D.is_dict;
        ndt += nt;
        if (!on) { D.npages = 0; continue; }
        // (splice: only the page after the last cut; probe: only the pages cut since the last probe)
        int64_t q = spec && !cuts[c].empty() ? cuts[c].back() : (p_from ? cuts[c][p_from - 1] : s);
        const size_t i_end = newonly ? cuts[c].size() - 1 : cuts[c].size();
        for (size_t i = spec ? cuts[c].size() : p_from; i <= i_end; i++) {
            const int64_t pe = i < cuts[c].size() ? std::min<int64_t>(cuts[c][i], e) : e;
            if (pe <= q) continue;
            ChunkDesc P;
            memset(&P, 0, sizeof(P));
            P.s = q; P.e = pe; P.col = c; P.rg = 0;
            P.is_dict = D.is_dict;
            P.smin = ~0ull; P.smax = 0;
            P.owner = c;
            P.dl_job = P.id_job = P.bool_job = P.dj0 = -1;
            if (cols[c].optional) {
                RleJob J;
                memset(&J, 0, sizeof(J));
                J.src.kind = 0; J.src.ptr = hc[c].pres; J.src.base = (uint64_t)P.s;
                J.len = (uint32_t)(pe - q); J.bw = 1;
                P.dl_job = (int32_t)ej.size();
                ej.push_back(J);
            }
            if (P.is_dict) {
                RleJob J;
                memset(&J, 0, sizeof(J));
                J.src.kind = 1; J.src.ptr = nullptr; J.src.base = 0;   // ptr below, base on the device
                J.len = (uint32_t)(pe - q); J.bw = 0;
                P.id_job = (int32_t)ej.size();
                ej.push_back(J);
            }
            if (v2_ && cols[c].phys == KPW_BOOLEAN) {   // RunLengthBitPackingHybridValuesWriter(1)
                RleJob J;
                memset(&J, 0, sizeof(J));
                J.src.kind = 0; J.src.ptr = cbits_[bool_pos[c]];
                J.src.base = cols[c].optional ? 0 : (uint64_t)P.s;   // optional: rank of P.s, set on the device
                J.len = (uint32_t)(pe - q); J.bw = 1;
                P.bool_job = (int32_t)ej.size();
                ej.push_back(J);
            }
            if (v2_ && P.is_dict && (cols[c].phys == KPW_INT32 || cols[c].phys == KPW_INT64 || cols[c].phys == KPW_BYTE_ARRAY)) {
                // DefaultV2ValuesWriterFactory fallback writers, one DELTA stream per page
                // (reset with the page); base = the page's rank offset, set on the device
                const int32_t prev0 = pg.size() > (size_t)D.first_page ? pg.back().dj0 : -1;   // this chunk's previous page
                P.dj0 = (int32_t)dj.size();
                const bool ba = cols[c].phys == KPW_BYTE_ARRAY;
                const uint64_t plen = (uint64_t)(pe - q);
                const uint32_t nblk = (uint32_t)std::max<uint64_t>(1, plen > 1 ? (plen - 1 + 127) / 128 : 1);
                for (int k = 0; k < (ba ? 2 : 1); k++) {
                    DeltaJob Dj;
                    memset(&Dj, 0, sizeof(Dj));
                    Dj.flags = DJ_INACTIVE | (cols[c].phys == KPW_INT64 ? DJ_LONG : 0u) | (ba ? DJ_U32_SRC : 0u);
                    Dj.blk0 = (uint32_t)dblk_job.size();
                    Dj.nblk = nblk;
                    Dj.prev = prev0 >= 0 ? prev0 + k : -1;
                    dblk_job.insert(dblk_job.end(), nblk, (uint32_t)dj.size());
                    dj.push_back(Dj);
                }
            }
            const uint32_t pt = (uint32_t)std::max<uint64_t>(1, ((uint64_t)(pe - q) + KPW_TILE_P_H - 1) / KPW_TILE_P_H);
            pfirst.push_back(npt);
            pcount.push_back(pt);
            npt += pt;
            pg.push_back(P);
            k7_on.push_back(!k7_from || (i >= (*k7_from)[c] && i < cuts[c].size()));
            q = pe;
        }
        D.npages = (int32_t)pg.size() - D.first_page;
    }
    const int npg = (int)pg.size();
    // dictionary insertion order (tile k of every chunk before tile k + 1, expanded on the device)
    // and per round of round_tiles its slice
    std::vector<uint32_t> dlist, droff, rlen, rend;
    uint32_t ndict_tiles = 0;
    dict_order(dcount, ddict, ndict_tiles, dlist, droff);
    const uint32_t maxnt = (uint32_t)droff.size() - 1;
    for (uint32_t k = 0, rt = round_tiles; k < maxnt; k += rt, rt = std::min(round_max, 2 * rt)) {
        rlen.push_back(droff[std::min(maxnt, k + rt)] - droff[k]);
        rend.push_back(std::min(maxnt, k + rt));   // tiles per chunk through this round
    }
    // page descriptors use the engine's chunk buffers; dictionary descriptors their own
    // chunk descriptors, then 4 words of string-statistics metadata per chunk (one readback)
    static_assert(sizeof(ChunkDesc) % 8 == 0, "metadata words follow the descriptors");
    ENS(d_chunks, npg * (sizeof(ChunkDesc) + 32));
    ENS(d_tile_raw, npt * 8); ENS(d_tile_raw_off, npt * 8); ENS(d_tile_smin, npt * 8); ENS(d_tile_smax, npt * 8);
    ENS(d_tile_cnt, npt * 4); ENS(d_tile_sz, npt * 8);
    ENS(mp_dch, nc * sizeof(ChunkDesc));
    ENS(mp_dtile_raw, ndt * 8); ENS(mp_dtile_smin, ndt * 8); ENS(mp_dtile_smax, ndt * 8); ENS(mp_dtile_cnt, ndt * 4);
    ENS(mp_dtile_sz, ndt * 8); ENS(d_fmask, (uint64_t)std::max(npt, ndt) * KPW_BLOCK_H);
    ENS(d_ht, std::max<uint64_t>(1, ht_off) * sizeof(HtSlot));
    ENS(d_ids, std::max<uint64_t>(1, ids_off) * 4); ENS(d_ent_rec, std::max<uint64_t>(1, ids_off) * 8);
    ENS(d_ent_boff, std::max<uint64_t>(1, ids_off) * 8);
    // page table as in Engine::encode: totals, collision flags, then per page slot its offset,
    // length, level prefix, compressed offset and length
    const size_t P2 = 2 * (size_t)npg;
    // (+ room behind it for the dictionary and page descriptors: the compression's sync reads all
    // three back with one copy)
    ENS(d_ptab, (4 + 5 * P2) * 8 + nc * sizeof(ChunkDesc) + npg * (sizeof(ChunkDesc) + 32) + 8);
    uint64_t *const pt = d_ptab.as<uint64_t>();
    uint64_t *const d_poff = pt + 4, *const d_plen = d_poff + P2, *const d_ppre = d_plen + P2;
    uint64_t *const d_pcoff = d_ppre + P2, *const d_pclen = d_pcoff + P2;
    uint32_t *const d_coll = (uint32_t *)(pt + 2);
    std::vector<uint64_t> ptab(4 + 5 * P2);
    for (auto &J : ej) if (J.src.kind == 1) J.src.ptr = pd_on_ ? pd_ids.p : d_ids.p;
    DeltaArgs dla{};
    if (v2_) {
        ENS(d_dense, std::max<uint64_t>(1, ids_off) * 8); ENS(d_pre, std::max<uint64_t>(1, ids_off) * 4);
        ENS(d_sfx, std::max<uint64_t>(1, ids_off) * 4);
        ENS(d_tile_sfx, npt * 8); ENS(d_tile_sfx_off, npt * 8); ENS(d_chunk_sfx, npg * 8);
        CK(hipMemsetAsync(d_chunk_sfx.p, 0, npg * 8, st));
        for (const ChunkDesc &P : pg) {
            if (P.dj0 < 0) continue;
            if (cols[P.col].phys == KPW_BYTE_ARRAY) { dj[P.dj0].vals = d_pre.p; dj[P.dj0 + 1].vals = d_sfx.p; }
            else dj[P.dj0].vals = d_dense.p;
        }
        const size_t nb = std::max<size_t>(1, dblk_job.size());
        ENS(d_djobs, std::max<size_t>(1, dj.size()) * sizeof(DeltaJob)); ENS(d_blk_job, nb * 4); ENS(d_blk_min, nb * 8);
        ENS(d_blk_w, nb * 4); ENS(d_blk_sz, nb * 8); ENS(d_blk_off, nb * 8); ENS(d_btot, std::max<size_t>(1, dj.size()) * 8);
        if (!dblk_job.empty()) CK(xh2d(d_blk_job.p, dblk_job.data(), dblk_job.size() * 4, st));
        dla.jobs = d_djobs.as<DeltaJob>(); dla.njobs = (uint32_t)dj.size(); dla.nblk = (uint32_t)dblk_job.size();
        dla.blk_job = d_blk_job.as<uint32_t>(); dla.blk_min = d_blk_min.as<uint64_t>(); dla.blk_w = d_blk_w.as<uint32_t>();
        dla.blk_sz = d_blk_sz.as<uint64_t>(); dla.blk_off = d_blk_off.as<uint64_t>(); dla.btot = d_btot.as<uint64_t>();
        dla.seg = &seg_;
    }
    // first tile and tile count per page and per dictionary chunk, the dictionary chunks and their
    // per-round offsets in one copy; the tile maps and the insertion order expanded from them
    std::vector<uint8_t *> tp;
    if (int rs = upload_parts(d_ctile, {{pfirst.data(), (size_t)npg * 4}, {pcount.data(), (size_t)npg * 4},
                                        {dfirst.data(), (size_t)nc * 4}, {dcount.data(), (size_t)nc * 4},
                                        {dlist.data(), dlist.size() * 4}, {droff.data(), droff.size() * 4}}, tp))
        return rs;
    ENS(d_ctj, std::max<uint64_t>(1, npt) * 4); ENS(mp_dtj, std::max<uint64_t>(1, ndt) * 4);
    ENS(d_dorder, std::max<uint64_t>(1, ndict_tiles) * 4);
    {
        TileMapArgs ta{};
        ta.nm = 2;
        ta.m[0] = TileMapSpec{(const uint32_t *)tp[0], (const uint32_t *)tp[1], 1u, (uint32_t)npg, d_ctj.as<uint32_t>()};
        ta.m[1] = TileMapSpec{(const uint32_t *)tp[2], (const uint32_t *)tp[3], 1u, (uint32_t)nc, mp_dtj.as<uint32_t>()};
        launch_tile_maps(ta, st);
        launch_dict_order((const uint32_t *)tp[4], (uint32_t)dlist.size(), (const uint32_t *)tp[2], (const uint32_t *)tp[3],
                          (const uint32_t *)tp[5], maxnt, d_dorder.as<uint32_t>(), st);
        CK(hipGetLastError());
    }

    ChunkArgs ap{};
    ap.ch = d_chunks.as<ChunkDesc>(); ap.nchunks = npg; ap.nctiles = npt; ap.cols = d_cols.as<DevCol>(); ap.data = d_data;
    ap.ctile_chunk = d_ctj.as<uint32_t>(); ap.ctile_first = (uint32_t *)tp[0];
    ap.ctile_count = (uint32_t *)tp[1]; ap.tile_raw = d_tile_raw.as<uint64_t>();
    ap.tile_raw_off = d_tile_raw_off.as<uint64_t>(); ap.tile_smin = d_tile_smin.as<uint64_t>();
    ap.tile_smax = d_tile_smax.as<uint64_t>(); ap.tile_cnt = d_tile_cnt.as<uint32_t>(); ap.tile_sz = d_tile_sz.as<uint64_t>();
    ap.ht = d_ht.as<HtSlot>();
    ap.ids = d_ids.as<uint32_t>(); ap.ent_rec = d_ent_rec.as<uint64_t>(); ap.ent_boff = d_ent_boff.as<uint64_t>();
    if (pd_on_) {   // every dictionary (and so every page's ids) in the kept continuation buffers
        ap.ht = pd_ht.as<HtSlot>();
        ap.ids = pd_ids.as<uint32_t>(); ap.ent_rec = pd_ent_rec.as<uint64_t>(); ap.ent_boff = pd_ent_boff.as<uint64_t>();
        for (int c = 0; c < nc; c++)   // a column's first probe of the open row group: an empty table
            if (dch[c].is_dict && pd_[c].done == 0 && !pd_[c].stopped && dch[c].npages > 0)
                CK(hipMemsetAsync(ap.ht + dch[c].ht_off, 0xFF, (pd_ht_cap_ + 1) * sizeof(HtSlot), st));
    }
    ap.fmask = d_fmask.as<uint8_t>();
    ap.max_dict_bytes = (uint32_t)props.dictionary_page_size;
    ap.data_end = d_off + n; ap.collision = d_coll;
    ap.page_pre = d_ppre;
    ap.mp = 1;
    ap.seg = &seg_;
    ap.v2 = v2_ ? 1 : 0;
    if (v2_) { ap.djobs = dla.jobs; ap.djobs_w = dla.jobs; ap.chunk_sfx = d_chunk_sfx.as<uint64_t>(); }
    ChunkArgs ad = ap;
    ad.ch = mp_dch.as<ChunkDesc>(); ad.nchunks = nc; ad.nctiles = ndt;
    ad.ctile_chunk = mp_dtj.as<uint32_t>(); ad.ctile_first = (uint32_t *)tp[2];
    ad.ctile_count = (uint32_t *)tp[3]; ad.tile_raw = mp_dtile_raw.as<uint64_t>(); ad.tile_raw_off = nullptr;
    ad.tile_smin = mp_dtile_smin.as<uint64_t>(); ad.tile_smax = mp_dtile_smax.as<uint64_t>();
    ad.tile_cnt = mp_dtile_cnt.as<uint32_t>(); ad.tile_sz = mp_dtile_sz.as<uint64_t>();
    ad.max_dict_bytes = 0xFFFFFFFFu;   // the dictPageSize limit is applied per page (k_mp_dict_decide)
    ad.dict_order = d_dorder.as<uint32_t>(); ad.ndict_tiles = ndict_tiles;
    ad.mp_round_end = rend.data(); ad.mp_nrounds = (uint32_t)rlen.size(); ad.mp_round_len = rlen.data();
    ad.mp_dict_limit = (uint32_t)props.dictionary_page_size;
    ad.dict_wide = probe_ ? 1u : 0u;

    uint32_t enpt = 0, enet = 0;
    RleScratch esc{};
    uint64_t body_tot = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        ap.exact_strings = ad.exact_strings = pd_on_ ? (pd_exact_ ? 1 : 0) : attempt;
        CK(xh2d(d_chunks.p, pg.data(), npg * sizeof(ChunkDesc), st));
        CK(xh2d(mp_dch.p, dch.data(), nc * sizeof(ChunkDesc), st));
        if (v2_ && !dj.empty()) CK(xh2d(d_djobs.p, dj.data(), dj.size() * sizeof(DeltaJob), st));
        ap.ht_clear = d_ht.as<HtSlot>(); ap.ht_clear_n = ht_off;   // K6 empties the hash tables and the flags
        ap.flags_clear = (uint64_t *)d_coll;
        launch_chunk_stats(ap, st);                          // K6 per page (+ nn, raw bytes)
        if (!ej.empty()) {
            int rs = run_rle(ej, enpt, enet, esc);
            if (rs) return rs;
            if (v2_) launch_v2_bool_jobs(ap, d_jobs.as<RleJob>(), st);   // optional booleans: page rank base + length
        }
        launch_mp_pages_init(ap.ch, npg, ad.ch, ap.cols, d_jobs.as<RleJob>(), st);
        if (!spec) launch_dict(ad, d_jobs.as<RleJob>(), st);   // K2 per column chunk (splice: spec's)
        launch_page_str_stats(ap, st);
        launch_mp_dict_decide(ap.ch, npg, ad.ch, ap.cols, ap.ent_rec, ap.ent_boff, (uint32_t)props.dictionary_page_size,
                              d_jobs.as<RleJob>(), st);
        CK(hipGetLastError());
        if (!ej.empty()) launch_rle_structure(d_jobs.as<RleJob>(), (int)ej.size(), enpt, enet, esc, st);
        launch_mp_satisfy(ap.ch, ad.ch, nc, ap.cols, ap.ent_rec, ap.ent_boff, d_jobs.as<RleJob>(), st);
        if (v2_) {   // the fallback pages' DELTA streams
            launch_v2_delta_jobs(ap, dla.jobs, st);
            launch_v2_dense(ap, d_dense.as<uint64_t>(), d_pre.as<uint32_t>(), d_sfx.as<uint32_t>(), d_tile_sfx.as<uint64_t>(),
                            d_tile_sfx_off.as<uint64_t>(), d_chunk_sfx.as<uint64_t>(), st);
            launch_delta_structure(dla, st);
        }
        launch_layout(ap, d_jobs.as<RleJob>(), d_poff, d_plen, pt, st);
        CK(hipGetLastError());
        CK(xd2h(ptab.data(), pt, (4 + (v2_ ? 3 : 2) * P2) * 8, st));   // totals, flags, offsets, lengths (v2: prefixes)
        // (the dictionary descriptors come back with the compression's sync: a D2H into pageable
        // memory holds the host until the stream reaches it, an idle gap before every later launch)
        CK(xsync(st));
        body_tot = ptab[0];
        const uint32_t coll = (uint32_t)ptab[2];
        if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "segmented scan scratch allocation failed");
        if (!coll) break;
        // a continuation's kept tables hold hash keys of earlier probes: the probe restarts the open
        // row group's dictionaries in exact mode (probe_mp)
        if (pd_on_) return pd_exact_ ? fail(KPW_ERR_DEVICE, "string dictionary verification failed in exact mode") : kPdRetry;
        if (attempt == 1) return fail(KPW_ERR_DEVICE, "string dictionary verification failed in exact mode");
        for (int c = 0; c < nc; c++) {   // restore the host descriptors for the exact re-run
            dch[c].nn = 0; dch[c].dict_bytes = 0; dch[c].dict_n = 0; dch[c].fallback = 0; dch[c].overflow = 0;
            dch[c].stop_tile = 0;
        }
    }
    ENS(d_body, body_tot + 512 + 4096);   // + 4 KiB: the writer D2Hs whole 4 KiB units
    // only the tail K7's windows may read and the PLAIN boolean values are cleared (k_chunk_prep,
    // launch_chunk_write); every other body byte is written by its kernel (KPW_BODY_POISON=1 fills
    // the body with 0xAB first: the GPU parity suite checks that)
    if (body_poison()) CK(hipMemsetAsync(d_body.p, 0xAB, body_tot, st));
    ap.body_tail = body_tot;
    launch_mp_dictpage_off(ap.ch, ad.ch, nc, st);
    if (!k7_from) launch_dict_page(ad, d_body.as<uint8_t>(), st);   // (a probe needs no dictionary page bytes)
    launch_chunk_write(ap, d_jobs.as<RleJob>(), d_body.as<uint8_t>(), st);
    if (!ej.empty()) launch_rle_write(d_jobs.as<RleJob>(), enpt, enet, esc, d_body.as<uint8_t>(), st);
    if (v2_) {
        launch_delta_write(dla, d_body.as<uint8_t>(), st);
        launch_dba_suffixes(ap, d_pre.as<uint32_t>(), dla.jobs, d_tile_sfx_off.as<uint64_t>(), d_body.as<uint8_t>(), st);
    }
    CK(hipGetLastError());
    // page metadata (the dictionary descriptors, the page descriptors and their binary statistics'
    // offsets / lengths) queued now, so they come back with the compression's results in its sync
    uint64_t *const d_smeta = (uint64_t *)(d_chunks.as<ChunkDesc>() + npg);
    static thread_local std::vector<uint8_t> md;
    md.resize(npg * (sizeof(ChunkDesc) + 32));
    launch_stats_gather(d_chunks.as<ChunkDesc>(), npg, d_cols.as<DevCol>(), d_data, d_smeta, nullptr, st);
    // their readback is queued behind the compression's launches (queue_meta), so the host issues
    // K7 without waiting for the stream; no sync here: the page offsets and lengths came back with
    // the layout
    auto queue_meta = [&]() -> hipError_t {
        hipError_t e = xd2h(dch.data(), mp_dch.p, nc * sizeof(ChunkDesc), st);
        return e != hipSuccess ? e : xd2h(md.data(), d_chunks.p, md.size(), st);
    };
    std::vector<uint64_t> poff(ptab.begin() + 4, ptab.begin() + 4 + P2), plen(ptab.begin() + 4 + P2, ptab.begin() + 4 + 2 * P2);
    std::vector<uint64_t> pcoff(P2), pclen(P2), ppre(P2, 0);
    if (v2_) ppre.assign(ptab.begin() + 4 + 2 * P2, ptab.begin() + 4 + 3 * P2);
    // ---------------------------------------------------------------- K7
    if (props.codec == KPW_SNAPPY) {
        std::vector<uint32_t> fpage, fidx, pfrag0(2 * npg);
        for (int p = 0; p < 2 * npg; p++) {
            pfrag0[p] = (uint32_t)fpage.size();
            if (k7_from && (!(p & 1) || !k7_on[p >> 1])) continue;   // a probe: only the newly cut pages
            const uint64_t nf = (plen[p] + SNAPPY_FRAG - 1) / SNAPPY_FRAG;
            for (uint64_t k = 0; k < nf; k++) { fpage.push_back((uint32_t)p); fidx.push_back((uint32_t)k); }
        }
        const uint32_t nf = (uint32_t)fpage.size();
        ENS(d_frag_out, (uint64_t)std::max<uint32_t>(1, nf) * SNAPPY_FRAG_CAP); ENS(d_frag_len, std::max<uint32_t>(1, nf) * 4);
        ENS(d_frag_coff, std::max<uint32_t>(1, nf) * 8);
        ENS(d_comp, body_tot + (uint64_t)nf * 64 + 2 * npg * 8 + 64 + 4096);
        std::vector<uint8_t *> kt;   // fragment -> page, index in page, first fragment per page: one copy
        if (int rs = upload_parts(d_ktab, {{fpage.data(), (size_t)nf * 4}, {fidx.data(), (size_t)nf * 4}, {pfrag0.data(), (size_t)2 * npg * 4}},
                                  kt))
            return rs;
        SnappyArgs sa{};
        sa.in = d_body.as<uint8_t>(); sa.page_off = d_poff; sa.page_len = d_plen;
        sa.npages = 2 * npg; sa.nfrags = nf; sa.frag_page = (uint32_t *)kt[0]; sa.frag_idx = (uint32_t *)kt[1];
        sa.frag_out = d_frag_out.as<uint8_t>(); sa.frag_len = d_frag_len.as<uint32_t>();
        sa.page_coff = d_pcoff; sa.page_clen = d_pclen;
        sa.frag_coff = d_frag_coff.as<uint64_t>(); sa.out = d_comp.as<uint8_t>(); sa.tot = pt + 1;
        sa.page_pre = v2_ ? d_ppre : nullptr;   // v2: levels in front, uncompressed
        if (seg_args(sa)) return KPW_ERR_NOMEM;
        launch_snappy(sa, st);
        launch_snappy_finish(sa, (const uint32_t *)kt[2], st);
        CK(hipGetLastError());
        {   // compressed total, offsets, lengths + the descriptors, gathered on the device (copies
            // that do not hold the host) and read back at once: each D2H into pageable memory
            // holds the host ~17 us before it can issue the next (r06bt probe trace)
            const size_t pb = (4 + 5 * P2) * 8, db = nc * sizeof(ChunkDesc);
            uint8_t *const rb = (uint8_t *)pt;
            CK(hipMemcpyAsync(rb + pb, mp_dch.p, db, hipMemcpyDeviceToDevice, st));
            CK(hipMemcpyAsync(rb + pb + db, d_chunks.p, md.size(), hipMemcpyDeviceToDevice, st));
            const size_t xb = rb_extra_src_ ? 8 : 0;   // + the caller's word (probe_mp: K1's verdict)
            if (xb) CK(hipMemcpyAsync(rb + pb + db + md.size(), rb_extra_src_, 8, hipMemcpyDeviceToDevice, st));
            static thread_local std::vector<uint8_t> rbh;
            rbh.resize(pb + db + md.size() + xb);
            CK(xd2h(rbh.data(), rb, rbh.size(), st));
            CK(xsync(st));
            memcpy(ptab.data(), rbh.data(), pb);
            memcpy(dch.data(), rbh.data() + pb, db);
            memcpy(md.data(), rbh.data() + pb + db, md.size());
            if (xb) { memcpy(&rb_extra_val_, rbh.data() + pb + db + md.size(), 8); rb_extra_done_ = true; }
        }
        const uint64_t ctot = ptab[1];
        pcoff.assign(ptab.begin() + 4 + 3 * P2, ptab.begin() + 4 + 4 * P2);
        pclen.assign(ptab.begin() + 4 + 4 * P2, ptab.begin() + 4 + 5 * P2);
        pages_dev_ = d_comp.as<uint8_t>();
        pages_len_ = ctot;
    } else if (props.codec == KPW_GZIP) {
        // a probe (k7_from) compresses only the data pages cut since its previous probe
        std::vector<char> on(2 * npg, 1);
        if (k7_from)
            for (int p = 0; p < 2 * npg; p++) on[p] = (p & 1) && k7_on[p >> 1];
        uint64_t cap = 4096;
        for (int p = 0; p < 2 * npg; p++) cap += ppre[p] + dfl_member_bound(plen[p]);
        ENS(d_comp, cap);
        if (int rs = gzip_pages(d_body.as<uint8_t>(), body_tot, d_poff, v2_ ? d_ppre : nullptr, poff, plen, on, d_pcoff,
                                d_pclen, pt + 1, pt + 3, st))
            return rs;
        CK(queue_meta());
        CK(xd2h(ptab.data(), pt, (4 + 5 * P2) * 8, st));   // compressed total, overflow, offsets, lengths
        CK(xsync(st));
        if (ptab[3]) return fail(KPW_ERR_DEVICE, "gzip member overflowed its scratch slot");
        pcoff.assign(ptab.begin() + 4 + 3 * P2, ptab.begin() + 4 + 4 * P2);
        pclen.assign(ptab.begin() + 4 + 4 * P2, ptab.begin() + 4 + 5 * P2);
        pages_dev_ = d_comp.as<uint8_t>();
        pages_len_ = ptab[1];
    } else {   // uncompressed: a (v2) page body starts at its level prefix
        for (int p = 0; p < 2 * npg; p++) { pcoff[p] = poff[p] - ppre[p]; pclen[p] = plen[p] + ppre[p]; }
        pages_dev_ = d_body.as<uint8_t>();
        pages_len_ = body_tot;
        CK(queue_meta());
        CK(xsync(st));
    }
    if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "segmented scan scratch allocation failed");
    for (int c = 0; c < nc; c++)
        if (dch[c].is_dict && dch[c].overflow) return fail(KPW_ERR_DEVICE, "multi-page dictionary table overflow");
    // ---------------------------------------------------------------- page metadata
    // (read back above, with the compression's sync)
    std::vector<uint64_t> smeta(4 * npg, 0);
    memcpy(pg.data(), md.data(), npg * sizeof(ChunkDesc));
    for (auto &C : pg) chunk_stats_derive(C);
    memcpy(smeta.data(), md.data() + npg * sizeof(ChunkDesc), npg * 32);
    std::vector<std::string> bmin(npg), bmax(npg);
    {
        uint64_t blob_len = 0;
        std::vector<uint64_t> boff(npg);
        for (int p = 0; p < npg; p++) {
            boff[p] = blob_len;
            if (cols[pg[p].col].phys == KPW_BYTE_ARRAY && pg[p].has_minmax) blob_len += smeta[4 * p + 1] + smeta[4 * p + 3];
        }
        // a probe needs the page headers' sizes only: the min / max lengths, and whether min ==
        // max (write_stats then also writes the deprecated fields), which k_stats_gather flags
        // (bit 63 of the max offset word), so no bytes come back
        if (blob_len && probe_) {
            for (int p = 0; p < npg; p++)
                if (cols[pg[p].col].phys == KPW_BYTE_ARRAY && pg[p].has_minmax) {
                    const bool eq = (smeta[4 * p + 2] >> 63) != 0;
                    bmin[p].assign(smeta[4 * p + 1], 'a');
                    bmax[p].assign(smeta[4 * p + 3], eq ? 'a' : 'b');
                }
        } else if (blob_len) {
            std::vector<uint8_t> blob(blob_len);
            ENS(d_sblob, blob_len);
            launch_stats_gather(d_chunks.as<ChunkDesc>(), npg, d_cols.as<DevCol>(), d_data, d_smeta,
                                d_sblob.as<uint8_t>(), st);
            CK(xd2h(blob.data(), d_sblob.p, blob_len, st));
            CK(xsync(st));
            for (int p = 0; p < npg; p++) {
                if (cols[pg[p].col].phys != KPW_BYTE_ARRAY || !pg[p].has_minmax) continue;
                const uint64_t l1 = smeta[4 * p + 1], l2 = smeta[4 * p + 3];
                bmin[p].assign((const char *)blob.data() + boff[p], l1);
                bmax[p].assign((const char *)blob.data() + boff[p] + l1, l2);
            }
        }
    }
    for (int p = 0; p < npg; p++) {
        const ChunkDesc &C = pg[p];
        const ColInfo &col = cols[C.col];
        std::vector<PageOut> &out = run.cols[C.col];
        if (C.dictpage_len) {   // ColumnChunkPageWriter: the dictionary page first
            PageOut d;
            d.page_type = KPW_DICTIONARY_PAGE;
            d.num_values = (int32_t)dch[C.col].dict_n;
            d.encoding = v2_ ? KPW_ENC_PLAIN : KPW_ENC_PLAIN_DICTIONARY;   // DictionaryValuesWriter v1 / v2 page encoding
            d.dl_encoding = d.rl_encoding = 0;
            d.has_stats = 0;
            d.uncompressed_size = (int64_t)plen[2 * p];
            d.compressed_size = (int64_t)pclen[2 * p];
            d.offset = pcoff[2 * p];
            d.null_count = 0;
            d.has_min_max = 0;
            out.push_back(d);
        }
        PageOut q;
        q.page_type = v2_ ? KPW_DATA_PAGE_V2 : KPW_DATA_PAGE;
        q.num_values = (int32_t)(C.e - C.s);
        if (!v2_) {
            q.encoding = (C.is_dict && !C.fallback) ? KPW_ENC_PLAIN_DICTIONARY : KPW_ENC_PLAIN;
        } else if (col.phys == KPW_BOOLEAN) {
            q.encoding = KPW_ENC_RLE;
        } else if (C.is_dict && !C.fallback) {
            q.encoding = KPW_ENC_RLE_DICTIONARY;
        } else {   // DefaultV2ValuesWriterFactory fallback writers
            q.encoding = col.phys == KPW_BYTE_ARRAY ? KPW_ENC_DELTA_BYTE_ARRAY
                       : (col.phys == KPW_INT32 || col.phys == KPW_INT64) ? KPW_ENC_DELTA_BINARY_PACKED : KPW_ENC_PLAIN;
        }
        q.dl_encoding = col.optional ? KPW_ENC_RLE : KPW_ENC_BIT_PACKED;
        q.rl_encoding = KPW_ENC_BIT_PACKED;
        q.has_stats = 1;
        q.dl_byte_length = v2_ ? (int32_t)C.dl_len : 0;
        q.rl_byte_length = v2_ ? C.rl0_len : 0;
        q.uncompressed_size = (int64_t)(plen[2 * p + 1] + ppre[2 * p + 1]);
        q.compressed_size = (int64_t)pclen[2 * p + 1];
        q.offset = pcoff[2 * p + 1];
        q.num_rows = (int32_t)(C.e - C.s);
        q.null_count = (int64_t)C.null_count;
        q.has_min_max = C.has_minmax ? 1 : 0;
        if (C.has_minmax) {
            if (col.phys == KPW_BYTE_ARRAY) {
                q.min = bmin[p];
                q.max = bmax[p];
            } else {
                auto unkey = [&](uint64_t k) -> uint64_t {
                    switch (col.phys) {
                    case KPW_INT32: return (uint32_t)k ^ 0x80000000u;
                    case KPW_INT64: return k ^ 0x8000000000000000ull;
                    case KPW_FLOAT: { uint32_t b = (uint32_t)k; return (b >> 31) ? (b & 0x7fffffffu) : (uint32_t)~b; }
                    case KPW_DOUBLE: return (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
                    default: return k;
                    }
                };
                auto le = [&](uint64_t v) {
                    std::string s2;
                    const int nb = col.phys == KPW_BOOLEAN ? 1 : col.vsize;
                    for (int i = 0; i < nb; i++) s2.push_back((char)(uint8_t)(v >> (8 * i)));
                    return s2;
                };
                q.min = le(unkey(C.smin));
                q.max = le(unkey(C.smax));
            }
        }
        out.push_back(q);
    }
    run.pg = std::move(pg);
    run.dch = std::move(dch);
    return KPW_OK;
}

// KPW_PROBE_EXACT=1 (test infrastructure): continuation probes compare string keys byte for byte
// from a row group's first probe on, the mode a hash collision switches to (tests/pipeline_options_child.py)
static bool pd_exact_forced()
{
    static const bool on = [] { const char *e = getenv("KPW_PROBE_EXACT"); return e && e[0] == '1'; }();
    return on;
}

void Engine::pd_reset()
{
    for (ProbeDict &Q : pd_) Q = ProbeDict();
    pd_exact_ = pd_exact_forced();
}

// The continuation buffers for a probe of [0, ne): per dictionary column a hash table and entry
// arrays sized for one dictionary (dictPageSize of the smallest entries + 1, plus one insertion
// round) and one id per record so far (grown by doubling, the kept ids copied).
int Engine::pd_prepare(uint64_t ne)
{
    const int nc = (int)cols.size();
    if ((int)pd_slot_.size() != nc) {
        pd_slot_.assign(nc, -1);
        int k = 0;
        for (int c = 0; c < nc; c++) if (cols[c].dict) pd_slot_[c] = k++;
    }
    uint64_t nd = 0;
    for (int c = 0; c < nc; c++) nd += pd_slot_[c] >= 0 ? 1 : 0;
    if (!nd) return KPW_OK;
    hipStream_t st = stream;
    if (!pd_ht_cap_) {
        pd_ent_cap_ = (uint64_t)props.dictionary_page_size / 4 + 1 + (uint64_t)kMpRoundTiles * KPW_TILE_P_H;
        pd_ht_cap_ = next_pow2_mp(2 * pd_ent_cap_);
        ENS(pd_ht, nd * (pd_ht_cap_ + 1) * sizeof(HtSlot));
        ENS(pd_ent_rec, nd * pd_ent_cap_ * 8);
        ENS(pd_ent_boff, nd * pd_ent_cap_ * 8);
    }
    if (ne > pd_ids_cap_) {
        const uint64_t cap = std::max<uint64_t>(2 * ne, 1u << 16);
        DevBuf nb;
        ENS(nb, nd * cap * 4);
        if (pd_ids_cap_)
            for (uint64_t k = 0; k < nd; k++)
                CK(hipMemcpyAsync(nb.as<uint32_t>() + k * cap, pd_ids.as<uint32_t>() + k * pd_ids_cap_, pd_ids_cap_ * 4,
                                  hipMemcpyDeviceToDevice, st));
        CK(xsync(st));   // (the old buffer is released when nb goes)
        pd_ids.swap(nb);
        pd_ids_cap_ = cap;
    }
    return KPW_OK;
}

// probe_pages: the open row group's prefix [0, ne) with its page cuts `pc` (cuts <= ne, a cut at
// ne included) -> per probed column the pages cut inside it and their header + compressed
// bytes, i.e. ColumnChunkPageWriter.getMemSize() after record ne - 1
int Engine::probe_mp(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, uint64_t ne, const std::vector<DevCol> &hc,
                     const std::vector<std::vector<int64_t>> &pc, BatchOut &out)
{
    hipStream_t st = stream;
    const int nc = (int)cols.size();
    MpRun pr;
    // pages cut in an earlier probe of this row group keep their sizes: only the ones cut since
    // are compressed (a cached page whose end moved would be a bug: recompute them all)
    probe_cache_.resize(nc);
    std::vector<uint32_t> from(nc, 0);
    for (int c = 0; c < nc; c++) {
        std::vector<CutPage> &pcache = probe_cache_[c];
        bool ok = pcache.size() <= pc[c].size();
        for (size_t i = 0; ok && i < pcache.size(); i++) ok = pcache[i].end == pc[c][i];
        if (!ok) { pcache.clear(); if (pd_.size() > (size_t)c) pd_[c] = ProbeDict(); }
        from[c] = (uint32_t)pcache.size();
    }
    probe_mode_.resize(nc, 0);
    for (int c = 0; c < nc; c++) if (from[c] == 0) probe_mode_[c] = 0;
    pd_on_ = pd_enabled() && !v2_;
    if (pd_on_) {
        pd_.resize(nc);
        for (int c = 0; c < nc; c++) if (from[c] == 0) pd_[c] = ProbeDict();   // (its row group's first probe)
        if (int rs = pd_prepare(ne)) { pd_on_ = false; return rs; }
    }
    // K1's verdict, not read before the probe (encode_impl: model probes): the pipeline reads it
    // back with its last copy (a D2H of its own into pageable memory would hold the host until
    // K1 and the presence scans finish, before the pipeline's host setup: r06bt trace)
    rb_extra_src_ = probe_err_dev_;
    rb_extra_done_ = false;
    auto ms_now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double tq0 = ms_now();
    probe_t[0] += tq0 - t_encode_in_;
    int rs = mp_pipeline(d_data, d_off, n, hc, 0, (int64_t)ne, pc, pr, probe_mask_, &from);
    if (rs == kPdRetry) {
        pd_reset();
        pd_exact_ = true;
        rs = mp_pipeline(d_data, d_off, n, hc, 0, (int64_t)ne, pc, pr, probe_mask_, &from);
    }
    rb_extra_src_ = nullptr;
    if (rs) {
        (void)hipStreamSynchronize(st);
        (void)hipGetLastError();
        pd_on_ = false;
        pd_reset();
        return rs;
    }
    const double tq1 = ms_now();
    probe_t[1] += tq1 - tq0;
    uint64_t err_idx = rb_extra_val_;
    if (!rb_extra_done_) {   // (GZIP / uncompressed pipelines: read it now)
        CK(xd2h(&err_idx, probe_err_dev_, 8, st));
        CK(xsync(st));
    }
    if (pd_on_) {   // what the run inserted stays for the next probe of the row group
        for (int c = 0; c < nc; c++) {
            const ChunkDesc &D = pr.dch[c];
            if (!cols[c].dict || D.npages <= 0 || !D.is_dict) continue;
            ProbeDict &Q = pd_[c];
            Q.n = D.dict_all;
            Q.bytes = D.dict_bytes;
            if (!Q.stopped) {
                Q.done = (int64_t)ne;
                Q.stopped = D.stop_tile != 0 || D.dict_bytes > (uint64_t)props.dictionary_page_size;
            }
        }
        pd_on_ = false;
    }
    probe_npages_.assign(nc, 0);
    probe_flushed_.assign(nc, 0);
    for (int c = 0; c < nc; c++) {
        if (probe_mask_ && !(*probe_mask_)[c]) { probe_npages_[c] = -1; probe_flushed_[c] = -1; continue; }
        std::vector<CutPage> &pcache = probe_cache_[c];
        // the chunk's first page encoded in this run: its dictionary outcome for later probes
        // (k_mp_satisfy: every page PLAIN when it failed isCompressionSatisfying or fell back)
        if (from[c] == 0 && !pr.cols[c].empty() && !pr.dch.empty() && pr.dch[c].npages > 0)
            probe_mode_[c] = (!cols[c].dict || pr.pg[pr.dch[c].first_page].fallback) ? 2u : 1u;
        size_t i = v2_ ? 0 : from[c];   // the run's data pages: the column's pages from[c] on (v2: all)
        for (const PageOut &p : pr.cols[c]) {
            if (p.page_type == KPW_DICTIONARY_PAGE) continue;
            if (i < pc[c].size() && i >= pcache.size())
                pcache.push_back(CutPage{pc[c][i], (int64_t)page_header(p, cols[c].phys).size() + p.compressed_size});
            i++;
        }
        for (const CutPage &cp : pcache) probe_flushed_[c] += cp.bytes;
        probe_npages_[c] = (int32_t)pcache.size();
    }
    out.records_consumed = 0;
    out.open_records = (int64_t)ne;
    CK(xsync(st));   // (nothing queued after the pipeline's last sync: returns at once)
    if (err_idx < n) out.invalid_record = (int64_t)err_idx;
    probe_t[2] += ms_now() - tq1;
    return KPW_OK;
}

// The speculative horizon's hint across engines: the records of the last row group any engine
// cut for the same schema and properties.  A writer opens two fresh engines per file, and a first
// horizon from the raw bytes alone (2 x blockSize) falls short where flushed pages count
// compressed (C2 Rec8 1 MiB pages: 4.3 M against 6.5 M records per row group), costing each
// engine's first job a second speculative pass.  Only the horizon depends on it, never a byte.
static std::mutex g_horizon_mu;
static std::unordered_map<uint64_t, int64_t> g_horizon;

// KPW_MP_LAZY=0: Engine::lazy_open is ignored (A/B)
static bool lazy_on()
{
    static const bool on = [] { const char *e = getenv("KPW_MP_LAZY"); return !(e && e[0] == '0'); }();
    return on;
}

// Speculative horizon past the last row group's records, in percent (KPW_MP_HORIZON_PCT, default
// 12): a larger margin encodes more pages past the cut per pass, a too small one misses the cut
// and pays a second pass over twice the range (r06l, bulk_multipage, two alternations: 25 %
// 24.3 / 23.7, 12 % 24.6 / 24.7, 6 % 24.1 / 24.1 GB/s; rounds 4-5 used 25 %)
static int64_t horizon_pct()
{
    static const int64_t v = [] { const char *e = getenv("KPW_MP_HORIZON_PCT"); const long long x = e ? atoll(e) : 12; return (int64_t)(x > 0 ? x : 12); }();
    return v;
}

// KPW_MP_SPLICE=0: every exact pass re-encodes the whole row group (A/B of the splice)
static bool splice_on()
{
    static const bool on = [] { const char *e = getenv("KPW_MP_SPLICE"); return !(e && e[0] == '0'); }();
    return on;
}

static uint64_t horizon_key(const std::vector<ColInfo> &cols, const kpw_props &p)
{
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    for (const ColInfo &c : cols) { mix((uint64_t)c.field_number); mix((uint64_t)c.phys); mix((uint64_t)c.optional); mix((uint64_t)c.dict); }
    mix((uint64_t)p.block_size); mix((uint64_t)p.page_size); mix((uint64_t)p.dictionary_page_size); mix((uint64_t)p.codec);
    mix((uint64_t)p.writer_version);
    return h;
}

int64_t Engine::rg_records_hint() const
{
    std::lock_guard<std::mutex> g(g_horizon_mu);
    auto it = g_horizon.find(horizon_key(cols, props));
    return it == g_horizon.end() ? 0 : it->second;
}

int Engine::encode_mp(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, uint64_t ne, bool final_flush, int64_t T,
                      const std::vector<DevCol> &hc, uint64_t gend_stride, uint64_t ev_stride, BatchOut &out)
{
    hipStream_t st = stream;
    const int nc = (int)cols.size();
    if (probe_ && probe_cuts_) return probe_mp(d_data, d_off, n, ne, hc, *probe_cuts_, out);
    // per BYTE_ARRAY column: exclusive prefix of (4 + len) over present values
    std::vector<const uint64_t *> sp(nc, nullptr);
    std::vector<int32_t> cstream(nc, -1);
    mp_sp.resize(nc);
    for (size_t k = 0; k < opt_idx_.size(); k++) cstream[opt_idx_[k]] = (int32_t)k;
    for (int c = 0; c < nc; c++) {
        if (cols[c].phys != KPW_BYTE_ARRAY) continue;
        ENS(mp_sp[c], (ne + 1) * 8); ENS(mp_ssz, ne * 4 + 4);
        launch_str_sizes(d_cols.as<DevCol>(), c, ne, mp_ssz.as<uint32_t>(), st);
        launch_prefix_raw(mp_ssz.as<uint32_t>(), ne, mp_sp[c].as<uint64_t>(), &seg_, st);
        if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "scan scratch allocation failed");
        sp[c] = mp_sp[c].as<uint64_t>();
    }
    std::vector<int32_t> bstream(nc, -1);   // v2: planner stream of each BOOLEAN column's values
    if (v2_)
        for (size_t k = 0; k < bool_idx_.size(); k++) bstream[bool_idx_[k]] = (int32_t)(opt_idx_.size() + k);
    ENS(mp_spp, nc * sizeof(uint64_t *)); ENS(mp_cstream, nc * 4); ENS(mp_bstream, nc * 4);
    CK(xh2d(mp_spp.p, sp.data(), nc * sizeof(uint64_t *), st));
    CK(xh2d(mp_cstream.p, cstream.data(), nc * 4, st));
    CK(xh2d(mp_bstream.p, bstream.data(), nc * 4, st));
    uint64_t Ptot = 0;
    CK(xd2h(&Ptot, d_P.as<uint64_t>() + ev_stride / 8, 8, st));   // P8's total
    CK(xsync(st));
    if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "segmented scan scratch allocation failed");

    PageCutArgs a{};
    a.n = ne; a.ncols = nc; a.page_size = props.page_size; a.cols = d_cols.as<DevCol>();
    a.col_stream = mp_cstream.as<int32_t>(); a.E8 = d_E.as<uint32_t>(); a.ev = d_ev.as<uint8_t>(); a.ev_stride = ev_stride;
    a.gend = d_gend.as<uint64_t>();
    a.gend_stride = gend_stride;
    a.sp = mp_spp.as<const uint64_t *>(); a.next_rg_size = T;
    a.col_bstream = mp_bstream.as<int32_t>(); a.streams = d_streams.as<PlanStream>(); a.v2 = v2_ ? 1 : 0;
    static const int str_spec = [] { const char *e = getenv("KPW_PAGE_CUT_SPEC"); return e && e[0] == '0' ? 0 : 1; }();
    a.str_spec = str_spec;
    if (opt_idx_.empty() && !(v2_ && !bool_idx_.empty())) { a.E8 = nullptr; a.ev = nullptr; a.gend = nullptr; }   // no planner streams

    if (probe_) {   // probe_pages: the open row group's prefix [0, ne); its page cuts from the GPU planner
        std::vector<std::vector<int64_t>> pc;
        int rs = mp_cuts(a, 0, (int64_t)ne, pc);
        if (rs) return rs;
        return probe_mp(d_data, d_off, n, ne, hc, pc, out);
    }
    uint64_t acc_len = 0;
    const uint64_t per_rec = std::max<uint64_t>(1, Ptot / ne);
    // first horizon: 2 x the raw records of a row group, or 1.25 x the last row group this engine
    // cut (flushed pages count compressed, so a row group holds more than T of raw bytes; a short
    // horizon costs a second speculative encode, C2 1 MiB pages: 4.3 M -> 8.5 M for a 6.7 M cut)
    int64_t guess = std::max<int64_t>(1000, (int64_t)(2 * (uint64_t)T / per_rec));
    const uint64_t hkey = horizon_key(cols, props);
    if (mp_last_rg_ <= 0) {
        std::lock_guard<std::mutex> g(g_horizon_mu);
        auto it = g_horizon.find(hkey);
        if (it != g_horizon.end()) mp_last_rg_ = it->second;
    }
    if (mp_last_rg_ > 0) guess = std::max<int64_t>(guess, mp_last_rg_ + mp_last_rg_ * horizon_pct() / 100 + 200);
    int64_t s0 = 0;
    std::vector<std::vector<int64_t>> cuts;
    MpRun run;
    auto append = [&](int64_t s, int64_t e) -> int {
        if (grow_keep(mp_acc, acc_len + pages_len_ + 64 + 4096, acc_len)) return KPW_ERR_NOMEM;
        if (pages_len_) CK(hipMemcpyAsync(mp_acc.as<uint8_t>() + acc_len, pages_dev_, pages_len_, hipMemcpyDeviceToDevice, st));
        out.rgs.push_back(RowGroupOut{s, e - s, (int32_t)out.chunks.size()});
        for (int c = 0; c < nc; c++) {
            ChunkOut co;
            co.column = c;
            co.first_page = (int32_t)out.pages.size();
            co.num_values = e - s;
            co.has_dictionary = 0;
            for (PageOut p : run.cols[c]) {
                if (p.page_type == KPW_DICTIONARY_PAGE) co.has_dictionary = 1;
                p.offset += acc_len;
                out.pages.push_back(p);
            }
            co.num_pages = (int32_t)out.pages.size() - co.first_page;
            out.chunks.push_back(co);
        }
        acc_len += pages_len_;
        return KPW_OK;
    };
    // Splice: the kept pages of the speculative `run` (per column its data pages before the last
    // cut <= e, contiguous in pages_dev_) go to the output first, then the exact pass over the
    // last pages (which reuses the device buffers) and its pages.
    auto append_splice = [&](int64_t s, int64_t e) -> int {
        MpRun sp = std::move(run);
        std::vector<uint64_t> ko0(nc, 0), kofs(nc, 0);
        uint64_t kept_total = 0;
        for (int c = 0; c < nc; c++) {
            kofs[c] = kept_total;
            const size_t k = cuts[c].size();
            if (!k) continue;
            size_t first = 0;
            while (first < sp.cols[c].size() && sp.cols[c][first].page_type == KPW_DICTIONARY_PAGE) first++;
            if (first + k + 1 > sp.cols[c].size()) return fail(KPW_ERR_DEVICE, "multi-page splice: page list mismatch");
            const PageOut &a0 = sp.cols[c][first], &a1 = sp.cols[c][first + k - 1];
            ko0[c] = a0.offset;
            kept_total += a1.offset + (uint64_t)a1.compressed_size - a0.offset;
        }
        if (grow_keep(mp_acc, acc_len + kept_total + 64 + 4096, acc_len)) return KPW_ERR_NOMEM;
        const uint64_t kept_base = acc_len;
        for (int c = 0; c < nc; c++) {
            const uint64_t l = (c + 1 < nc ? kofs[c + 1] : kept_total) - kofs[c];
            if (l) CK(hipMemcpyAsync(mp_acc.as<uint8_t>() + kept_base + kofs[c], pages_dev_ + ko0[c], l, hipMemcpyDeviceToDevice, st));
        }
        acc_len += kept_total;
        int rs = mp_pipeline(d_data, d_off, n, hc, s, e, cuts, run, nullptr, nullptr, &sp);
        if (rs) return rs;
        if (grow_keep(mp_acc, acc_len + pages_len_ + 64 + 4096, acc_len)) return KPW_ERR_NOMEM;
        if (pages_len_) CK(hipMemcpyAsync(mp_acc.as<uint8_t>() + acc_len, pages_dev_, pages_len_, hipMemcpyDeviceToDevice, st));
        out.rgs.push_back(RowGroupOut{s, e - s, (int32_t)out.chunks.size()});
        for (int c = 0; c < nc; c++) {
            ChunkOut co;
            co.column = c;
            co.first_page = (int32_t)out.pages.size();
            co.num_values = e - s;
            co.has_dictionary = 0;
            size_t t = 0;   // the exact pass: [dictionary page] last page
            for (; t < run.cols[c].size() && run.cols[c][t].page_type == KPW_DICTIONARY_PAGE; t++) {
                PageOut p = run.cols[c][t];
                co.has_dictionary = 1;
                p.offset += acc_len;
                out.pages.push_back(p);
            }
            const size_t k = cuts[c].size();
            size_t first = 0;
            while (first < sp.cols[c].size() && sp.cols[c][first].page_type == KPW_DICTIONARY_PAGE) first++;
            for (size_t i = 0; i < k; i++) {
                PageOut p = sp.cols[c][first + i];
                p.offset = p.offset - ko0[c] + kept_base + kofs[c];
                out.pages.push_back(p);
            }
            for (; t < run.cols[c].size(); t++) {
                PageOut p = run.cols[c][t];
                p.offset += acc_len;
                out.pages.push_back(p);
            }
            co.num_pages = (int32_t)out.pages.size() - co.first_page;
            out.chunks.push_back(co);
        }
        acc_len += pages_len_;
        return KPW_OK;
    };
    // Non-final batches planned as a whole (no HDFS alignment): every row group's cut first (the
    // speculative passes), then the cuts and the carry go to the caller (on_plan: the next job
    // starts on the other worker), then each row group's exact pass.  Interleaved, the next job
    // waited for every exact pass of this one.
    const bool defer = !final_flush && max_cuts <= 0;
    struct PlannedRg { int64_t s, e; std::vector<std::vector<int64_t>> cuts; };
    std::vector<PlannedRg> planned;
    PlannedRg late{-1, -1, {}};   // lazy_open: the last row group's splice, after on_plan
    int n_spliced = 0;
    // KPW_TRACE=1: wall time per phase (page cuts, speculative encodes, row-group checks, splices,
    // full exact passes); the phases end in host syncs, so the clock brackets their device work
    const bool tr = getenv("KPW_TRACE") && getenv("KPW_TRACE")[0] == '1';
    double tph[5] = {0, 0, 0, 0, 0};
    auto tnow = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double tm = tr ? tnow() : 0.0;
    const double t_pre = tr ? tm - t_encode_in_ : 0.0;   // decode, planner inputs, size prefixes
    auto lap = [&](int k) { if (tr) { const double t = tnow(); tph[k] += t - tm; tm = t; } };
    while (s0 < (int64_t)ne) {
        int64_t h = std::min<int64_t>((int64_t)ne, s0 + guess);
        int64_t po[2] = {-1, 0};
        for (;;) {
            int rs = mp_cuts(a, s0, h, cuts);
            if (rs) return rs;
            lap(0);
            rs = mp_pipeline(d_data, d_off, n, hc, s0, h, cuts, run);
            if (rs) return rs;
            lap(1);
            // header + compressed bytes of every cut page (the open page per column is last),
            // column c's at pb_off[c] (compact: the cut capacity per column is (h - s) / 2 + 2,
            // and a strided table of that size cost a 100+ MB host fill and H2D per row group)
            std::vector<uint64_t> pb, pboff(nc);
            for (int c = 0; c < nc; c++) {
                pboff[c] = pb.size();
                size_t i = 0;
                for (const PageOut &p : run.cols[c]) {
                    if (p.page_type == KPW_DICTIONARY_PAGE) continue;
                    if (i < cuts[c].size()) pb.push_back(page_header(p, cols[c].phys).size() + (uint64_t)p.compressed_size);
                    i++;
                }
            }
            pb.push_back(0);
            ENS(mp_pbytes, pb.size() * 8); ENS(mp_pboff, nc * 8);
            // (pb / pboff outlive the copies: the stream is synchronised below)
            CK(xh2d(mp_pbytes.p, pb.data(), pb.size() * 8, st));
            CK(xh2d(mp_pboff.p, pboff.data(), nc * 8, st));
            a.pbytes = mp_pbytes.as<uint64_t>();
            a.pb_off = mp_pboff.as<uint64_t>();
            a.s = s0; a.h = h;
            launch_plan_mp(a, st);
            CK(hipGetLastError());
            CK(xd2h(po, a.out, 16, st));
            CK(xsync(st));
            lap(2);
            if (po[0] >= 0 || h == (int64_t)ne) break;
            h = std::min<int64_t>((int64_t)ne, s0 + 2 * (h - s0));
        }
        if (po[0] >= 0) {
            const int64_t r = po[0];
            for (auto &v : cuts) v.erase(std::remove_if(v.begin(), v.end(), [r](int64_t x) { return x > r; }), v.end());
            // Splice (v1): every page before a column's last cut <= r is the speculative pass's,
            // byte for byte (its cut, ids, bit width and fallback / first-page decisions do not
            // depend on where the row group ends), so the exact pass encodes only each column's
            // last page and dictionary page.  A column cut exactly at r (its dictionary page would
            // have no page to ride with) and the v2 DELTA streams take the whole exact pass.
            bool splice = splice_on() && !v2_ && planned.empty();
            for (int c = 0; c < nc && splice; c++) splice = cuts[c].empty() || cuts[c].back() < r;
            // lazy_open: fewer records after r than this row group holds are the next job's carry
            // (it plans them from r, so a cut among them is found there); this row group's
            // splice then runs after on_plan
            const bool last = lazy_open && lazy_on() && !final_flush && max_cuts <= 0 && (int64_t)ne - r < r - s0;
            if (splice && last) {
                late = PlannedRg{s0, r, {}};
            } else if (splice) {
                int rs = append_splice(s0, r);
                if (rs) return rs;
                n_spliced++;
                lap(3);
            } else if (defer) {
                planned.push_back(PlannedRg{s0, r, cuts});
            } else {
                int rs = mp_pipeline(d_data, d_off, n, hc, s0, r, cuts, run);
                if (rs) return rs;
                rs = append(s0, r);
                if (rs) return rs;
                lap(4);
            }
            guess = std::max<int64_t>(1000, (r - s0) + (r - s0) * horizon_pct() / 100 + 200);
            mp_last_rg_ = r - s0;
            {
                std::lock_guard<std::mutex> g(g_horizon_mu);
                g_horizon[hkey] = mp_last_rg_;
            }
            s0 = r;
            if (max_cuts > 0 && (int32_t)out.rgs.size() >= max_cuts) break;   // re-planned by the caller
            if (last) {
                out.open_buffered = -1;
                break;
            }
            continue;
        }
        if (final_flush) {   // [s0, ne) was just encoded with its final pages
            int rs = append(s0, (int64_t)ne);
            if (rs) return rs;
            s0 = (int64_t)ne;
        } else {
            out.open_buffered = po[1];
        }
        break;
    }
    CK(xsync(st));
    out.records_consumed = s0;
    out.open_records = (int64_t)ne - s0;
    if (final_flush) out.open_buffered = 0;
    if (on_plan) on_plan(out);
    lap(2);
    if (late.s >= 0) {   // (the speculative run and cuts of this row group are still in place)
        int rs = append_splice(late.s, late.e);
        if (rs) return rs;
        n_spliced++;
        lap(3);
    }
    for (const PlannedRg &g : planned) {   // (defer) the exact passes
        int rs = mp_pipeline(d_data, d_off, n, hc, g.s, g.e, g.cuts, run);
        if (rs) return rs;
        rs = append(g.s, g.e);
        if (rs) return rs;
        lap(4);
    }
    CK(xsync(st));
    lap(4);
    if (tr)
        fprintf(stderr, "[kpw] multi-page encode: %zu row groups, %d spliced; ms: decode + inputs %.2f, page cuts %.2f, speculative %.2f, "
                        "checks %.2f, splices %.2f, exact %.2f\n", out.rgs.size(), n_spliced, t_pre, tph[0], tph[1], tph[2], tph[3], tph[4]);
    out.d_pages = mp_acc.as<uint8_t>();
    out.pages_len = acc_len;
    pages_dev_ = mp_acc.as<uint8_t>();
    pages_len_ = acc_len;
    CK(hipEventRecord(ev_[7], st));
    CK(hipEventSynchronize(ev_[7]));
    for (int i = 0; i < 10; i++) stage_ms[i] = 0;
    CK(hipEventElapsedTime(&stage_ms[7], ev_[0], ev_[7]));
    return KPW_OK;
}

int Engine::probe_pages(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, std::vector<int32_t> &npages,
                        std::vector<int64_t> &flushed, const std::vector<char> *cols_mask, uint64_t rg_token,
                        const std::vector<std::vector<int64_t>> *cuts)
{
    if (!mp_) return fail(KPW_ERR_STATE, "probe_pages: single-page regime (no page cuts inside row groups)");
    if (rg_token != probe_token_ || rg_token == ~0ull) { probe_cache_.clear(); pd_reset(); }
    probe_token_ = rg_token;
    probe_cuts_ = v2_ || !cuts || cuts->size() != cols.size() ? nullptr : cuts;
    BatchOut out;
    probe_ = true;
    probe_mask_ = cols_mask;
    const int st = encode(d_data, d_off, n, false, props.block_size, nullptr, out);
    probe_ = false;
    probe_mask_ = nullptr;
    probe_cuts_ = nullptr;
    if (st) return st;
    if (out.invalid_record >= 0) return fail(KPW_ERR_INVALID_PROTO, "probe_pages: invalid record in a modelled row group");
    npages = probe_npages_;
    flushed = probe_flushed_;
    return KPW_OK;
}

}  // namespace kpw
