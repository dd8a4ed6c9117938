// engine.cpp — host orchestration: one handle = one device + one HIP stream.
//
// encode(): device-resident record batch -> row groups exactly where parquet-mr would cut
// them -> per column chunk: dictionary page (if any) + one data page, compressed.
// Host syncs per batch: decode error index, row-group plan, page layout, (snappy sizes),
// chunk metadata — all small; every byte of record/page data stays in HBM.
#include <chrono>
#include "engine.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

namespace {
thread_local hipStream_t tl_order = nullptr;   // StreamOrder: the stream this thread's buffers are used on
}
StreamOrder::StreamOrder(hipStream_t s) : prev_(tl_order) { tl_order = s; }
StreamOrder::~StreamOrder() { tl_order = prev_; }

// Buffers come from the process-wide cache (memcache.h).  Growing one may replace a block
// that queued work (e.g. a D2H of the previous job's pages) still reads: under a StreamOrder
// the old block returns to the cache once that stream has passed this point (work queued
// later on it may already use the new block); without one the device is synchronised first
// (what hipFree used to imply).
int DevBuf::ensure(size_t bytes)
{
    if (bytes <= cap && p) return 0;
    if (p) {
        if (tl_order) dev_free_after(p, tl_order);
        else { device_sync_for_free(); dev_free(p); }
        p = nullptr;
        cap = 0;
    }
    size_t c = bytes < 256 ? 256 : bytes + bytes / 8;
    p = dev_alloc(c);
    if (!p) return -1;
    cap = c;
    return 0;
}
// owners free their buffers only after synchronising the stream that used them
DevBuf::~DevBuf() { dev_free(p); }

Engine::~Engine()
{
    const bool tr = getenv("KPW_TRACE") && getenv("KPW_TRACE")[0] == '1' && stream;
    const auto t0 = std::chrono::steady_clock::now();
    for (auto &e : ev_) if (e) (void)hipEventDestroy(e);
    for (auto &e : kev_) if (e) (void)hipEventDestroy(e);
    for (int k = 0; k < UP_RING; k++)
        if (up_ev_[k]) {
            if (up_used_[k]) (void)hipEventSynchronize(up_ev_[k]);
            (void)hipEventDestroy(up_ev_[k]);
        }
    if (stream) (void)hipStreamSynchronize(stream);
    seg_scratch_free(seg_);
    if (stream && stream != given_stream) (void)hipStreamDestroy(stream);
    if (tr)
        fprintf(stderr, "[kpw] engine free: events+stream %.1f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

int Engine::fail(int code, const std::string &msg)
{
    err_ = msg;
    return code;
}

static int proto_phys(int pt, int &wt, int &utf8, int &vsize)
{
    utf8 = 0;
    vsize = 0;
    switch (pt) {
    case KPW_PT_DOUBLE: wt = 1; vsize = 8; return KPW_DOUBLE;
    case KPW_PT_FLOAT: wt = 5; vsize = 4; return KPW_FLOAT;
    case KPW_PT_INT64: case KPW_PT_UINT64: case KPW_PT_SINT64: wt = 0; vsize = 8; return KPW_INT64;
    case KPW_PT_FIXED64: case KPW_PT_SFIXED64: wt = 1; vsize = 8; return KPW_INT64;
    case KPW_PT_INT32: case KPW_PT_UINT32: case KPW_PT_SINT32: wt = 0; vsize = 4; return KPW_INT32;
    case KPW_PT_FIXED32: case KPW_PT_SFIXED32: wt = 5; vsize = 4; return KPW_INT32;
    case KPW_PT_BOOL: wt = 0; return KPW_BOOLEAN;
    case KPW_PT_STRING: wt = 2; utf8 = 1; return KPW_BYTE_ARRAY;
    case KPW_PT_BYTES: wt = 2; return KPW_BYTE_ARRAY;
    default: return -1;
    }
}

int Engine::init(int dev, const kpw_schema *schema, const kpw_props *pr)
{
    if (!schema || !pr || !schema->columns || schema->num_columns <= 0 || !schema->message_name)
        return fail(KPW_ERR_INVALID_ARG, "null schema/props");
    if (schema->num_columns > MAX_COLS) return fail(KPW_ERR_UNSUPPORTED, "more than 256 columns");
    if (pr->writer_version != 1 && pr->writer_version != 2) return fail(KPW_ERR_UNSUPPORTED, "writer_version must be 1 or 2");
    // PARQUET_2_0 without a dictionary writes DELTA streams directly, and their page-size
    // accounting (DeltaBinaryPacking getBufferedSize = flushed blocks) is not planned here.
    // The reference can never turn the dictionary off (ParquetFile.java:48-50).
    if (pr->writer_version == 2 && !pr->enable_dictionary)
        return fail(KPW_ERR_UNSUPPORTED, "PARQUET_2_0 requires the dictionary on (the only setting the reference produces)");
    if (pr->codec != KPW_UNCOMPRESSED && pr->codec != KPW_SNAPPY && pr->codec != KPW_GZIP) return fail(KPW_ERR_UNSUPPORTED, "codec");
    if (pr->block_size <= 0 || pr->page_size <= 0 || pr->dictionary_page_size <= 0) return fail(KPW_ERR_INVALID_ARG, "sizes");
    props = *pr;
    v2_ = pr->writer_version == 2;
    // pages cut inside row groups: ColumnWriterV1 page checks / ColumnWriteStoreV2 size checks
    // + compressed-size row-group checks.  v2 cuts a page once a column's buffered size is within
    // 10% of pageSize, which a column can reach before its row group flushes even when pageSize
    // >= blockSize (the reference default pageSize = blockSize): v2 plans pages unless pageSize
    // is at least twice blockSize (the single-page path keeps a guard for that case).
    mp_ = pr->page_size < pr->block_size || (v2_ && pr->page_size / 2 < pr->block_size);
    message_name = schema->message_name;
    proto_class = schema->proto_class ? schema->proto_class : schema->message_name;
    for (int c = 0; c < schema->num_columns; c++) {
        const kpw_column_desc &d = schema->columns[c];
        ColInfo ci;
        int wt, utf8, vsize;
        int phys = proto_phys(d.proto_type, wt, utf8, vsize);
        if (phys < 0 || !d.name || d.field_number <= 0 || (d.label != KPW_LABEL_OPTIONAL && d.label != KPW_LABEL_REQUIRED))
            return fail(KPW_ERR_UNSUPPORTED, std::string("column ") + (d.name ? d.name : "?") + ": unsupported proto field");
        ci.name = d.name;
        ci.field_number = d.field_number;
        ci.proto_type = d.proto_type;
        ci.label = d.label;
        ci.phys = phys;
        ci.wire_type = wt;
        ci.optional = d.label == KPW_LABEL_OPTIONAL;
        ci.utf8 = utf8;
        ci.vsize = vsize;
        ci.dict = props.enable_dictionary && phys != KPW_BOOLEAN;
        cols.push_back(ci);
        if (ci.optional) opt_idx_.push_back((uint32_t)c);
        if (phys == KPW_BOOLEAN) bool_idx_.push_back((uint32_t)c);
    }
    device = dev;
    CK(hipSetDevice(dev));
    if (given_stream) stream = given_stream;   // (a writer's stream set, released by the writer)
    else CK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (auto &e : ev_) CK(hipEventCreate(&e));
    for (auto &e : kev_) CK(hipEventCreate(&e));
    for (auto &e : up_ev_) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const size_t nc = cols.size();
    col_vals.resize(nc); col_shash.resize(nc); col_spfx.resize(nc); col_soff.resize(nc); col_slen.resize(nc); col_pres.resize(nc); col_vbits.resize(nc); col_pcnt.resize(nc);
    col_cbits.resize(bool_idx_.size());
    std::vector<int16_t> fmap(FMAP_SIZE, -1);
    for (size_t c = 0; c < nc; c++)
        if (cols[c].field_number < FMAP_SIZE) fmap[cols[c].field_number] = (int16_t)c;
    if (d_fmap.ensure(FMAP_SIZE * sizeof(int16_t))) return fail(KPW_ERR_NOMEM, "fmap");
    CK(hipMemcpy(d_fmap.p, fmap.data(), FMAP_SIZE * sizeof(int16_t), hipMemcpyHostToDevice));
    if (d_opt.ensure(std::max<size_t>(1, opt_idx_.size()) * 4) || d_bool.ensure(std::max<size_t>(1, bool_idx_.size()) * 4))
        return fail(KPW_ERR_NOMEM, "idx");
    if (!opt_idx_.empty()) CK(hipMemcpy(d_opt.p, opt_idx_.data(), opt_idx_.size() * 4, hipMemcpyHostToDevice));
    if (!bool_idx_.empty()) CK(hipMemcpy(d_bool.p, bool_idx_.data(), bool_idx_.size() * 4, hipMemcpyHostToDevice));
    return KPW_OK;
}

#define ENS(buf, bytes) do { if ((buf).ensure(bytes)) return fail(KPW_ERR_NOMEM, "device allocation failed: " #buf); } while (0)

// KPW_COPY_TRACE=1: every small host <-> device copy of the engine (size) on stderr
static bool copy_trace()
{
    static const bool v = [] { const char *e = getenv("KPW_COPY_TRACE"); return e && e[0] == '1'; }();
    return v;
}

// The engine's small host tables and readbacks.  Measured (r04, C2 writer A/B on one box):
// staging them through a pinned arena so they run on SDMA instead of one blit kernel each cost
// 7-10 % (every SDMA copy between two kernels of the stream is a cross-engine wait), so they
// stay plain pageable copies; the readbacks are synchronous, xsync keeps the call sites'
// ordering explicit.  Re-measured in r05 (profiles/r05h_small_copies.md) with every upload and
// readback as a hipMemcpyDeviceToDeviceNoCU copy through pinned staging: C2 140 -> 152-154 ms
// per step, C3 284-297 -> 296-303.
int Engine::upload_parts(DevBuf &buf, const std::vector<HostPart> &parts, std::vector<uint8_t *> &dev, size_t tail_room)
{
    const int k = up_k_;
    up_k_ = (up_k_ + 1) % UP_RING;
    if (up_used_[k]) {   // the copy that last read this slot has completed (at once in practice)
        up_used_[k] = false;
        CK(hipEventSynchronize(up_ev_[k]));
    }
    std::vector<uint8_t> &host = up_host_[k];
    size_t tot = 0;
    for (const HostPart &q : parts) tot += (q.bytes + 255) & ~(size_t)255;
    ENS(buf, std::max<size_t>(tot + tail_room, 256));
    host.resize(tot);
    dev.clear();
    size_t at = 0;
    for (const HostPart &q : parts) {
        if (q.bytes) memcpy(host.data() + at, q.p, q.bytes);
        dev.push_back(buf.as<uint8_t>() + at);
        at += (q.bytes + 255) & ~(size_t)255;
    }
    CK(xh2d(buf.p, host.data(), tot, stream));
    CK(hipEventRecord(up_ev_[k], stream));
    up_used_[k] = true;
    return KPW_OK;
}

hipError_t Engine::xh2d(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    if (copy_trace() && bytes) fprintf(stderr, "[kpw] copy h2d %zu B\n", bytes);
    return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
}

hipError_t Engine::xd2h(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    if (copy_trace() && bytes) fprintf(stderr, "[kpw] copy d2h %zu B\n", bytes);
    return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s) : hipSuccess;
}

hipError_t Engine::xsync(hipStream_t s) { return hipStreamSynchronize(s); }

// Lays out tiles for the given jobs (first tile and tile count per job) and sizes the scratch.
int Engine::rle_layout(std::vector<RleJob> &jobs, uint32_t &npt, uint32_t &net)
{
    npt = net = 0;
    uint32_t nlt = 0;
    uint64_t e0 = 0;
    for (size_t j = 0; j < jobs.size(); j++) {
        RleJob &J = jobs[j];
        const uint64_t len = J.len;
        J.tile0 = npt;
        J.ntiles = (uint32_t)std::max<uint64_t>(1, (len + KPW_TILE_P_H - 1) / KPW_TILE_P_H);
        npt += J.ntiles;
        J.ltile0 = nlt;
        J.nltiles = (uint32_t)std::max<uint64_t>(1, (len + KPW_TILE_L_H - 1) / KPW_TILE_L_H);
        nlt += J.nltiles;
        const uint64_t cap = len / 8 + 2;
        J.etile0 = net;
        J.netiles = (uint32_t)((cap + 255) / 256);
        net += J.netiles;
        J.e0 = e0;
        e0 += (uint64_t)J.netiles * 256;
        J.n_long = J.n_rle = 0;
        J.total_bytes = J.total_groups = J.final_gap_off = J.final_gap_groups = J.final_gap_start = 0;
    }
    r_nlt_ = nlt;
    ENS(r_last, nlt * 8); ENS(r_prev, nlt * 8); ENS(r_lrcnt, nlt * 4); ENS(r_lroff, nlt * 4);
    ENS(r_lra, e0 * 4); ENS(r_lrb, e0 * 4); ENS(r_lrf, e0); ENS(r_rg, e0 * 4);
    ENS(r_rb, e0 * 4); ENS(r_rboff, e0 * 8); ENS(r_rgoff, e0 * 8);
    ENS(r_ptj, std::max<uint64_t>(1, npt) * 4); ENS(r_etj, std::max<uint64_t>(1, net) * 4); ENS(r_ltj, std::max<uint64_t>(1, nlt) * 4);
    return KPW_OK;
}

// The scratch of the jobs laid out last.
void Engine::rle_bind(RleScratch &sc)
{
    sc.ptile_job = r_ptj.as<uint32_t>();
    sc.ltile_job = r_ltj.as<uint32_t>();
    sc.n_ltiles = r_nlt_;
    sc.last_brk = r_last.as<int64_t>();
    sc.prev_brk = r_prev.as<int64_t>();
    sc.lr_cnt = r_lrcnt.as<uint32_t>();
    sc.lr_off = r_lroff.as<uint32_t>();
    sc.etile_job = r_etj.as<uint32_t>();
    sc.lr_a = r_lra.as<uint32_t>();
    sc.lr_b = r_lrb.as<uint32_t>();
    sc.lr_rle = nullptr;   // kept by the planning jobs only (set by the caller)
    sc.r_g = r_rg.as<uint32_t>();
    sc.r_b = r_rb.as<uint32_t>();
    sc.r_boff = r_rboff.as<uint64_t>();
    sc.r_goff = r_rgoff.as<uint64_t>();
    sc.seg = &seg_;
}

// The position / element / long-run tile -> job maps of the jobs laid out last, expanded on the device from
// their uploaded table (k_maps.hip), and the scratch bound.
int Engine::rle_maps(const RleJob *jobs_d, uint32_t njobs, RleScratch &sc)
{
    static_assert(sizeof(RleJob) % 4 == 0, "job words");
    TileMapArgs ta{};
    ta.nm = 3;
    ta.m[0] = TileMapSpec{&jobs_d->tile0, &jobs_d->ntiles, (uint32_t)(sizeof(RleJob) / 4), njobs, r_ptj.as<uint32_t>()};
    ta.m[1] = TileMapSpec{&jobs_d->etile0, &jobs_d->netiles, (uint32_t)(sizeof(RleJob) / 4), njobs, r_etj.as<uint32_t>()};
    ta.m[2] = TileMapSpec{&jobs_d->ltile0, &jobs_d->nltiles, (uint32_t)(sizeof(RleJob) / 4), njobs, r_ltj.as<uint32_t>()};
    launch_tile_maps(ta, stream);
    CK(hipGetLastError());
    rle_bind(sc);
    return KPW_OK;
}

// Lays out tiles for the given jobs, uploads the job table (d_jobs), expands its maps and binds
// the scratch.
int Engine::run_rle(std::vector<RleJob> &jobs, uint32_t &npt, uint32_t &net, RleScratch &sc)
{
    if (int st = rle_layout(jobs, npt, net)) return st;
    std::vector<uint8_t *> dp;
    if (int st = upload_parts(d_jobs, {{jobs.data(), jobs.size() * sizeof(RleJob)}}, dp)) return st;
    return rle_maps(d_jobs.as<RleJob>(), (uint32_t)jobs.size(), sc);
}

// Host side of the dictionary insertion order (k_dict_order): the dictionary chunks in chunk
// order and, per round k, the tiles of rounds < k (chunks with more than k' tiles, k' < k).
int Engine::dict_order(const std::vector<uint32_t> &count, const std::vector<uint8_t> &is_dict, uint32_t &ndict_tiles,
                       std::vector<uint32_t> &list, std::vector<uint32_t> &roff)
{
    list.clear();
    uint32_t maxnt = 0;
    for (size_t ci = 0; ci < count.size(); ci++)
        if (is_dict[ci]) { list.push_back((uint32_t)ci); maxnt = std::max(maxnt, count[ci]); }
    std::vector<uint32_t> hist(maxnt + 1, 0);
    for (uint32_t ci : list) hist[count[ci]]++;
    roff.assign(maxnt + 1, 0);
    uint32_t more = (uint32_t)list.size() - hist[0];   // chunks with more than k tiles, k = 0
    for (uint32_t k = 0; k < maxnt; k++) {
        roff[k + 1] = roff[k] + more;
        more -= hist[k + 1];
    }
    ndict_tiles = roff[maxnt];
    return KPW_OK;
}

static inline uint64_t next_pow2(uint64_t x)
{
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// RLE streams whose emitted bytes count in checkBlockSizeReached: definition levels of optional
// columns; in v2 also the boolean values (RunLengthBitPackingHybridValuesWriter).  Job k = stream
// k, its events at k * ev_stride.
int Engine::plan_inputs(const std::vector<DevCol> &hc, uint64_t ne, uint64_t nwords, std::vector<PlanStream> &hs,
                        std::vector<RleJob> &pj)
{
    hipStream_t s = stream;
    const uint32_t nopt = (uint32_t)opt_idx_.size();
    const uint32_t nbool = (uint32_t)bool_idx_.size();
    const uint32_t nstreams = nopt + (v2_ ? nbool : 0);
    const uint64_t ev_stride = (ne + 1 + 7) & ~7ull;
    std::vector<uint64_t *> &cbits = cbits_;
    cbits.assign(nbool, nullptr);
    if (v2_) {
        for (uint32_t i = 0; i < nbool; i++) {
            const uint32_t c = bool_idx_[i];
            if (cols[c].optional) {
                ENS(col_cbits[i], nwords * 8);
                CK(hipMemsetAsync(col_cbits[i].p, 0, nwords * 8, s));
                cbits[i] = col_cbits[i].as<uint64_t>();
            } else {
                cbits[i] = hc[c].vbits;   // required: the record-indexed value bits are the stream
            }
        }
    }
    hs.resize(nstreams);
    pj.resize(nstreams);
    for (uint32_t k = 0; k < nstreams; k++) {
        PlanStream &S = hs[k];
        S.pad = 0;
        S.len = ne;
        if (k < nopt) { S.bits = hc[opt_idx_[k]].pres; S.rank_col = -1; }
        else {
            const uint32_t c = bool_idx_[k - nopt];
            S.bits = cbits[k - nopt];
            S.rank_col = cols[c].optional ? (int32_t)c : -1;   // optional: length set on the device
        }
        RleJob &J = pj[k];
        memset(&J, 0, sizeof(J));
        J.src.kind = 0;
        J.src.ptr = S.bits;
        J.src.base = 0;
        J.len = (uint32_t)ne;    // upper bound; optional boolean streams are shortened on the device
        J.bw = 1;
        J.out_off = (uint64_t)k * ev_stride;
    }
    return KPW_OK;
}

int Engine::encode(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, bool final_flush, int64_t next_rg_size,
                   hipStream_t user_stream, BatchOut &out)
{
    t_encode_in_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    const int st = encode_impl(d_data, d_off, n, final_flush, next_rg_size, user_stream, out);
    if (st) return st;
    // look-backs that waited past their bound and recomputed the predecessor (kpw_lookback.h):
    // exact either way, counted for kpw_writer_stats (a page-size probe's engine reports none:
    // its count is never read, which saves the probe a readback and a host sync)
    if (probe_) { lb_fallbacks = 0; return KPW_OK; }
    const int lf = lb_failures(&seg_, stream);
    if (lf < 0) return fail(KPW_ERR_DEVICE, "scan status unreadable");
    lb_fallbacks = (uint32_t)lf;
    return KPW_OK;
}

int Engine::encode_impl(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, bool final_flush, int64_t next_rg_size,
                        hipStream_t user_stream, BatchOut &out)
{
    out = BatchOut();
    CK(hipSetDevice(device));
    StreamOrder order(stream);
    if (user_stream) {  // order our stream after the caller's work
        CK(hipEventRecord(ev_[8], user_stream));
        CK(hipStreamWaitEvent(stream, ev_[8], 0));
    }
    hipStream_t s = stream;
    const int nc = (int)cols.size();
    const uint32_t nopt = (uint32_t)opt_idx_.size();
    CK(hipEventRecord(ev_[0], s));
    if (n == 0) {
        for (int i = 0; i < 10; i++) stage_ms[i] = 0;
        return KPW_OK;
    }
    if (n >= 0xFFFFFFF0ull) return fail(KPW_ERR_LIMIT, "batch too large (>= 2^32 records)");
    const uint64_t nwords = n / 64 + 2;

    // ---------------------------------------------------------------- K1 decode
    std::vector<DevCol> hc(nc);
    for (int c = 0; c < nc; c++) {
        const ColInfo &ci = cols[c];
        DevCol &d = hc[c];
        memset(&d, 0, sizeof(d));
        d.phys = ci.phys; d.proto_type = ci.proto_type; d.wire_type = ci.wire_type; d.optional = ci.optional;
        d.field_number = ci.field_number; d.vsize = ci.vsize; d.dict = ci.dict;
        if (ci.vsize) { ENS(col_vals[c], n * ci.vsize); d.vals = col_vals[c].p; }
        if (ci.phys == KPW_BYTE_ARRAY) {
            ENS(col_soff[c], n * 8); ENS(col_slen[c], n * 4); ENS(col_spfx[c], n * 16);
            d.soff = col_soff[c].as<uint64_t>(); d.slen = col_slen[c].as<uint32_t>(); d.spfx = col_spfx[c].as<uint64_t>();
            if (ci.dict) { ENS(col_shash[c], n * 8); d.shash = col_shash[c].as<uint64_t>(); }
        }
        if (ci.optional) {
            ENS(col_pres[c], nwords * 8); ENS(col_pcnt[c], (nwords + 1) * 4);   // K1 writes every word
            d.pres = col_pres[c].as<uint64_t>(); d.pcnt = col_pcnt[c].as<uint32_t>();
        }
        if (ci.phys == KPW_BOOLEAN) {
            ENS(col_vbits[c], nwords * 8);
            d.vbits = col_vbits[c].as<uint64_t>();
        }
    }
    // column descriptors and K1's first-invalid-record word (all ones: none) in one copy; the
    // single-page path (which plans before it knows K1's verdict) adds the planner's inputs for
    // all n records: its RLE jobs, their tile maps and the stream table
    const uint32_t nbool = (uint32_t)bool_idx_.size();
    const uint32_t nstreams = nopt + (v2_ ? nbool : 0);
    const bool plan = nstreams && !(probe_ && probe_cuts_);   // (a v1 probe with the size model's page cuts: none)
    const bool pre = plan && !mp_;
    std::vector<PlanStream> hs;
    std::vector<RleJob> pj;
    uint32_t npt = 0, net = 0;
    static const uint64_t kNoErr = ~0ull;
    std::vector<HostPart> parts{{hc.data(), nc * sizeof(DevCol)}, {&kNoErr, 8}};
    if (pre) {
        if (int st = plan_inputs(hc, n, nwords, hs, pj)) return st;
        if (int st = rle_layout(pj, npt, net)) return st;
        parts.push_back({pj.data(), pj.size() * sizeof(RleJob)});
        parts.push_back({hs.data(), hs.size() * sizeof(PlanStream)});
    }
    std::vector<uint8_t *> cp;
    if (int st = upload_parts(d_cols, parts, cp)) return st;
    RleScratch sc{};
    if (pre) {
        if (int st = rle_maps((const RleJob *)cp[2], nstreams, sc)) return st;
    }
    unsigned long long *const d_err = (unsigned long long *)cp[1];
    ENS(d_raw, n * 4);
    DecodeArgs da;
    da.data = d_data; da.off = d_off; da.n = n; da.cols = d_cols.as<DevCol>(); da.ncols = nc; da.pad = 0;
    da.fmap = d_fmap.as<int16_t>(); da.raw = d_raw.as<uint32_t>(); da.err_min = d_err;
    da.nwords = nwords;
    CK(hipEventRecord(kev_[0], s));
    launch_decode(da, s);
    CK(hipEventRecord(kev_[1], s));
    CK(hipGetLastError());
    CK(hipEventRecord(ev_[1], s));
    // K1's first invalid record bounds the batch.  The single-page path does not wait for it: it
    // plans over all n records and learns the verdict with the plan (k_plan copies it), re-planning
    // over the valid prefix in the rare batch that has one; the multi-page path reads it now.
    uint64_t err_idx = ~0ull;
    // a page-size probe of the size model's row group: the host model validated every record
    // (an invalid one never reaches a probe), so the verdict is read back with the probe's last
    // sync and checked there (probe_mp) instead of costing a sync here
    const bool model_probe = probe_ && probe_cuts_;
    probe_err_dev_ = d_err;
    const bool optimistic = !mp_ || model_probe;
    if (!optimistic) {
        CK(xd2h(&err_idx, d_err, 8, s));
        CK(xsync(s));
    }
    uint64_t ne = std::min<uint64_t>(n, err_idx);

    // ---------------------------------------------------------------- planning inputs
    if (nopt) launch_pcnt_scan(d_cols.as<DevCol>(), d_opt.as<uint32_t>(), nopt, nwords, &seg_, s);
    if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "scan scratch allocation failed");
replan:
    out.invalid_record = err_idx < n ? (int64_t)err_idx : -1;
    if (ne == 0) {
        out.records_consumed = 0;
        out.open_records = 0;
        if (on_plan) on_plan(out);
        CK(xsync(s));
        return KPW_OK;
    }
    const uint64_t ev_stride = (ne + 1 + 7) & ~7ull;   // event bytes per stream (positions 0..ne, 8-aligned)
    const bool pre_ok = pre && ne == n;   // the uploaded inputs are this plan's
    RleJob *pjobs = pre_ok ? (RleJob *)cp[2] : nullptr;   // (d_jobs is set, and may move, in run_rle)
    PlanStream *pstreams = pre_ok ? (PlanStream *)cp[3] : nullptr;
    if (plan) {
        if (pre_ok) {
            rle_bind(sc);   // (maps expanded after the upload)
        } else {
            if (int st = plan_inputs(hc, ne, nwords, hs, pj)) return st;
            ENS(d_streams, nstreams * sizeof(PlanStream));
            CK(xh2d(d_streams.p, hs.data(), nstreams * sizeof(PlanStream), s));
            pstreams = d_streams.as<PlanStream>();
            if (int st = run_rle(pj, npt, net, sc)) return st;
            pjobs = d_jobs.as<RleJob>();
        }
        sc.lr_rle = r_lrf.as<uint8_t>();   // k_plan's walkers read the global parse's decision per long run
        if (v2_ && nbool) {
            ENS(d_cbits_ptr, nbool * sizeof(uint64_t *));
            CK(xh2d(d_cbits_ptr.p, cbits_.data(), nbool * sizeof(uint64_t *), s));
            launch_bool_streams(d_cols.as<DevCol>(), d_bool.as<uint32_t>(), nbool, ne, d_cbits_ptr.as<uint64_t *>(), pjobs, nopt,
                                pstreams, nopt, s);
        }
        ENS(d_ev, (uint64_t)nstreams * ev_stride);
        ENS(d_E, (uint64_t)nstreams * (ev_stride / 8 + 1) * 4);
        CK(hipMemsetAsync(d_ev.p, 0, (uint64_t)nstreams * ev_stride, s));
        // the RLE-run end bitmaps: only the multi-page planners' walkers read them (k_plan's
        // read the per-long-run decisions)
        if (mp_) {
            ENS(d_gend, (uint64_t)nstreams * nwords * 8);
            CK(hipMemsetAsync(d_gend.p, 0, (uint64_t)nstreams * nwords * 8, s));
        }
        launch_rle_structure(pjobs, (int)nstreams, npt, net, sc, s);
        launch_rle_events(pjobs, npt, net, sc, d_ev.as<uint8_t>(), mp_ ? d_gend.as<uint64_t>() : nullptr, nwords, s);
    }
    // one scan for the planner's prefixes per group of 8 positions: the event streams' E8, the raw
    // record sizes' P8 and, for the single-page planner of a wide schema, Q8 over raw + the
    // record-indexed streams' global event bytes (k_plan folds converged streams into one load)
    uint32_t nfold = 0;
    for (const PlanStream &S : hs) nfold += S.rank_col < 0 ? 1 : 0;
    // (few streams: the planner's evaluations are cheap already and the fold's extra pass over
    // the batch costs more, C2 4 streams: +0.8 ms per 100 M records; C3 199 streams: -6 ms per 10 M)
    const bool fold = plan && !mp_ && nfold >= 16 && !fold_off();
    const uint64_t groups = ev_stride / 8;
    ENS(d_P, (groups + 1) * 8);
    if (fold) {
        ENS(d_Q, (groups + 1) * 8);
        ENS(d_qv, ne * 4);
        launch_plan_fold(d_ev.as<uint8_t>(), ev_stride, pstreams, nstreams, d_raw.as<uint32_t>(), ne,
                         d_qv.as<uint32_t>(), s);
    }
    if (!model_probe)   // (a model probe takes its page cuts from the host: no planner prefixes)
        launch_plan_prefix(plan ? d_ev.as<uint8_t>() : nullptr, plan ? d_E.as<uint32_t>() : nullptr, plan ? nstreams : 0,
                           ev_stride, d_raw.as<uint32_t>(), fold ? d_qv.as<uint32_t>() : nullptr, ne, d_P.as<uint64_t>(),
                           fold ? d_Q.as<uint64_t>() : nullptr, &seg_, s);
    if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "scan scratch allocation failed");
    if (mp_) return encode_mp(d_data, d_off, n, ne, final_flush, next_rg_size, hc, nwords, ev_stride, out);
    // ---------------------------------------------------------------- A9 plan
    // plan buffer (int64): [out 4 | pad 4 | (start, end) per row group]: the result and the first
    // kPlanHead row groups come back in one copy
    constexpr int32_t kPlanHead = 64;
    const int32_t max_rgs = (int32_t)(ne / 100 + 4);
    ENS(d_plan, (8 + 2 * (size_t)max_rgs) * 8);
    PlanArgs pa{};
    pa.n = ne; pa.final_flush = final_flush ? 1 : 0; pa.ncols = nc; pa.next_rg_size = next_rg_size;
    pa.P8 = d_P.as<uint64_t>(); pa.raw = d_raw.as<uint32_t>(); pa.cols = d_cols.as<DevCol>();
    pa.Q8 = fold ? d_Q.as<uint64_t>() : nullptr; pa.qv = fold ? d_qv.as<uint32_t>() : nullptr;
    pa.jobs = pjobs; pa.lr_a = sc.lr_a; pa.lr_b = sc.lr_b; pa.lr_off = sc.lr_off; pa.lr_rle = sc.lr_rle;
    pa.streams = pstreams; pa.nstreams = (int32_t)nstreams;
    pa.nbool = v2_ ? 0 : (int32_t)nbool; pa.bool_cols = d_bool.as<uint32_t>();
    pa.E8 = nstreams ? d_E.as<uint32_t>() : nullptr; pa.ev = nstreams ? d_ev.as<uint8_t>() : nullptr; pa.ev_stride = ev_stride;
    pa.gend = nstreams ? d_gend.as<uint64_t>() : nullptr; pa.gend_stride = nwords;
    pa.rg = d_plan.as<int64_t>() + 8; pa.max_rgs = max_rgs;
    pa.err = d_err;
    pa.max_cuts = max_cuts;
    pa.out = d_plan.as<int64_t>();
    launch_plan(pa, s);
    CK(hipGetLastError());
    const int32_t head = std::min<int32_t>(max_rgs, kPlanHead);
    std::vector<int64_t> pl(8 + 2 * (size_t)head);
    CK(xd2h(pl.data(), d_plan.p, pl.size() * 8, s));
    CK(xsync(s));
    CK(hipEventRecord(ev_[2], s));
    const int64_t *po = pl.data();
    if (optimistic && ne == n && (uint64_t)po[4] < n) {   // K1 found an invalid record: plan its prefix
        err_idx = ne = (uint64_t)po[4];
        goto replan;
    }
    const int nrg = (int)po[0];
#ifdef KPW_PLAN_PROF
    fprintf(stderr, "[plan_prof] rgs %d total %.3f ms walk %.3f ms (%lld) conv (%lld) points %lld\n", nrg, po[5] / 1e5,
            po[6] / 1e5, (long long)(po[7] & 0x1fffff), (long long)((po[7] >> 21) & 0x1fffff), (long long)(po[7] >> 42));
#endif
    if (po[3]) return fail(KPW_ERR_DEVICE, "planner row-group table overflow");
    if (nrg > head) {   // more row groups than the first copy held
        pl.resize(8 + 2 * (size_t)nrg);
        CK(xd2h(pl.data() + 8 + 2 * head, d_plan.as<int64_t>() + 8 + 2 * head, 2 * (size_t)(nrg - head) * 8, s));
        CK(xsync(s));
        po = pl.data();
    }
    std::vector<int64_t> rs(nrg), re(nrg);
    for (int r = 0; r < nrg; r++) { rs[r] = pl[8 + 2 * r]; re[r] = pl[8 + 2 * r + 1]; }
    out.records_consumed = po[1];
    out.open_records = (int64_t)ne - po[1];
    out.open_buffered = po[2];
    for (int r = 0; r < nrg; r++) out.rgs.push_back(RowGroupOut{rs[r], re[r] - rs[r], r * nc});
    if (on_plan) on_plan(out);
    if (nrg == 0 || plan_only) {   // plan_only: cuts + open buffered size, no pages (out.rgs carry no chunks)
        for (int i = 3; i < 8; i++) CK(hipEventRecord(ev_[i], s));
        CK(xsync(s));
        return KPW_OK;
    }

    // ---------------------------------------------------------------- chunk descriptors
    const int nch = nrg * nc;
    std::vector<ChunkDesc> ch(nch);
    std::vector<uint32_t> cfirst(nch), ccount(nch);
    std::vector<uint8_t> cdict(nch);
    uint32_t nct = 0;
    std::vector<RleJob> ej;
    std::vector<DeltaJob> dj;          // v2 DELTA streams (INT32/INT64: 1, BYTE_ARRAY: prefix + suffix lengths)
    std::vector<uint32_t> dblk_job;    // job of each DELTA block tile
    std::vector<int> bool_pos(nc, -1);
    for (uint32_t i = 0; i < nbool; i++) bool_pos[bool_idx_[i]] = (int)i;
    uint64_t ht_off = 0, ids_off = 0;
    for (int r = 0; r < nrg; r++) {
        for (int c = 0; c < nc; c++) {
            const int ci = r * nc + c;
            ChunkDesc &C = ch[ci];
            memset(&C, 0, sizeof(C));
            C.s = rs[r]; C.e = re[r]; C.col = c; C.rg = r;
            C.is_dict = cols[c].dict ? 1 : 0;
            C.smin = ~0ull; C.smax = 0;
            const uint64_t len = (uint64_t)(C.e - C.s);
            C.ids_off = ids_off;
            C.ent_off = ids_off;
            ids_off += len;
            C.dl_job = C.id_job = -1;
            if (cols[c].optional) {
                RleJob J;
                memset(&J, 0, sizeof(J));
                J.src.kind = 0; J.src.ptr = hc[c].pres; J.src.base = (uint64_t)C.s;
                J.len = (uint32_t)len; J.bw = 1;
                C.dl_job = (int32_t)ej.size();
                ej.push_back(J);
            }
            if (C.is_dict) {
                RleJob J;
                memset(&J, 0, sizeof(J));
                J.src.kind = 1; J.src.ptr = nullptr; J.src.base = C.ids_off;   // ptr patched below
                J.len = (uint32_t)len; J.bw = 0;
                C.id_job = (int32_t)ej.size();
                ej.push_back(J);
            }
            C.bool_job = -1;
            C.dj0 = -1;
            if (v2_ && cols[c].phys == KPW_BOOLEAN) {   // RunLengthBitPackingHybridValuesWriter(1)
                RleJob J;
                memset(&J, 0, sizeof(J));
                J.src.kind = 0; J.src.ptr = cbits_[bool_pos[c]];
                J.src.base = cols[c].optional ? 0 : (uint64_t)C.s;   // optional: rank of C.s, set on the device
                J.len = (uint32_t)len; J.bw = 1;
                C.bool_job = (int32_t)ej.size();
                ej.push_back(J);
            }
            if (v2_ && C.is_dict && (cols[c].phys == KPW_INT32 || cols[c].phys == KPW_INT64 || cols[c].phys == KPW_BYTE_ARRAY)) {
                C.dj0 = (int32_t)dj.size();
                const bool ba = cols[c].phys == KPW_BYTE_ARRAY;
                const uint32_t nblk = (uint32_t)std::max<uint64_t>(1, len > 1 ? (len - 1 + 127) / 128 : 1);
                for (int k = 0; k < (ba ? 2 : 1); k++) {
                    DeltaJob D;
                    memset(&D, 0, sizeof(D));
                    D.vals = nullptr;   // patched below: dense values (u64) or prefix/suffix lengths (u32)
                    D.base = C.ids_off;
                    D.flags = DJ_INACTIVE | (cols[c].phys == KPW_INT64 ? DJ_LONG : 0u) | (ba ? DJ_U32_SRC : 0u);
                    D.blk0 = (uint32_t)dblk_job.size();
                    D.nblk = nblk;
                    D.prev = -1;   // one page per chunk: a fresh fallback writer
                    dblk_job.insert(dblk_job.end(), nblk, (uint32_t)dj.size());
                    dj.push_back(D);
                }
            }
            const uint32_t nt = (uint32_t)std::max<uint64_t>(1, (len + KPW_TILE_P_H - 1) / KPW_TILE_P_H);
            cfirst[ci] = nct;
            ccount[ci] = nt;
            cdict[ci] = C.is_dict;
            nct += nt;
        }
    }
    // Dictionary hash tables.  Full size: >= 2x the most entries the dictionary can hold before
    // its fallback (dictionaryByteSize > dictPageSize: entries of >= 4 / 8 bytes), so probe
    // chains stay short until the fallback; a table that fills anyway means more entries than
    // that, i.e. a fallback (overflow).  Hinted: 4x the entries the column's chunks reached in
    // the previous encode (dict_hint_), with a probe limit; a hinted table that hits the limit
    // flags a retry and the chunk phase is redone at full size, so the hint never changes bytes.
    // Low-cardinality columns (C3: 199 of 200) then fill and touch kilobytes instead of MiBs.
    auto assign_tables = [&](bool hinted) {
        ht_off = 0;
        for (int ci = 0; ci < nch; ci++) {
            ChunkDesc &C = ch[ci];
            if (!C.is_dict) continue;
            const int c = C.col;
            const uint64_t len = (uint64_t)(C.e - C.s);
            const uint64_t esz = (cols[c].phys == KPW_INT64 || cols[c].phys == KPW_DOUBLE) ? 8 : 4;
            const uint64_t maxent = (uint64_t)props.dictionary_page_size / esz + 1;
            uint64_t cap = std::min<uint64_t>(next_pow2(std::max<uint64_t>(16, 2 * std::min<uint64_t>(len, maxent))), 1u << 20);
            C.ht_plim = 0;
            if (hinted && dict_hint_[c]) {
                const uint64_t hc = next_pow2(std::max<uint64_t>(256, 4ull * dict_hint_[c]));
                if (hc < cap) { cap = hc; C.ht_plim = 64; }
            }
            C.ht_cap = (uint32_t)cap;
            C.ht_off = ht_off;
            ht_off += cap + 1;
        }
    };
    if (dict_hint_.size() != (size_t)nc) dict_hint_.assign(nc, 0);
    static const bool hints_off = [] { const char *e = getenv("KPW_DICT_HINTS"); return e && e[0] == '0'; }();
    assign_tables(!hints_off);
    // Dictionary insertion order: tile k of every dictionary chunk before tile k+1 of any, so
    // each chunk is scanned roughly in record order and a chunk that crosses the 1 MiB
    // fallback threshold stops after a few tiles instead of inserting all of its values.
    // (expanded on the device, k_dict_order, from the dictionary chunks and per-round offsets)
    static thread_local std::vector<uint32_t> dlist, droff;
    uint32_t ndict_tiles = 0;
    dict_order(ccount, cdict, ndict_tiles, dlist, droff);
    // chunk descriptors, then 4 words of string-statistics metadata per chunk (one readback)
    static_assert(sizeof(ChunkDesc) % 8 == 0, "metadata words follow the descriptors");
    ENS(d_tile_raw, nct * 8); ENS(d_tile_raw_off, nct * 8); ENS(d_tile_smin, nct * 8); ENS(d_tile_smax, nct * 8);
    ENS(d_tile_cnt, nct * 4); ENS(d_tile_sz, nct * 8); ENS(d_fmask, (uint64_t)nct * KPW_BLOCK_H);
    ENS(d_ht, std::max<uint64_t>(1, ht_off) * sizeof(HtSlot));
    ENS(d_ids, std::max<uint64_t>(1, ids_off) * 4); ENS(d_ent_rec, std::max<uint64_t>(1, ids_off) * 8);
    ENS(d_ent_boff, std::max<uint64_t>(1, ids_off) * 8);
    // page table (u64 words): [body / compressed totals 2 | collision flags 1 | pad 1 | page offsets,
    // lengths, level prefixes, compressed offsets, compressed lengths: 2 per chunk each], so the
    // layout's results come back in one copy and K7's in another
    const size_t P2 = 2 * (size_t)nch;
    ENS(d_ptab, (4 + 5 * P2) * 8);
    uint64_t *const pt = d_ptab.as<uint64_t>();
    uint64_t *const d_poff = pt + 4, *const d_plen = d_poff + P2, *const d_ppre = d_plen + P2;
    uint64_t *const d_pcoff = d_ppre + P2, *const d_pclen = d_pcoff + P2;
    uint32_t *const d_coll = (uint32_t *)(pt + 2);
    for (auto &J : ej) if (J.src.kind == 1) J.src.ptr = d_ids.p;
    // one upload: descriptors, first tile and tile count per chunk, the dictionary chunks and
    // their per-round tile offsets; the chunk tile -> chunk map and the dictionary insertion order
    // are expanded from them on the device, the descriptors' statistics metadata zeroed there
    const size_t desc_bytes = (size_t)nch * sizeof(ChunkDesc);
    std::vector<uint8_t *> ctp;
    if (int st = upload_parts(d_chunks, {{cfirst.data(), (size_t)nch * 4}, {ccount.data(), (size_t)nch * 4},
                                         {dlist.data(), dlist.size() * 4}, {droff.data(), droff.size() * 4},
                                         {ch.data(), desc_bytes}}, ctp, (size_t)nch * 32))
        return st;
    ChunkDesc *const d_ch = (ChunkDesc *)ctp[4];   // descriptors, then their metadata words
    CK(hipMemsetAsync(ctp[4] + desc_bytes, 0, (size_t)nch * 32, s));
    ENS(d_ctj, std::max<uint64_t>(1, nct) * 4); ENS(d_dorder, std::max<uint64_t>(1, ndict_tiles) * 4);
    {
        TileMapArgs ta{};
        ta.nm = 1;
        ta.m[0] = TileMapSpec{(const uint32_t *)ctp[0], (const uint32_t *)ctp[1], 1u, (uint32_t)nch, d_ctj.as<uint32_t>()};
        launch_tile_maps(ta, s);
        launch_dict_order((const uint32_t *)ctp[2], (uint32_t)dlist.size(), (const uint32_t *)ctp[0], (const uint32_t *)ctp[1],
                          (const uint32_t *)ctp[3], (uint32_t)droff.size() - 1, d_dorder.as<uint32_t>(), s);
        CK(hipGetLastError());
    }
    ChunkArgs a{};
    a.ch = d_ch; a.nchunks = nch; a.nctiles = nct; a.cols = d_cols.as<DevCol>(); a.data = d_data;
    a.ctile_chunk = d_ctj.as<uint32_t>(); a.ctile_first = (uint32_t *)ctp[0];
    a.ctile_count = (uint32_t *)ctp[1]; a.tile_raw = d_tile_raw.as<uint64_t>();
    a.tile_raw_off = d_tile_raw_off.as<uint64_t>(); a.tile_smin = d_tile_smin.as<uint64_t>();
    a.tile_smax = d_tile_smax.as<uint64_t>(); a.tile_cnt = d_tile_cnt.as<uint32_t>(); a.tile_sz = d_tile_sz.as<uint64_t>();
    a.ht = d_ht.as<HtSlot>();
    a.ids = d_ids.as<uint32_t>(); a.ent_rec = d_ent_rec.as<uint64_t>(); a.ent_boff = d_ent_boff.as<uint64_t>();
    a.fmask = d_fmask.as<uint8_t>();
    a.max_dict_bytes = (uint32_t)props.dictionary_page_size;
    a.data_end = d_off + n;
    a.collision = d_coll;
    a.dict_order = d_dorder.as<uint32_t>(); a.ndict_tiles = ndict_tiles;
    a.v2 = v2_ ? 1 : 0;
    a.seg = &seg_;
    // v2 DELTA streams: dense inputs share the chunks' rank-indexed id space (ids_off)
    DeltaArgs dla{};
    a.page_pre = d_ppre;
    if (v2_) {
        ENS(d_dense, std::max<uint64_t>(1, ids_off) * 8); ENS(d_pre, std::max<uint64_t>(1, ids_off) * 4);
        ENS(d_sfx, std::max<uint64_t>(1, ids_off) * 4);
        ENS(d_tile_sfx, nct * 8); ENS(d_tile_sfx_off, nct * 8); ENS(d_chunk_sfx, nch * 8);
        CK(hipMemsetAsync(d_chunk_sfx.p, 0, nch * 8, s));
        for (int ci = 0; ci < nch; ci++) {
            const ChunkDesc &C = ch[ci];
            if (C.dj0 < 0) continue;
            if (cols[C.col].phys == KPW_BYTE_ARRAY) { dj[C.dj0].vals = d_pre.p; dj[C.dj0 + 1].vals = d_sfx.p; }
            else dj[C.dj0].vals = d_dense.p;
        }
        const size_t nb = std::max<size_t>(1, dblk_job.size());
        ENS(d_djobs, std::max<size_t>(1, dj.size()) * sizeof(DeltaJob)); ENS(d_blk_job, nb * 4); ENS(d_blk_min, nb * 8);
        ENS(d_blk_w, nb * 4); ENS(d_blk_sz, nb * 8); ENS(d_blk_off, nb * 8); ENS(d_btot, std::max<size_t>(1, dj.size()) * 8);
        if (!dblk_job.empty()) CK(xh2d(d_blk_job.p, dblk_job.data(), dblk_job.size() * 4, s));
        dla.jobs = d_djobs.as<DeltaJob>(); dla.njobs = (uint32_t)dj.size(); dla.nblk = (uint32_t)dblk_job.size();
        dla.blk_job = d_blk_job.as<uint32_t>(); dla.blk_min = d_blk_min.as<uint64_t>(); dla.blk_w = d_blk_w.as<uint32_t>();
        dla.blk_sz = d_blk_sz.as<uint64_t>(); dla.blk_off = d_blk_off.as<uint64_t>(); dla.btot = d_btot.as<uint64_t>();
        dla.seg = &seg_;
        a.djobs = dla.jobs; a.djobs_w = dla.jobs; a.chunk_sfx = d_chunk_sfx.as<uint64_t>();
    }
    uint32_t enpt = 0, enet = 0;
    RleScratch esc{};
    std::vector<uint64_t> ptab;   // host copy of the page table
    uint64_t body_tot = 0;
    // BYTE_ARRAY dictionaries are keyed by a 64-bit hash and verified byte-for-byte; a
    // verified collision re-runs the chunk phase with byte comparisons (exact_strings).
    // A hint-sized table that overflowed (flag word 1) re-runs the phase at full size.
    for (bool exact = false, first = true;; first = false) {
        a.exact_strings = exact ? 1 : 0;
        if (!first) CK(xh2d(d_ch, ch.data(), nch * sizeof(ChunkDesc), s));   // a re-run starts from the host's
        if (v2_ && !dj.empty()) CK(xh2d(d_djobs.p, dj.data(), dj.size() * sizeof(DeltaJob), s));
        // ------------------------------------------------------------ K6 + K2
        a.ht_clear = d_ht.as<HtSlot>(); a.ht_clear_n = ht_off;   // K6 empties the hash tables and the flags
        a.flags_clear = (uint64_t *)d_coll;
        launch_chunk_stats(a, s);
        CK(hipGetLastError());
        if (!ej.empty()) {
            int st = run_rle(ej, enpt, enet, esc);
            if (st) return st;
            if (v2_) launch_v2_bool_jobs(a, d_jobs.as<RleJob>(), s);
        }
        launch_dict(a, d_jobs.as<RleJob>(), s);
        CK(hipGetLastError());
        CK(hipEventRecord(ev_[3], s));
        // ------------------------------------------------------------ K3 (dl + ids + v2 booleans)
        if (!ej.empty()) launch_rle_structure(d_jobs.as<RleJob>(), (int)ej.size(), enpt, enet, esc, s);
        CK(hipGetLastError());
        // ------------------------------------------------------------ A10 (v2 fallback: DELTA streams)
        if (v2_) {
            launch_v2_decide(a, d_jobs.as<RleJob>(), dla.jobs, s);
            launch_v2_dense(a, d_dense.as<uint64_t>(), d_pre.as<uint32_t>(), d_sfx.as<uint32_t>(), d_tile_sfx.as<uint64_t>(),
                            d_tile_sfx_off.as<uint64_t>(), d_chunk_sfx.as<uint64_t>(), s);
            launch_delta_structure(dla, s);
            CK(hipGetLastError());
        }
        CK(hipEventRecord(ev_[4], s));
        // ------------------------------------------------------------ layout
        launch_layout(a, d_jobs.as<RleJob>(), d_poff, d_plen, pt, s);
        ptab.resize(4 + 5 * P2);
        CK(xd2h(ptab.data(), pt, (4 + (v2_ ? 3 : 2) * P2) * 8, s));   // totals, flags, offsets, lengths (v2: prefixes)
        CK(xsync(s));
        body_tot = ptab[0];
        uint32_t flags[2];
        memcpy(flags, &ptab[2], 8);
        if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "segmented scan scratch allocation failed");
        if (flags[1]) {
            assign_tables(false);
            ENS(d_ht, std::max<uint64_t>(1, ht_off) * sizeof(HtSlot));
            a.ht = d_ht.as<HtSlot>();
            continue;
        }
        if (!flags[0]) break;
        if (exact) return fail(KPW_ERR_DEVICE, "string dictionary verification failed in exact mode");
        exact = true;
    }
    // +512: K7 reads its input through 256-byte register windows that may run past the last page
    ENS(d_body, body_tot + 512 + 4096);   // + 4 KiB: the writer D2Hs whole 4 KiB units
    // only the tail K7's windows may read and the PLAIN boolean values are cleared (k_chunk_prep,
    // launch_chunk_write); every other body byte is written by its kernel (KPW_BODY_POISON=1 fills
    // the body with 0xAB first: the GPU parity suite checks that)
    if (body_poison()) CK(hipMemsetAsync(d_body.p, 0xAB, body_tot, s));
    a.body_tail = body_tot;
    launch_chunk_write(a, d_jobs.as<RleJob>(), d_body.as<uint8_t>(), s);
    if (!ej.empty()) launch_rle_write(d_jobs.as<RleJob>(), enpt, enet, esc, d_body.as<uint8_t>(), s);
    if (v2_) {
        launch_delta_write(dla, d_body.as<uint8_t>(), s);
        launch_dba_suffixes(a, d_pre.as<uint32_t>(), dla.jobs, d_tile_sfx_off.as<uint64_t>(), d_body.as<uint8_t>(), s);
    }
    CK(hipGetLastError());
    CK(hipEventRecord(ev_[5], s));
    // (no sync here: the page offsets and lengths came back with the layout)
    std::vector<uint64_t> poff(ptab.begin() + 4, ptab.begin() + 4 + P2), plen(ptab.begin() + 4 + P2, ptab.begin() + 4 + 2 * P2);
    std::vector<uint64_t> ppre(P2, 0), pcoff, pclen;
    if (v2_) ppre.assign(ptab.begin() + 4 + 2 * P2, ptab.begin() + 4 + 3 * P2);
    // ---------------------------------------------------------------- K7
    if (props.codec == KPW_SNAPPY) {
        std::vector<uint32_t> fpage, fidx, pfrag0(2 * nch);
        for (int p = 0; p < 2 * nch; p++) {
            pfrag0[p] = (uint32_t)fpage.size();
            const uint64_t nf = (plen[p] + SNAPPY_FRAG - 1) / SNAPPY_FRAG;
            for (uint64_t k = 0; k < nf; k++) { fpage.push_back((uint32_t)p); fidx.push_back((uint32_t)k); }
        }
        const uint32_t nf = (uint32_t)fpage.size();
        ENS(d_frag_out, (uint64_t)std::max<uint32_t>(1, nf) * SNAPPY_FRAG_CAP); ENS(d_frag_len, std::max<uint32_t>(1, nf) * 4);
        ENS(d_frag_coff, std::max<uint32_t>(1, nf) * 8);
        ENS(d_comp, body_tot + (uint64_t)nf * 64 + 2 * nch * 8 + 64 + 4096);
        SnappyArgs sa{};
        sa.in = d_body.as<uint8_t>(); sa.page_off = d_poff; sa.page_len = d_plen;
        sa.npages = 2 * nch; sa.nfrags = nf;
        sa.frag_out = d_frag_out.as<uint8_t>(); sa.frag_len = d_frag_len.as<uint32_t>();
        sa.page_coff = d_pcoff; sa.page_clen = d_pclen;
        sa.frag_coff = d_frag_coff.as<uint64_t>(); sa.out = d_comp.as<uint8_t>(); sa.tot = pt + 1;
        sa.page_pre = v2_ ? d_ppre : nullptr;
        // Longest-first dispatch.  K7's waves are latency-bound and a fragment's time depends on
        // its data (one PLAIN int64 fragment of slowly-growing timestamps: ~9 ms; an
        // incompressible one: ~50 us), so the kernel's tail is set by the long fragments
        // dispatched last.  Every fragment records its [start, end] clock; the longest duration
        // seen per (column, page kind, fragment index in the page) in the previous batch ranks
        // this batch's fragments, longest first (per (column, page kind) when the index is new).
        // Output is unchanged (fragments are independent; slots are indexed by fragment).
        const size_t nkind = 2 * cols.size();
        if (sn_cost_.size() != nkind) sn_cost_.assign(nkind, 0.0);
        auto kind_of = [&](uint32_t p) { return ((p / 2) % cols.size()) * 2 + (p & 1); };
        auto fkey = [&](uint32_t f) { return ((uint64_t)kind_of(fpage[f]) << 32) | fidx[f]; };
        auto cost_of = [&](uint32_t f) {
            auto it = sn_fcost_.find(fkey(f));
            return it != sn_fcost_.end() ? it->second : sn_cost_[kind_of(fpage[f])];
        };
        bool have_cost = false;
        for (double c : sn_cost_) have_cost |= c > 0;
        sn_order_.clear();
        if (nf) {
            ENS(d_sprof, (uint64_t)nf * 16);
            sa.ftime = d_sprof.as<uint64_t>();
            if (have_cost) {
                sn_order_.resize(nf);
                std::vector<std::pair<double, uint32_t>> ranked(nf);
                for (uint32_t f = 0; f < nf; f++) ranked[f] = {-cost_of(f), f};
                std::sort(ranked.begin(), ranked.end());
                for (uint32_t f = 0; f < nf; f++) sn_order_[f] = ranked[f].second;
            }
        }
        // fragment -> page, index in page, first fragment per page, dispatch order: one copy
        std::vector<uint8_t *> kt;
        if (int st = upload_parts(d_ktab, {{fpage.data(), (size_t)nf * 4}, {fidx.data(), (size_t)nf * 4},
                                           {pfrag0.data(), (size_t)2 * nch * 4}, {sn_order_.data(), sn_order_.size() * 4}}, kt))
            return st;
        sa.frag_page = (uint32_t *)kt[0]; sa.frag_idx = (uint32_t *)kt[1];
        const uint32_t *page_frag0 = (const uint32_t *)kt[2];
        if (!sn_order_.empty()) sa.order = (uint32_t *)kt[3];
        if (seg_args(sa)) return KPW_ERR_NOMEM;
        // K7 window (stage_ms[9]): every kernel from the first fragment kernel to the compressed
        // pages in place (k_snappy_v, k_snappy_s_rest, k_snappy_seg, k_snappy_v, k_snappy_s_rest,
        // k_snappy_page_sizes, k_snappy_copy; one 4-byte fill of the fragment counter)
        CK(hipEventRecord(kev_[2], s));
        launch_snappy(sa, s);
        launch_snappy_finish(sa, page_frag0, s);
        CK(hipEventRecord(kev_[3], s));
        if (nf) {
            sn_ft_.resize(2 * (size_t)nf);
            CK(xd2h(sn_ft_.data(), d_sprof.p, sn_ft_.size() * 8, s));
        }
        CK(hipGetLastError());
        CK(xd2h(ptab.data(), pt, (4 + 5 * P2) * 8, s));   // compressed total, offsets, lengths
        CK(xsync(s));
        const uint64_t ctot = ptab[1];
        pcoff.assign(ptab.begin() + 4 + 3 * P2, ptab.begin() + 4 + 4 * P2);
        pclen.assign(ptab.begin() + 4 + 4 * P2, ptab.begin() + 4 + 5 * P2);
        if (nf) {
            // per-kind mean duration (fragments handed to k_snappy_s_rest count their short
            // k_snappy_v attempt); KPW_SNAPPY_PROFILE=<file> also dumps the raw records
            std::vector<double> mx(nkind, 0.0);
            sn_fcost_.clear();
            for (uint32_t f = 0; f < nf; f++) {
                const uint64_t e = sn_ft_[2 * f + 1] & ~(1ull << 63);
                const double d = std::max(1.0, (double)(e - sn_ft_[2 * f]));
                const size_t k = kind_of(fpage[f]);
                mx[k] = std::max(mx[k], d);
                double &c = sn_fcost_[fkey(f)];
                c = std::max(c, d);
            }
            for (size_t k = 0; k < nkind; k++)
                if (mx[k] > 0) sn_cost_[k] = mx[k];
            static const char *sprof = getenv("KPW_SNAPPY_PROFILE");
            if (sprof) {
                if (FILE *fp = fopen(sprof, "wb")) {
                    // per fragment: page, index in page, page length, column, start, end (bit 63: handed on)
                    for (uint32_t f = 0; f < nf; f++) {
                        const uint64_t rec[6] = {fpage[f], fidx[f], plen[fpage[f]], (uint64_t)((fpage[f] / 2) % cols.size()),
                                                 sn_ft_[2 * f], sn_ft_[2 * f + 1]};
                        fwrite(rec, 8, 6, fp);
                    }
                    fclose(fp);
                }
            }
        }
        pages_dev_ = d_comp.as<uint8_t>();
        pages_len_ = ctot;
    } else if (props.codec == KPW_GZIP) {
        uint64_t cap = 4096;
        for (int p = 0; p < 2 * nch; p++) cap += ppre[p] + dfl_member_bound(plen[p]);
        ENS(d_comp, cap);
        CK(hipEventRecord(kev_[2], s));
        if (int st = gzip_pages(d_body.as<uint8_t>(), body_tot, d_poff, v2_ ? d_ppre : nullptr, poff, plen,
                                std::vector<char>(2 * nch, 1), d_pcoff, d_pclen, pt + 1, pt + 3, s))
            return st;
        CK(hipEventRecord(kev_[3], s));
        CK(xd2h(ptab.data(), pt, (4 + 5 * P2) * 8, s));   // compressed total, overflow, offsets, lengths
        CK(xsync(s));
        if (ptab[3]) return fail(KPW_ERR_DEVICE, "gzip member overflowed its scratch slot");
        pcoff.assign(ptab.begin() + 4 + 3 * P2, ptab.begin() + 4 + 4 * P2);
        pclen.assign(ptab.begin() + 4 + 4 * P2, ptab.begin() + 4 + 5 * P2);
        pages_dev_ = d_comp.as<uint8_t>();
        pages_len_ = ptab[1];
    } else {   // uncompressed: a (v2) page body starts at its level prefix
        pcoff.resize(2 * nch);
        pclen.resize(2 * nch);
        for (int p = 0; p < 2 * nch; p++) { pcoff[p] = poff[p] - ppre[p]; pclen[p] = plen[p] + ppre[p]; }
        pages_dev_ = d_body.as<uint8_t>();
        pages_len_ = body_tot;
    }
    CK(hipEventRecord(ev_[6], s));
    if (seg_failed_reset()) return fail(KPW_ERR_NOMEM, "segmented scan scratch allocation failed");
    // ---------------------------------------------------------------- metadata
    // binary min/max bytes: gather (offset, len) pairs, then the bytes into one blob
    std::vector<uint64_t> smeta(4 * nch, 0);
    uint64_t *const d_smeta = (uint64_t *)(d_ch + nch);
    launch_stats_gather(d_ch, nch, d_cols.as<DevCol>(), d_data, d_smeta, nullptr, s);
    {   // descriptors + metadata in one copy
        static thread_local std::vector<uint8_t> md;
        md.resize(nch * (sizeof(ChunkDesc) + 32));
        CK(xd2h(md.data(), d_ch, md.size(), s));
        CK(xsync(s));
        memcpy(ch.data(), md.data(), nch * sizeof(ChunkDesc));
        for (auto &C : ch) chunk_stats_derive(C);
        memcpy(smeta.data(), md.data() + nch * sizeof(ChunkDesc), nch * 32);
    }
    {   // next encode's table hints: the most entries of each column's chunks, none after a fallback
        std::vector<uint32_t> most(nc, 0);
        std::vector<char> seen(nc, 0), fell(nc, 0);
        for (int ci = 0; ci < nch; ci++) {
            const ChunkDesc &C = ch[ci];
            if (!cols[C.col].dict) continue;
            seen[C.col] = 1;
            if (!C.is_dict || C.fallback || C.overflow) fell[C.col] = 1;
            else most[C.col] = std::max(most[C.col], C.dict_n);
        }
        for (int c = 0; c < nc; c++)
            if (seen[c]) dict_hint_[c] = fell[c] ? 0 : std::max<uint32_t>(1, most[c]);
    }
    std::vector<std::string> bmin(nch), bmax(nch);
    {
        uint64_t blob_len = 0;
        std::vector<uint64_t> boff(nch);
        for (int ci = 0; ci < nch; ci++) {
            boff[ci] = blob_len;
            if (cols[ch[ci].col].phys == KPW_BYTE_ARRAY && ch[ci].has_minmax) blob_len += smeta[4 * ci + 1] + smeta[4 * ci + 3];
        }
        if (blob_len) {
            std::vector<uint8_t> blob(blob_len);
            ENS(d_sblob, blob_len);
            launch_stats_gather(d_ch, nch, d_cols.as<DevCol>(), d_data, d_smeta,
                                d_sblob.as<uint8_t>(), s);
            CK(xd2h(blob.data(), d_sblob.p, blob_len, s));
            CK(xsync(s));
            for (int ci = 0; ci < nch; ci++) {
                if (cols[ch[ci].col].phys != KPW_BYTE_ARRAY || !ch[ci].has_minmax) continue;
                const uint64_t l1 = smeta[4 * ci + 1], l2 = smeta[4 * ci + 3];
                bmin[ci].assign((const char *)blob.data() + boff[ci], l1);
                bmax[ci].assign((const char *)blob.data() + boff[ci] + l1, l2);
            }
        }
    }
    CK(hipEventRecord(ev_[7], s));
    CK(hipEventSynchronize(ev_[7]));
    for (int i = 0; i < 7; i++) CK(hipEventElapsedTime(&stage_ms[i], ev_[i], ev_[i + 1]));
    CK(hipEventElapsedTime(&stage_ms[7], ev_[0], ev_[7]));
    CK(hipEventElapsedTime(&stage_ms[8], kev_[0], kev_[1]));
    stage_ms[9] = 0;
    if (props.codec == KPW_SNAPPY || props.codec == KPW_GZIP) CK(hipEventElapsedTime(&stage_ms[9], kev_[2], kev_[3]));

    // ---------------------------------------------------------------- results
    for (int ci = 0; ci < nch; ci++) {
        const ChunkDesc &C = ch[ci];
        const ColInfo &col = cols[C.col];
        ChunkOut co;
        co.column = C.col;
        co.first_page = (int32_t)out.pages.size();
        co.num_values = C.e - C.s;
        co.has_dictionary = C.dictpage_len > 0;
        if (C.dictpage_len) {
            PageOut p;
            p.page_type = KPW_DICTIONARY_PAGE;
            p.num_values = (int32_t)C.dict_n;
            p.encoding = v2_ ? KPW_ENC_PLAIN : KPW_ENC_PLAIN_DICTIONARY;   // DictionaryValuesWriter v1 / v2 page encoding
            p.dl_encoding = p.rl_encoding = 0;
            p.has_stats = 0;
            p.uncompressed_size = (int64_t)plen[2 * ci];
            p.compressed_size = (int64_t)pclen[2 * ci];
            p.offset = pcoff[2 * ci];
            p.null_count = 0;
            p.has_min_max = 0;
            out.pages.push_back(p);
        }
        PageOut p;
        p.page_type = v2_ ? KPW_DATA_PAGE_V2 : KPW_DATA_PAGE;
        p.num_values = (int32_t)(C.e - C.s);
        if (!v2_) {
            p.encoding = (C.is_dict && !C.fallback) ? KPW_ENC_PLAIN_DICTIONARY : KPW_ENC_PLAIN;
        } else if (col.phys == KPW_BOOLEAN) {
            p.encoding = KPW_ENC_RLE;
        } else if (C.is_dict && !C.fallback) {
            p.encoding = KPW_ENC_RLE_DICTIONARY;
        } else {   // DefaultV2ValuesWriterFactory fallback writers
            p.encoding = col.phys == KPW_BYTE_ARRAY ? KPW_ENC_DELTA_BYTE_ARRAY
                       : (col.phys == KPW_INT32 || col.phys == KPW_INT64) ? KPW_ENC_DELTA_BINARY_PACKED : KPW_ENC_PLAIN;
        }
        p.dl_encoding = col.optional ? KPW_ENC_RLE : KPW_ENC_BIT_PACKED;
        p.rl_encoding = KPW_ENC_BIT_PACKED;
        p.has_stats = 1;
        p.uncompressed_size = (int64_t)(plen[2 * ci + 1] + ppre[2 * ci + 1]);
        p.compressed_size = (int64_t)pclen[2 * ci + 1];
        p.offset = pcoff[2 * ci + 1];
        p.dl_byte_length = v2_ ? (int32_t)C.dl_len : 0;
        p.rl_byte_length = v2_ ? C.rl0_len : 0;
        p.num_rows = (int32_t)(C.e - C.s);
        p.null_count = (int64_t)C.null_count;
        p.has_min_max = C.has_minmax ? 1 : 0;
        if (C.has_minmax) {
            if (col.phys == KPW_BYTE_ARRAY) {
                p.min = bmin[ci];
                p.max = bmax[ci];
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
                p.min = le(unkey(C.smin));
                p.max = le(unkey(C.smax));
            }
        }
        out.pages.push_back(p);
        co.num_pages = (int32_t)out.pages.size() - co.first_page;
        out.chunks.push_back(co);
        // single-page regime guard: ColumnWriterV1.accountForValueWritten never cut a page iff
        // the column's buffered size stayed <= pageSize up to the row-group flush;
        // ColumnWriteStoreV2.sizeCheck cuts once pageSize - usedMem <= (long)(pageSize * 0.1f)
        // (checked conservatively on the final sizes: no cut can have happened below them).
        if (!v2_) {
            const uint64_t colmem = (col.phys == KPW_BOOLEAN ? (C.nn + 7) / 8 : C.raw_bytes) + C.dl_len;
            if (colmem > (uint64_t)props.page_size)
                return fail(KPW_ERR_UNSUPPORTED, "column '" + col.name + "' would be split into several pages "
                                                 "(pageSize smaller than a column chunk): multi-page chunks are the next round");
        } else {
            const int64_t tol = (int64_t)((float)props.page_size * 0.1f);
            // buffered sizes: a width-0 level encoder emits nothing before toBytes
            const int64_t colmem = (col.optional ? (int64_t)C.dl_len : 0) + (int64_t)(col.phys == KPW_BOOLEAN ? C.val_len - 4 : C.raw_bytes);
            if ((int64_t)props.page_size - colmem <= tol)
                return fail(KPW_ERR_UNSUPPORTED, "column '" + col.name + "' could be split into several v2 pages "
                                                 "(within 10% of pageSize): multi-page chunks are the next round");
        }
    }
    out.d_pages = pages_dev_;
    out.pages_len = pages_len_;
    return KPW_OK;
}

int Engine::copy_pages(uint64_t off, uint64_t len, void *host)
{
    if (!pages_dev_ || off + len > pages_len_) return fail(KPW_ERR_INVALID_ARG, "copy_pages range");
    CK(hipMemcpy(host, pages_dev_ + off, len, hipMemcpyDeviceToHost));
    return KPW_OK;
}

// GZIP (CompressionCodecName.GZIP, ParquetFile.java:45): k_deflate.hip on the listed page slots.
// Per input byte the match finder keeps a chain distance (2 B), two match results (8 B) and a
// symbol slot (4 B); each member is built in its own scratch slot, then the pages are packed.
int Engine::gzip_pages(const uint8_t *body, uint64_t body_len, const uint64_t *d_poff, const uint64_t *d_ppre,
                       const std::vector<uint64_t> &poff, const std::vector<uint64_t> &plen, const std::vector<char> &on,
                       uint64_t *d_pcoff, uint64_t *d_pclen, uint64_t *tot, uint64_t *overflow, hipStream_t s)
{
    const uint32_t nslots = (uint32_t)plen.size();
    std::vector<DflPage> pages;
    std::vector<DflTile> tiles;
    std::vector<DflSeg> segs;
    std::vector<DflBlk> blks;
    std::vector<uint32_t> page_seg0, page_blk0, page_tile0;
    std::vector<int32_t> slot_page(nslots, -1);
    uint64_t gz = 0;
    for (uint32_t p = 0; p < nslots; p++) {
        // a dictionary page slot (even) with no bytes has no page; a data page always has one
        // (an empty v2 values section still gets its 20-byte member)
        if (!on[p] || (!(p & 1) && plen[p] == 0)) continue;
        const uint32_t pg = (uint32_t)pages.size();
        slot_page[p] = (int32_t)pg;
        const uint64_t cap = (dfl_member_bound(plen[p]) + 16 + 255) & ~255ull;   // (the stream starts at slot + 16)
        pages.push_back(DflPage{poff[p], plen[p], gz, cap});
        page_tile0.push_back((uint32_t)tiles.size());
        for (uint64_t t = 0; t * 32768 < plen[p]; t++) tiles.push_back(DflTile{pg, (uint32_t)t});
        page_seg0.push_back((uint32_t)segs.size());
        const uint64_t ns = std::max<uint64_t>(1, (plen[p] + DFL_SEG - 1) / DFL_SEG);
        for (uint64_t k = 0; k < ns; k++) segs.push_back(DflSeg{pg, (uint32_t)k});
        page_blk0.push_back((uint32_t)blks.size());
        const uint64_t nb = (plen[p] + 1) / DFL_BLK + 2;   // blocks of 16383 symbols, at most one per byte (+ the final)
        for (uint64_t j = 0; j < nb; j++) blks.push_back(DflBlk{pg, (uint32_t)j});
        gz += cap;
    }
    page_tile0.push_back((uint32_t)tiles.size());
    page_seg0.push_back((uint32_t)segs.size());
    page_blk0.push_back((uint32_t)blks.size());
    const uint32_t np = (uint32_t)pages.size(), nt = (uint32_t)tiles.size();
    const uint32_t nsegs = (uint32_t)segs.size(), nblks = (uint32_t)blks.size();
    ENS(d_dfl_pdist, std::max<uint64_t>(body_len, 1) * 2 + 64);
    ENS(d_dfl_m128, std::max<uint64_t>(body_len, 1) * 4 + 64);
    ENS(d_dfl_m32, std::max<uint64_t>(body_len, 1) * 4 + 64);
    ENS(d_dfl_sym, std::max<uint64_t>(body_len, 1) * 4 + 64);
    ENS(d_dfl_dsym, (body_len + np + 64) * 4);
    ENS(d_dfl_dpos, (body_len + np + 64) * 4);
    ENS(d_dfl_gz, std::max<uint64_t>(gz, 256));
    ENS(d_dfl_glen, std::max<uint32_t>(np, 1) * 8);
    ENS(d_dfl_seg, std::max<uint64_t>(nsegs, 1) * (2 * sizeof(DflSt) + 12));
    ENS(d_dfl_page, std::max<uint64_t>(np, 1) * 12 + std::max<uint64_t>(nt, 1) * 4 + 64);
    ENS(d_dfl_blk, std::max<uint64_t>(nblks, 1) * 20);
    std::vector<uint8_t *> tp;
    if (int st = upload_parts(d_dfl_tab, {{pages.data(), pages.size() * sizeof(DflPage)}, {tiles.data(), tiles.size() * sizeof(DflTile)},
                                          {slot_page.data(), slot_page.size() * 4}, {segs.data(), segs.size() * sizeof(DflSeg)},
                                          {blks.data(), blks.size() * sizeof(DflBlk)}, {page_seg0.data(), page_seg0.size() * 4},
                                          {page_blk0.data(), page_blk0.size() * 4}, {page_tile0.data(), page_tile0.size() * 4}},
                              tp))
        return st;
    DflArgs a{};
    a.in = body; a.pages = (const DflPage *)tp[0]; a.tiles = (const DflTile *)tp[1];
    a.pdist = d_dfl_pdist.as<uint16_t>(); a.m128 = d_dfl_m128.as<uint32_t>(); a.m32 = d_dfl_m32.as<uint32_t>();
    a.sym = d_dfl_sym.as<uint32_t>(); a.gz = d_dfl_gz.as<uint8_t>(); a.glen = d_dfl_glen.as<uint64_t>();
    a.nslots = nslots; a.slot_page = (const int32_t *)tp[2];
    a.page_off = d_poff; a.page_pre = d_ppre; a.page_coff = d_pcoff; a.page_clen = d_pclen;
    a.out = d_comp.as<uint8_t>(); a.tot = tot; a.overflow = overflow;
    a.segs = (const DflSeg *)tp[3]; a.nsegs = nsegs; a.blks = (const DflBlk *)tp[4]; a.nblks = nblks;
    a.page_seg0 = (const uint32_t *)tp[5]; a.page_blk0 = (const uint32_t *)tp[6]; a.page_tile0 = (const uint32_t *)tp[7];
    {   // per segment: entry and exit states, dirty flag, symbol count and offset
        uint8_t *q = d_dfl_seg.as<uint8_t>();
        a.seg_entry = (DflSt *)q; q += (size_t)nsegs * sizeof(DflSt);
        a.seg_exit = (DflSt *)q; q += (size_t)nsegs * sizeof(DflSt);
        a.seg_dirty = (uint32_t *)q; q += (size_t)nsegs * 4;
        a.seg_cnt = (uint32_t *)q; q += (size_t)nsegs * 4;
        a.seg_sym0 = (uint32_t *)q;
    }
    {   // per page: symbols, blocks, CRC; per tile: CRC; the round flag
        uint32_t *q = d_dfl_page.as<uint32_t>();
        a.page_T = q; q += np; a.page_nblk = q; q += np; a.page_crc = q; q += np;
        a.tile_crc = q; q += nt;
        a.flag = q;
    }
    {   // per block: bits (or stored bytes), offset, kind
        uint8_t *q = d_dfl_blk.as<uint8_t>();
        a.blk_bits = (uint64_t *)q; q += (size_t)nblks * 8;
        a.blk_off = (uint64_t *)q; q += (size_t)nblks * 8;
        a.blk_kind = (uint32_t *)q;
    }
    a.dsym = d_dfl_dsym.as<uint32_t>(); a.dpos = d_dfl_dpos.as<uint32_t>();
    CK(hipMemsetAsync(overflow, 0, 8, s));
    launch_deflate_prep(a, nt, s);
    CK(hipGetLastError());
    // parse rounds until no segment's entry changes (the converged prefix grows by at least one
    // segment per round, so this ends; every dumped page took 2)
    for (uint32_t round = 0;; round++) {
        CK(hipMemsetAsync(a.flag, 0, 4, s));
        launch_deflate_round(a, s);
        CK(hipGetLastError());
        uint32_t changed = 0;
        CK(xd2h(&changed, a.flag, 4, s));
        CK(xsync(s));
        if (!changed) break;
        if (round > nsegs + 1) return fail(KPW_ERR_DEVICE, "gzip parse did not converge");
    }
    launch_deflate_finish(a, np, s);
    CK(hipMemsetAsync(d_dfl_gz.p, 0, std::max<uint64_t>(gz, 256), s));   // the emit pass ors bits into zeroed words
    launch_deflate_emit(a, np, s);
    CK(hipGetLastError());
    return KPW_OK;
}

// k_snappy_seg needs one scratch block per workgroup and runs one workgroup per CU
int Engine::seg_args(SnappyArgs &sa)
{
    static const bool off = [] { const char *e = getenv("KPW_SNAPPY_SEG"); return e && e[0] == '0'; }();
    if (off || !sa.nfrags) return 0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    ENS(d_seg_scratch, snappy_seg_scratch_bytes((uint32_t)cus));
    void *const old_counter = d_seg_counter.p;
    ENS(d_seg_counter, 64);
    if (d_seg_counter.p != old_counter && hipMemsetAsync(d_seg_counter.p, 0, 64, stream) != hipSuccess)   // once
        return fail(KPW_ERR_DEVICE, "fragment counter clear failed");
    sa.seg_scratch = d_seg_scratch.as<uint8_t>();
    sa.seg_counter = d_seg_counter.as<uint32_t>();
    {   // KPW_SEG_RESERVE_CUS: CUs kept out of the persistent segment kernel's grid (its workgroup
        // holds a CU's whole VGPR file, so nothing else runs beside it: the other encode worker's
        // kernels wait for it unless CUs are left over)
        static const int reserve = [] { const char *e = getenv("KPW_SEG_RESERVE_CUS"); return e ? atoi(e) : 0; }();
        sa.seg_grid = (uint32_t)std::max(1, cus - std::max(0, reserve));
    }
    return 0;
}

}  // namespace kpw
