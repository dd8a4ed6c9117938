// engine.h — host orchestration of one encoder handle (one device, one stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <functional>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kpw_types.h"
#include "kpw_kernels.h"

namespace kpw {

// KPW_BODY_POISON=1: fill each job's page-body buffer with 0xAB before the writers run (test
// infrastructure: shows that no output byte depends on the buffer's previous contents)
inline bool body_poison()
{
    static const bool on = [] { const char *e = getenv("KPW_BODY_POISON"); return e && e[0] == '1'; }();
    return on;
}
// KPW_PLAN_FOLD=0: the planner evaluates every stream per check point instead of the folded
// prefix Q (A/B and parity of the two evaluations)
inline bool fold_off()
{
    static const bool off = [] { const char *e = getenv("KPW_PLAN_FOLD"); return e && e[0] == '0'; }();
    return off;
}
struct SnappyArgs;

struct ColInfo {
    std::string name;
    int32_t field_number, proto_type, label;
    int32_t phys, wire_type, optional, utf8, vsize, dict;
};

struct PageOut {
    int32_t page_type, num_values, encoding, dl_encoding, rl_encoding, has_stats;
    int64_t uncompressed_size, compressed_size;
    uint64_t offset;            // into the device page buffer
    int64_t null_count;
    int32_t has_min_max;
    int32_t dl_byte_length = 0; // DataPageV2: uncompressed definition-level bytes after the repetition levels
    int32_t rl_byte_length = 0; // DataPageV2: uncompressed repetition-level bytes at the body start
    int32_t num_rows = 0;       // DataPageV2
    std::string min, max;       // Statistics.getMinBytes / getMaxBytes
};

struct ChunkOut {
    int32_t column;
    int32_t first_page, num_pages, has_dictionary;
    int64_t num_values;
};

struct RowGroupOut {
    int64_t first_record, num_records;
    int32_t first_chunk;
};

struct BatchOut {
    std::vector<RowGroupOut> rgs;
    std::vector<ChunkOut> chunks;
    std::vector<PageOut> pages;
    const uint8_t *d_pages = nullptr;   // device
    uint64_t pages_len = 0;
    int64_t records_consumed = 0, open_records = 0, open_buffered = 0, invalid_record = -1;
};

// multi-page regime: one encode of [s, e) -> per column its pages (dictionary page first)
struct MpRun {
    std::vector<std::vector<PageOut>> cols;
    std::vector<ChunkDesc> pg, dch;   // the run's page and dictionary descriptors as the device left them
};

// While alive, DevBuf::ensure on this thread orders the release of a replaced block after the
// work already queued on `s` (every reader of the thread's buffers runs on s or waits on it)
// instead of synchronising the whole device.
class StreamOrder {
public:
    explicit StreamOrder(hipStream_t s);
    ~StreamOrder();
    StreamOrder(const StreamOrder &) = delete;
    StreamOrder &operator=(const StreamOrder &) = delete;

private:
    hipStream_t prev_;
};

class DevBuf {
public:
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes);
    void swap(DevBuf &o) { std::swap(p, o.p); std::swap(cap, o.cap); }
    ~DevBuf();
    template <typename T> T *as() const { return (T *)p; }
};

class Engine {
public:
    Engine() = default;
    ~Engine();
    int init(int device, const kpw_schema *schema, const kpw_props *props);
    int encode(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, bool final_flush, int64_t next_rg_size,
               hipStream_t user_stream, BatchOut &out);
    int copy_pages(uint64_t off, uint64_t len, void *host);
    // Multi-page regime: the records [0, n) are the open row group's prefix (no row-group cut
    // inside it).  Per column: the pages ColumnWriterV1 cut within them (a cut after record
    // n - 1 included) and those pages' header + compressed bytes, which is what
    // ColumnChunkPageWriter.getMemSize() adds to getBufferedSize() (the writer's size model).
    // `cols_mask` (optional): only those columns are encoded (the ones that cut a page since the
    // last probe; the others' pages are unchanged, so their npages / flushed come back as -1).
    // `rg_token` names the open row group (the caller's fill-buffer generation): a cut page never
    // changes afterwards, so its header + compressed size is kept per (column, page) across the
    // probes of one token and only the pages cut since are compressed.
    // `cuts` (optional, v1): the page cuts of [0, n) per column as the caller's size model has
    // them, so the probe skips the GPU planner's page-cut pass and its inputs.
    int probe_pages(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, std::vector<int32_t> &npages,
                    std::vector<int64_t> &flushed, const std::vector<char> *cols_mask = nullptr, uint64_t rg_token = ~0ull,
                    const std::vector<std::vector<int64_t>> *cuts = nullptr);
    const std::string &error() const { return err_; }
    // Alternate the page output buffers between encodes, so the previous encode's pages can
    // still be read (D2H on another stream) while this one runs.  The caller orders this
    // encode after any reader of the buffers it now gets back (two encodes ago).
    void swap_page_buffers() { d_body.swap(d_body_alt); d_comp.swap(d_comp_alt); }
    bool multi_page() const { return mp_; }   // pages accumulate in one buffer (no alternation)
    // Single-page regime only: encode() stops after the row-group planner (records_consumed,
    // open_buffered and the cut positions; no chunks, pages or statistics)
    bool plan_only = false;
    // Called once per successful encode as soon as the row-group cuts are known (records_consumed,
    // open_records, invalid_record set; pages not yet), on the encoding thread; work it queues on
    // `stream` runs before the rest of the encode.  The writer places the next job's carried
    // records from here, so the next job can start while this one still encodes.
    std::function<void(const BatchOut &)> on_plan;
    // > 0: plan at most this many row groups per encode (the rest stays unconsumed, also on a
    // final flush).  HDFS block alignment re-plans after each row group with the next limit.
    int32_t max_cuts = 0;
    // Multi-page, non-final: after a row-group cut whose remaining records are less than a row
    // group's raw bytes, stop (they are the next job's carry, which plans them again) instead of
    // encoding them to look for a cut; open_buffered is then -1 (unknown).  The writer's
    // write-path jobs only: getDataSize plans the open row group when it needs the size.
    bool lazy_open = false;
    // Multi-page: records of the last row group an engine of this schema and properties cut (0: none yet)
    int64_t rg_records_hint() const;
    std::vector<ColInfo> cols;
    kpw_props props{};
    std::string message_name, proto_class;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t given_stream = nullptr;   // set before init: the engine's stream (the owner's to release)
    float stage_ms[10] = {0};   // 0-7 stages, 8 k_decode, 9 K7 (k_snappy_v, k_snappy_seg, k_snappy_s_rest)
    uint32_t lb_fallbacks = 0;  // look-backs of the last encode that recomputed a predecessor (kpw_lookback.h)
    // page-size probes, host wall per phase (ms, summed): encode entry -> probe_mp (K1 and its
    // launches), the multi-page pipeline, after it (page headers, caches)
    double probe_t[3] = {0, 0, 0};

private:
    int encode_impl(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, bool final_flush, int64_t next_rg_size,
                    hipStream_t user_stream, BatchOut &out);
    int fail(int code, const std::string &msg);
    SegScratch seg_;   // segmented-scan scratch of this handle (freed in ~Engine)
    bool seg_failed_reset() { const bool f = seg_.failed; seg_.failed = false; return f; }
    std::string err_;
    // decode buffers
    std::vector<DevBuf> col_vals, col_shash, col_spfx, col_soff, col_slen, col_pres, col_vbits, col_pcnt;
    std::vector<uint32_t> dict_hint_;  // per column: most dictionary entries in the previous encode (0: none)
    DevBuf d_cols, d_fmap, d_raw, d_P, d_Q, d_qv, d_opt, d_bool;   // d_cols: descriptors + error word
    // planning
    DevBuf d_ev, d_E, d_gend, d_plan;
    // rle scratch (shared by planning and encoding)
    DevBuf r_last, r_prev, r_lrcnt, r_lroff, r_lra, r_lrb, r_lrf, r_rg, r_rb, r_rboff, r_rgoff, d_jobs;   // d_jobs: the job table
    DevBuf r_ptj, r_etj, r_ltj, d_ctj, mp_dtj, d_dorder;
    uint32_t r_nlt_ = 0;                     // long-run tiles of the RLE jobs laid out last   // tile -> job maps and the dictionary order (built by k_maps)
    // chunks
    DevBuf d_fmask;   // k_dict_firsts: first occurrences per chunk tile and thread (u8)
    DevBuf d_chunks, d_ctile, d_tile_raw, d_tile_raw_off, d_tile_smin, d_tile_smax,
        d_tile_cnt, d_tile_sz, d_ht, d_ids, d_ent_rec, d_ent_boff, d_ptab,   // d_ptab: page table (engine.cpp)
        d_body;
    // snappy
    DevBuf d_ktab, d_frag_out, d_frag_len, d_frag_coff, d_comp;   // d_ktab: K7's host tables
    DevBuf d_sblob, d_sprof;
    DevBuf d_seg_scratch, d_seg_counter;   // k_snappy_seg (one scratch block per CU)
    int seg_args(SnappyArgs &sa);          // fills sa.seg_* (KPW_SNAPPY_SEG=0: sequential kernels only)
    // K7 for GZIP: members of the page slots with `on[p]` into d_comp (offsets / lengths in
    // d_pcoff / d_pclen, total at tot[0]); the caller reads them back as for Snappy
    int gzip_pages(const uint8_t *body, uint64_t body_len, const uint64_t *d_poff, const uint64_t *d_ppre,
                   const std::vector<uint64_t> &poff, const std::vector<uint64_t> &plen, const std::vector<char> &on,
                   uint64_t *d_pcoff, uint64_t *d_pclen, uint64_t *tot, uint64_t *overflow, hipStream_t s);
    DevBuf d_dfl_tab, d_dfl_pdist, d_dfl_m128, d_dfl_m32, d_dfl_sym, d_dfl_gz, d_dfl_glen, d_dfl_dsym, d_dfl_dpos,
        d_dfl_seg, d_dfl_page, d_dfl_blk;
    DevBuf d_body_alt, d_comp_alt;
    std::vector<double> sn_cost_;       // K7 mean fragment duration per (column, page kind), previous batch
    std::unordered_map<uint64_t, double> sn_fcost_;   // per (kind, fragment index)
    std::vector<uint32_t> sn_order_;
    std::vector<uint64_t> sn_ft_;
    // v2 (PARQUET_2_0): boolean value streams, planner streams, DELTA streams
    bool v2_ = false;
    std::vector<DevBuf> col_cbits;
    std::vector<uint64_t *> cbits_;    // per BOOLEAN column (bool_idx_ order): its value stream bits (this encode)
    DevBuf d_cbits_ptr, d_streams, d_djobs, d_blk_job, d_blk_min, d_blk_w, d_blk_sz, d_blk_off, d_btot, d_dense, d_pre, d_sfx,
        d_tile_sfx, d_tile_sfx_off, d_chunk_sfx;
    hipEvent_t ev_[9] = {};
    hipEvent_t kev_[4] = {};
    // upload_parts' pageable host staging: a ring of buffers, each reused only after the event
    // recorded behind its copy has completed (correct whether or not hipMemcpyAsync has consumed
    // a pageable source by the time it returns)
    static constexpr int UP_RING = 4;
    std::vector<uint8_t> up_host_[UP_RING];
    hipEvent_t up_ev_[UP_RING] = {};
    bool up_used_[UP_RING] = {};
    int up_k_ = 0;
    std::vector<uint32_t> opt_idx_, bool_idx_;
    int run_rle(std::vector<RleJob> &jobs, uint32_t &nptiles, uint32_t &netiles, RleScratch &sc);
    int rle_layout(std::vector<RleJob> &jobs, uint32_t &npt, uint32_t &net);
    void rle_bind(RleScratch &sc);
    int rle_maps(const RleJob *jobs_d, uint32_t njobs, RleScratch &sc);
    int dict_order(const std::vector<uint32_t> &count, const std::vector<uint8_t> &is_dict, uint32_t &ndict_tiles,
                   std::vector<uint32_t> &list, std::vector<uint32_t> &roff);
    // the planner's streams and RLE jobs over the first ne records (v2: clears the optional
    // booleans' compacted bit arrays on the stream)
    int plan_inputs(const std::vector<DevCol> &hc, uint64_t ne, uint64_t nwords, std::vector<PlanStream> &hs,
                    std::vector<RleJob> &pj);
    // multi-page regime (engine_mp.cpp)
    bool mp_ = false;
    int64_t mp_last_rg_ = 0;               // records of the last row group the multi-page path cut (horizon hint)
    double t_encode_in_ = 0.0;             // steady clock (ms) at the last encode() entry (KPW_TRACE)
    bool probe_ = false;                 // encode() is a probe_pages call
    std::vector<int32_t> probe_npages_;
    const std::vector<char> *probe_mask_ = nullptr;
    uint64_t probe_token_ = ~0ull;       // open row group of the cached page sizes (~0: none)
    const std::vector<std::vector<int64_t>> *probe_cuts_ = nullptr;   // v1 probe: the caller's page cuts
    const unsigned long long *probe_err_dev_ = nullptr;   // K1's first-invalid-record word of this encode
    // an 8-byte device word mp_pipeline reads back with its last (compression) copy, so the
    // caller needs no readback of its own: source, value, whether it was read
    const void *rb_extra_src_ = nullptr;
    uint64_t rb_extra_val_ = 0;
    bool rb_extra_done_ = false;
    struct CutPage { int64_t end; int64_t bytes; };   // a cut page: end record, header + compressed bytes
    std::vector<std::vector<CutPage>> probe_cache_;   // per column, in page order
    std::vector<uint32_t> probe_mode_;                // per column: first page satisfied (1) / all PLAIN (2), 0 unknown
    // Probe continuation (v1 page-size probes, engine_mp.cpp): each dictionary column's hash table,
    // ids and entries stay on the device between the probes of one open row group, so a probe
    // inserts only the records since the column's previous probe (KPW_PROBE_CONT=0: off).
    struct ProbeDict {
        int64_t done = 0;       // records [0, done) inserted
        uint32_t n = 0;         // entries (in first-occurrence order)
        uint64_t bytes = 0;     // their dictionaryByteSize
        bool stopped = false;   // past dictPageSize: later records fall in PLAIN pages, need no ids
    };
    std::vector<ProbeDict> pd_;
    bool pd_on_ = false;        // mp_pipeline runs a continuation probe
    bool pd_exact_ = false;     // the open row group's string keys are compared byte for byte
    uint64_t pd_ht_cap_ = 0, pd_ent_cap_ = 0, pd_ids_cap_ = 0;   // per dictionary column: table slots, entries, values
    std::vector<int32_t> pd_slot_;   // column -> its region in the pd_ buffers (-1: no dictionary)
    DevBuf pd_ht, pd_ids, pd_ent_rec, pd_ent_boff;
    int pd_prepare(uint64_t ne);   // buffers for a probe of [0, ne)
    void pd_reset();
    std::vector<int64_t> probe_flushed_;
    int encode_mp(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, uint64_t ne, bool final_flush, int64_t T,
                  const std::vector<DevCol> &hc, uint64_t gend_stride, uint64_t ev_stride, BatchOut &out);
    int mp_cuts(PageCutArgs &a, int64_t s, int64_t h, std::vector<std::vector<int64_t>> &cuts);
    int probe_mp(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, uint64_t ne, const std::vector<DevCol> &hc,
                 const std::vector<std::vector<int64_t>> &pc, BatchOut &out);
    // k7_from (probe): per column the first cut page to compress; the dictionary page, the open
    // page and the cut pages before k7_from[c] are not compressed (their compressed sizes in
    // `run` are then meaningless)
    // spec (splice, v1): `run` is only each column's page after its last cut (cuts[c] < e) plus
    // its dictionary page, encoded with the dictionary `spec` (the speculative pass over a range
    // starting at s) left on the device: the pages before are spec's, byte for byte
    int mp_pipeline(const uint8_t *d_data, const uint64_t *d_off, uint64_t n, const std::vector<DevCol> &hc, int64_t s, int64_t e,
                    const std::vector<std::vector<int64_t>> &cuts, MpRun &run, const std::vector<char> *mask = nullptr,
                    const std::vector<uint32_t> *k7_from = nullptr, const MpRun *spec = nullptr);
    int grow_keep(DevBuf &b, size_t bytes, size_t keep);
    // the engine's small host <-> device transfers (engine.cpp: why they stay pageable copies)
    // Several host tables in one H2D copy into `buf` (256-byte aligned parts): their device
    // addresses in `dev`.  One copy instead of one per table (each is a blit kernel).
    struct HostPart { const void *p; size_t bytes; };
    // tail_room: bytes reserved on the device after the last part (not copied)
    int upload_parts(DevBuf &buf, const std::vector<HostPart> &parts, std::vector<uint8_t *> &dev, size_t tail_room = 0);
    hipError_t xh2d(void *dst, const void *src, size_t bytes, hipStream_t s);
    hipError_t xd2h(void *dst, const void *src, size_t bytes, hipStream_t s);
    hipError_t xsync(hipStream_t s);
    std::vector<DevBuf> mp_sp;
    DevBuf mp_ncuts, mp_cutpos, mp_pbytes, mp_pboff, mp_flag, mp_dch, mp_dtile_raw,
        mp_dtile_smin, mp_dtile_smax, mp_dtile_cnt, mp_dtile_sz, mp_ssz, mp_spp, mp_cstream, mp_bstream, mp_acc;
    uint8_t *pages_dev_ = nullptr;
    uint64_t pages_len_ = 0;
};

}  // namespace kpw
