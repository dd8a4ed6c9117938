// kpw_kernels.h — structs shared by host orchestration (engine.cpp) and the HIP kernels,
// plus the host-side launch wrappers.  Internal to libkpw_gpu.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kpw {

constexpr int MAX_COLS = 256;
constexpr int FMAP_SIZE = 1024;
constexpr uint64_t KPW_TILE_P_H = 2048;   // host copy of KPW_TILE_P
constexpr uint64_t KPW_TILE_L_H = 16384;  // host copy of KPW_TILE_L
constexpr uint64_t KPW_BLOCK_H = 256;     // host copy of KPW_BLOCK

// One schema column as the device sees it (decode outputs live in these buffers).
struct DevCol {
    int32_t phys;          // kpw_physical_type
    int32_t proto_type;    // kpw_proto_type
    int32_t wire_type;     // expected proto wire type
    int32_t optional;
    int32_t field_number;
    int32_t vsize;         // 4 / 8 fixed width, 0 for BYTE_ARRAY and BOOLEAN
    int32_t dict;          // dictionary-capable (non-boolean and dictionary enabled)
    int32_t pad;
    void *vals;            // u32 / u64 [n] (fixed width)
    uint64_t *soff;        // BYTE_ARRAY: absolute byte offset of the value in the batch data
    uint32_t *slen;        // BYTE_ARRAY: length
    uint64_t *pres;        // optional: presence bits [nwords]
    uint64_t *vbits;       // BOOLEAN: value bits [nwords]
    uint32_t *pcnt;        // optional: exclusive prefix popcount of pres per word [nwords+1]
    uint64_t *shash;       // BYTE_ARRAY: 64-bit hash of the value bytes (dictionary key)
    uint64_t *spfx;        // BYTE_ARRAY: first 16 value bytes, zero padded (2 words per record)
};

struct DecodeArgs {
    const uint8_t *data;
    const uint64_t *off;
    uint64_t n;
    const DevCol *cols;
    int32_t ncols;
    int32_t pad;
    const int16_t *fmap;   // field number -> column (-1), size FMAP_SIZE
    uint32_t *raw;         // per record: raw (plain-equivalent) bytes of non-boolean present values
    unsigned long long *err_min;
    uint64_t nwords;       // words of every presence / boolean bitmask (K1 zeroes those past n)
};

// Device scratch of the multi-block segmented scans (k_scan.hip), owned by one encoder
// handle (Engine::seg_) and grown on demand.  Scans of one handle run in order on its own
// stream, so they share it; handles never share one (concurrent writers, C5).
struct SegScratch {
    void *p = nullptr;             // single-pass scans: tile status words (kpw_lookback.h)
    size_t bytes = 0;
    uint32_t *fails = nullptr;     // look-back fallbacks since the last lb_failures (its own word:
                                   // the status words' growth and epoch-wrap clears never touch it)
    uint32_t epoch = 0;            // of the last launch (status words carry it)
    void *tmp = nullptr;           // reduce-then-scan tile sums (never the status words: any
    size_t tmp_bytes = 0;          // value written there could pose as a status of a later epoch)
    bool failed = false;           // an allocation failed since the engine last checked
};

// Generic RLE/bit-packing hybrid job (one encoded stream).
struct ValSrcH {
    uint32_t kind, pad;
    const void *ptr;
    uint64_t base;
};
struct RleJob {
    ValSrcH src;
    uint32_t len;          // number of values (device may lower it; upper bound used for tiling)
    uint32_t bw;           // bit width (device may set it)
    uint32_t tile0, ntiles;        // position tiles [tile0, tile0+ntiles)
    uint32_t etile0, netiles;      // element tiles (long runs / RLE runs)
    uint32_t ltile0, nltiles;      // long-run tiles [ltile0, ltile0+nltiles) (KPW_TILE_L positions each)
    uint64_t e0;                   // base index into element arrays (capacity netiles*KPW_TILE_E)
    uint64_t out_off;              // encode: output byte offset; plan: event array base (positions)
    // results (device written)
    uint32_t n_long, n_rle;
    uint64_t total_bytes;
    uint64_t total_groups;
    uint64_t final_gap_off;        // byte offset of the final gap
    uint64_t final_gap_groups;
    uint64_t final_gap_start;      // position where the final gap starts
};

struct RleScratch {
    uint32_t *ptile_job;           // position tile -> job
    uint32_t *ltile_job;           // long-run tile -> job
    uint32_t n_ltiles;
    int64_t *last_brk, *prev_brk;  // per long-run tile: its last value break / the one before it
    uint32_t *lr_cnt, *lr_off;     // per long-run tile: long runs ending in it / their offset
    uint32_t *etile_job;           // element tile -> job
    uint32_t *lr_a, *lr_b;         // long runs (a, b)
    uint8_t *lr_rle;               // per long run: the parse took it as an RLE run (planning; null: not kept)
    uint32_t *r_g, *r_b;           // RLE runs (g, b)
    uint64_t *r_boff, *r_goff;     // per RLE run: byte offset of its gap, groups before its gap
    SegScratch *seg;               // the handle's scan scratch (look-back status words)
};

// Plan / chunk descriptors -------------------------------------------------------------

// One RLE-encoded bit stream whose emitted bytes count in the row-group size check: the
// definition levels of an optional column (record-indexed presence bits) or, in v2, the
// values of a boolean column (RunLengthBitPackingHybridValuesWriter: record-indexed value
// bits when required, rank-indexed compacted bits when optional).
struct PlanStream {
    const uint64_t *bits;
    uint64_t len;                  // stream length (device-set for rank-indexed streams)
    int32_t rank_col;              // -1: position = record; else position = rank in this column
    int32_t pad;
};
constexpr int MAX_STREAMS = 2 * MAX_COLS;

struct PlanArgs {
    uint64_t n;                    // records in the batch
    int32_t final_flush;           // close(): flush the trailing row group
    int32_t ncols;
    int64_t next_rg_size;          // nextRowGroupSize
    const uint64_t *P8;            // raw record bytes before record 8g [n/8 + 1] ...
    const uint32_t *raw;           // ... plus those of the group's records before r (pref8)
    const unsigned long long *err; // K1's first invalid record (copied to out[4])
    const RleJob *jobs;            // the streams' K3 planning jobs (job k = stream k) and long runs
    const uint32_t *lr_a, *lr_b, *lr_off;
    const uint8_t *lr_rle;
    const uint64_t *Q8;            // the same over val = raw + the global parse's event bytes of every
    const uint32_t *qv;            // record-indexed stream (null: not folded); see k_plan_fold
    const DevCol *cols;
    const PlanStream *streams;     // RLE streams counted by emitted bytes
    int32_t nstreams;
    int32_t nbool;                 // boolean columns counted as ceil(values/8) (v1); 0 in v2
    const uint32_t *bool_cols;     // indices of boolean columns
    // emitted bytes of the global parse of stream k before position q (ev_prefix): per group of 8
    // positions E8[k * (ev_stride / 8 + 1) + q / 8], plus the event bytes ev[k * ev_stride + ...]
    // of the positions before q in its group (one 8-byte load)
    const uint32_t *E8;
    const uint8_t *ev;
    uint64_t ev_stride;            // bytes per stream in ev (a multiple of 8, > n)
    const uint64_t *gend;          // per stream k: bitmask of global RLE ends [(n/64+2)]
    uint64_t gend_stride;          // words per stream
    // outputs
    int64_t *rg;                   // [max_rgs] (start, end) pairs
    int32_t max_rgs;
    int32_t max_cuts;              // > 0: stop after this many cuts (HDFS alignment plans one row group at a time)
    int64_t *out;                  // [0]=n_rgs [1]=open_start [2]=open_buffered [3]=overflow
};

// Multi-page (v1, pageSize < blockSize) planning of one row group at a time (k_plan.hip):
// ColumnWriterV1.accountForValueWritten page cuts per column from the row-group start s up
// to a horizon h, then InternalParquetRecordWriter.checkBlockSizeReached with the flushed
// pages' header + compressed bytes (ColumnChunkPageWriter.getMemSize) in memSize.
struct PageCutArgs {
    uint64_t n;                    // records in the batch (valid prefix)
    int64_t s, h;                  // row-group start, horizon (exclusive)
    int32_t ncols;
    int32_t pad;
    int64_t page_size;
    const DevCol *cols;
    const int32_t *col_stream;     // per column: definition-level stream (E/gend index) or -1
    const uint32_t *E8;            // as PlanArgs
    const uint8_t *ev;
    uint64_t ev_stride;
    const uint64_t *gend;
    uint64_t gend_stride;
    const uint64_t *const *sp;     // per column: exclusive prefix of (4 + len) over present BYTE_ARRAY values
    uint32_t cap;                  // cut capacity per column
    uint32_t *ncuts;               // [ncols]
    int64_t *cuts;                 // [ncols * cap] page ends (exclusive record index), increasing
    int32_t *overflow;
    const uint64_t *pbytes;        // k_plan_mp: header + compressed bytes of each cut page, column c's
    const uint64_t *pb_off;        // at pbytes[pb_off[c] + i] (compact: sum of ncuts entries)
    int64_t next_rg_size;
    int64_t *out;                  // k_plan_mp: [0] row-group end or -1, [1] memSize at n (open buffered)
    // PARQUET_2_0: BOOLEAN values are a RunLengthBitPackingHybridValuesWriter stream (buffered
    // size = RLE bytes emitted, walked like the level streams); pages are cut by the store
    const int32_t *col_bstream;    // per column: its boolean value stream (E/gend index) or -1
    const PlanStream *streams;     // the planner streams (bits / length of the boolean ones)
    int32_t v2;
    int32_t str_spec;              // k_page_cuts: speculative batches for REQUIRED BYTE_ARRAY columns (KPW_PAGE_CUT_SPEC=0: off)
};
void launch_str_sizes(const DevCol *cols, int c, uint64_t n, uint32_t *sz, hipStream_t s);
void launch_page_cuts(const PageCutArgs &a, hipStream_t s);   // v1 per column, v2 per store
void launch_plan_mp(const PageCutArgs &a, hipStream_t s);

struct ChunkDesc {
    int64_t s, e;                  // record range in the batch
    int32_t col, rg;
    uint32_t nn;                   // non-null values (device)
    uint32_t is_dict;              // dictionary attempted (device may clear on fallback)
    uint64_t raw_bytes;            // plain-equivalent bytes (rawDataByteSize / plain size)
    uint64_t dict_bytes;           // dictionaryByteSize
    uint32_t dict_n;               // dictionary entries
    uint32_t fallback;             // 1 = PLAIN (fallback or not satisfying)
    uint32_t overflow;             // hash table overflow -> fallback
    uint32_t bw;                   // id bit width
    // hash table
    uint64_t ht_off;               // slot offset
    uint32_t ht_cap;               // power of two
    uint32_t ht_plim;              // probe limit of a hint-sized table (0: none, full-size table)
    uint64_t ids_off;              // ids array offset (nn entries)
    uint64_t ent_off;              // dictionary entries array offset (first-occurrence value index)
    // stats
    uint64_t smin, smax;           // fixed: canonical bits; binary: value index of min/max
    uint32_t has_minmax;
    uint32_t stop_tile;            // multi-page dictionary descriptor: tiles >= this one (within
                                   // the chunk) are skipped, the dictionary having passed
                                   // dictPageSize before them (0: none)
    uint64_t null_count;
    // layout
    uint64_t dl_len;               // RLE def-level bytes (without the 4-byte prefix)
    uint64_t val_len;              // values part of the data page
    uint64_t dictpage_len;         // dictionary page bytes (0 if none)
    uint64_t body_off;             // byte offset of this chunk's uncompressed bodies (dict page, then data page)
    uint64_t dl_scratch, id_scratch;   // offsets of RLE outputs in the rle output scratch
    int32_t dl_job, id_job;
    // v2 (PARQUET_2_0)
    int32_t bool_job;              // RLE job of the boolean values (-1 none)
    int32_t dj0;                   // first DELTA stream (INT: 1, BYTE_ARRAY: 2), -1 none
    uint64_t val_off;              // absolute offset of the values part of the data page
    // multi-page (v1): page descriptors point at their column chunk's dictionary descriptor;
    // a dictionary descriptor lists its pages [first_page, first_page + npages)
    int32_t owner;                 // page: dictionary descriptor index (-1 single-page regime)
    int32_t first_page, npages;    // dictionary descriptor: its pages
    int32_t rl0_len;               // v2: bytes of the width-0 repetition-level stream (layout)
    // multi-page splice (engine_mp.cpp): an exact pass that re-encodes only each column's last
    // page reuses the speculative pass's dictionary descriptor
    uint32_t dict_all;             // dictionary descriptor: K2's entries (k_mp_satisfy then narrows dict_n)
    uint32_t tail_mode;            // 0: the chunk's first page is in this run; 1: kept first page, dictionary
                                   // satisfying; 2: kept first page, every page of the chunk PLAIN
    uint32_t tail_dict_n;          // mode 1: dict_n of the last kept dictionary-encoded page (0: none)
    // probe continuation (engine_mp.cpp, a page-size probe's dictionary descriptor): the table,
    // ids and entries of [s, s + tile_skip) are kept on the device from the previous probes of the
    // open row group; this run inserts only [s + tile_skip, e), new entries numbered from ent_base
    // with dictionary-page offsets from boff_base.  0 / 0 / 0 everywhere else.
    uint32_t ent_base;
    uint64_t tile_skip;
    uint64_t boff_base;
};

// One DELTA_BINARY_PACKED stream (k_delta.hip).
constexpr uint32_t DJ_LONG = 1;      // 64-bit arithmetic (ForLong)
constexpr uint32_t DJ_U32_SRC = 2;   // source values are u32 (else u64)
constexpr uint32_t DJ_INACTIVE = 4;  // not written (chunk kept its dictionary)
struct DeltaJob {
    const void *vals;              // dense values, rank order
    uint64_t base;                 // index of value 0
    uint32_t n;                    // values (device-set)
    uint32_t flags;
    uint32_t blk0, nblk;           // block tiles [blk0, blk0+nblk) (host: upper bound, >= 1)
    uint64_t out_off;              // absolute output offset (device-set by the layout)
    uint64_t hdr;                  // header bytes (device)
    uint64_t total;                // header + blocks (device)
    int32_t prev;                  // multi-page: the same stream of the chunk's previous page (the
                                   // fallback writer is reset, not rebuilt, between pages), or -1
    int32_t pad;
};

// ---------------------------------------------------------------- launch wrappers
void launch_decode(const DecodeArgs &a, hipStream_t s);
void launch_prefix_raw(const uint32_t *raw, uint64_t n, uint64_t *P, SegScratch *sc, hipStream_t s);
// P[0] = 0, P[k] = base + raw[1] + ... + raw[k-1] (k >= 1) for u8 (width 1) / u16 (width 2) raw
void launch_prefix_narrow(const void *raw, int width, uint64_t base, uint64_t n, uint64_t *P, SegScratch *sc, hipStream_t s);

void launch_rle_structure(RleJob *jobs_d, int njobs, uint32_t n_ptiles, uint32_t n_etiles,
                          const RleScratch &sc, hipStream_t s);
void launch_rle_write(RleJob *jobs_d, uint32_t n_ptiles, uint32_t n_etiles, const RleScratch &sc,
                      uint8_t *out, hipStream_t s);
void launch_rle_events(RleJob *jobs_d, uint32_t n_ptiles, uint32_t n_etiles, const RleScratch &sc,
                       uint8_t *ev, uint64_t *gend, uint64_t gend_stride, hipStream_t s);

// k_maps.hip: tile -> job maps expanded from the job tables' (first tile, tile count) words
// (job j's words at first[j * stride], count[j * stride]); up to 4 maps per launch
struct TileMapSpec {
    const uint32_t *first, *count;
    uint32_t stride, n;            // words between jobs; jobs
    uint32_t *map;
};
struct TileMapArgs {
    TileMapSpec m[4];
    uint32_t nm;
};
void launch_tile_maps(const TileMapArgs &a, hipStream_t s);
// dictionary insertion order: tile k of every listed chunk (list order) before tile k + 1 of
// any; round_off[k] = tiles of rounds < k
void launch_dict_order(const uint32_t *list, uint32_t nl, const uint32_t *first, const uint32_t *count,
                       const uint32_t *round_off, uint32_t nrounds, uint32_t *out, hipStream_t s);

void launch_plan(const PlanArgs &a, hipStream_t s);
void launch_plan_fold(const uint8_t *ev, uint64_t ev_stride, const PlanStream *streams, uint32_t nstreams, const uint32_t *raw,
                      uint64_t n, uint32_t *val, hipStream_t s);
// k_asm.hip: one job's file bytes gathered in HBM (pieces of <= 64 KiB: dst offset in `out`,
// src = device address (dev) or offset into the host-built header blob)
struct AsmPiece {
    uint64_t dst, src;
    uint32_t len, dev;
};
void launch_asm_gather(const AsmPiece *pc, uint32_t npieces, const uint8_t *blob, uint8_t *out, hipStream_t s);

}  // namespace kpw
