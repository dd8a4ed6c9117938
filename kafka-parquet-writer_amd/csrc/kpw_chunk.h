// kpw_chunk.h — chunk-kernel arguments and launchers (k_chunk.hip, k_snappy.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kpw_kernels.h"
#include "kpw_scan.h"

namespace kpw {

// One dictionary hash-table slot: key, first rank and entry id share a 16-byte slot, so a probe
// (key compare + atomicMin of the rank) and the later id lookups touch one cache line.  An
// all-0xFF fill is the empty table (key HT_EMPTY, rank UINT32_MAX).
struct HtSlot {
    uint64_t key;
    uint32_t min;
    uint32_t id;
};

// host side of the statistics K6 leaves in a read-back descriptor
inline void chunk_stats_derive(ChunkDesc &C)
{
    C.null_count = (uint64_t)(C.e - C.s) - C.nn;
    C.has_minmax = C.nn > 0;
}

struct ChunkArgs {
    ChunkDesc *ch;
    int32_t nchunks;
    uint32_t nctiles;
    const DevCol *cols;
    const uint8_t *data;
    const uint32_t *ctile_chunk;   // chunk of each chunk tile
    const uint32_t *ctile_first;   // per chunk: first tile
    const uint32_t *ctile_count;   // per chunk: number of tiles
    uint64_t *tile_raw, *tile_raw_off, *tile_smin, *tile_smax;
    uint32_t *tile_cnt;
    uint64_t *tile_sz;
    HtSlot *ht;                    // dictionary hash tables (per chunk at ChunkDesc::ht_off)
    HtSlot *ht_clear;              // k_chunk_stats empties these slots (all ones) on the way: the
    uint64_t ht_clear_n;           // dictionary phase follows it (one dispatch fewer than a fill)
    uint64_t *flags_clear;         // and zeroes this word (the collision / retry flags)
    uint64_t body_tail;            // page writers: the body's end (k_chunk_prep clears 512 bytes from there)
    uint32_t *ids;
    uint64_t *ent_rec, *ent_boff;
    uint8_t *fmask;                // per chunk tile and thread: its first occurrences (k_dict_firsts' count pass)
    uint32_t max_dict_bytes;
    int32_t exact_strings;         // 1: BYTE_ARRAY dictionary keys compared byte-for-byte (collision retry)
    const uint64_t *data_end;      // device pointer to offsets[n] (end of the record bytes)
    uint32_t *collision;           // device flag: a hash-keyed string dictionary failed verification
    const uint32_t *dict_order;    // dictionary chunk tiles, interleaved across chunks
    uint32_t ndict_tiles;
    int32_t v2;                    // PARQUET_2_0 page layout (levels unprefixed, DELTA fallback, RLE booleans)
    const DeltaJob *djobs;         // v2: DELTA streams (layout reads their totals)
    DeltaJob *djobs_w;             // v2: same array (layout sets out_off)
    const uint64_t *chunk_sfx;     // v2: DELTA_BYTE_ARRAY suffix bytes per chunk
    uint64_t *page_pre;            // v2: uncompressed level bytes in front of each page's values
    int32_t mp;                    // multi-page regime: descriptors are pages (dictionary decided per chunk)
    // multi-page dictionary insertion in rounds (host-side, read by launch_dict): round j is
    // dict_order[sum(len[0..j)), +len[j]) = tiles [end[j - 1], end[j]) of every chunk; between
    // rounds a chunk past dict_limit bytes stops (ChunkDesc::stop_tile)
    const uint32_t *mp_round_end;
    uint32_t mp_nrounds;
    const uint32_t *mp_round_len;
    uint32_t mp_dict_limit;
    uint32_t dict_wide;            // K2 insertion with 1024-thread tiles (page-size probes: few tiles)
    SegScratch *seg;               // the handle's segmented-scan scratch
};

// Multi-page (v1): page descriptors `pg` (ChunkArgs of the pages) and dictionary
// descriptors `dch` (one per column chunk; dictionary kernels run on them).
void launch_mp_pages_init(ChunkDesc *pg, int npg, const ChunkDesc *dch, const DevCol *cols, RleJob *jobs, hipStream_t s);
void launch_dict_page(const ChunkArgs &a, uint8_t *out, hipStream_t s);
void launch_mp_dict_decide(ChunkDesc *pg, int npg, const ChunkDesc *dch, const DevCol *cols, const uint64_t *ent_rec,
                           const uint64_t *ent_boff, uint32_t max_dict_bytes, RleJob *jobs, hipStream_t s);
void launch_mp_satisfy(ChunkDesc *pg, ChunkDesc *dch, int ndch, const DevCol *cols, const uint64_t *ent_rec,
                       const uint64_t *ent_boff, const RleJob *jobs, hipStream_t s);
void launch_mp_dictpage_off(const ChunkDesc *pg, ChunkDesc *dch, int ndch, hipStream_t s);
void launch_page_str_stats(const ChunkArgs &a, hipStream_t s);

// DELTA streams of a batch (k_delta.hip)
struct DeltaArgs {
    DeltaJob *jobs;
    uint32_t njobs;
    uint32_t nblk;                 // block tiles
    const uint32_t *blk_job;
    uint64_t *blk_min, *blk_sz, *blk_off, *btot;
    uint32_t *blk_w;
    SegScratch *seg;
};
void launch_delta_structure(const DeltaArgs &d, hipStream_t s);
void launch_delta_write(const DeltaArgs &d, uint8_t *out, hipStream_t s);
void launch_v2_decide(const ChunkArgs &a, const RleJob *jobs, DeltaJob *djobs, hipStream_t s);
void launch_v2_delta_jobs(const ChunkArgs &a, DeltaJob *djobs, hipStream_t s);
void launch_v2_dense(const ChunkArgs &a, uint64_t *dense, uint32_t *pre, uint32_t *sfx, uint64_t *tile_sfx, uint64_t *tile_sfx_off,
                     uint64_t *chunk_sfx, hipStream_t s);
void launch_dba_suffixes(const ChunkArgs &a, const uint32_t *pre, const DeltaJob *djobs, const uint64_t *tile_sfx_off, uint8_t *out,
                         hipStream_t s);
void launch_v2_bool_jobs(const ChunkArgs &a, RleJob *jobs, hipStream_t s);
void launch_bool_streams(const DevCol *cols, const uint32_t *bool_cols, uint32_t nbool, uint64_t n, uint64_t *const *cbits,
                         RleJob *jobs, uint32_t job0, PlanStream *streams, uint32_t stream0, hipStream_t s);

inline void seg_tile_scan_u32(const uint32_t *in, uint32_t *out, const uint32_t *seg, uint32_t n, SegScratch *sc, hipStream_t s)
{
    seg_tile_scan<uint32_t, OpSum32>(in, out, seg, n, nullptr, sc, s);
}
inline void seg_tile_scan_u64(const uint64_t *in, uint64_t *out, const uint32_t *seg, uint32_t n, SegScratch *sc, hipStream_t s)
{
    seg_tile_scan<uint64_t, OpSum64>(in, out, seg, n, nullptr, sc, s);
}

void launch_chunk_stats(const ChunkArgs &a, hipStream_t s);
void launch_dict(const ChunkArgs &a, RleJob *jobs, hipStream_t s);
void launch_layout(const ChunkArgs &a, RleJob *jobs, uint64_t *page_off, uint64_t *page_len, uint64_t *tot, hipStream_t s);
void launch_chunk_write(const ChunkArgs &a, const RleJob *jobs, uint8_t *out, hipStream_t s);

// Snappy (K7)
struct SnappyArgs {
    const uint8_t *in;           // uncompressed page bodies
    const uint64_t *page_off;    // [npages]
    const uint64_t *page_len;
    uint32_t npages;
    uint32_t nfrags;             // total fragments (host computed)
    const uint32_t *frag_page;   // [nfrags]
    const uint32_t *frag_idx;    // fragment index within its page
    uint8_t *frag_out;           // nfrags * SNAPPY_FRAG_CAP
    uint32_t *frag_len;
    uint64_t *page_coff;         // exclusive compressed offsets [npages]
    uint64_t *page_clen;         // compressed lengths
    uint64_t *frag_coff;         // per fragment output offset
    uint8_t *out;                // compressed pages
    uint64_t *tot;               // [0] total compressed bytes
    const uint64_t *page_pre;    // v2: uncompressed level bytes right before page_off (nullptr: none)
    uint64_t *ftime;             // per fragment [start, end] wall clock of k_snappy_v (nullptr: off)
    const uint32_t *order;       // k_snappy_v: block b compresses fragment order[b] (nullptr: b)
    uint8_t *seg_scratch;        // k_snappy_seg: per-workgroup scratch (nullptr: k_snappy_v on every fragment)
    uint32_t *seg_counter;       // k_snappy_seg: next fragment slot
    uint32_t seg_grid;           // k_snappy_seg: workgroups (one per CU)
    uint32_t v_only_handed_on;   // k_snappy_v: only the fragments k_snappy_seg handed on
    uint32_t seg_only_marked;    // k_snappy_seg: only the fragments k_snappy_v marked SEG_TODO
    uint32_t v_budget;           // k_snappy_v: decisions before it marks a fragment SEG_TODO (0: no limit)
    uint32_t s_budget;           // k_snappy_s_rest: search batches + copies before SEG_TODO (0: no limit)
    uint64_t *seg_prof;          // k_snappy_seg phase cycle counters (microbench; nullptr: off)
    volatile uint32_t *seg_dbg;  // k_snappy_seg progress per workgroup (microbench; nullptr: off)
};
constexpr uint32_t SNAPPY_FRAG = 65536;
// per-fragment output slot: max compressed length (32 + n + n/6) rounded up to the 256-byte
// output window, plus one window of slack for the final partial flush
constexpr uint32_t SNAPPY_FRAG_CAP = ((32 + SNAPPY_FRAG + SNAPPY_FRAG / 6 + 255) / 256) * 256 + 256;
void launch_snappy(const SnappyArgs &a, hipStream_t s);

// K7 for GZIP (k_deflate.hip): one gzip member per listed page slot
struct DflPage {
    uint64_t off, len;   // page bytes in `in`
    uint64_t slot, cap;  // its member's scratch slot in `gz` and the slot's size
};
struct DflTile {
    uint32_t page, tile;  // listed page, 32 KiB tile of it
};
struct DflSeg {
    uint32_t page, seg;   // listed page, DFL_SEG-position segment of it
};
struct DflBlk {
    uint32_t page, j;     // listed page, deflate block j of it (blocks past the page's count: idle)
};
struct DflSt {
    uint32_t p, ms, ml, ma;   // deflate_slow loop-top state: strstart, match_start, match_length, match_available
};
constexpr uint32_t DFL_SEG = 2048;       // positions per parse segment (one thread each)
constexpr uint32_t DFL_BLK = 16383;      // symbols per deflate block (zlib's lit_bufsize - 1 at level 6)
struct DflArgs {
    const uint8_t *in;
    const DflPage *pages;        // listed pages
    const DflTile *tiles;
    uint16_t *pdist;             // per input byte: distance to the previous same-hash position (0: none)
    uint32_t *m128, *m32;        // per input byte: longest_match, length | distance << 9
    uint32_t *sym;               // per input byte: the symbol the parse emits at that loop top (bit 31: present)
    uint8_t *gz;                 // member scratch (per page: the deflate stream at slot + 16)
    uint64_t *glen;              // per listed page: member length (~0: did not fit)
    uint32_t nslots;             // page slots
    const int32_t *slot_page;    // page slot -> listed page (-1: not compressed)
    const uint64_t *page_off, *page_pre;   // per slot (page_pre: v2 level prefix, or nullptr)
    uint64_t *page_coff, *page_clen;       // per slot: compressed offset / length
    uint8_t *out;                // packed pages
    uint64_t *tot;               // [0] total bytes
    uint64_t *overflow;          // set to 1 when a member overflowed its slot (not expected: the slot is deflateBound)
    // the segment-parallel parse and the block-parallel bit stream (k_deflate.hip)
    const DflSeg *segs;
    uint32_t nsegs, nblks;
    const DflBlk *blks;
    const uint32_t *page_seg0, *page_blk0, *page_tile0;   // per listed page (+1 entry): first segment / block / tile
    DflSt *seg_entry, *seg_exit;
    uint32_t *seg_dirty, *seg_cnt, *seg_sym0;
    uint32_t *flag;              // a parse round changed an entry
    uint32_t *dsym, *dpos;       // per listed page, from P.off + page index: dense symbols and their loop tops
    uint32_t *page_T, *page_nblk, *page_crc, *tile_crc;
    uint64_t *blk_bits, *blk_off;
    uint32_t *blk_kind;          // 0 stored, 1 static, 2 dynamic (0xff: past the page's blocks)
};
// phases (the host runs the parse rounds until no entry changes, reading `flag` between them)
void launch_deflate_prep(const DflArgs &a, uint32_t ntiles, hipStream_t s);
void launch_deflate_round(const DflArgs &a, hipStream_t s);
void launch_deflate_finish(const DflArgs &a, uint32_t npages_listed, hipStream_t s);
void launch_deflate_emit(const DflArgs &a, uint32_t npages_listed, hipStream_t s);
// worst-case gzip member of n bytes (zlib's deflateBound for these parameters + framing)
inline uint64_t dfl_member_bound(uint64_t n) { return n + (n >> 12) + (n >> 14) + (n >> 25) + 13 + 18 + 64; }
size_t snappy_seg_scratch_bytes(uint32_t grid);
constexpr uint32_t SEG_ABORTED = 0xfffffffeu;   // frag_len: k_snappy_seg handed the fragment on
constexpr uint32_t SEG_TODO = 0xfffffffdu;      // frag_len: k_snappy_v ran past its budget (k_snappy_seg's work)

}  // namespace kpw
