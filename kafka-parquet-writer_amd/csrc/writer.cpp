// writer.cpp — kpw_writer_*: the ParquetFile drop-in (include/kpw_gpu.h), PCIe-inclusive.
//
// Reference seam: ParquetFile<T> (src/main/java/ir/sahab/kafka/reader/ParquetFile.java:24-100)
// driven by KafkaProtoParquetWriter.WorkerThread (write per record :277, getDataSize :281-285,
// 306-308, close :326-337).
//
// Pipeline (north_star "pinned staging ... overlapped with encoding of the previous
// row group"):
//
//   caller thread   write(): record bytes -> the fill stage buffer in HBM.  Pinned sources
//                   (kpw_host_alloc, where polled batches are meant to land) are DMA'd
//                   directly; other memory goes through pinned 32 MiB slots (one host copy).
//                   Only the u64 record ends stay on the host.  A full stage buffer is handed
//                   to the worker as a job and the caller goes on filling the next one.
//   worker thread   per job: wait for the buffer's copies, upload its offsets, encode on the
//                   handle's stream (K1..K7), carry the open row group's records to the next
//                   stage buffer device-to-device, release the buffer, D2H the pages.
//   assembly thread per job: page headers + bodies + row-group metadata into the file
//                   (overlaps the next job's encode).
//
// Three stage buffers: one encoding, one queued, one filling.  Each starts with a gap of
// `gap_` bytes where the previous job's open records are placed, so a job's records are
// contiguous: [carried records | appended records].
//
// getDataSize() for the per-record loop: an exact host model of parquet-mr's buffered size and
// row-group check (sizemodel.h) runs on every record of small writes, so getDataSize() is O(1)
// and row groups are cut on the host exactly where parquet-mr cuts them; the GPU encodes those
// records as complete row groups (jobs of kind EXACT).  Large writes (bulk path) leave the
// model: their cuts are planned on the GPU (jobs of kind PLANNED) and getDataSize() drains the
// pipeline and encodes what is staged.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kpw_gpu.h"
#include "engine.h"
#include "kpw_scan.h"
#include "filewriter.h"
#include "memcache.h"
#include "sizemodel.h"

using namespace kpw;

namespace {

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// KPW_TRACE=1: per-job timings of the writer pipeline on stderr
bool trace_on()
{
    static const bool v = [] { const char *e = getenv("KPW_TRACE"); return e && *e == '1'; }();
    return v;
}
uint64_t env_mb(const char *name, uint64_t dflt)
{
    const char *e = getenv(name);
    const long long v = e ? atoll(e) : 0;
    return (uint64_t)(v > 0 ? v : (long long)dflt) << 20;
}
// Bytes of appended records per job.  KPW_STAGE_FLUSH_MB overrides.
uint64_t stage_flush_bytes()
{
    static const uint64_t v = env_mb("KPW_STAGE_FLUSH_MB", 1024);
    return v;
}
// Eager jobs: a fill buffer holding at least this many appended bytes is submitted early when
// an encode worker is idle and nothing is queued (KPW_EAGER_MB, default 384; a negative value
// turns it off).  The GPU then starts on the data already in HBM instead of waiting for a full
// job, and close() finds less left to encode; jobs stay at the full size while the workers are
// busy.  C2 writer path 33.5 -> 35.8 GB/s, C5 28.4 -> 31.6 with 512 MiB in r02; with round 4's
// fewer dispatches and syncs per job 384 MiB measured better (alternating on one box: C2 5 runs
// 42.1-44.5 against 35.7-43.5 GB/s with 512, C3 42.6-45.8 against 42.2, C4 21.2-21.3 against
// 20.7-20.9, C5 unchanged; 256 MiB lower).
uint64_t eager_job_bytes()
{
    static const uint64_t b = [] {
        const char *e = getenv("KPW_EAGER_MB");
        const long long v = e ? atoll(e) : 384;
        return v > 0 ? (uint64_t)v << 20 : 0ull;
    }();
    return b;
}

// Multi-page writers (pageSize < blockSize) submit eager jobs while the workers are busy too, as
// long as fewer than this many jobs are queued (KPW_MP_EAGER_QUEUE, default 3; 0: as single-page).
// A multi-page job's row-group cuts need its speculative encodes, so jobs run one after another
// up to their cuts; jobs grown to the full stage size (1 GiB) carry open row groups larger than
// the buffers' gap (a rebuild per carry) and bigger page buffers.
int mp_eager_queue()
{
    static const int v = [] { const char *e = getenv("KPW_MP_EAGER_QUEUE"); return e ? atoi(e) : 3; }();
    return v;
}

// Writes of more records than this leave the per-record size model (bulk path).
uint64_t model_max_batch()
{
    static const uint64_t v = [] { const char *e = getenv("KPW_MODEL_MAX_BATCH"); return e ? (uint64_t)atoll(e) : 65536ull; }();
    return v;
}

// pinned host memory handed out by kpw_host_alloc (or used inside the library): direct-DMA sources
bool pinned_range(const void *p, size_t n) { return pin_contains(p, n); }

// Page-locked host memory owned by the library (from the pinned cache, memcache.h).  Its
// previous contents are never DMA targets or sources when it grows (callers ensure it).
struct PinnedBuf {
    uint8_t *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes)
    {
        if (bytes <= cap && p) return 0;
        pin_free(p);
        p = nullptr;
        cap = 0;
        const size_t c = bytes + bytes / 4 + 4096;
        p = (uint8_t *)pin_alloc(c);
        if (!p) return -1;
        cap = c;
        return 0;
    }
    ~PinnedBuf() { pin_free(p); }
};

// Growable u64 array without value-initialisation: the bulk path appends 500 k record ends per
// write and a zero-fill before overwriting them doubled the caller's memory traffic.  Storage
// comes from the pinned cache (memcache.h): a stage buffer's ends reach ~140 MB, and malloc'd
// arrays of that size were page-faulted in by every new writer and unmapped by every free
// (~45 ms per file).
class U64Vec {
public:
    U64Vec() = default;
    U64Vec(const U64Vec &) = delete;
    U64Vec &operator=(const U64Vec &) = delete;
    ~U64Vec() { pin_free(p_); }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    void clear() { n_ = 0; }
    uint64_t *data() { return p_; }
    const uint64_t *data() const { return p_; }
    uint64_t back() const { return p_[n_ - 1]; }
    uint64_t *begin() { return p_; }
    uint64_t *end() { return p_ + n_; }
    // n more entries, uninitialised; returns the first of them
    uint64_t *grow(size_t n)
    {
        if (n_ + n > cap_) {
            size_t c = std::max<size_t>(cap_ * 2, n_ + n);
            c = std::max<size_t>(c, 1u << 20);
            uint64_t *q = (uint64_t *)pin_alloc(c * 8);
            if (!q) throw std::bad_alloc();
            if (n_) memcpy(q, p_, n_ * 8);
            pin_free(p_);
            p_ = q;
            cap_ = c;
        }
        uint64_t *r = p_ + n_;
        n_ += n;
        return r;
    }
    void push_back(uint64_t v) { *grow(1) = v; }
    void resize(size_t n) { if (n <= n_) n_ = n; else grow(n - n_); }

private:
    uint64_t *p_ = nullptr;
    size_t n_ = 0, cap_ = 0;
};

enum { BUF_FREE = 0, BUF_FILLING = 1, BUF_QUEUED = 2 };
enum { JOB_PLANNED = 0, JOB_EXACT = 1, JOB_FINAL = 2 };

struct StageBuf {
    uint8_t *d = nullptr;
    size_t cap = 0;
    uint64_t gap = 0;                  // first appended byte; carried records end here
    uint64_t len = 0;                  // append position
    std::vector<uint64_t> carry;       // carried record boundaries (worker-written; ncarry+1 or empty)
    bool carry_in_store = false;       // carried records wait in kpw_writer::carry_store (did not fit the gap)
    U64Vec ends;                       // appended record ends (caller-written)
    int64_t ncarry_expected = 0;       // carried records, as the caller knows them (EXACT jobs)
    int64_t first_new_global = 0;      // file record index of the first appended record
    int state = BUF_FREE;
    hipEvent_t copied = nullptr;       // recorded on the copy stream after the last append
    // the appended records' lengths, narrowed ahead of the job by a waiting worker (prep_lengths):
    // they do not depend on the carried records, which are known only at the previous job's cuts
    PinnedBuf lp;
    int lp_width = 0;                  // bytes per length
    int lp_state = 0;                  // 0 not prepared, 1 being prepared, 2 ready (under kpw_writer::mu)
};

struct Job {
    int buf, kind, next;
    int64_t n_exact;                   // EXACT: records [0, n_exact) of the buffer form complete row groups
    uint64_t seq;                      // submission order (= file order)
    bool lazy;                         // PLANNED from the write path: the open row group's buffered
                                       // size may be left unknown (Engine::lazy_open)
};

}  // namespace

// One encode worker: its own engine (HIP stream, scratch, double-buffered page buffers) and thread.
struct Worker {
    Engine *eng = nullptr;
    DevBuf d_off;                      // device record offsets of the running job ([0] = 0, then offs)
    PinnedBuf h_off;                   // host record boundaries of the running job
    PinnedBuf h_len;                   // record lengths, u8 / u16 / u32 (H2D source: 1/8 .. 1/2 the bytes of offsets)
    int len_width = 1;                 // narrowest length width a job tries (KPW_LEN_BYTES)
    DevBuf d_len;                      // device lengths
    struct ScanScratch {               // the offsets scan's tile status words
        SegScratch sc;
        ~ScanScratch() { seg_scratch_free(sc); }
    } scan;
    const uint64_t *offs = nullptr;    // device record offsets handed to the engine
    hipEvent_t carry_ev = nullptr;     // recorded after this worker placed a job's carried records
    hipEvent_t enc_done = nullptr;     // recorded after a job's encode (the D2H of its pages waits on it)
    hipEvent_t d2h_ev[2] = {};         // D2H done, per page buffer set of the engine
    bool d2h_used[2] = {false, false};
    PinnedBuf h_asm;                   // device assembly: header blob + pieces (H2D source)
    hipEvent_t asm_ev = nullptr;       // after a job's assembly H2D, gather and D2H into the file
    bool asm_pending = false;          // asm_ev recorded and not yet waited for
    DevBuf d_asm_in, d_asm_out;        // device assembly: blob + pieces, the job's file bytes
    uint64_t njobs = 0;
    bool busy = false;
    std::thread th;
};

// The writer's stream set (memcache.h): eng, eng1, copy, d2h, and eng2 with three encode workers
// only.  Declared before the engines, so it is destroyed after them: the streams go back idle
// (every owner synchronised its own).  A fifth stream and a fifth stage buffer for the default two
// workers cost the bulk multi-page line 23.0-23.4 -> 19.8-21.3 GB/s (r06bm, same box: the writer
// ran ahead into more queued jobs and the close grew 62 -> 162 ms), so both follow the count.
constexpr int kSetStreams = 5;
struct StreamSetOwner {
    hipStream_t s[kSetStreams] = {};
    int n = 0;
    ~StreamSetOwner() { if (s[0]) stream_set_release(n, s); }
};

struct kpw_writer {
    static constexpr int kBufs = 5;    // up to three encoding, one queued, one filling (nbufs in use)
    int nbufs = 4;                     // 5 with three workers
    static constexpr int kSlots = 4;
    static constexpr size_t kSlotBytes = 32ull << 20;
    StreamSetOwner sset;
    Engine eng;                        // worker 0's engine (also the caller's, for write_until_full probes)
    Engine eng1;                       // worker 1's engine
    Engine eng2;                       // worker 2's engine (KPW_ENCODERS=3)
    int nworkers = 2;
    bool aligned = false;              // HDFS PaddingAlignment: row groups planned one at a time (run_job_aligned)
    Worker wk[3];
    FileWriter *fw = nullptr;
    hipStream_t copy_stream = nullptr;
    StageBuf buf[kBufs];
    int fill = -1;                     // buffer the caller appends to
    std::atomic<uint64_t> gap_{0};   // raised by the workers when a carry does not fit (place_carry)
    // pinned slots for non-pinned sources
    PinnedBuf slot[kSlots];
    hipEvent_t slot_ev[kSlots] = {};
    int cur_slot = 0;
    uint64_t slot_used = 0, slot_dev = 0;   // pending bytes in the current slot and their device offset
    hipEvent_t direct_ev = nullptr;
    bool direct_pending = false;       // a DMA from the caller's pinned batch is in flight
    // the record bytes' H2D span (kpw_writer_stats [17]): timing events on the copy stream before
    // the first record DMA and after the last one (recorded at close)
    hipEvent_t h2d_ev[2] = {nullptr, nullptr};
    int h2d_marks = 0;
    // kpw_writer_write_async: the DMAs of call k may still read the caller's batch until call
    // k+1 returns (call_ev[k & 1] follows them on the copy stream)
    bool async_call = false;
    hipEvent_t call_ev[2] = {nullptr, nullptr};
    bool call_pending[2] = {false, false};
    int call_k = 0;
    // caller-side state
    int64_t num_records = 0;           // ParquetFile.numWrittenRecords
    int64_t created_ms = 0;
    int64_t failed_record = -1;
    bool closed = false;
    std::string err;
    SizeModel model;
    bool model_ok = false;             // the configuration has a size model (PARQUET_1_0)
    bool model_on = false;             // the model tracks the open row group (per-record path)
    // multi-page regime: probes of the open row group's cut pages (Engine::probe_pages) on their
    // own engine (the workers' engines may be encoding row groups meanwhile)
    Engine peng;
    DevBuf pr_off;                     // device boundaries of the fill buffer's records
    PinnedBuf pr_h;
    uint64_t fill_gen = 0, pr_gen = ~0ull;   // fill buffer generation / the one pr_off describes
    size_t pr_up = 0;                  // boundaries of that generation already on the device
    bool dirty = false;                // records appended since the last PLANNED job (model off)
    bool size_polled = false;          // getDataSize() was called on the bulk path: later write-path
                                       // jobs plan their open row group (no lazy jobs), so
                                       // each later call does not submit a planning job of its own
    bool pending_cut = false;          // an EXACT job may not be in the file yet (lastRowGroupEndPos stale)
    DevBuf probe_off;                  // write_until_full on the bulk path: offsets of staged prefixes
    PinnedBuf probe_h;
    // job scheduling (under mu): a job starts once the previous job's row-group cuts are known
    // (its carried records are placed), and appends to the file once the previous job has
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Job> q;
    uint64_t next_seq = 0;             // next job's sequence number (caller)
    uint64_t plan_seq = 0;             // first job whose cuts are not known yet
    uint64_t asm_seq = 0;              // first job not yet appended to the file
    hipEvent_t last_carry_ev = nullptr;   // carry placement of job plan_seq - 1
    int inflight = 0;
    bool stop = false;
    int fatal_st = KPW_OK;             // first failure of the pipeline (sticky)
    std::string fatal_err;
    bool invalid_seen = false;         // a worker found an invalid record (bulk path)
    bool dev_bound = false;            // hipSetDevice done in this entry call (bind_device)
    std::atomic<bool> flagged{false};  // fatal_st or invalid_seen set (read without the lock)
    int64_t invalid_global = -1;
    // shared by the workers, used in job order only
    DevBuf carry_store;
    PinnedBuf host_pages[2];           // file mode: pages on the host for the assembly thread
    int page_slot = 0;
    hipEvent_t fd2h_ev[2] = {};
    hipStream_t d2h_stream = nullptr;  // memory mode: page bodies D2H straight into the in-memory file
    std::thread assembler;
    int asm_st = KPW_OK;
    std::string asm_err;
    BatchOut asm_out;
    int64_t last_rg_end = 0;           // InternalParquetRecordWriter.lastRowGroupEndPos
    int64_t open_buffered = 0;         // open row group's buffered size after the last PLANNED job
    std::atomic<int> n_materialize{0};
    double t_open = 0, t_encode = 0, t_dma = 0, t_acquire = 0, t_asm = 0, t_d2h_alloc = 0, t_turn = 0, t_gate = 0;
    double t_probe = 0;          // page-size probes (multi-page per-record path): wall time, count, records
    double t_probe_pre = 0;      // their staging flush + offsets upload before the probe
    uint64_t n_probe = 0, probe_recs = 0;
    double stats[18] = {0};            // kpw_writer_stats (job order; read after drain)

    ~kpw_writer();
    int init_pipeline(const kpw_schema *schema, const kpw_props *props);
};

static int wfail(kpw_writer *w, int st, const std::string &m)
{
    w->err = m;
    return st;
}

// Sticky pipeline failure (any thread).  Device / I/O failures lose records already taken off
// staging, so every later call reports it (close() cannot retry them).
static void set_fatal(kpw_writer *w, int st, const std::string &m)
{
    std::lock_guard<std::mutex> g(w->mu);
    if (!w->fatal_st) { w->fatal_st = st; w->fatal_err = m; }
    w->flagged.store(true, std::memory_order_release);
    w->cv.notify_all();
}

static int check_fatal(kpw_writer *w)
{
    std::lock_guard<std::mutex> g(w->mu);
    if (w->fatal_st) {
        w->err = w->fatal_err;
        return w->fatal_st;
    }
    return KPW_OK;
}

// ---------------------------------------------------------------- stage buffers

static int alloc_buf(kpw_writer *w, StageBuf &b, size_t cap)
{
    uint8_t *nd = (uint8_t *)dev_alloc(cap);
    if (!nd) return KPW_ERR_NOMEM;
    dev_free(b.d);   // a FREE buffer: its last job synchronised before releasing it
    b.d = nd;
    b.cap = cap;
    return KPW_OK;
}

// Take a free buffer for filling (waits while the worker still holds all of them).
static int acquire_fill(kpw_writer *w)
{
    int k = -1;
    const double ta = trace_on() ? now_ms() : 0.0;
    {
        std::unique_lock<std::mutex> lk(w->mu);
        for (;;) {
            for (int i = 0; i < w->nbufs; i++)   // (not while a worker still reads its lengths)
                if (w->buf[i].state == BUF_FREE && w->buf[i].lp_state != 1) { k = i; break; }
            if (k >= 0 || w->fatal_st) break;
            w->cv.wait(lk);
        }
        if (k < 0) return w->fatal_st;
        w->buf[k].state = BUF_FILLING;
    }
    StageBuf &b = w->buf[k];
    // one read of gap_: a worker may raise it (place_carry) while this runs, and the buffer's
    // gap must be the one its capacity was sized for
    const uint64_t gap = w->gap_.load();
    const size_t need = gap + stage_flush_bytes() + (64ull << 20);
    if (b.cap < need && alloc_buf(w, b, need)) {
        std::lock_guard<std::mutex> g(w->mu);
        b.state = BUF_FREE;   // not taken: the caller has no fill buffer (w->fill stays -1)
        w->cv.notify_all();
        return wfail(w, KPW_ERR_NOMEM, "device stage buffer allocation failed");
    }
    if (trace_on()) w->t_acquire += now_ms() - ta;
    b.gap = gap;
    b.len = gap;
    b.carry.clear();
    b.carry_in_store = false;
    b.ends.clear();
    b.ncarry_expected = 0;
    b.lp_state = 0;
    b.first_new_global = w->num_records;
    w->fill = k;
    w->fill_gen++;
    return KPW_OK;
}

// Issue the H2D of the bytes pending in the current slot.
// the first record DMA of the file: the H2D span starts (kpw_writer_stats [17])
static void mark_h2d_start(kpw_writer *w)
{
    if (w->h2d_marks == 0 && w->h2d_ev[0] && hipEventRecord(w->h2d_ev[0], w->copy_stream) == hipSuccess) w->h2d_marks = 1;
}

static int flush_slot(kpw_writer *w)
{
    if (!w->slot_used) return KPW_OK;
    mark_h2d_start(w);
    const int k = w->cur_slot;
    if (hipMemcpyAsync(w->buf[w->fill].d + w->slot_dev, w->slot[k].p, w->slot_used, hipMemcpyHostToDevice, w->copy_stream) !=
            hipSuccess ||
        hipEventRecord(w->slot_ev[k], w->copy_stream) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "H2D of staged records failed");
    w->cur_slot = (k + 1) % kpw_writer::kSlots;
    w->slot_used = 0;
    return KPW_OK;
}

// Append record bytes to the fill buffer at its append position.
static int stage_bytes(kpw_writer *w, const uint8_t *src, uint64_t len, bool allow_direct = true)
{
    StageBuf &F = w->buf[w->fill];
    if (allow_direct && pinned_range(src, len)) {
        // direct DMA from the caller's pinned batch; the caller waits for it (wait_direct)
        // before the write returns, so it may reuse the batch
        if (int st = flush_slot(w)) return st;
        mark_h2d_start(w);
        // (an async call's DMAs are marked once, by call_ev at its end: every marker on the copy
        // stream costs the SDMA queue ~1 % of a 31 MB batch, tests/microbench/h2d_streams.hip)
        if (hipMemcpyAsync(F.d + F.len, src, len, hipMemcpyHostToDevice, w->copy_stream) != hipSuccess ||
            (!w->async_call && hipEventRecord(w->direct_ev, w->copy_stream) != hipSuccess))
            return wfail(w, KPW_ERR_DEVICE, "H2D of a pinned batch failed");
        w->direct_pending = true;
        F.len += len;
        return KPW_OK;
    }
    while (len) {
        if (w->slot_used == 0) {
            // reuse of this slot waits for its previous DMA
            if (w->slot[w->cur_slot].p && hipEventSynchronize(w->slot_ev[w->cur_slot]) != hipSuccess)
                return wfail(w, KPW_ERR_DEVICE, "staging slot wait failed");
            if (w->slot[w->cur_slot].ensure(kpw_writer::kSlotBytes))
                return wfail(w, KPW_ERR_NOMEM, "pinned staging allocation failed");
            w->slot_dev = F.len;
        }
        const size_t piece = std::min<uint64_t>(len, kpw_writer::kSlotBytes - w->slot_used);
        par_copy(w->slot[w->cur_slot].p + w->slot_used, src, piece);
        w->slot_used += piece;
        F.len += piece;
        src += piece;
        len -= piece;
        if (w->slot_used == kpw_writer::kSlotBytes)
            if (int st = flush_slot(w)) return st;
    }
    return KPW_OK;
}

// Make room for `bytes` more in the fill buffer.  Growing moves the buffer, so the worker
// must not be placing a carry into it: wait for the pipeline to drain first.
static int drain(kpw_writer *w);
static int grow_fill(kpw_writer *w, uint64_t bytes)
{
    StageBuf &F = w->buf[w->fill];
    if (F.len + bytes + 64 <= F.cap) return KPW_OK;
    if (int st = drain(w)) return st;
    if (int st = flush_slot(w)) return st;
    if (hipStreamSynchronize(w->copy_stream) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "staging sync failed");
    const size_t cap = std::max<size_t>(F.cap * 2, F.len + bytes + (64ull << 20));
    uint8_t *nd = (uint8_t *)dev_alloc(cap);
    if (!nd) return wfail(w, KPW_ERR_NOMEM, "device stage buffer allocation failed");
    if (F.len && hipMemcpy(nd, F.d, F.len, hipMemcpyDeviceToDevice) != hipSuccess) {
        dev_free(nd);
        return wfail(w, KPW_ERR_DEVICE, "stage buffer grow copy failed");
    }
    dev_free(F.d);
    F.d = nd;
    F.cap = cap;
    return KPW_OK;
}

// Record boundaries of a buffer's records: carried then appended ([n+1] absolute offsets).
// fn(a, b) over [0, n) split over up to 4 host threads (for large n)
template <class Fn>
static void par_for(uint64_t n, Fn fn)
{
    static const unsigned hw = std::max(1u, std::min(4u, std::thread::hardware_concurrency() / 2));
    const uint64_t kMin = 128 * 1024;
    const unsigned t = (unsigned)std::min<uint64_t>(hw, n / kMin);
    if (t <= 1) { fn(0, n); return; }
    std::thread th[4];
    const uint64_t per = (n + t - 1) / t;
    for (unsigned i = 1; i < t; i++) th[i] = std::thread(fn, std::min(n, per * i), std::min(n, per * (i + 1)));
    fn(0, std::min(n, per));
    for (unsigned i = 1; i < t; i++) th[i].join();
}

static size_t nbounds(const StageBuf &B) { return (B.carry.empty() ? 1 : B.carry.size()) + B.ends.size(); }
// (a job's worker runs this between the previous job's cuts and its own start: 7 M records are
// 56 MB into pinned memory, ~5 ms on one thread, so the appended part is copied on up to 4)
static void boundaries(const StageBuf &B, uint64_t *hb)
{
    size_t k = 0;
    if (B.carry.empty()) hb[k++] = B.gap;
    else { memcpy(hb, B.carry.data(), B.carry.size() * 8); k = B.carry.size(); }
    const uint64_t *src = B.ends.data();
    uint64_t *dst = hb + k;
    static const bool par = [] { const char *e = getenv("KPW_PAR_BOUNDS"); return !(e && e[0] == '0'); }();   // (A/B)
    if (!par) { memcpy(dst, src, B.ends.size() * 8); return; }
    par_for(B.ends.size(), [=](uint64_t a, uint64_t b) { memcpy(dst + a, src + a, (b - a) * 8); });
}
static void boundaries(const StageBuf &B, std::vector<uint64_t> &hb)
{
    hb.resize(nbounds(B));
    boundaries(B, hb.data());
}

// ---------------------------------------------------------------- workers


// A carry that did not fit its buffer's gap waits in carry_store: rebuild the buffer as
// [carried | appended] on stream `s` (the caller is not appending to it: its job runs, or it
// drains; the store was filled by the previous job, which `s` already waits for).
static int materialize(kpw_writer *w, StageBuf &B, hipStream_t s)
{
    if (!B.carry_in_store) return KPW_OK;
    w->n_materialize++;
    const uint64_t cs = B.carry.back();                 // carried bytes (store offsets start at 0)
    const uint64_t app = B.len - B.gap;
    const size_t cap = std::max<size_t>(B.cap, cs + app + w->gap_ + (64ull << 20));
    uint8_t *nd = (uint8_t *)dev_alloc(cap);
    if (!nd) return KPW_ERR_NOMEM;
    if (hipStreamWaitEvent(s, B.copied, 0) != hipSuccess ||
        hipMemcpyAsync(nd, w->carry_store.p, cs, hipMemcpyDeviceToDevice, s) != hipSuccess ||
        (app && hipMemcpyAsync(nd + cs, B.d + B.gap, app, hipMemcpyDeviceToDevice, s) != hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess) {
        dev_free(nd);
        return KPW_ERR_DEVICE;
    }
    for (auto &e : B.ends) e = e - B.gap + cs;
    dev_free(B.d);
    B.d = nd;
    B.cap = cap;
    B.len = cs + app;
    B.gap = cs;
    B.carry_in_store = false;
    return KPW_OK;
}

static bool gap_adapt()
{
    static const bool on = [] { const char *e = getenv("KPW_GAP_ADAPT"); return !(e && e[0] == '0'); }();
    return on;
}

// Place records [hb[i0], hb[i1]) of buffer `src` in front of buffer `dst`'s appended records
// (on stream s).
template <class HB>
static int place_carry(kpw_writer *w, const StageBuf &src, const HB &hb, size_t i0, size_t i1, StageBuf &dst, hipStream_t s)
{
    const uint64_t b0 = hb[i0], c = hb[i1] - b0;
    uint64_t at;
    uint8_t *base;
    // A carry larger than the gap goes through carry_store and a rebuild of the whole buffer
    // (materialize: two device copies of up to a job's bytes and a stream sync).  Open row
    // groups of wide records (C3) carry more wire bytes than 2 x blockSize, so the gap of the
    // buffers acquired from now on grows to 1.25 x the largest carry seen.
    if (c > dst.gap && gap_adapt()) {
        const uint64_t want = (c + c / 4 + (1ull << 20) - 1) & ~((1ull << 20) - 1);
        uint64_t cur = w->gap_.load();
        while (cur < want && !w->gap_.compare_exchange_weak(cur, want)) {}
    }
    if (c <= dst.gap) {
        at = dst.gap - c;
        base = dst.d;
        dst.carry_in_store = false;
    } else {
        if (w->carry_store.ensure(c + 64)) return KPW_ERR_NOMEM;
        at = 0;
        base = w->carry_store.as<uint8_t>();
        dst.carry_in_store = true;
    }
    if (c && trace_on()) fprintf(stderr, "[kpw] carry %llu B (%zu records) %s\n", (unsigned long long)c, i1 - i0,
                                 dst.carry_in_store ? "to the carry store" : "into the gap");
    if (c && hipMemcpyAsync(base + at, src.d + b0, c, hipMemcpyDeviceToDevice, s) != hipSuccess) return KPW_ERR_DEVICE;
    dst.carry.resize(i1 - i0 + 1);
    for (size_t i = i0; i <= i1; i++) dst.carry[i - i0] = hb[i] - b0 + at;
    return KPW_OK;
}

// File mode: headers + bodies + metadata of one job on the assembly thread (fwrite; overlaps
// the next job's encode).  In-memory files are assembled in HBM instead (append_job).
static void start_assembly(kpw_writer *w, BatchOut &&out, int slot)
{
    w->asm_out = std::move(out);
    w->assembler = std::thread([w, slot] {
        // no exception may leave this thread (std::terminate would kill the host process)
        try {
            (void)hipSetDevice(w->eng.device);
            if (hipEventSynchronize(w->fd2h_ev[slot]) != hipSuccess) {
                w->asm_st = KPW_ERR_DEVICE;
                w->asm_err = "D2H of pages failed";
                return;
            }
            const double ta = trace_on() ? now_ms() : 0.0;
            for (size_t r = 0; r < w->asm_out.rgs.size(); r++) {
                const int st = w->fw->write_row_group(w->asm_out, (int)r, w->host_pages[slot].p, 0);
                if (st) {
                    w->asm_st = st;
                    w->asm_err = w->fw->error();
                    return;
                }
            }
            w->last_rg_end = w->fw->pos();
            if (trace_on()) w->t_asm += now_ms() - ta;
        } catch (const std::bad_alloc &) {
            w->asm_st = KPW_ERR_NOMEM;
            w->asm_err = "file assembly: host allocation failed";
        } catch (...) {
            w->asm_st = KPW_ERR_DEVICE;
            w->asm_err = "file assembly failed";
        }
    });
}

static int join_assembly(kpw_writer *w)
{
    if (w->assembler.joinable()) w->assembler.join();
    if (w->asm_st) {
        const int st = w->asm_st;
        w->asm_st = KPW_OK;
        set_fatal(w, st, w->asm_err);
        return st;
    }
    return KPW_OK;
}

// Append one encoded job to the file, in job order (called in the job's assembly turn).
static int append_job(kpw_writer *w, Worker &W, BatchOut &out, int set)
{
    Engine &E = *W.eng;
    hipStream_t s = E.stream;
    if (out.rgs.empty()) return KPW_OK;
    const double ta = trace_on() ? now_ms() : 0.0;
    static const bool per_page_d2h = [] { const char *e = getenv("KPW_D2H_PER_PAGE"); return e && e[0] == '1'; }();
    if (w->fw->memory_mode() && per_page_d2h) {
        // headers on the host; bodies D2H straight into the in-memory file on d2h_stream, after
        // this encode; the engine's next-but-one encode reuses these page buffers after d2h_ev.
        // (Measured: ROCm runs these per-page D2H copies as blit kernels that take CUs from the
        // encode; the default below is one DMA per job plus host copies.)
        if (hipEventRecord(W.enc_done, s) != hipSuccess || hipStreamWaitEvent(w->d2h_stream, W.enc_done, 0) != hipSuccess)
            return KPW_ERR_DEVICE;
        for (size_t r = 0; r < out.rgs.size(); r++) {
            if (int st = w->fw->write_row_group(out, (int)r, out.d_pages, 0, w->d2h_stream)) return st;
            w->last_rg_end = w->fw->pos();
        }
        if (hipEventRecord(W.d2h_ev[set], w->d2h_stream) != hipSuccess) return KPW_ERR_DEVICE;
        W.d2h_used[set] = true;
        if (trace_on()) w->t_asm += now_ms() - ta;
        return KPW_OK;
    }
    if (int st = join_assembly(w)) return st;
    if (w->fw->memory_mode()) {
        // in-memory file: headers on the host, the job's bytes gathered in HBM (k_asm.hip) and
        // DMA'd straight into the file's pinned chunks; no host thread touches the page bodies
        w->fw->device_assembly(true);
        int st = KPW_OK;
        for (size_t r = 0; r < out.rgs.size() && !st; r++) st = w->fw->write_row_group(out, (int)r, out.d_pages, 0);
        w->fw->device_assembly(false);
        std::string blob;
        std::vector<FileWriter::AsmSeg> segs;
        std::vector<std::pair<uint8_t *, size_t>> spans;
        uint64_t total = 0;
        const int st2 = w->fw->take_asm(blob, segs, total, spans);
        if (st) return st;
        if (st2) return st2;
        std::vector<AsmPiece> pcs;
        pcs.reserve(segs.size() + total / 65536 + 1);
        for (const auto &g : segs)
            for (uint32_t o = 0; o < g.len; o += 65536)
                pcs.push_back({g.dst + o, g.src + o, std::min<uint32_t>(65536u, g.len - o), g.dev});
        const size_t bb = (blob.size() + 15) & ~(size_t)15, pb = pcs.size() * sizeof(AsmPiece);
        // this worker's previous assembly may still read h_asm (H2D) and write d_asm_out's
        // D2H; the device side is stream-ordered, the host buffer is not
        if (W.asm_pending) {
            if (hipEventSynchronize(W.asm_ev) != hipSuccess) return KPW_ERR_DEVICE;
            W.asm_pending = false;
        }
        if (W.h_asm.ensure(bb + pb) || W.d_asm_in.ensure(bb + pb + 16) || W.d_asm_out.ensure(total + 64)) return KPW_ERR_NOMEM;
        memcpy(W.h_asm.p, blob.data(), blob.size());
        memcpy(W.h_asm.p + bb, pcs.data(), pb);
        if (hipMemcpyAsync(W.d_asm_in.p, W.h_asm.p, bb + pb, hipMemcpyHostToDevice, s) != hipSuccess) return KPW_ERR_DEVICE;
        launch_asm_gather((const AsmPiece *)(W.d_asm_in.as<uint8_t>() + bb), (uint32_t)pcs.size(), W.d_asm_in.as<uint8_t>(),
                          W.d_asm_out.as<uint8_t>(), s);
        if (hipGetLastError() != hipSuccess) return KPW_ERR_DEVICE;
        // KPW_ASM_D2H_STREAM=1: the file bytes' D2H on the writer's D2H stream (after the gather)
        // instead of the engine stream (A/B; d_asm_out is rewritten only after asm_ev, above)
        static const bool sep = [] { const char *e = getenv("KPW_ASM_D2H_STREAM"); return e && e[0] == '1'; }();
        hipStream_t ds = s;
        if (sep) {
            if (hipEventRecord(W.enc_done, s) != hipSuccess || hipStreamWaitEvent(w->d2h_stream, W.enc_done, 0) != hipSuccess)
                return KPW_ERR_DEVICE;
            ds = w->d2h_stream;
        }
        uint64_t at = 0;
        for (const auto &sp : spans) {
            if (hipMemcpyAsync(sp.first, W.d_asm_out.as<uint8_t>() + at, sp.second, hipMemcpyDeviceToHost, ds) != hipSuccess)
                return KPW_ERR_DEVICE;
            at += sp.second;
        }
        // not waited for here: the engine's next encode reuses the page buffers after the gather
        // in stream order, and drain() (close, getDataSize after a cut) waits for the file bytes
        if (hipEventRecord(W.asm_ev, ds) != hipSuccess) return KPW_ERR_DEVICE;
        W.asm_pending = true;
        w->last_rg_end = w->fw->pos();
        if (trace_on()) w->t_d2h_alloc += now_ms() - ta;
        return KPW_OK;
    }
    // file mode: pages -> pinned host buffer in one D2H (double-buffered against the previous
    // job's assembly), headers + bodies written by fwrite on the assembly thread
    const int slot = w->page_slot;
    w->page_slot ^= 1;
    // One DMA on the engine stream.  (Measured alternatives, tests/microbench/copy_ab.sh: the
    // same copy on a separate D2H stream, or a 32-workgroup copy kernel there, which alone reaches
    // 54 GB/s, both cost 10-12 % end to end.)
    if (out.pages_len) {
        if (w->host_pages[slot].ensure(out.pages_len)) return KPW_ERR_NOMEM;
        if (hipMemcpyAsync(w->host_pages[slot].p, out.d_pages, out.pages_len, hipMemcpyDeviceToHost, s) != hipSuccess)
            return KPW_ERR_DEVICE;
    }
    // the assembly thread waits for this D2H; the engine's next encode reuses the device page
    // buffers after it in stream order, and this slot's host pages again two jobs later, after
    // this job's assembly thread was joined
    if (hipEventRecord(w->fd2h_ev[slot], s) != hipSuccess) return KPW_ERR_DEVICE;
    if (trace_on()) w->t_d2h_alloc += now_ms() - ta;
    start_assembly(w, std::move(out), slot);
    // HDFS alignment: the next row group's size limit depends on where this one ends in the file
    if (w->aligned) return join_assembly(w);
    return KPW_OK;
}

// Record offsets of a job (`count` boundaries in W.h_off) onto the device, on the engine stream
// before the encode.  PCIe is the writer's ceiling, so they cross as u32 lengths
// (lens[0] = the first boundary) and a prefix scan rebuilds the u64 offsets in HBM.  (A per-worker
// copy stream measured 3-5 % slower end to end: profiles/r02d_copy_paths.md.)
// Lengths cross in the narrowest of u8 / u16 / u32 that holds every record of the job (C2's
// ~62-byte records: 1 byte each, a quarter of the u32 bytes): u8 is tried first, and the OR of
// the lengths that pass computes picks the width when it does not fit.
static int upload_offsets(Worker &W, size_t count, hipStream_t s)
{
    const uint64_t *hb = (const uint64_t *)W.h_off.p;
    if (hb[0] >= (1ull << 32)) {   // a carried prefix of >= 4 GiB: plain u64 offsets
        if (W.d_off.ensure(count * 8)) return KPW_ERR_NOMEM;
        W.offs = W.d_off.as<uint64_t>();
        return hipMemcpyAsync(W.d_off.p, hb, count * 8, hipMemcpyHostToDevice, s) == hipSuccess ? KPW_OK : KPW_ERR_DEVICE;
    }
    if (W.h_len.ensure(count * 4) || W.d_len.ensure(count * 4) || W.d_off.ensure((count + 1) * 8)) return KPW_ERR_NOMEM;
    // Every job starts at u8 (no ratchet: one long record must not keep the worker on wide
    // lengths for the rest of the file); the u8 pass ORs the lengths, so a job that
    // does not fit goes straight to the width that holds it (at most two host passes).
    int width = W.len_width;   // 1 unless KPW_LEN_BYTES forces wider lengths (A/B)
    for (;;) {
        std::atomic<uint64_t> all_or{0};
        bool over = false;
        if (width == 4) {
            uint32_t *len = (uint32_t *)W.h_len.p;
            len[0] = (uint32_t)hb[0];
            par_for(count - 1, [=](uint64_t a, uint64_t b) { for (uint64_t i = a; i < b; i++) len[i + 1] = (uint32_t)(hb[i + 1] - hb[i]); });
        } else {
            auto narrow = [&](auto *len, uint64_t lim) {
                len[0] = 0;
                par_for(count - 1, [=, &all_or](uint64_t a, uint64_t b) {
                    uint64_t m = 0;
                    for (uint64_t i = a; i < b; i++) {
                        const uint64_t d = hb[i + 1] - hb[i];
                        m |= d;
                        len[i + 1] = (decltype(+len[0]))d;
                    }
                    all_or.fetch_or(m, std::memory_order_relaxed);
                });
                over = all_or.load() > lim;   // an OR of lengths is > lim iff some length is
            };
            if (width == 1) narrow((uint8_t *)W.h_len.p, 0xff); else narrow((uint16_t *)W.h_len.p, 0xffff);
            if (over) { width = all_or.load() <= 0xffff ? 2 : 4; continue; }
        }
        if (hipMemcpyAsync(W.d_len.p, W.h_len.p, count * width, hipMemcpyHostToDevice, s) != hipSuccess) return KPW_ERR_DEVICE;
        if (width == 4) launch_prefix_raw(W.d_len.as<uint32_t>(), count, W.d_off.as<uint64_t>(), &W.scan.sc, s);
        else launch_prefix_narrow(W.d_len.p, width, hb[0], count, W.d_off.as<uint64_t>(), &W.scan.sc, s);
        if (W.scan.sc.failed) { W.scan.sc.failed = false; return KPW_ERR_NOMEM; }
        if (hipGetLastError() != hipSuccess) return KPW_ERR_DEVICE;
        W.offs = W.d_off.as<uint64_t>() + 1;   // P[k + 1] = boundary k
        return KPW_OK;
    }
}

// KPW_PREP_LENGTHS=0: every job narrows its record lengths itself, after its turn (A/B)
static bool prep_on()
{
    static const bool on = [] { const char *e = getenv("KPW_PREP_LENGTHS"); return !(e && e[0] == '0'); }();
    return on;
}

// A job's record boundaries without copying them: the carried ones, then the appended ends.
struct HostBounds {
    const uint64_t *carry;   // carried boundaries (nc1 of them), or null: one boundary, the gap
    size_t nc1;
    uint64_t gap;
    const uint64_t *ends;
    uint64_t operator[](size_t i) const { return i < nc1 ? (carry ? carry[i] : gap) : ends[i - nc1]; }
};

// Lengths of B's appended records (ends[k] - ends[k - 1], the first from the gap) at the
// narrowest of 1 / 2 bytes that holds them (0: wider lengths, the job's own pass handles them).
static void prep_lengths(StageBuf &B)
{
    const size_t n = B.ends.size();
    B.lp_width = 0;
    if (!n || B.lp.ensure(n * 2 + 64)) return;
    const uint64_t *e = B.ends.data();
    const uint64_t g = B.gap;
    for (int width = 1; width <= 2; width++) {
        std::atomic<uint64_t> all_or{0};
        auto run = [&](auto *len) {
            par_for(n, [=, &all_or](uint64_t a, uint64_t b) {
                uint64_t m = 0, prev = a ? e[a - 1] : g;
                for (uint64_t i = a; i < b; i++) {
                    const uint64_t d = e[i] - prev;
                    prev = e[i];
                    m |= d;
                    len[i] = (decltype(+len[0]))d;
                }
                all_or.fetch_or(m, std::memory_order_relaxed);
            });
        };
        if (width == 1) run((uint8_t *)B.lp.p); else run((uint16_t *)B.lp.p);
        const uint64_t o = all_or.load();
        if (o <= (width == 1 ? 0xffull : 0xffffull)) { B.lp_width = width; return; }
        if (o > 0xffff) return;
    }
}

// upload_offsets for a job whose appended records' lengths were prepared: the carried records'
// lengths are narrowed here (a few), both parts go up in two copies.  Returns 1 when it cannot
// (no preparation, wider lengths, a forced width): the caller takes upload_offsets.
static int upload_offsets_prepped(Worker &W, const StageBuf &B, const HostBounds &hb, size_t count, hipStream_t s)
{
    const size_t nc1 = hb.nc1, nnew = count > nc1 ? count - nc1 : 0;
    if (B.lp_width == 0 || W.len_width != 1 || nnew == 0 || nnew > B.ends.size() || hb[0] >= (1ull << 32)) return 1;
    uint64_t o = 0;
    for (size_t i = 1; i < nc1; i++) o |= hb[i] - hb[i - 1];
    const int width = std::max(B.lp_width, o <= 0xff ? 1 : o <= 0xffff ? 2 : 4);
    if (width != B.lp_width) return 1;
    if (W.h_len.ensure(nc1 * width) || W.d_len.ensure(count * width + 64) || W.d_off.ensure((count + 1) * 8)) return KPW_ERR_NOMEM;
    if (width == 1) { uint8_t *l = W.h_len.p; l[0] = 0; for (size_t i = 1; i < nc1; i++) l[i] = (uint8_t)(hb[i] - hb[i - 1]); }
    else { uint16_t *l = (uint16_t *)W.h_len.p; l[0] = 0; for (size_t i = 1; i < nc1; i++) l[i] = (uint16_t)(hb[i] - hb[i - 1]); }
    if (hipMemcpyAsync(W.d_len.p, W.h_len.p, nc1 * width, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(W.d_len.as<uint8_t>() + nc1 * width, B.lp.p, nnew * width, hipMemcpyHostToDevice, s) != hipSuccess)
        return KPW_ERR_DEVICE;
    launch_prefix_narrow(W.d_len.p, width, hb[0], count, W.d_off.as<uint64_t>(), &W.scan.sc, s);
    if (W.scan.sc.failed) { W.scan.sc.failed = false; return KPW_ERR_NOMEM; }
    if (hipGetLastError() != hipSuccess) return KPW_ERR_DEVICE;
    W.offs = W.d_off.as<uint64_t>() + 1;   // P[k + 1] = boundary k
    return KPW_OK;
}

static int run_job(kpw_writer *w, int x, const Job &j, hipEvent_t prev_carry)
{
    Worker &W = w->wk[x];
    Engine &E = *W.eng;
    StageBuf &B = w->buf[j.buf];
    hipStream_t s = E.stream;
    bool planned = false;
    const double t_in = trace_on() ? now_ms() : 0.0;
    double t_planned = 0.0, t_up = 0.0;
    auto plan_fail = [&](int st, const std::string &m) {
        set_fatal(w, st, m);
        return st;
    };
    // the previous job's carried records (and a carry_store it filled) come first
    if (prev_carry && hipStreamWaitEvent(s, prev_carry, 0) != hipSuccess) return plan_fail(KPW_ERR_DEVICE, "stream wait failed");
    {   // a worker may still be preparing this buffer's lengths (it reads B.ends)
        std::unique_lock<std::mutex> lk(w->mu);
        w->cv.wait(lk, [&] { return B.lp_state != 1; });
    }
    // admitted with the device's other writers' jobs in arrival order (memcache.h EncodeGate);
    // released once this job's encode has completed, before its turn to append
    EncodeGate gate(E.device);
    {
        std::lock_guard<std::mutex> g(w->mu);
        w->t_gate += gate.waited_ms();
    }
    if (int st = materialize(w, B, s)) return plan_fail(st, "stage buffer rebuild failed");
    bool after_invalid;
    {
        std::lock_guard<std::mutex> g(w->mu);
        after_invalid = w->invalid_seen;
    }
    if (after_invalid) { B.ends.clear(); B.len = B.gap; }   // records behind an invalid one are never written
    const size_t nb = nbounds(B);
    const HostBounds hb{B.carry.empty() ? nullptr : B.carry.data(), B.carry.empty() ? (size_t)1 : B.carry.size(), B.gap,
                        B.ends.data()};
    const int64_t nrec = (int64_t)nb - 1;
    const int64_t ncarry = B.carry.empty() ? 0 : (int64_t)B.carry.size() - 1;
    const int64_t n_enc = j.kind == JOB_EXACT ? std::min<int64_t>(j.n_exact, nrec) : nrec;
    const double t0 = now_ms();
    if (hipStreamWaitEvent(s, B.copied, 0) != hipSuccess) return plan_fail(KPW_ERR_DEVICE, "stream wait failed");
    const int set = (int)(W.njobs & 1);
    if (w->fw->memory_mode() && n_enc > 0) {
        // the page buffers this encode gets back were last read by the D2H of this engine's
        // job before last
        E.swap_page_buffers();
        for (int k = 0; k < 2; k++)
            if (W.d2h_used[k] && (k == set || E.multi_page()) && hipStreamWaitEvent(s, W.d2h_ev[k], 0) != hipSuccess)
                return plan_fail(KPW_ERR_DEVICE, "stream wait failed");
    }
    // the row-group cuts: carried records -> the next buffer, then the next job may start
    int64_t consumed = 0, keep_end = nrec;
    auto on_plan = [&](const BatchOut &o) {
        consumed = o.records_consumed;
        int64_t inv = -1;
        if (o.invalid_record >= 0) { keep_end = o.invalid_record; inv = B.first_new_global - ncarry + o.invalid_record; }
        if (j.kind == JOB_FINAL) keep_end = consumed;
        int st = KPW_OK;
        if (keep_end > consumed && j.next >= 0)
            st = place_carry(w, B, hb, (size_t)consumed, (size_t)keep_end, w->buf[j.next], s);
        if (!st && hipEventRecord(W.carry_ev, s) != hipSuccess) st = KPW_ERR_DEVICE;
        std::lock_guard<std::mutex> g(w->mu);
        if (st) {
            if (!w->fatal_st) { w->fatal_st = st; w->fatal_err = "carry-over copy failed"; }
            w->flagged.store(true, std::memory_order_release);
        } else if (inv >= 0) {
            w->invalid_seen = true;
            w->invalid_global = inv;
            w->flagged.store(true, std::memory_order_release);
        }
        w->last_carry_ev = W.carry_ev;
        w->plan_seq = j.seq + 1;
        planned = true;
        if (trace_on()) t_planned = now_ms();
        w->cv.notify_all();
    };
    BatchOut out;
    if (n_enc > 0) {
        int st2 = B.lp_state == 2 && !after_invalid ? upload_offsets_prepped(W, B, hb, (size_t)n_enc + 1, s) : 1;
        if (st2 == 1) {   // boundaries into the pinned offset buffer, lengths narrowed here
            if (W.h_off.ensure(nb * 8)) return plan_fail(KPW_ERR_NOMEM, "offset staging allocation failed");
            boundaries(B, (uint64_t *)W.h_off.p);
            st2 = upload_offsets(W, (size_t)n_enc + 1, s);
        }
        if (st2) return plan_fail(st2, "H2D of offsets failed");
        if (trace_on()) t_up = now_ms();
        // EXACT jobs are encoded non-final: the GPU planner must cut the same single row group
        // the host size model cut (checked below), so every such row group cross-checks the model
        E.on_plan = on_plan;
        E.lazy_open = j.lazy;
        const int st = E.encode(B.d, W.offs, (uint64_t)n_enc, j.kind == JOB_FINAL, E.props.block_size, nullptr, out);
        E.on_plan = nullptr;
        E.lazy_open = false;
        if (st) return plan_fail(st, E.error());
    } else {
        on_plan(out);
    }
    if (!planned) return plan_fail(KPW_ERR_DEVICE, "encode returned without a plan");
    const double t1 = now_ms();
    if (out.invalid_record < 0 && j.kind == JOB_EXACT && (consumed != n_enc || out.rgs.size() != 1))
        // the host size model and the GPU planner restate the same cut: a mismatch is a bug
        return plan_fail(KPW_ERR_DEVICE, "row-group cut of the size model and the GPU planner differ");
    if (hipStreamSynchronize(s) != hipSuccess) return plan_fail(KPW_ERR_DEVICE, "encode sync failed");
    gate.release();
    {
        std::lock_guard<std::mutex> g(w->mu);
        B.state = BUF_FREE;   // the carried records were copied out before the rest of the encode
        w->cv.notify_all();
    }
    // append to the file in job order
    {
        const double ta = trace_on() ? now_ms() : 0.0;
        std::unique_lock<std::mutex> lk(w->mu);
        w->cv.wait(lk, [&] { return w->asm_seq == j.seq || w->fatal_st; });
        if (w->fatal_st) return w->fatal_st;
        if (trace_on()) w->t_turn += now_ms() - ta;
    }
    for (const PageOut &pg : out.pages) {
        w->stats[3] += (double)pg.uncompressed_size;
        w->stats[4] += (double)pg.compressed_size;
    }
    if (n_enc > 0) {
        w->stats[0] += 1;
        w->stats[1] += (double)n_enc;
        w->stats[2] += (double)(hb[n_enc] - hb[0]);
        for (int k = 0; k < 10; k++) w->stats[5 + k] += E.stage_ms[k];
        w->stats[15] += t1 - t0;
        w->stats[16] += E.lb_fallbacks;
        W.njobs++;
    }
    if (j.kind == JOB_PLANNED) w->open_buffered = out.open_buffered;
    w->t_encode += t1 - t0;
    const double tq = trace_on() ? now_ms() : 0.0;
    if (int st = append_job(w, W, out, set)) return plan_fail(st, "file assembly failed: " + w->fw->error());
    if (trace_on())
        fprintf(stderr, "[kpw] job %llu worker %d kind=%d records=%lld (carried %lld) encode %.2f ms; at %.1f: turn to plan "
                        "(buffer + boundaries %.1f), start, offsets up %.1f, cuts known %.1f, encoded %.1f, turn %.1f, appended %.1f\n",
                (unsigned long long)j.seq, x, j.kind, (long long)n_enc, (long long)ncarry, t1 - t0, t_in - w->t_open,
                t0 - t_in, t_up ? t_up - w->t_open : 0.0, t_planned ? t_planned - w->t_open : 0.0, t1 - w->t_open,
                tq - w->t_open, now_ms() - w->t_open);
    {
        std::lock_guard<std::mutex> g(w->mu);
        w->asm_seq = j.seq + 1;
        w->cv.notify_all();
    }
    return KPW_OK;
}

// HDFS block alignment (props.dfs_block_size > 0: ParquetFileWriter's PaddingAlignment).
// Each row group's size limit is min(blockSize, bytes left in the HDFS block after the row
// group before it) (InternalParquetRecordWriter.flushRowGroupToStore: nextRowGroupSize), so a
// cut depends on the compressed bytes of every row group before it.  One worker; the job's
// row groups are planned and encoded one at a time (the planner stops after one cut), and
// each is in the file before the next limit is read from the file position.
static int run_job_aligned(kpw_writer *w, const Job &j, hipEvent_t prev_carry)
{
    Worker &W = w->wk[0];
    Engine &E = *W.eng;
    StageBuf &B = w->buf[j.buf];
    hipStream_t s = E.stream;
    auto jfail = [&](int st, const std::string &m) {
        set_fatal(w, st, m);
        return st;
    };
    if (prev_carry && hipStreamWaitEvent(s, prev_carry, 0) != hipSuccess) return jfail(KPW_ERR_DEVICE, "stream wait failed");
    EncodeGate gate(E.device);   // (the job's row groups one at a time: the slot is held throughout)
    w->t_gate += gate.waited_ms();
    if (int st = materialize(w, B, s)) return jfail(st, "stage buffer rebuild failed");
    bool after_invalid;
    {
        std::lock_guard<std::mutex> g(w->mu);
        after_invalid = w->invalid_seen;
    }
    if (after_invalid) { B.ends.clear(); B.len = B.gap; }
    const size_t nb = nbounds(B);
    if (W.h_off.ensure(nb * 8)) return jfail(KPW_ERR_NOMEM, "offset staging allocation failed");
    uint64_t *hb = (uint64_t *)W.h_off.p;
    boundaries(B, hb);
    const int64_t nrec = (int64_t)nb - 1;
    const int64_t ncarry = B.carry.empty() ? 0 : (int64_t)B.carry.size() - 1;
    int64_t lim = j.kind == JOB_EXACT ? std::min<int64_t>(j.n_exact, nrec) : nrec;
    if (hipStreamWaitEvent(s, B.copied, 0) != hipSuccess) return jfail(KPW_ERR_DEVICE, "stream wait failed");
    if (lim > 0) {
        if (int st2 = upload_offsets(W, (size_t)lim + 1, s)) return jfail(st2, "H2D of offsets failed");
    }
    {   // file order (one worker: the previous job is in the file already)
        std::unique_lock<std::mutex> lk(w->mu);
        w->cv.wait(lk, [&] { return w->asm_seq == j.seq || w->fatal_st; });
        if (w->fatal_st) return w->fatal_st;
    }
    int64_t s0 = 0, inv = -1;
    if (j.kind == JOB_PLANNED) w->open_buffered = 0;
    while (s0 < lim) {
        const int64_t T = w->fw->next_row_group_size();
        const int set = (int)(W.njobs & 1);
        if (w->fw->memory_mode()) {
            E.swap_page_buffers();
            for (int k = 0; k < 2; k++)
                if (W.d2h_used[k] && (k == set || E.multi_page()) && hipStreamWaitEvent(s, W.d2h_ev[k], 0) != hipSuccess)
                    return jfail(KPW_ERR_DEVICE, "stream wait failed");
        }
        const double t0 = now_ms();
        BatchOut out;
        E.max_cuts = 1;
        const int st = E.encode(B.d, W.offs + s0, (uint64_t)(lim - s0), j.kind == JOB_FINAL, T, nullptr, out);
        E.max_cuts = 0;
        if (st) return jfail(st, E.error());
        W.njobs++;   // page buffer sets alternate per encode
        if (out.invalid_record >= 0) {
            // records from the invalid one on are never written (KafkaProtoParquetWriter.java:270-276)
            lim = s0 + out.invalid_record;
            inv = B.first_new_global - ncarry + lim;
        }
        if (inv < 0 && j.kind == JOB_EXACT && (out.records_consumed != lim - s0 || out.rgs.size() != 1))
            return jfail(KPW_ERR_DEVICE, "row-group cut of the size model and the GPU planner differ");
        if (hipStreamSynchronize(s) != hipSuccess) return jfail(KPW_ERR_DEVICE, "encode sync failed");
        const double t1 = now_ms();
        for (const PageOut &pg : out.pages) {
            w->stats[3] += (double)pg.uncompressed_size;
            w->stats[4] += (double)pg.compressed_size;
        }
        w->stats[0] += 1;
        w->stats[1] += (double)out.records_consumed;
        w->stats[2] += (double)(hb[s0 + out.records_consumed] - hb[s0]);
        for (int k = 0; k < 10; k++) w->stats[5 + k] += E.stage_ms[k];
        w->stats[15] += t1 - t0;
        w->stats[16] += E.lb_fallbacks;
        w->t_encode += t1 - t0;
        if (out.rgs.empty()) {   // no cut in [s0, lim): the open row group
            if (j.kind == JOB_PLANNED) w->open_buffered = out.open_buffered;
            break;
        }
        s0 += out.records_consumed;
        if (int st2 = append_job(w, W, out, set)) return jfail(st2, "file assembly failed: " + w->fw->error());
        if (trace_on())
            fprintf(stderr, "[kpw] job %llu row group at %lld: %lld records, limit %lld, file at %lld\n",
                    (unsigned long long)j.seq, (long long)(s0 - out.records_consumed), (long long)out.records_consumed,
                    (long long)T, (long long)w->fw->pos());
    }
    // the open row group -> the next buffer; then the next job may start
    int st = KPW_OK;
    if (j.kind != JOB_FINAL && lim > s0 && j.next >= 0) st = place_carry(w, B, hb, (size_t)s0, (size_t)lim, w->buf[j.next], s);
    if (!st && hipEventRecord(W.carry_ev, s) != hipSuccess) st = KPW_ERR_DEVICE;
    if (!st && hipStreamSynchronize(s) != hipSuccess) st = KPW_ERR_DEVICE;
    if (st) return jfail(st, "carry-over copy failed");
    std::lock_guard<std::mutex> g(w->mu);
    if (inv >= 0) {
        w->invalid_seen = true;
        w->invalid_global = inv;
        w->flagged.store(true, std::memory_order_release);
    }
    w->last_carry_ev = W.carry_ev;
    w->plan_seq = j.seq + 1;
    B.state = BUF_FREE;
    w->asm_seq = j.seq + 1;
    w->cv.notify_all();
    return KPW_OK;
}

static void worker_main(kpw_writer *w, int x)
{
    (void)hipSetDevice(w->eng.device);
    Worker &W = w->wk[x];
    StreamOrder order(W.eng->stream);   // this worker's buffers are used on its engine stream
    for (;;) {
        Job j;
        hipEvent_t prev_carry;
        {
            std::unique_lock<std::mutex> lk(w->mu);
            // the next job starts once the previous job's cuts are known; meanwhile a waiting
            // worker narrows a queued job's appended record lengths (prep_lengths)
            for (;;) {
                if ((w->stop && w->q.empty()) || (!w->q.empty() && w->q.front().seq == w->plan_seq)) break;
                StageBuf *pb = nullptr;
                if (!w->aligned && prep_on())
                    for (const Job &qj : w->q)
                        if (w->buf[qj.buf].lp_state == 0) { pb = &w->buf[qj.buf]; break; }
                if (pb) {
                    pb->lp_state = 1;
                    lk.unlock();
                    prep_lengths(*pb);
                    lk.lock();
                    pb->lp_state = 2;
                    w->cv.notify_all();
                    continue;
                }
                w->cv.wait(lk);
            }
            if (w->q.empty()) break;   // stop requested and nothing queued
            j = w->q.front();
            w->q.pop_front();
            prev_carry = j.seq ? w->last_carry_ev : nullptr;
            W.busy = true;
            w->inflight++;
        }
        bool failed;
        {
            std::lock_guard<std::mutex> g(w->mu);
            failed = w->fatal_st != KPW_OK;
        }
        try {
            if (!failed) (void)(w->aligned ? run_job_aligned(w, j, prev_carry) : run_job(w, x, j, prev_carry));
        } catch (const std::bad_alloc &) {
            set_fatal(w, KPW_ERR_NOMEM, "host allocation failed in an encode worker");
        } catch (...) {
            set_fatal(w, KPW_ERR_DEVICE, "encode worker failed");
        }
        {
            std::lock_guard<std::mutex> g(w->mu);
            if (w->fatal_st) {
                // nothing after a failure is encoded: release its buffers, let every job pass
                for (auto &k : w->buf) if (k.state == BUF_QUEUED) k.state = BUF_FREE;
                w->buf[j.buf].state = BUF_FREE;
                for (auto &q : w->q) w->plan_seq = std::max(w->plan_seq, q.seq + 1);
                w->q.clear();
                w->plan_seq = std::max(w->plan_seq, j.seq + 1);
                w->asm_seq = std::max(w->asm_seq, j.seq + 1);
            }
            W.busy = false;
            w->inflight--;
            w->cv.notify_all();
        }
    }
}

// Hand the fill buffer to the workers and start filling the next one.
static int submit(kpw_writer *w, int kind, int64_t n_exact, bool exact_open = false)
{
    if (int st = flush_slot(w)) return st;
    StageBuf &F = w->buf[w->fill];
    if (hipEventRecord(F.copied, w->copy_stream) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "event record failed");
    const int f = w->fill;
    const int64_t nrec = F.ncarry_expected + (int64_t)F.ends.size();
    int next = -1;
    if (kind != JOB_FINAL) {
        w->fill = -1;
        {
            std::lock_guard<std::mutex> g(w->mu);
            F.state = BUF_QUEUED;
        }
        if (int st = acquire_fill(w)) {
            // F's records were accepted by earlier writes and cannot be encoded now: sticky,
            // so every later write / getDataSize / close reports it instead of a short file
            {
                std::lock_guard<std::mutex> g(w->mu);
                F.state = BUF_FREE;
            }
            set_fatal(w, st, "stage buffer for the next records unavailable: " + w->err);
            return st;
        }
        next = w->fill;
        w->buf[next].ncarry_expected = kind == JOB_EXACT ? nrec - n_exact : 0;
    } else {
        std::lock_guard<std::mutex> g(w->mu);
        F.state = BUF_QUEUED;
        w->fill = -1;
    }
    {
        std::lock_guard<std::mutex> g(w->mu);
        if (trace_on())
            fprintf(stderr, "[kpw] submit job %llu kind=%d new records=%lld (%.0f MiB) at %.1f ms, %d in flight, %d queued\n",
                    (unsigned long long)w->next_seq, kind, (long long)F.ends.size(), (F.len - F.gap) / 1048576.0,
                    now_ms() - w->t_open, w->inflight, (int)w->q.size());
        w->q.push_back(Job{f, kind, next, n_exact, w->next_seq++, kind == JOB_PLANNED && !exact_open && !w->size_polled});
        w->cv.notify_all();
    }
    if (kind == JOB_PLANNED) w->dirty = false;
    return KPW_OK;
}

// Wait until every submitted job is encoded and in the file (memory mode: its pages landed).
static int drain(kpw_writer *w)
{
    {
        std::unique_lock<std::mutex> lk(w->mu);
        w->cv.wait(lk, [w] { return w->q.empty() && w->inflight == 0; });
    }
    // no job runs now: the file-mode assembly thread and the D2H stream are the caller's
    (void)join_assembly(w);
    for (int x = 0; x < w->nworkers; x++) {   // in-memory files: the last jobs' bytes have landed
        Worker &W = w->wk[x];
        if (W.asm_pending) {
            if (hipEventSynchronize(W.asm_ev) != hipSuccess) set_fatal(w, KPW_ERR_DEVICE, "D2H of pages failed");
            W.asm_pending = false;
        }
    }
    if (w->d2h_stream && hipStreamSynchronize(w->d2h_stream) != hipSuccess) set_fatal(w, KPW_ERR_DEVICE, "D2H of pages failed");
    std::lock_guard<std::mutex> g(w->mu);
    if (w->fatal_st) {
        w->err = w->fatal_err;
        return w->fatal_st;
    }
    return KPW_OK;
}

static uint64_t env_workers()
{
    const char *e = getenv("KPW_ENCODERS");
    const long v = e ? atol(e) : 2;
    return v == 1 ? 1 : v >= 3 ? 3 : 2;
}

int kpw_writer::init_pipeline(const kpw_schema *schema, const kpw_props *props)
{
    if (hipSetDevice(eng.device) != hipSuccess) return KPW_ERR_DEVICE;
    nworkers = (int)env_workers();
    aligned = props->dfs_block_size > 0 && props->max_padding_size > 0;
    if (aligned) nworkers = 1;   // each row group's limit follows the file position after the one before
    nbufs = nworkers >= 3 ? 5 : 4;
    if (nworkers > 1) {
        if (int st = eng1.init(eng.device, schema, props)) return st;
    }
    if (nworkers > 2) {
        if (int st = eng2.init(eng.device, schema, props)) return st;
    }
    wk[0].eng = &eng;
    wk[1].eng = &eng1;
    wk[2].eng = &eng2;
    copy_stream = sset.s[2];
    d2h_stream = sset.s[3];
    for (auto &e : slot_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
    for (auto &e : fd2h_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
    if (hipEventCreateWithFlags(&direct_ev, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
    for (auto &e : h2d_ev)
        if (hipEventCreate(&e) != hipSuccess) return KPW_ERR_DEVICE;
    for (auto &e : call_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
    for (auto &b : buf)
        if (hipEventCreateWithFlags(&b.copied, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
    for (int x = 0; x < nworkers; x++) {
        Worker &W = wk[x];
        if (hipEventCreateWithFlags(&W.carry_ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&W.enc_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&W.d2h_ev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&W.d2h_ev[1], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&W.asm_ev, hipEventDisableTiming) != hipSuccess)
            return KPW_ERR_DEVICE;
    }
    // the open row group of a job lands in the next buffer's gap (its wire bytes are a small
    // multiple of its buffered size for every schema but pathological ones; see materialize)
    gap_ = std::max<uint64_t>(64ull << 20, 2 * (uint64_t)eng.props.block_size) + 4096;
    model_ok = model.init(eng.cols, eng.props);
    model_on = model_ok;
    if (model_ok && model.multi_page()) {
        if (int st = peng.init(eng.device, schema, props)) return st;
    }
    {   // KPW_LEN_BYTES=4: record lengths always cross as u32 (A/B of the narrow lengths)
        const char *e = getenv("KPW_LEN_BYTES");
        const int lw = e && (atoi(e) == 2 || atoi(e) == 4) ? atoi(e) : 1;
        for (int x = 0; x < nworkers; x++) wk[x].len_width = lw;
    }
    for (int x = 0; x < nworkers; x++) wk[x].th = std::thread(worker_main, this, x);
    return acquire_fill(this);
}

kpw_writer::~kpw_writer()
{
    const double tf0 = trace_on() ? now_ms() : 0.0;
    double tf[5] = {0, 0, 0, 0, 0};
    {
        std::lock_guard<std::mutex> g(mu);
        stop = true;
        cv.notify_all();
    }
    for (auto &W : wk)
        if (W.th.joinable()) W.th.join();
    if (assembler.joinable()) assembler.join();
    if (trace_on()) tf[0] = now_ms();
    (void)hipSetDevice(eng.device);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    if (d2h_stream) (void)hipStreamSynchronize(d2h_stream);
    if (eng.stream) (void)hipStreamSynchronize(eng.stream);
    if (eng1.stream) (void)hipStreamSynchronize(eng1.stream);
    if (eng2.stream) (void)hipStreamSynchronize(eng2.stream);
    if (trace_on()) tf[1] = now_ms();
    for (auto &b : buf) {
        dev_free(b.d);
        if (b.copied) (void)hipEventDestroy(b.copied);
    }
    for (auto &e : slot_ev) if (e) (void)hipEventDestroy(e);
    for (auto &e : h2d_ev) if (e) (void)hipEventDestroy(e);
    for (auto &e : fd2h_ev) if (e) (void)hipEventDestroy(e);
    for (auto &W : wk) {
        for (hipEvent_t e : {W.carry_ev, W.enc_done, W.d2h_ev[0], W.d2h_ev[1], W.asm_ev}) if (e) (void)hipEventDestroy(e);
    }
    if (direct_ev) (void)hipEventDestroy(direct_ev);
    for (auto &e : call_ev) if (e) (void)hipEventDestroy(e);
    if (trace_on()) tf[2] = now_ms();
    // (the stream set goes back to the pool once the engines are gone: StreamSetOwner)
    if (trace_on()) tf[3] = now_ms();
    delete fw;
    if (trace_on()) {
        tf[4] = now_ms();
        fprintf(stderr, "[kpw] free: joins %.1f ms, syncs %.1f ms, buffers+events %.1f ms, streams %.1f ms, file %.1f ms\n",
                tf[0] - tf0, tf[1] - tf[0], tf[2] - tf[1], tf[3] - tf[2], tf[4] - tf[3]);
    }
}

// ---------------------------------------------------------------- C-ABI

extern "C" void *kpw_host_alloc(uint64_t bytes, int *status)
{
    void *p = bytes ? pin_alloc(bytes) : nullptr;
    if (!p) {
        if (status) *status = bytes ? KPW_ERR_NOMEM : KPW_ERR_INVALID_ARG;
        return nullptr;
    }
    if (status) *status = KPW_OK;
    return p;
}

extern "C" void kpw_host_free(void *p)
{
    pin_free(p);   // kept pinned for the next kpw_host_alloc
}

extern "C" kpw_writer *kpw_writer_open(int device, const kpw_schema *schema, const kpw_props *props, const char *path, int *status)
{
    try {
        kpw_writer *w = new kpw_writer();
        const int ns = env_workers() >= 3 ? 5 : 4;
        int st = hipSetDevice(device) == hipSuccess && stream_set_acquire(ns, w->sset.s) == hipSuccess ? KPW_OK : KPW_ERR_DEVICE;
        if (!st) w->sset.n = ns;
        w->eng.given_stream = w->sset.s[0];
        w->eng1.given_stream = w->sset.s[1];
        w->eng2.given_stream = w->sset.s[4];   // (null with four streams: eng2 is not used)
        if (!st) st = w->eng.init(device, schema, props);
        if (!st) {
            w->fw = new FileWriter(w->eng.cols, w->eng.message_name, w->eng.proto_class, w->eng.props);
            st = w->fw->open(path);
        }
        if (!st) st = w->init_pipeline(schema, props);
        if (st) {
            if (status) *status = st;
            delete w;
            return nullptr;
        }
        w->t_open = now_ms();
        w->created_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::system_clock::now().time_since_epoch()).count();
        if (status) *status = KPW_OK;
        return w;
    } catch (const std::bad_alloc &) {
        if (status) *status = KPW_ERR_NOMEM;
    } catch (...) {
        if (status) *status = KPW_ERR_DEVICE;
    }
    return nullptr;
}

// A reported pipeline failure; an invalid record found by the worker (bulk path) also fixes
// the record count: it and everything after it were never written.
static int observe_failure(kpw_writer *w)
{
    // per-record calls (write + getDataSize per record) skip the lock while no worker has
    // flagged a failure and the caller's own thread recorded none
    if (!w->flagged.load(std::memory_order_acquire) && w->failed_record < 0) return KPW_OK;
    std::lock_guard<std::mutex> g(w->mu);
    if (w->invalid_seen && w->failed_record < 0) {
        w->failed_record = w->invalid_global;
        w->num_records = w->invalid_global;
    }
    if (w->fatal_st) {
        w->err = w->fatal_err;
        return w->fatal_st;
    }
    if (w->failed_record >= 0) {
        w->err = "Invalid proto message received (record " + std::to_string(w->failed_record) + ")";
        return KPW_ERR_INVALID_PROTO;
    }
    return KPW_OK;
}


// Wait for a direct DMA from the caller's pinned batch (issued by stage_bytes).
static int wait_direct(kpw_writer *w)
{
    if (!w->direct_pending) return KPW_OK;
    const double ta = trace_on() ? now_ms() : 0.0;
    w->direct_pending = false;
    if (hipEventSynchronize(w->direct_ev) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "H2D of a pinned batch failed");
    if (trace_on()) w->t_dma += now_ms() - ta;
    return KPW_OK;
}

// Every batch an earlier kpw_writer_write_async may still be reading is released (its DMAs are
// done): called by every entry point except the async write itself.
static int release_batches(kpw_writer *w)
{
    for (int k = 0; k < 2; k++) {
        if (!w->call_pending[k]) continue;
        const double ta = trace_on() ? now_ms() : 0.0;
        w->call_pending[k] = false;
        if (hipEventSynchronize(w->call_ev[k]) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "H2D of a pinned batch failed");
        if (trace_on()) w->t_dma += now_ms() - ta;
    }
    return KPW_OK;
}

// End of an async write: the DMAs this call issued are marked by call_ev[call_k]; the previous
// call's batch is released (waited for) now, so the copy stream always has the next batch
// queued behind the current one.
static int finish_async_call(kpw_writer *w)
{
    const int k = w->call_k;
    if (w->direct_pending) {
        w->direct_pending = false;
        if (hipEventRecord(w->call_ev[k], w->copy_stream) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "event record failed");
        w->call_pending[k] = true;
    }
    w->call_k ^= 1;
    if (w->call_pending[k ^ 1]) {
        const double ta = trace_on() ? now_ms() : 0.0;
        w->call_pending[k ^ 1] = false;
        if (hipEventSynchronize(w->call_ev[k ^ 1]) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "H2D of a pinned batch failed");
        if (trace_on()) w->t_dma += now_ms() - ta;
    }
    return KPW_OK;
}

// Rewind the fill buffer's append position to `new_len` (records after it were not accepted).
// Bytes still pending in the current slot are dropped with it; bytes already sent are simply
// overwritten by later appends (same copy stream, in order).
static void rewind_fill(kpw_writer *w, uint64_t new_len)
{
    StageBuf &F = w->buf[w->fill];
    if (w->slot_used) w->slot_used = new_len > w->slot_dev ? std::min<uint64_t>(w->slot_used, new_len - w->slot_dev) : 0;
    F.len = new_len;
}

// One record through the pinned slot (the size-model path: small writes).
static int stage_record(kpw_writer *w, const uint8_t *src, uint64_t len)
{
    if (w->slot_used + len > kpw_writer::kSlotBytes || w->slot_used == 0) return stage_bytes(w, src, len, false);
    StageBuf &F = w->buf[w->fill];
    memcpy(w->slot[w->cur_slot].p + w->slot_used, src, len);
    w->slot_used += len;
    F.len += len;
    return KPW_OK;
}

// boundary i of a buffer's records (carried, then appended), as boundaries() lays them out
static uint64_t boundary_at(const StageBuf &B, size_t i)
{
    if (B.carry.empty()) return i == 0 ? B.gap : B.ends.data()[i - 1];
    return i < B.carry.size() ? B.carry[i] : B.ends.data()[i - B.carry.size()];
}

// Multi-page regime: the pages every column cut in the open row group up to its record m - 1,
// and their header + compressed bytes (ColumnChunkPageWriter.getMemSize), from a GPU encode of
// the open row group's first m records.  In the model path those are the fill buffer's first m
// records (an EXACT job leaves the next buffer with no carried records; a resynchronisation
// materialises its carried ones in place first).
static int probe_flushed(kpw_writer *w, size_t m, std::vector<int32_t> &np, std::vector<int64_t> &fl)
{
    const double tp0 = trace_on() ? now_ms() : 0.0;
    StageBuf &F = w->buf[w->fill];
    Engine &P = w->peng;
    StreamOrder order(P.stream);
    if (int st = flush_slot(w)) return st;
    if (hipEventRecord(F.copied, w->copy_stream) != hipSuccess || hipStreamWaitEvent(P.stream, F.copied, 0) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "probe: staging order failed");
    // boundaries [0, m] on the device, uploaded incrementally (records are only appended)
    if (w->pr_gen != w->fill_gen) { w->pr_gen = w->fill_gen; w->pr_up = 0; }
    const size_t nb = m + 1;
    if (nb * 8 > w->pr_off.cap) {
        if (w->pr_off.ensure(std::max<size_t>(nb * 16, 1u << 20))) return wfail(w, KPW_ERR_NOMEM, "probe offsets");
        w->pr_up = 0;
    }
    if (nb > w->pr_up) {
        const size_t k = nb - w->pr_up;
        if (w->pr_h.ensure(k * 8)) return wfail(w, KPW_ERR_NOMEM, "probe offsets");
        uint64_t *h = (uint64_t *)w->pr_h.p;
        for (size_t i = 0; i < k; i++) h[i] = boundary_at(F, w->pr_up + i);
        if (hipMemcpyAsync(w->pr_off.as<uint64_t>() + w->pr_up, h, k * 8, hipMemcpyHostToDevice, P.stream) != hipSuccess)
            return wfail(w, KPW_ERR_DEVICE, "probe: H2D of offsets failed");
        w->pr_up = nb;
    }
    // only the columns that cut a page since the last probe are encoded (the others' cut pages,
    // hence their flushed bytes, are unchanged)
    std::vector<char> mask;
    w->model.cut_columns(mask);
    std::vector<std::vector<int64_t>> cuts;   // the model's page cuts: the probe skips the GPU's page-cut pass
    w->model.page_cuts(cuts);
    const double tp = trace_on() ? now_ms() : 0.0;
    if (int st = P.probe_pages(F.d, w->pr_off.as<uint64_t>(), m, np, fl, &mask, w->fill_gen, &cuts))
        return wfail(w, st, P.error());
    if (trace_on()) { w->t_probe += now_ms() - tp; w->t_probe_pre += tp - tp0; w->n_probe++; w->probe_recs += m; }
    return KPW_OK;
}

// A record the model reported PAGES for: its row-group check with the cut pages' sizes.
static int model_pages(kpw_writer *w, size_t m, int &r)
{
    std::vector<int32_t> np;
    std::vector<int64_t> fl;
    if (int st = probe_flushed(w, m, np, fl)) {
        set_fatal(w, st, "page-size probe failed: " + w->err);   // the record is staged: no retry
        return st;
    }
    r = w->model.finish_pages(np, fl);
    if (r == SizeModel::MISMATCH) {
        set_fatal(w, KPW_ERR_DEVICE, "page cuts of the size model and the GPU differ");
        return KPW_ERR_DEVICE;
    }
    return KPW_OK;
}

// write / write_until_full with the size model on: records go one by one through the model
// (O(columns) each, plus a GPU probe of the open row group when a column cuts a page) and the
// slot; an invalid record stops the batch right there (the reference throws at parseFrom,
// KafkaProtoParquetWriter.java:270-276); a row-group cut hands the fill buffer, which then
// holds exactly that row group, to the worker.
// The calling thread's current device, set once per entry call and only when it issues device
// work: hipSetDevice costs ~70 ns (r06s), more than half of what the per-record loop's write
// otherwise spends per record.
static int bind_device(kpw_writer *w)
{
    if (w->dev_bound) return KPW_OK;
    if (hipSetDevice(w->eng.device) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "hipSetDevice failed");
    w->dev_bound = true;
    return KPW_OK;
}

static int write_modelled(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n, int64_t max_file_size,
                          uint64_t *n_accepted, int *full)
{
    uint64_t i = 0;
    int rc = KPW_OK;
    for (; i < n; i++) {
        const uint8_t *rec = data + offsets[i];
        const uint64_t len = offsets[i + 1] - offsets[i];
        int r = w->model.add(rec, len);
        if (r == SizeModel::INVALID) {
            w->failed_record = w->num_records;
            w->err = "Invalid proto message received (record " + std::to_string(w->failed_record) + ")";
            rc = KPW_ERR_INVALID_PROTO;
            break;
        }
        if (r != SizeModel::OK || w->slot_used == 0 || w->slot_used + len > kpw_writer::kSlotBytes ||
            w->buf[w->fill].len + len + 64 > w->buf[w->fill].cap)
            if (int st = bind_device(w)) return st;   // a probe, job, slot flush or buffer growth
        if (int st = grow_fill(w, len)) return st;
        if (int st = stage_record(w, rec, len)) return st;
        StageBuf &F = w->buf[w->fill];
        F.ends.push_back(F.len);
        w->num_records++;
        if (r == SizeModel::PAGES) {
            if (int st = model_pages(w, nbounds(F) - 1, r)) return st;
        }
        if (r == SizeModel::CUT) {
            const int64_t nrec = F.ncarry_expected + (int64_t)F.ends.size();
            if (int st = submit(w, JOB_EXACT, nrec)) return st;
            w->pending_cut = true;
            if (w->aligned) {
                // the next row group's limit follows from this one's end in the file
                if (int st = drain(w)) return st;
                w->pending_cut = false;
                w->model.set_next_rg_size(w->fw->next_row_group_size());
            }
        }
        if (max_file_size >= 0) {
            // getDataSize() = lastRowGroupEndPos + columnStore.getBufferedSize()
            if (w->pending_cut) {
                if (int st = drain(w)) return st;
                w->pending_cut = false;
            }
            if (w->last_rg_end + w->model.buffered() >= max_file_size) {
                i++;
                if (full) *full = 1;
                break;
            }
        }
    }
    if (n_accepted) *n_accepted = i;
    return rc;
}

// Back to the per-record model after bulk writes (GPU-planned cuts): encode what is staged
// (the row groups it completes reach the file; the open row group's records are carried to
// the fill buffer), then replay the open row group's records through the model from its start
// (page probes included).  The GPU planner left them open, so the replay cannot cut.
static int model_resync(kpw_writer *w)
{
    if (w->dirty)
        if (int st = submit(w, JOB_PLANNED, 0)) return st;
    if (int st = drain(w)) return st;
    if (int st = observe_failure(w)) return st;
    StageBuf &F = w->buf[w->fill];
    if (int st = flush_slot(w)) return st;
    if (hipEventRecord(F.copied, w->copy_stream) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "event record failed");
    if (int st = materialize(w, F, w->eng.stream)) return wfail(w, st, "stage buffer rebuild failed");
    std::vector<uint64_t> hb;
    boundaries(F, hb);
    const size_t nrec = hb.size() - 1;
    w->model.restart(w->aligned ? w->fw->next_row_group_size() : w->eng.props.block_size);
    w->fill_gen++;   // boundaries changed in place: re-upload probe offsets
    F.ncarry_expected = (int64_t)(F.carry.empty() ? 0 : F.carry.size() - 1);
    if (nrec) {
        std::vector<uint8_t> bytes(hb[nrec] - hb[0]);
        if (hipStreamSynchronize(w->copy_stream) != hipSuccess ||
            hipMemcpy(bytes.data(), F.d + hb[0], bytes.size(), hipMemcpyDeviceToHost) != hipSuccess)
            return wfail(w, KPW_ERR_DEVICE, "model resync: D2H of the open row group failed");
        for (size_t i = 0; i < nrec; i++) {
            int r = w->model.add(bytes.data() + (hb[i] - hb[0]), hb[i + 1] - hb[i]);
            if (r == SizeModel::PAGES)
                if (int st = model_pages(w, i + 1, r)) return st;
            if (r != SizeModel::OK) {
                set_fatal(w, KPW_ERR_DEVICE, "model resync: the open row group does not replay as open");
                return KPW_ERR_DEVICE;
            }
        }
    }
    w->model_on = true;
    w->dirty = false;
    return KPW_OK;
}

// e[i] = offsets[i + 1] + delta for i < n, split over a few host threads for large batches
// (one poll() batch is 500 k records: 4 MB in and out, which one core streams no faster than
// the batch's own DMA)
static void rebase_ends(uint64_t *e, const uint64_t *offsets, uint64_t n, uint64_t delta)
{
    par_for(n, [=](uint64_t a, uint64_t b) { for (uint64_t i = a; i < b; i++) e[i] = offsets[i + 1] + delta; });
}

// Bulk write: the whole batch in one copy (direct DMA when the batch is pinned).
static int write_bulk(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n)
{
    const uint64_t bytes = offsets[n] - offsets[0];
    if (int st = grow_fill(w, bytes)) return st;
    StageBuf &F = w->buf[w->fill];
    const uint64_t delta = F.len - offsets[0];
    if (int st = stage_bytes(w, data + offsets[0], bytes)) return st;
    // the record ends are rebased while the batch's DMA runs
    rebase_ends(F.ends.grow(n), offsets, n, delta);
    w->num_records += (int64_t)n;
    w->dirty = true;
    return w->async_call ? KPW_OK : wait_direct(w);   // async: finish_async_call waits a call later
}

// Plain bulk write: a batch that does not fit the fill buffer's capacity (gap + job size +
// 64 MiB) is split where it stops fitting and the full buffer is submitted first, so the buffer
// never has to grow (grow_fill drains the pipeline and copies the buffer: C3's 690 MB poll
// batches did that on every second batch).  Batches that fit are appended whole, as before
// (jobs end at the first batch that reaches the job size).
// Multi-page writers: appended records per eager job, about one row group's (the last one an
// engine of this schema and properties cut, +2 %), so a job cuts one row group and carries a few
// records; a byte or batch-granular size lets the carry grow by the difference every job until it
// outgrows the buffers' gap.  0: no target (single-page, no row group cut yet, or turned off).
static uint64_t mp_job_records(kpw_writer *w)
{
    if (mp_eager_queue() <= 0 || !eager_job_bytes() || !w->eng.multi_page()) return 0;
    const int64_t R = w->eng.rg_records_hint();
    return R > 0 ? (uint64_t)((double)R * 1.02) : 0;
}

// An eager job may be submitted now: an encode worker is idle and nothing is queued (multi-page:
// fewer than mp_eager_queue() jobs are queued).
static bool eager_go(kpw_writer *w)
{
    std::lock_guard<std::mutex> g(w->mu);
    if (mp_eager_queue() > 0 && w->eng.multi_page()) return (int)w->q.size() < mp_eager_queue();
    return w->q.empty() && w->inflight < w->nworkers;
}

static int write_bulk_split(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n)
{
    while (n) {
        const StageBuf &F = w->buf[w->fill];
        const uint64_t used = F.len - F.gap;
        const uint64_t room = F.cap > F.len + 64 ? F.cap - F.len - 64 : 0;
        // largest k with offsets[k] - offsets[0] <= room
        uint64_t k = (uint64_t)(std::upper_bound(offsets, offsets + n + 1, offsets[0] + room) - offsets) - 1;
        const uint64_t ke = mp_job_records(w);
        if (ke && F.ends.size() < ke && F.ends.size() + std::min(k, n) > ke) {   // the job's row group ends in this batch
            const uint64_t m = ke - F.ends.size();
            if (int st = write_bulk(w, data, offsets, m)) return st;
            offsets += m;
            n -= m;
            if (eager_go(w))
                if (int st = submit(w, JOB_PLANNED, 0)) return st;
            continue;
        }
        if (k >= n) return write_bulk(w, data, offsets, n);
        if (k == 0 && used == 0) k = 1;   // one record larger than a job: the buffer grows
        if (k)
            if (int st = write_bulk(w, data, offsets, k)) return st;
        if (int st = submit(w, JOB_PLANNED, 0)) return st;
        offsets += k;
        n -= k;
    }
    return KPW_OK;
}

// getDataSize() after the first m records of the (drained) fill buffer, without flushing:
// an encode of [0, m) gives the row groups parquet-mr would have completed by then (their
// header + compressed bytes follow lastRowGroupEndPos) and the open row group's buffered size.
static int ds_prefix(kpw_writer *w, uint64_t m, int64_t &ds, BatchOut &out)
{
    out = BatchOut();
    StageBuf &F = w->buf[w->fill];
    int st = w->eng.encode(F.d, w->probe_off.as<uint64_t>(), m, false, w->eng.props.block_size, nullptr, out);
    if (st) return wfail(w, st, w->eng.error());
    int64_t t = w->last_rg_end;
    for (size_t r = 0; r < out.rgs.size(); r++) t += w->fw->row_group_size(out, (int)r);
    ds = t + out.open_buffered;
    return KPW_OK;
}

// The WorkerThread rotation loop (KafkaProtoParquetWriter.java:268-285,306-308) on the bulk
// path: records are written in order and the file is full right after the first record with
// getDataSize() >= max.  Within a row group getDataSize() only grows and a flush swaps the
// group's buffered size for its encoded bytes, so the first crossing is found segment by
// segment (before each planned cut, at the cut) and by bisection inside the crossing segment;
// each probe encodes a staged prefix (cuts are causal).  Multi-page chunks can shrink the
// buffered size inside a row group: that regime keeps write + getDataSize per record.
static int write_until_full_bulk(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                 int64_t max_file_size, uint64_t *n_accepted, int *full)
{
    // a page cut can shrink the buffered size inside a row group, and alignment moves each limit:
    // those regimes are record-at-a-time through the size model (write_entry), never here
    if (w->eng.multi_page() || w->aligned)
        return wfail(w, KPW_ERR_UNSUPPORTED, "write_until_full: no bulk search with page cuts or HDFS alignment");
    if (int st = drain(w)) return st;
    StreamOrder order(w->eng.stream);
    if (int st = flush_slot(w)) return st;
    if (hipEventRecord(w->buf[w->fill].copied, w->copy_stream) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "event record failed");
    if (int st = materialize(w, w->buf[w->fill], w->eng.stream)) return wfail(w, st, "stage buffer rebuild failed");
    StageBuf &F0 = w->buf[w->fill];
    const uint64_t base = (F0.carry.empty() ? 0 : F0.carry.size() - 1) + F0.ends.size();
    if (int st = write_bulk(w, data, offsets, n)) return st;
    if (int st = flush_slot(w)) return st;
    StageBuf &F = w->buf[w->fill];
    if (hipEventRecord(F.copied, w->copy_stream) != hipSuccess || hipStreamWaitEvent(w->eng.stream, F.copied, 0) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "staging order failed");
    std::vector<uint64_t> hb;
    boundaries(F, hb);
    if (w->probe_off.ensure(hb.size() * 8) || w->probe_h.ensure(hb.size() * 8))
        return wfail(w, KPW_ERR_NOMEM, "offset staging allocation failed");
    memcpy(w->probe_h.p, hb.data(), hb.size() * 8);
    if (hipMemcpyAsync(w->probe_off.p, w->probe_h.p, hb.size() * 8, hipMemcpyHostToDevice, w->eng.stream) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "H2D of offsets failed");
    auto truncate = [&](uint64_t keep) {   // keep the first `keep` records of this batch staged
        F.ends.resize(F.ends.size() - (n - keep));
        rewind_fill(w, F.ends.empty() ? F.gap : F.ends.back());
        w->num_records -= (int64_t)(n - keep);
    };
    BatchOut out;
    int64_t ds_end = 0;
    if (int st = ds_prefix(w, base + n, ds_end, out)) return st;
    uint64_t valid = n;
    if (out.invalid_record >= 0) {
        if ((uint64_t)out.invalid_record < base) {   // a record staged by an earlier write(): keep what precedes it
            truncate(0);
            const uint64_t keep = (uint64_t)out.invalid_record;
            const uint64_t nc = F.carry.empty() ? 0 : F.carry.size() - 1;
            if (keep >= nc) {
                F.ends.resize(keep - nc);
            } else {
                F.ends.clear();
                F.carry.resize(keep + 1);
                if (keep == 0) F.carry.clear();
            }
            rewind_fill(w, F.ends.empty() ? F.gap : F.ends.back());
            w->failed_record = F.first_new_global - (int64_t)nc + (int64_t)keep;
            w->num_records = w->failed_record;
            return wfail(w, KPW_ERR_INVALID_PROTO,
                         "Invalid proto message received (record " + std::to_string(w->failed_record) + ")");
        }
        valid = (uint64_t)out.invalid_record - base;
        if (int st = ds_prefix(w, base + valid, ds_end, out)) return st;
    }
    std::vector<int64_t> cut, end;   // row-group ends (records from the buffer start), file pos after each
    {
        int64_t e = w->last_rg_end;
        for (size_t r = 0; r < out.rgs.size(); r++) {
            e += w->fw->row_group_size(out, (int)r);
            cut.push_back(out.rgs[r].first_record + out.rgs[r].num_records);
            end.push_back(e);
        }
    }
    BatchOut tmp;
    // getDataSize() after record j of this batch, j inside the segment that follows `seg_end`
    // (the file position after the row groups cut before it): the cuts before j are causal, so
    // they are the ones already known and only the open row group's buffered size is new; a
    // plan-only encode of the prefix (K1 + planner, no dictionary / RLE / pages / Snappy) gives
    // it.  (Each probe used to encode the whole staged prefix in full.)
    int64_t seg_end = w->last_rg_end;
    auto ds = [&](uint64_t j, int64_t &v) {
        tmp = BatchOut();
        StageBuf &G = w->buf[w->fill];
        w->eng.plan_only = true;
        const int st = w->eng.encode(G.d, w->probe_off.as<uint64_t>(), base + j, false, w->eng.props.block_size, nullptr, tmp);
        w->eng.plan_only = false;
        if (st) return wfail(w, st, w->eng.error());
        v = seg_end + tmp.open_buffered;
        return (int)KPW_OK;
    };
    auto bisect = [&](uint64_t lo, uint64_t hi, uint64_t &res) {   // first j in [lo, hi] with ds(j) >= max
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo) / 2;
            int64_t v = 0;
            if (int e2 = ds(mid, v)) return e2;
            if (v >= max_file_size) hi = mid; else lo = mid + 1;
        }
        res = lo;
        return (int)KPW_OK;
    };
    uint64_t a = 0, found = 0;
    for (size_t i = 0; i < cut.size() && !found; i++) {
        const int64_t b = cut[i] - (int64_t)base;
        if (b < 1) continue;
        if ((uint64_t)b - 1 >= a + 1) {
            int64_t v = 0;
            if (int st = ds((uint64_t)b - 1, v)) return st;
            if (v >= max_file_size) {
                if (int st = bisect(a + 1, (uint64_t)b - 1, found)) return st;
                break;
            }
        }
        if (end[i] >= max_file_size) { found = (uint64_t)b; break; }
        a = (uint64_t)b;
        seg_end = end[i];
    }
    if (!found && valid >= a + 1 && ds_end >= max_file_size)
        if (int st = bisect(a + 1, valid, found)) return st;
    if (found) {
        truncate(found);
        *n_accepted = found;
        *full = 1;
    } else {
        truncate(valid);
        *n_accepted = valid;
        if (valid < n) {
            w->failed_record = w->num_records;
            w->err = "Invalid proto message received (record " + std::to_string(w->failed_record) + ")";
            return KPW_ERR_INVALID_PROTO;
        }
    }
    return KPW_OK;
}

static int write_entry(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n, int64_t max_file_size,
                       uint64_t *n_accepted, int *full)
{
    if (n_accepted) *n_accepted = 0;
    if (full) *full = 0;
    if (w->closed) return KPW_ERR_STATE;
    if (!w->async_call)
        if (int st = release_batches(w)) return st;
    if (int st = observe_failure(w)) return st;
    if (w->fill < 0) return wfail(w, KPW_ERR_STATE, "no stage buffer (an earlier failure)");
    if (!n) return KPW_OK;
    w->dev_bound = false;
    if (w->model_ok) {
        // write_until_full is record-at-a-time where the bulk search is not exact (multi-page
        // chunks: a page cut can shrink the buffered size inside a row group; HDFS alignment:
        // each limit follows the previous row group's end); otherwise large writes take the
        // bulk path (GPU-planned cuts) and small ones the per-record model
        const bool bulk_search = !w->model.multi_page() && !w->aligned;
        const bool modelled = (max_file_size >= 0 && !bulk_search) || n <= model_max_batch();
        if (!modelled) w->model_on = false;
        else if (!w->model_on) {
            if (int st = bind_device(w)) return st;
            if (int st = model_resync(w)) return st;
        }
    }
    if (!w->model_on)
        if (int st = bind_device(w)) return st;
    int rc;
    if (w->model_on) {
        rc = write_modelled(w, data, offsets, n, max_file_size, n_accepted, full);
    } else if (max_file_size >= 0) {
        rc = write_until_full_bulk(w, data, offsets, n, max_file_size, n_accepted, full);
    } else {
        rc = write_bulk_split(w, data, offsets, n);
        if (n_accepted && !rc) *n_accepted = n;
    }
    if (rc) return rc;
    StageBuf &F = w->buf[w->fill];
    if (!w->model_on) {
        const uint64_t used = F.len - F.gap;
        if (used >= stage_flush_bytes()) return submit(w, JOB_PLANNED, 0);
        const uint64_t ke = mp_job_records(w);
        if (ke ? F.ends.size() >= ke : eager_job_bytes() && used >= eager_job_bytes())
            if (eager_go(w)) return submit(w, JOB_PLANNED, 0);
    }
    return KPW_OK;
}

extern "C" int kpw_writer_write(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n)
{
    if (!w || (n && (!data || !offsets))) return KPW_ERR_INVALID_ARG;
    try {
        return write_entry(w, data, offsets, n, -1, nullptr, nullptr);
    } catch (const std::bad_alloc &) {
        set_fatal(w, KPW_ERR_NOMEM, "host staging allocation failed");
        return KPW_ERR_NOMEM;
    } catch (...) {
        set_fatal(w, KPW_ERR_DEVICE, "unexpected failure");
        return KPW_ERR_DEVICE;
    }
}

extern "C" int kpw_writer_write_async(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n)
{
    if (!w || (n && (!data || !offsets))) return KPW_ERR_INVALID_ARG;
    try {
        // the modelled path (small writes) stages through the library's own pinned slots, so it
        // never reads the batch after returning; only the bulk path's direct DMA is deferred
        w->async_call = true;
        int st = write_entry(w, data, offsets, n, -1, nullptr, nullptr);
        w->async_call = false;
        const int st2 = finish_async_call(w);
        return st ? st : st2;
    } catch (const std::bad_alloc &) {
        w->async_call = false;
        set_fatal(w, KPW_ERR_NOMEM, "host staging allocation failed");
        return KPW_ERR_NOMEM;
    } catch (...) {
        w->async_call = false;
        set_fatal(w, KPW_ERR_DEVICE, "unexpected failure");
        return KPW_ERR_DEVICE;
    }
}

extern "C" int kpw_writer_write_until_full(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                           int64_t max_file_size, uint64_t *n_accepted, int *full)
{
    if (!w || !n_accepted || !full || (n && (!data || !offsets)) || max_file_size < 0) return KPW_ERR_INVALID_ARG;
    try {
        return write_entry(w, data, offsets, n, max_file_size, n_accepted, full);
    } catch (const std::bad_alloc &) {
        set_fatal(w, KPW_ERR_NOMEM, "host allocation failed");
        return KPW_ERR_NOMEM;
    } catch (...) {
        set_fatal(w, KPW_ERR_DEVICE, "unexpected failure");
        return KPW_ERR_DEVICE;
    }
}

// getDataSize() (ParquetFile.java:77-79 -> InternalParquetRecordWriter.getDataSize).
extern "C" int64_t kpw_writer_data_size(kpw_writer *w)
{
    if (!w) return -1;
    try {
        if (w->closed) return w->fw->pos();
        if (release_batches(w)) return -1;
        if (observe_failure(w)) return -1;
        if (w->model_on) {
            if (w->pending_cut) {
                if (drain(w)) return -1;
                w->pending_cut = false;
            }
            return w->last_rg_end + w->model.buffered();
        }
        w->size_polled = true;
        if (w->dirty && submit(w, JOB_PLANNED, 0, true)) return -1;   // encode what is staged (completed row groups flushed)
        if (drain(w)) return -1;
        if (observe_failure(w)) return -1;
        if (w->open_buffered < 0) {   // the last job left the open row group to the next one: plan it now
            if (submit(w, JOB_PLANNED, 0, true)) return -1;
            if (drain(w)) return -1;
            if (observe_failure(w)) return -1;
        }
        return w->last_rg_end + w->open_buffered;
    } catch (...) {
        return -1;
    }
}

// The getters are entry points too: the batch of an earlier kpw_writer_write_async is free
// once any kpw_writer_* call returns (kpw_gpu.h), so each releases it first (nothing to wait
// for when no DMA is pending).  The handle is const in the C-ABI only as a promise about the
// file it describes; its pipeline state is the library's.
static void release_from_getter(const kpw_writer *w)
{
    try {
        (void)release_batches(const_cast<kpw_writer *>(w));   // a failed DMA is recorded (wfail)
    } catch (...) {
    }
}
extern "C" int64_t kpw_writer_num_records(const kpw_writer *w)
{
    if (!w) return -1;
    release_from_getter(w);
    return w->num_records;
}
extern "C" int64_t kpw_writer_creation_time_ms(const kpw_writer *w)
{
    if (!w) return -1;
    release_from_getter(w);
    return w->created_ms;
}
extern "C" int64_t kpw_writer_failed_record(const kpw_writer *w)
{
    if (!w) return -1;
    release_from_getter(w);
    return w->failed_record;
}
extern "C" const char *kpw_writer_last_error(const kpw_writer *w)
{
    if (!w) return "null handle";
    release_from_getter(w);
    return w->err.c_str();
}

// close() (ParquetFile.java:65-68): flush everything staged (after an invalid record: only
// the records before it), then the footer.  Idempotent.
extern "C" int kpw_writer_close(kpw_writer *w)
{
    if (!w) return KPW_ERR_INVALID_ARG;
    if (w->closed) return KPW_OK;
    const double t_close = now_ms();
    try {
        if (hipSetDevice(w->eng.device) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "hipSetDevice failed");
        if (int st = release_batches(w)) return st;
        {
            std::lock_guard<std::mutex> g(w->mu);
            if (w->fatal_st) { w->err = w->fatal_err; return w->fatal_st; }
        }
        (void)observe_failure(w);   // an invalid record: only what came before it is flushed
        if (w->fill >= 0) {
            if (int st = submit(w, JOB_FINAL, 0)) return st;
        }
        if (w->h2d_marks == 1 && hipEventRecord(w->h2d_ev[1], w->copy_stream) == hipSuccess) w->h2d_marks = 2;
        if (int st = drain(w)) return st;
        int st = w->fw->close();
        if (st) return wfail(w, st, w->fw->error());
        w->closed = true;
        if (trace_on())
            fprintf(stderr, "[kpw] close: entered at %.1f, footer done at %.1f ms\n", t_close - w->t_open, now_ms() - w->t_open);
        if (trace_on())
            fprintf(stderr, "[kpw] close: worker encode %.1f ms, encode gate waits %.1f ms; caller: pinned DMA waits %.1f ms, "
                            "buffer acquire %.1f ms; worker: page buffer alloc + D2H issue %.1f ms; assembly %.1f ms; "
                            "buffers rebuilt for a carry %d, gap %.0f MiB\n",
                    w->t_encode, w->t_gate, w->t_dma, w->t_acquire, w->t_d2h_alloc, w->t_asm, w->n_materialize.load(),
                    w->gap_.load() / 1048576.0);
        if (trace_on() && w->n_probe)
            fprintf(stderr, "[kpw] close: %llu page-size probes, %.1f ms (%.3f ms each, %.0f records each); per probe: "
                            "staging + offsets %.3f, encode entry to pipeline %.3f, pipeline %.3f, after %.3f ms\n",
                    (unsigned long long)w->n_probe, w->t_probe, w->t_probe / w->n_probe, (double)w->probe_recs / w->n_probe,
                    w->t_probe_pre / w->n_probe, w->peng.probe_t[0] / w->n_probe, w->peng.probe_t[1] / w->n_probe,
                    w->peng.probe_t[2] / w->n_probe);
        return KPW_OK;
    } catch (...) {
        set_fatal(w, KPW_ERR_DEVICE, "close failed");
        return KPW_ERR_DEVICE;
    }
}

extern "C" int kpw_writer_file_bytes(const kpw_writer *w, const uint8_t **bytes, uint64_t *len)
{
    if (!w || !bytes || !len) return KPW_ERR_INVALID_ARG;
    if (!w->closed) return KPW_ERR_STATE;
    *bytes = w->fw->memory_data();
    *len = w->fw->memory_size();
    if (!*bytes && *len) {   // the contiguous copy of a multi-chunk file could not be allocated
        *len = 0;
        return KPW_ERR_NOMEM;
    }
    return KPW_OK;
}

extern "C" void kpw_writer_free(kpw_writer *w)
{
    const double t0 = trace_on() ? now_ms() : 0.0;
    if (w) release_from_getter(w);   // no DMA may still read a caller's batch once the handle is gone
    const double t1 = trace_on() ? now_ms() : 0.0;
    delete w;
    if (trace_on()) fprintf(stderr, "[kpw] writer free: release %.1f ms, delete (members included) %.1f ms\n", t1 - t0, now_ms() - t1);
}

extern "C" int kpw_writer_stats(kpw_writer *w, double *out, int cap)
{
    if (!w || !out || cap <= 0) return 0;
    if (release_batches(w) || drain(w)) return 0;
    if (w->h2d_marks == 2) {
        float ms = 0.f;
        if (hipEventSynchronize(w->h2d_ev[1]) == hipSuccess && hipEventElapsedTime(&ms, w->h2d_ev[0], w->h2d_ev[1]) == hipSuccess)
            w->stats[17] = ms;
        else
            (void)hipGetLastError();
    }
    const int n = cap < 18 ? cap : 18;
    for (int i = 0; i < n; i++) out[i] = w->stats[i];
    return n;
}
