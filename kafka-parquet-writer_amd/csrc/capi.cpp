// capi.cpp — extern "C" boundary of libkpw_gpu.so (include/kpw_gpu.h).
// No C++ exception crosses this file: every entry point catches and maps to a status.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kpw_gpu.h"
#include "engine.h"
#include "filewriter.h"

using namespace kpw;

// ---------------------------------------------------------------- encoder (flush path)

struct kpw_encoder {
    Engine eng;
    BatchOut out;
    std::vector<kpw_row_group_info> rgs;
    std::vector<kpw_chunk_info> chunks;
    std::vector<kpw_page_info> pages;
    std::string stats;
    std::string err;
};

extern "C" kpw_encoder *kpw_encoder_create(int device, const kpw_schema *schema, const kpw_props *props, int *status)
{
    try {
        kpw_encoder *e = new kpw_encoder();
        int st = e->eng.init(device, schema, props);
        if (st) {
            if (status) *status = st;
            delete e;
            return nullptr;
        }
        if (status) *status = KPW_OK;
        return e;
    } catch (const std::bad_alloc &) {
        if (status) *status = KPW_ERR_NOMEM;
    } catch (...) {
        if (status) *status = KPW_ERR_DEVICE;
    }
    return nullptr;
}

extern "C" void kpw_encoder_destroy(kpw_encoder *e) { delete e; }

extern "C" const char *kpw_encoder_last_error(const kpw_encoder *e)
{
    if (!e) return "null handle";
    return e->err.empty() ? e->eng.error().c_str() : e->err.c_str();
}

static void fill_info(kpw_encoder *e, kpw_batch_info *info)
{
    const BatchOut &o = e->out;
    e->rgs.clear(); e->chunks.clear(); e->pages.clear(); e->stats.clear();
    for (auto &r : o.rgs) e->rgs.push_back(kpw_row_group_info{r.first_record, r.num_records, r.first_chunk, 0});
    for (auto &c : o.chunks) e->chunks.push_back(kpw_chunk_info{c.column, c.first_page, c.num_pages, c.has_dictionary, c.num_values});
    for (auto &p : o.pages) {
        kpw_page_info q;
        memset(&q, 0, sizeof(q));
        q.page_type = p.page_type; q.num_values = p.num_values; q.encoding = p.encoding; q.dl_encoding = p.dl_encoding;
        q.rl_encoding = p.rl_encoding; q.has_stats = p.has_stats; q.uncompressed_size = p.uncompressed_size;
        q.compressed_size = p.compressed_size; q.offset = p.offset; q.null_count = p.null_count; q.has_min_max = p.has_min_max;
        q.min_len = (int32_t)p.min.size(); q.max_len = (int32_t)p.max.size();
        q.dl_byte_length = p.dl_byte_length; q.num_rows = p.num_rows;
        q.min_off = e->stats.size(); e->stats += p.min;
        q.max_off = e->stats.size(); e->stats += p.max;
        e->pages.push_back(q);
    }
    memset(info, 0, sizeof(*info));
    info->num_row_groups = (int32_t)e->rgs.size();
    info->num_chunks = (int32_t)e->chunks.size();
    info->num_pages = (int32_t)e->pages.size();
    info->row_groups = e->rgs.data();
    info->chunks = e->chunks.data();
    info->pages = e->pages.data();
    info->stats_bytes = (const uint8_t *)e->stats.data();
    info->stats_len = e->stats.size();
    info->device_pages = o.d_pages;
    info->device_pages_len = o.pages_len;
    info->records_consumed = o.records_consumed;
    info->open_records = o.open_records;
    info->open_buffered_size = o.open_buffered;
    info->invalid_record = o.invalid_record;
}

extern "C" int kpw_encoder_encode(kpw_encoder *e, const uint8_t *d_data, const uint64_t *d_offsets, uint64_t n, int final,
                                  int64_t next_row_group_size, void *hip_stream, kpw_batch_info *info)
{
    if (!e || !info || (n && (!d_data || !d_offsets))) return KPW_ERR_INVALID_ARG;
    try {
        e->err.clear();
        const int64_t T = next_row_group_size > 0 ? next_row_group_size : e->eng.props.block_size;
        int st = e->eng.encode(d_data, d_offsets, n, final != 0, T, (hipStream_t)hip_stream, e->out);
        if (st) return st;
        fill_info(e, info);
        return KPW_OK;
    } catch (const std::bad_alloc &) {
        return KPW_ERR_NOMEM;
    } catch (...) {
        return KPW_ERR_DEVICE;
    }
}

extern "C" int kpw_encoder_copy_pages(kpw_encoder *e, uint64_t off, uint64_t len, void *host_dst)
{
    if (!e || !host_dst) return KPW_ERR_INVALID_ARG;
    return e->eng.copy_pages(off, len, host_dst);
}

extern "C" int kpw_encoder_stage_times(const kpw_encoder *e, float *ms, int cap)
{
    if (!e || !ms) return 0;
    int n = cap < 10 ? cap : 10;
    for (int i = 0; i < n; i++) ms[i] = e->eng.stage_ms[i];
    return n;
}

// ---------------------------------------------------------------- ParquetFile drop-in

// Pinned host memory (page-locked: DMA-able without a bounce through pageable buffers).
struct PinnedBuf {
    uint8_t *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes)
    {
        if (bytes <= cap && p) return 0;
        if (p) { (void)hipHostFree(p); p = nullptr; cap = 0; }
        const size_t c = bytes + bytes / 4 + 4096;
        if (hipHostMalloc((void **)&p, c, hipHostMallocDefault) != hipSuccess) { p = nullptr; return -1; }
        cap = c;
        return 0;
    }
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
};

// Staging: record bytes go straight to HBM as they are written.  write()
// copies each batch into one of kSlots pinned slots and queues its H2D on a side stream
// (copy_stream) into the device stage at the append position, so the DMA of one slot
// overlaps the host copy of the next and the caller's own work between write() calls.  The
// host keeps only the u64 offsets.  At a flush the encode stream waits on the side stream
// (one event), encodes in place, and the open row group's records are carried over by a
// device-to-device copy into the second stage buffer (never re-sent over PCIe).
struct kpw_writer {
    static constexpr int kSlots = 4;
    static constexpr size_t kSlotBytes = 32ull << 20;
    Engine eng;
    FileWriter *fw = nullptr;
    uint8_t *d_stage[2] = {nullptr, nullptr};   // device record bytes (current + carry-over target)
    size_t stage_cap = 0;
    int cur = 0;
    uint64_t stage_len = 0;                      // bytes staged on the device (queued copies included)
    std::vector<uint64_t> offs{0};               // record offsets into d_stage[cur]
    hipStream_t copy_stream = nullptr;
    hipEvent_t slot_ev[kSlots] = {}, copied = nullptr;
    PinnedBuf slot[kSlots];
    int next_slot = 0;
    double t_enter = 0, t_slotwait = 0, t_copy = 0;
    uint64_t staged_bytes_at_encode = ~0ull;
    int64_t num_records = 0;         // ParquetFile.numWrittenRecords
    int64_t last_rg_end = 0;         // InternalParquetRecordWriter.lastRowGroupEndPos
    int64_t open_buffered = 0;
    int64_t failed_record = -1;
    int64_t created_ms = 0;
    bool closed = false, dead = false;
    std::string err;
    DevBuf d_off;
    PinnedBuf h_off, host_pages;
    // file assembly of a flush runs on `bg` (waits for the pages' D2H, writes headers + bodies)
    // while the caller goes on staging records; joined before anything reads the file state
    std::thread bg;
    int bg_st = KPW_OK;
    std::string bg_err;
    BatchOut bg_out;
    hipEvent_t d2h_done = nullptr;
    int init_staging()
    {
        if (hipSetDevice(eng.device) != hipSuccess) return KPW_ERR_DEVICE;
        if (hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking) != hipSuccess) return KPW_ERR_DEVICE;
        for (auto &e : slot_ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
        if (hipEventCreateWithFlags(&copied, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
        if (hipEventCreateWithFlags(&d2h_done, hipEventDisableTiming) != hipSuccess) return KPW_ERR_DEVICE;
        return KPW_OK;
    }
    ~kpw_writer()
    {
        if (bg.joinable()) bg.join();
        (void)hipSetDevice(eng.device);
        if (copy_stream) (void)hipStreamSynchronize(copy_stream);
        if (eng.stream) (void)hipStreamSynchronize(eng.stream);
        for (auto &b : d_stage) if (b) (void)hipFree(b);
        for (auto &e : slot_ev) if (e) (void)hipEventDestroy(e);
        if (copied) (void)hipEventDestroy(copied);
        if (d2h_done) (void)hipEventDestroy(d2h_done);
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        delete fw;
    }
};

static int wfail(kpw_writer *w, int st, const std::string &m)
{
    w->err = m;
    if (st != KPW_ERR_IO) w->dead = true;
    return st;
}

// Wait for the previous flush's file assembly; surface its failure.  A failed assembly is
// fatal even for KPW_ERR_IO: its records were already dropped from staging, so a retried
// close()/getDataSize() could otherwise "succeed" with rows missing from the file.
static int join_bg(kpw_writer *w)
{
    if (w->bg.joinable()) w->bg.join();
    if (w->bg_st) {
        const int st = w->bg_st;
        w->bg_st = KPW_OK;
        wfail(w, st, w->bg_err);
        w->dead = true;
        return st;
    }
    return KPW_OK;
}

// Grow both device stage buffers to hold `need` bytes (+16 B of read slack), keeping the
// staged bytes of the current one.
static int grow_stage(kpw_writer *w, size_t need)
{
    need += 16;
    if (need <= w->stage_cap) return KPW_OK;
    size_t c = std::max(need, w->stage_cap * 2);
    c = std::max<size_t>(c, 64ull << 20);
    uint8_t *nb[2] = {nullptr, nullptr};
    for (auto &b : nb)
        if (hipMalloc((void **)&b, c) != hipSuccess) {
            if (nb[0]) (void)hipFree(nb[0]);
            return wfail(w, KPW_ERR_NOMEM, "device staging allocation failed");
        }
    if (hipStreamSynchronize(w->copy_stream) != hipSuccess || hipStreamSynchronize(w->eng.stream) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "staging sync failed");
    if (w->stage_len && hipMemcpy(nb[0], w->d_stage[w->cur], w->stage_len, hipMemcpyDeviceToDevice) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "staging grow copy failed");
    for (auto &b : w->d_stage) if (b) (void)hipFree(b);
    w->d_stage[0] = nb[0];
    w->d_stage[1] = nb[1];
    w->cur = 0;
    w->stage_cap = c;
    return KPW_OK;
}

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// KPW_TRACE=1: per-flush timings of the writer path on stderr
static bool trace_on()
{
    static const bool v = [] { const char *e = getenv("KPW_TRACE"); return e && *e == '1'; }();
    return v;
}

// Queue `len` host bytes for the device stage (through the pinned slots).
static int stage_bytes(kpw_writer *w, const uint8_t *src, uint64_t len)
{
    while (len) {
        const int k = w->next_slot;
        w->next_slot = (k + 1) % kpw_writer::kSlots;
        const size_t piece = std::min<uint64_t>(len, kpw_writer::kSlotBytes);
        const double ta = trace_on() ? now_ms() : 0.0;
        if (w->slot[k].p && hipEventSynchronize(w->slot_ev[k]) != hipSuccess)
            return wfail(w, KPW_ERR_DEVICE, "staging slot wait failed");
        const double tb = trace_on() ? now_ms() : 0.0;
        if (w->slot[k].ensure(kpw_writer::kSlotBytes)) return wfail(w, KPW_ERR_NOMEM, "pinned staging allocation failed");
        par_copy(w->slot[k].p, src, piece);
        if (trace_on()) { w->t_slotwait += tb - ta; w->t_copy += now_ms() - tb; }
        if (hipMemcpyAsync(w->d_stage[w->cur] + w->stage_len, w->slot[k].p, piece, hipMemcpyHostToDevice, w->copy_stream) !=
                hipSuccess ||
            hipEventRecord(w->slot_ev[k], w->copy_stream) != hipSuccess)
            return wfail(w, KPW_ERR_DEVICE, "H2D failed");
        w->stage_len += piece;
        src += piece;
        len -= piece;
    }
    return KPW_OK;
}

// Stage n records (bytes through the pinned slots, offsets on the host).
static int append_records(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n)
{
    const uint64_t bytes = offsets[n] - offsets[0];
    if (hipSetDevice(w->eng.device) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "hipSetDevice failed");
    if (grow_stage(w, w->stage_len + bytes)) return KPW_ERR_NOMEM;
    const uint64_t base = w->stage_len;
    int st = stage_bytes(w, data + offsets[0], bytes);
    if (st) return st;
    const size_t o0 = w->offs.size();
    w->offs.resize(o0 + n);
    uint64_t *od = w->offs.data() + o0;
    const uint64_t delta = base - offsets[0];
    for (uint64_t i = 1; i <= n; i++) od[i - 1] = offsets[i] + delta;
    w->num_records += (int64_t)n;
    return KPW_OK;
}

// Offsets of every staged record to the device, ordered after the side stream's byte copies.
static int upload_offsets(kpw_writer *w)
{
    const uint64_t n = w->offs.size() - 1;
    if (w->d_off.ensure((n + 1) * 8) || w->h_off.ensure((n + 1) * 8))
        return wfail(w, KPW_ERR_NOMEM, "offset staging allocation failed");
    hipStream_t s = w->eng.stream;
    memcpy(w->h_off.p, w->offs.data(), (n + 1) * 8);
    if (hipEventRecord(w->copied, w->copy_stream) != hipSuccess || hipStreamWaitEvent(s, w->copied, 0) != hipSuccess ||
        hipMemcpyAsync(w->d_off.p, w->h_off.p, (n + 1) * 8, hipMemcpyHostToDevice, s) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "H2D failed");
    return KPW_OK;
}

// Encode the staged records: flush every row group parquet-mr would have completed (all of
// them if final), keep the open row group's records staged.
static int process(kpw_writer *w, bool final)
{
    int jst = join_bg(w);
    if (jst) return jst;
    const uint64_t n = w->offs.size() - 1;
    if (!final && w->staged_bytes_at_encode == w->stage_len) return KPW_OK;  // nothing new
    if (hipSetDevice(w->eng.device) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "hipSetDevice failed");
    if (trace_on()) w->t_enter = now_ms();
    if (grow_stage(w, w->stage_len)) return KPW_ERR_NOMEM;
    if (int ust = upload_offsets(w)) return ust;
    hipStream_t s = w->eng.stream;
    const double t0 = trace_on() ? ((void)hipStreamSynchronize(s), now_ms()) : 0.0;
    BatchOut out;
    int st = w->eng.encode(w->d_stage[w->cur], w->d_off.as<uint64_t>(), n, final, w->eng.props.block_size, nullptr, out);
    if (st) return wfail(w, st, w->eng.error());
    if (out.pages_len) {
        if (w->host_pages.ensure(out.pages_len)) return wfail(w, KPW_ERR_NOMEM, "pinned page buffer allocation failed");
        if (hipMemcpyAsync(w->host_pages.p, out.d_pages, out.pages_len, hipMemcpyDeviceToHost, s) != hipSuccess)
            return wfail(w, KPW_ERR_DEVICE, "D2H of pages failed");
    }
    if (hipEventRecord(w->d2h_done, s) != hipSuccess) return wfail(w, KPW_ERR_DEVICE, "event record failed");
    if (trace_on())
        fprintf(stderr, "[kpw] flush n=%llu bytes=%llu rgs=%zu pages=%llu: wait %.2f ms, encode %.2f ms\n",
                (unsigned long long)n, (unsigned long long)w->stage_len, out.rgs.size(), (unsigned long long)out.pages_len,
                t0 - w->t_enter, now_ms() - t0);
    const int64_t records_consumed = out.records_consumed, invalid_record = out.invalid_record,
                  open_buffered = out.open_buffered;
    if (!out.rgs.empty()) {
        w->bg_out = std::move(out);
        w->bg = std::thread([w] {
            // no exception may leave this thread (std::terminate would kill the host process)
            try {
                (void)hipSetDevice(w->eng.device);
                const double tf = trace_on() ? now_ms() : 0.0;
                if (hipEventSynchronize(w->d2h_done) != hipSuccess) {
                    w->bg_st = KPW_ERR_DEVICE;
                    w->bg_err = "D2H of pages failed";
                    return;
                }
                for (size_t r = 0; r < w->bg_out.rgs.size(); r++) {
                    const int st2 = w->fw->write_row_group(w->bg_out, (int)r, w->host_pages.p, 0);
                    if (st2) {
                        w->bg_st = st2;
                        w->bg_err = w->fw->error();
                        return;
                    }
                    w->last_rg_end = w->fw->pos();
                }
                if (trace_on()) fprintf(stderr, "[kpw] file assembly (d2h wait + write) %.2f ms\n", now_ms() - tf);
            } catch (const std::bad_alloc &) {
                w->bg_st = KPW_ERR_NOMEM;
                w->bg_err = "file assembly: host allocation failed";
            } catch (...) {
                w->bg_st = KPW_ERR_DEVICE;
                w->bg_err = "file assembly failed";
            }
        });
    }
    // keep [records_consumed, valid end) staged
    const uint64_t keep0 = (uint64_t)records_consumed;
    uint64_t keep1 = n;
    int rc = KPW_OK;
    if (invalid_record >= 0) {
        keep1 = (uint64_t)invalid_record;
        const int64_t dropped = (int64_t)(n - keep1);
        w->failed_record = w->num_records - dropped;
        w->num_records -= dropped;
        rc = KPW_ERR_INVALID_PROTO;
        w->err = "Invalid proto message received (record " + std::to_string(w->failed_record) + ")";
    }
    const uint64_t b0 = w->offs[keep0], b1 = w->offs[keep1];
    if (b0 > 0 && b1 > b0) {
        // carry the open row group over on the device (ordered after the encode on `s`; the
        // side stream's next copies land past b1 - b0 in the new buffer)
        if (hipMemcpyAsync(w->d_stage[1 - w->cur], w->d_stage[w->cur] + b0, b1 - b0, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return wfail(w, KPW_ERR_DEVICE, "carry-over copy failed");
        if (hipEventRecord(w->copied, s) != hipSuccess || hipStreamWaitEvent(w->copy_stream, w->copied, 0) != hipSuccess)
            return wfail(w, KPW_ERR_DEVICE, "carry-over ordering failed");
        w->cur = 1 - w->cur;
    }
    // shift the kept offsets to the front in place (the vector keeps its capacity, so the
    // next batch's appends do not reallocate)
    uint64_t *o = w->offs.data();
    for (uint64_t i = keep0; i <= keep1; i++) o[i - keep0] = o[i] - b0;
    w->offs.resize(keep1 - keep0 + 1);
    w->stage_len = b1 - b0;
    w->open_buffered = final ? 0 : open_buffered;
    if (rc) {
        // the open row group may have been cut by the invalid record: re-plan it next time
        w->staged_bytes_at_encode = ~0ull;
        w->dead = true;
        return rc;
    }
    w->staged_bytes_at_encode = w->stage_len;
    return KPW_OK;
}

extern "C" kpw_writer *kpw_writer_open(int device, const kpw_schema *schema, const kpw_props *props, const char *path, int *status)
{
    try {
        kpw_writer *w = new kpw_writer();
        int st = w->eng.init(device, schema, props);
        if (!st) {
            w->fw = new FileWriter(w->eng.cols, w->eng.message_name, w->eng.proto_class, w->eng.props);
            st = w->fw->open(path);
        }
        if (!st) st = w->init_staging();
        if (st) {
            if (status) *status = st;
            delete w;
            return nullptr;
        }
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

// Records are encoded once this many bytes beyond one row group are staged.  512 MiB measured
// best for the PCIe-inclusive rate (profiles/r01e_writer.md: 2 and 4 GiB flushes lose more to
// the unoverlapped last flush and bigger pinned buffers than they gain per batch).
// KPW_STAGE_FLUSH_MB overrides it.
static uint64_t stage_flush_bytes()
{
    static const uint64_t v = [] {
        const char *e = getenv("KPW_STAGE_FLUSH_MB");
        const long long mb = e ? atoll(e) : 0;
        return (uint64_t)(mb > 0 ? mb : 512) << 20;
    }();
    return v;
}

extern "C" int kpw_writer_write(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n)
{
    if (!w || (n && (!data || !offsets))) return KPW_ERR_INVALID_ARG;
    if (w->closed || w->dead) return KPW_ERR_STATE;
    try {
        int st = append_records(w, data, offsets, n);
        if (st) return st;
        if (w->stage_len >= stage_flush_bytes() + (uint64_t)w->eng.props.block_size) return process(w, false);
        return KPW_OK;
    } catch (const std::bad_alloc &) {
        return wfail(w, KPW_ERR_NOMEM, "host staging allocation failed");
    } catch (...) {
        return wfail(w, KPW_ERR_DEVICE, "unexpected failure");
    }
}

// getDataSize() after the first m staged records, without flushing anything: an encode of
// [0, m) gives the row groups parquet-mr would have completed by then (their header +
// compressed bytes follow lastRowGroupEndPos) and the open row group's buffered size.
static int ds_prefix(kpw_writer *w, uint64_t m, int64_t &ds, BatchOut &out)
{
    out = BatchOut();
    int st = w->eng.encode(w->d_stage[w->cur], w->d_off.as<uint64_t>(), m, false, w->eng.props.block_size, nullptr, out);
    if (st) return wfail(w, st, w->eng.error());
    int64_t t = w->last_rg_end;
    for (size_t r = 0; r < out.rgs.size(); r++) t += w->fw->row_group_size(out, (int)r);
    ds = t + out.open_buffered;
    return KPW_OK;
}

// The WorkerThread loop (KafkaProtoParquetWriter.java:268-285,306-308) over a batch: records
// are written one at a time and the file is full right after the first record for which
// getDataSize() >= max_file_size.  Within one row group getDataSize() only grows (raw column
// sizes and level bytes are appended), and a row-group flush replaces the group's buffered
// size by its encoded bytes, so the first crossing is found segment by segment: at the last
// record before each cut, at the cut itself, and by bisection inside the segment that crosses.
// Every probe is an encode of a staged prefix (row-group cuts are causal: a prefix plans the
// same cuts).  Multi-page chunks can shrink the buffered size inside a row group (a page cut
// swaps raw bytes for compressed ones), so that regime keeps the per-record getDataSize() path.
extern "C" int kpw_writer_write_until_full(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                           int64_t max_file_size, uint64_t *n_accepted, int *full)
{
    if (!w || !n_accepted || !full || (n && (!data || !offsets))) return KPW_ERR_INVALID_ARG;
    *n_accepted = 0;
    *full = 0;
    if (w->closed || w->dead) return KPW_ERR_STATE;
    if (w->eng.props.writer_version == 1 && w->eng.props.page_size < w->eng.props.block_size) {
        w->err = "write_until_full: pageSize < blockSize (multi-page chunks) — use write + getDataSize per record";
        return KPW_ERR_UNSUPPORTED;
    }
    try {
        int st = join_bg(w);
        if (st) return st;
        if (!n) return KPW_OK;
        const uint64_t base = w->offs.size() - 1;
        st = append_records(w, data, offsets, n);
        if (st) return st;
        w->staged_bytes_at_encode = ~0ull;
        auto truncate = [&](uint64_t keep) {   // keep the first `keep` records of this batch staged
            w->offs.resize(base + keep + 1);
            w->stage_len = w->offs.back();
            w->num_records -= (int64_t)(n - keep);
        };
        if ((st = upload_offsets(w))) return st;
        BatchOut out;
        int64_t ds_end = 0;
        if ((st = ds_prefix(w, base + n, ds_end, out))) return st;
        uint64_t valid = n;
        if (out.invalid_record >= 0) {
            if ((uint64_t)out.invalid_record < base) {   // a record staged by an earlier write()
                truncate(0);
                return process(w, false);
            }
            valid = (uint64_t)out.invalid_record - base;
            if ((st = ds_prefix(w, base + valid, ds_end, out))) return st;
        }
        std::vector<int64_t> cut, end;   // row-group ends (records from the staging start), file pos after each
        {
            int64_t e = w->last_rg_end;
            for (size_t r = 0; r < out.rgs.size(); r++) {
                e += w->fw->row_group_size(out, (int)r);
                cut.push_back(out.rgs[r].first_record + out.rgs[r].num_records);
                end.push_back(e);
            }
        }
        BatchOut tmp;
        auto ds = [&](uint64_t j, int64_t &v) { return ds_prefix(w, base + j, v, tmp); };
        // first j in [lo, hi] with ds(j) >= max, given ds(hi) >= max
        auto bisect = [&](uint64_t lo, uint64_t hi, uint64_t &res) {
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
                if ((st = ds((uint64_t)b - 1, v))) return st;
                if (v >= max_file_size) {
                    if ((st = bisect(a + 1, (uint64_t)b - 1, found))) return st;
                    break;
                }
            }
            if (end[i] >= max_file_size) { found = (uint64_t)b; break; }
            a = (uint64_t)b;
        }
        if (!found && valid >= a + 1 && ds_end >= max_file_size)
            if ((st = bisect(a + 1, valid, found))) return st;
        if (found) {
            truncate(found);
            *n_accepted = found;
            *full = 1;
        } else {
            truncate(valid);
            *n_accepted = valid;
            if (valid < n) {
                w->failed_record = w->num_records;
                w->dead = true;
                w->err = "Invalid proto message received (record " + std::to_string(w->failed_record) + ")";
                return KPW_ERR_INVALID_PROTO;
            }
        }
        if (w->stage_len >= stage_flush_bytes() + (uint64_t)w->eng.props.block_size) return process(w, false);
        return KPW_OK;
    } catch (const std::bad_alloc &) {
        return wfail(w, KPW_ERR_NOMEM, "host allocation failed");
    } catch (...) {
        return wfail(w, KPW_ERR_DEVICE, "unexpected failure");
    }
}

extern "C" int64_t kpw_writer_data_size(kpw_writer *w)
{
    if (!w) return -1;
    if (w->closed) return w->fw->pos();
    if (!w->dead) {
        try {
            if (process(w, false) || join_bg(w)) return -1;
        } catch (...) {
            return -1;
        }
    } else if (w->bg.joinable()) {
        w->bg.join();
    }
    return w->last_rg_end + w->open_buffered;
}

extern "C" int64_t kpw_writer_num_records(const kpw_writer *w) { return w ? w->num_records : -1; }
extern "C" int64_t kpw_writer_creation_time_ms(const kpw_writer *w) { return w ? w->created_ms : -1; }
extern "C" int64_t kpw_writer_failed_record(const kpw_writer *w) { return w ? w->failed_record : -1; }
extern "C" const char *kpw_writer_last_error(const kpw_writer *w) { return w ? w->err.c_str() : "null handle"; }

extern "C" int kpw_writer_close(kpw_writer *w)
{
    if (!w) return KPW_ERR_INVALID_ARG;
    if (w->closed) return KPW_OK;
    try {
        int st = KPW_OK;
        if (!w->dead) st = process(w, true);
        else if (w->offs.size() > 1) {  // invalid record seen: flush what was valid
            w->dead = false;
            st = process(w, true);
        }
        if (!st) st = join_bg(w);
        if (st) return st;
        if (trace_on()) fprintf(stderr, "[kpw] staging: slot waits %.1f ms, host copies %.1f ms\n", w->t_slotwait, w->t_copy);
        st = w->fw->close();
        if (st) return wfail(w, st, w->fw->error());
        w->closed = true;
        return KPW_OK;
    } catch (...) {
        return wfail(w, KPW_ERR_DEVICE, "close failed");
    }
}

extern "C" int kpw_writer_file_bytes(const kpw_writer *w, const uint8_t **bytes, uint64_t *len)
{
    if (!w || !bytes || !len) return KPW_ERR_INVALID_ARG;
    if (!w->closed) return KPW_ERR_STATE;
    *bytes = w->fw->memory_data();
    *len = w->fw->memory_size();
    return KPW_OK;
}

extern "C" void kpw_writer_free(kpw_writer *w) { delete w; }
