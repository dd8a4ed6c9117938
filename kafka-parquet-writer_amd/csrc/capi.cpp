// capi.cpp — extern "C" boundary of libkpw_gpu.so (include/kpw_gpu.h).
// No C++ exception crosses this file: every entry point catches and maps to a status.
#include <chrono>
#include <cstring>
#include <new>
#include <string>
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

struct kpw_writer {
    Engine eng;
    FileWriter *fw = nullptr;
    std::vector<uint8_t> data;       // staged record bytes (records of the open row group + new ones)
    std::vector<uint64_t> offs{0};
    uint64_t staged_bytes_at_encode = ~0ull;
    int64_t num_records = 0;         // ParquetFile.numWrittenRecords
    int64_t last_rg_end = 0;         // InternalParquetRecordWriter.lastRowGroupEndPos
    int64_t open_buffered = 0;
    int64_t failed_record = -1;
    int64_t created_ms = 0;
    bool closed = false, dead = false;
    std::string err;
    DevBuf d_in, d_off;
    std::vector<uint8_t> host_pages;
    ~kpw_writer() { delete fw; }
};

static int wfail(kpw_writer *w, int st, const std::string &m)
{
    w->err = m;
    if (st != KPW_ERR_IO) w->dead = true;
    return st;
}

// Encode the staged records: flush every row group parquet-mr would have completed (all of
// them if final), keep the open row group's records staged.
static int process(kpw_writer *w, bool final)
{
    const uint64_t n = w->offs.size() - 1;
    if (!final && w->staged_bytes_at_encode == w->data.size()) return KPW_OK;  // nothing new
    if (w->d_in.ensure(w->data.size() + 16) || w->d_off.ensure((n + 1) * 8))
        return wfail(w, KPW_ERR_NOMEM, "device staging allocation failed");
    hipStream_t s = w->eng.stream;
    if (!w->data.empty() && hipMemcpyAsync(w->d_in.p, w->data.data(), w->data.size(), hipMemcpyHostToDevice, s) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "H2D failed");
    if (hipMemcpyAsync(w->d_off.p, w->offs.data(), (n + 1) * 8, hipMemcpyHostToDevice, s) != hipSuccess)
        return wfail(w, KPW_ERR_DEVICE, "H2D failed");
    BatchOut out;
    int st = w->eng.encode(w->d_in.as<uint8_t>(), w->d_off.as<uint64_t>(), n, final, w->eng.props.block_size, nullptr, out);
    if (st) return wfail(w, st, w->eng.error());
    if (out.pages_len) {
        w->host_pages.resize(out.pages_len);
        st = w->eng.copy_pages(0, out.pages_len, w->host_pages.data());
        if (st) return wfail(w, st, w->eng.error());
    }
    for (size_t r = 0; r < out.rgs.size(); r++) {
        st = w->fw->write_row_group(out, (int)r, w->host_pages.data(), 0);
        if (st) return wfail(w, st, w->fw->error());
        w->last_rg_end = w->fw->pos();
    }
    // keep [records_consumed, valid end) staged
    const uint64_t keep0 = (uint64_t)out.records_consumed;
    uint64_t keep1 = n;
    int rc = KPW_OK;
    if (out.invalid_record >= 0) {
        keep1 = (uint64_t)out.invalid_record;
        const int64_t dropped = (int64_t)(n - keep1);
        w->failed_record = w->num_records - dropped;
        w->num_records -= dropped;
        rc = KPW_ERR_INVALID_PROTO;
        w->err = "Invalid proto message received (record " + std::to_string(w->failed_record) + ")";
    }
    const uint64_t b0 = w->offs[keep0], b1 = w->offs[keep1];
    std::vector<uint8_t> nd(w->data.begin() + b0, w->data.begin() + b1);
    std::vector<uint64_t> no;
    no.reserve(keep1 - keep0 + 1);
    for (uint64_t i = keep0; i <= keep1; i++) no.push_back(w->offs[i] - b0);
    w->data.swap(nd);
    w->offs.swap(no);
    w->open_buffered = final ? 0 : out.open_buffered;
    if (rc) {
        // the open row group may have been cut by the invalid record: re-plan it next time
        w->staged_bytes_at_encode = ~0ull;
        w->dead = true;
        return rc;
    }
    w->staged_bytes_at_encode = w->data.size();
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

static const uint64_t kStageFlushBytes = 512ull << 20;

extern "C" int kpw_writer_write(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n)
{
    if (!w || (n && (!data || !offsets))) return KPW_ERR_INVALID_ARG;
    if (w->closed || w->dead) return KPW_ERR_STATE;
    try {
        const uint64_t base = w->data.size();
        w->data.insert(w->data.end(), data + offsets[0], data + offsets[n]);
        for (uint64_t i = 1; i <= n; i++) w->offs.push_back(base + offsets[i] - offsets[0]);
        w->num_records += (int64_t)n;
        if (w->data.size() >= kStageFlushBytes + (uint64_t)w->eng.props.block_size) return process(w, false);
        return KPW_OK;
    } catch (const std::bad_alloc &) {
        return wfail(w, KPW_ERR_NOMEM, "host staging allocation failed");
    } catch (...) {
        return wfail(w, KPW_ERR_DEVICE, "unexpected failure");
    }
}

extern "C" int kpw_writer_write_until_full(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                           int64_t max_file_size, uint64_t *n_accepted, int *full)
{
    (void)data; (void)offsets; (void)n; (void)max_file_size; (void)n_accepted; (void)full;
    if (!w) return KPW_ERR_INVALID_ARG;
    w->err = "write_until_full: per-record size rotation on the GPU path is the next round";
    return KPW_ERR_UNSUPPORTED;
}

extern "C" int64_t kpw_writer_data_size(kpw_writer *w)
{
    if (!w) return -1;
    if (w->closed) return w->fw->pos();
    if (!w->dead) {
        try {
            if (process(w, false)) return -1;
        } catch (...) {
            return -1;
        }
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
        if (st) return st;
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
    *bytes = w->fw->memory().data();
    *len = w->fw->memory().size();
    return KPW_OK;
}

extern "C" void kpw_writer_free(kpw_writer *w) { delete w; }
