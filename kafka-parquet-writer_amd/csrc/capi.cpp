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
        q.dl_byte_length = p.dl_byte_length; q.num_rows = p.num_rows; q.rl_byte_length = p.rl_byte_length;
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

// The ParquetFile drop-in (kpw_writer_*) and kpw_host_alloc live in writer.cpp.

// ---------------------------------------------------------------- device memory (flush-path batches)

extern "C" void *kpw_device_alloc(int device, uint64_t bytes, int *status)
{
    void *p = nullptr;
    int st = KPW_OK;
    if (hipSetDevice(device) != hipSuccess) st = KPW_ERR_DEVICE;
    else if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) { st = KPW_ERR_NOMEM; p = nullptr; }
    if (status) *status = st;
    return p;
}

extern "C" void kpw_device_free(void *d_ptr)
{
    if (d_ptr) (void)hipFree(d_ptr);
}

extern "C" int kpw_copy_h2d(int device, void *d_dst, const void *src, uint64_t bytes)
{
    if (!bytes) return KPW_OK;
    if (!d_dst || !src) return KPW_ERR_INVALID_ARG;
    if (hipSetDevice(device) != hipSuccess) return KPW_ERR_DEVICE;
    return hipMemcpy(d_dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? KPW_OK : KPW_ERR_DEVICE;
}

extern "C" int kpw_copy_d2h(int device, void *dst, const void *d_src, uint64_t bytes)
{
    if (!bytes) return KPW_OK;
    if (!dst || !d_src) return KPW_ERR_INVALID_ARG;
    if (hipSetDevice(device) != hipSuccess) return KPW_ERR_DEVICE;
    return hipMemcpy(dst, d_src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? KPW_OK : KPW_ERR_DEVICE;
}
