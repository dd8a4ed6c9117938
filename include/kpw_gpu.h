/*
 * kpw_gpu.h — C-ABI of the MI355X-native Parquet column-chunk encoder (libkpw_gpu.so).
 *
 * Two layers, both plain C (pointers + sizes, integer status codes, no C++ exceptions,
 * no torch/HIP types in any signature):
 *
 *  (1) kpw_writer_*  — the drop-in for the reference seam ParquetFile<T>
 *      (src/main/java/ir/sahab/kafka/reader/ParquetFile.java:24-100): open / write /
 *      getDataSize / getNumWrittenRecords / close, fed with the raw record values the
 *      caller already holds (KafkaProtoParquetWriter.java:270 `record.value()`), so
 *      parser.parseFrom + ProtoWriteSupport shredding run on the GPU (K1).  The host part
 *      of parquet-mr that north_star keeps on the host (Thrift page headers, footer, file
 *      bytes) is done here on the CPU side of the library.
 *
 *  (2) kpw_encoder_* — the flush-path primitive a JVM host binds when it keeps its own
 *      ParquetFileWriter: device-resident record batch -> encoded pages + per-page
 *      metadata for every row group parquet-mr would cut (replaces
 *      InternalParquetRecordWriter.flushRowGroupToStore -> ColumnWriteStoreV1.flush ->
 *      ColumnChunkPageWriter.writePage, parquet-mr 1.10.1).
 *
 * Threading: handles are independent; one handle is used by one thread at a time
 * (ParquetFile is documented not thread-safe, ParquetFile.java:19-20).  Each handle owns
 * its HIP streams and device buffers on the device it was opened on.
 */
#ifndef KPW_GPU_H
#define KPW_GPU_H

#include <stdint.h>
#include "kpw_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ (1) ParquetFile drop-in */

typedef struct kpw_writer kpw_writer;

/* new ParquetFile(filePath, protoClass, properties) — ParquetFile.java:36-54.
 * path == NULL keeps the file in memory (kpw_writer_file_bytes); otherwise the file is
 * created/overwritten (Mode.OVERWRITE, ParquetFile.java:46).  device = HIP ordinal. */
kpw_writer *kpw_writer_open(int device, const kpw_schema *schema, const kpw_props *props,
                            const char *path, int *status);

/* n x { parser.parseFrom(value); ParquetFile.write(T) } — KafkaProtoParquetWriter.java:268-277,
 * ParquetFile.java:59-62.  data/offsets are host memory; record i is
 * data[offsets[i] .. offsets[i+1]); the caller may reuse both when the call returns.  Data in a
 * kpw_host_alloc buffer is DMA'd to the device directly; other memory takes one host copy.
 * On an invalid record the call returns KPW_ERR_INVALID_PROTO: the records before it are
 * written, it and the rest are not (kpw_writer_failed_record).  For writes of <= 65536 records
 * that is reported by this call (the reference throws at parseFrom); larger writes are
 * validated on the GPU and the error surfaces at the next call (write / getDataSize / close),
 * with kpw_writer_num_records corrected then.  The writer accepts no records after it;
 * close() writes the ones before it. */
int kpw_writer_write(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n);

/* kpw_writer_write for a consumer that polls into a ring of >= 2 kpw_host_alloc batches
 * (north_star: polled batches in pinned staging, moved to HBM by hipMemcpyAsync on a side
 * stream): the call returns once the batch's DMA is queued, and the DMA may still read `data`
 * until the NEXT kpw_writer_* call on this handle returns (any entry point, getters and
 * kpw_writer_free included, waits for it before returning; the next async write waits for it
 * then, with its own DMA already queued behind it, so the copy stream never idles between
 * poll batches).  `offsets` may be reused at once.  Same records, file and errors as
 * kpw_writer_write; memory outside kpw_host_alloc is copied before the call returns. */
int kpw_writer_write_async(kpw_writer *w, const uint8_t *data, const uint64_t *offsets, uint64_t n);

/* Pinned (page-locked) host memory for record batches: where polled Kafka batches are meant
 * to land (north_star: "pinned host staging buffers"), so kpw_writer_write can DMA them to
 * HBM without a host copy.  Thread-safe; any writer handle on any device may read them. */
void *kpw_host_alloc(uint64_t bytes, int *status);
void kpw_host_free(void *p);

/* The library keeps freed HBM and pinned blocks for the next writer (a writer is one file and
 * files rotate; hipFree synchronises the device): up to KPW_DEV_CACHE_GB per device (default:
 * 96 GB or the device's peak live bytes, whichever is larger, at most 3/4 of the device) and
 * KPW_PIN_CACHE_GB pinned per process (default 48 GB divided by LOCAL_WORLD_SIZE, the ranks
 * sharing the host), read once per process.  This releases every idle block and idle pooled
 * stream set now (e.g. before a co-located consumer or framework allocates).  Thread-safe.  No
 * reference counterpart (the JVM writer allocates on the Java heap). */
void kpw_trim_caches(void);

/* Allocator figures of this process: [0] device cache cap (bytes, the current device's), [1] pinned cache cap,
 * [2] device bytes live, [3] device bytes idle in the cache, [4] pinned bytes live, [5] pinned
 * bytes idle, [6] hipMalloc calls, [7] their host ms, [8] hipFree calls, [9] their ms,
 * [10] hipHostMalloc calls, [11] ms, [12] hipHostFree calls, [13] ms, [14] device cache hits,
 * [15] pinned cache hits, [16] hipMalloc failures retried after releasing the idle blocks,
 * [17] device-wide synchronisations before freeing a grown buffer, [18] their host ms,
 * [19] writer jobs admitted by the device encode gate (KPW_DEVICE_ENCODES), [20] their host
 * ms of waiting for admission.
 * Returns the number of entries written (<= cap).  Diagnostics; no reference counterpart. */
int kpw_cache_stats(double *out, int cap);

/* The WorkerThread size-rotation loop (KafkaProtoParquetWriter.java:277-285,306-308):
 * writes records in order and stops right after the first one for which
 * getDataSize() >= max_file_size.  *n_accepted = records written, *full = 1 if the stop
 * condition fired (the caller then closes this file and opens the next).  Single-page chunks
 * without HDFS alignment: the stop point is found by encoding staged prefixes (segment checks +
 * bisection).  Multi-page chunks (page cuts shrink the buffered size inside a row group) and
 * HDFS alignment: record at a time through the host getDataSize model, page sizes from GPU
 * probes of the open row group.  Both are identical to the per-record loop.  An invalid record
 * ends the batch as in kpw_writer_write. */
int kpw_writer_write_until_full(kpw_writer *w, const uint8_t *data, const uint64_t *offsets,
                                uint64_t n, int64_t max_file_size, uint64_t *n_accepted, int *full);

/* getDataSize() — ParquetFile.java:77-79, parquet-mr InternalParquetRecordWriter.getDataSize()
 * (lastRowGroupEndPos + buffered).  With writes of <= 65536 records (the WorkerThread loop) an
 * exact host model answers in O(1) and cuts row groups on the host; after a larger write the
 * staged records are encoded to answer.  -1 on failure (see kpw_writer_failed_record). */
int64_t kpw_writer_data_size(kpw_writer *w);
int64_t kpw_writer_num_records(const kpw_writer *w); /* getNumWrittenRecords() ParquetFile.java:81-83 */
int64_t kpw_writer_creation_time_ms(const kpw_writer *w); /* getCreationDate()  ParquetFile.java:70-72 */
int kpw_writer_close(kpw_writer *w);                 /* close() (idempotent)   ParquetFile.java:65-68 */
int kpw_writer_file_bytes(const kpw_writer *w, const uint8_t **bytes, uint64_t *len);
int64_t kpw_writer_failed_record(const kpw_writer *w); /* -1 if none */

/* Pipeline statistics of this writer, accumulated over its encode jobs (waits for queued
 * jobs).  [0] jobs, [1] records encoded, [2] record bytes encoded, [3] uncompressed page
 * bytes, [4] compressed page bytes, [5..14] device milliseconds per stage summed over jobs
 * (HIP events on the encoder's stream, kpw_encoder_stage_times order), [15] encode wall
 * milliseconds of the worker thread, [16] scan look-backs that recomputed a predecessor tile
 * instead of waiting longer (exact either way; every look-back scan runs inside the encoders —
 * the writer's own record-offsets scan is reduce-then-scan and has none), [17] milliseconds from
 * the file's first record DMA to the completion of its last (the H2D span, after close; 0
 * before).  Returns the number of entries written (<= cap). */
int kpw_writer_stats(kpw_writer *w, double *out, int cap);
const char *kpw_writer_last_error(const kpw_writer *w);
void kpw_writer_free(kpw_writer *w);

/* ------------------------------------------------------------------ (2) flush-path encoder */

typedef struct kpw_encoder kpw_encoder;

kpw_encoder *kpw_encoder_create(int device, const kpw_schema *schema, const kpw_props *props, int *status);
void kpw_encoder_destroy(kpw_encoder *e);
const char *kpw_encoder_last_error(const kpw_encoder *e);

/* Per-page metadata of one encoded page (data or dictionary). */
typedef struct kpw_page_info {
    int32_t page_type;          /* KPW_DATA_PAGE / KPW_DATA_PAGE_V2 (writer_version 2) / KPW_DICTIONARY_PAGE */
    int32_t num_values;         /* data: values incl. nulls; dictionary: entries */
    int32_t encoding;           /* values encoding (data) or dictionary encoding */
    int32_t dl_encoding;        /* v1: KPW_ENC_RLE (optional) / KPW_ENC_BIT_PACKED (required) */
    int32_t rl_encoding;        /* v1: KPW_ENC_BIT_PACKED (DevNull, no repeated fields) */
    int32_t has_stats;          /* 0 for dictionary pages */
    int64_t uncompressed_size;  /* v2: level bytes + uncompressed values */
    int64_t compressed_size;    /* v2: level bytes + compressed values */
    uint64_t offset;            /* byte offset of the (compressed) body in the batch output */
    int64_t null_count;
    int32_t has_min_max;
    int32_t min_len, max_len;   /* stats bytes (Statistics.getMinBytes/getMaxBytes) */
    int32_t dl_byte_length;     /* v2: definition-level bytes after the repetition levels (never compressed) */
    uint64_t min_off, max_off;  /* offsets into kpw_batch_info.stats_bytes */
    int32_t num_rows;           /* v2 DataPageHeaderV2.num_rows (= num_values: no repeated fields) */
    int32_t rl_byte_length;     /* v2: repetition-level bytes at the start of the body (never compressed) */
} kpw_page_info;

typedef struct kpw_chunk_info {
    int32_t column;
    int32_t first_page;         /* index into kpw_batch_info.pages; dictionary page first */
    int32_t num_pages;
    int32_t has_dictionary;
    int64_t num_values;
} kpw_chunk_info;

typedef struct kpw_row_group_info {
    int64_t first_record;       /* index within the batch */
    int64_t num_records;
    int32_t first_chunk;        /* index into kpw_batch_info.chunks (schema order) */
    int32_t reserved;
} kpw_row_group_info;

typedef struct kpw_batch_info {
    int32_t num_row_groups;
    int32_t num_chunks;
    int32_t num_pages;
    int32_t reserved;
    const kpw_row_group_info *row_groups;
    const kpw_chunk_info *chunks;
    const kpw_page_info *pages;
    const uint8_t *stats_bytes;         /* host memory */
    uint64_t stats_len;
    const uint8_t *device_pages;        /* device pointer to all page bodies (valid until next call) */
    uint64_t device_pages_len;
    int64_t records_consumed;           /* records covered by the returned row groups */
    int64_t open_records;               /* records left in the open (unflushed) row group */
    int64_t open_buffered_size;         /* columnStore.getBufferedSize() of the open row group */
    int64_t invalid_record;             /* first invalid record index, -1 if none */
} kpw_batch_info;

/* Encode a device-resident batch of n records (d_data/d_offsets are device pointers,
 * d_offsets has n+1 entries, offsets relative to d_data).  Cuts row groups exactly where
 * InternalParquetRecordWriter.checkBlockSizeReached would (starting a fresh row group at
 * record 0); if `final` the trailing open row group is flushed too (close()).  Blocking;
 * the returned info stays valid until the next call on this encoder.  hip_stream may be
 * NULL (the encoder's own stream). */
int kpw_encoder_encode(kpw_encoder *e, const uint8_t *d_data, const uint64_t *d_offsets, uint64_t n,
                       int final, int64_t next_row_group_size, void *hip_stream, kpw_batch_info *info);

/* Copy page bodies [off, off+len) of the last batch to host memory. */
int kpw_encoder_copy_pages(kpw_encoder *e, uint64_t off, uint64_t len, void *host_dst);

/* Timing of the last encode: device milliseconds measured with HIP events on the encoder's
 * stream.  Index order: [0] decode, [1] plan, [2] stats+dictionary, [3] rle,
 * [4] layout+plain+write, [5] compress, [6] metadata, [7] total, [8] k_decode kernel alone,
 * [9] K7 Snappy kernels alone (k_snappy_v x2, k_snappy_s_rest x2, k_snappy_seg, k_snappy_page_sizes,
 * k_snappy_copy; 0 when uncompressed).  Returns entries written (<= cap). */
int kpw_encoder_stage_times(const kpw_encoder *e, float *ms, int cap);

/* Device memory for kpw_encoder_encode's batches, from this library's own HIP runtime (a JVM
 * host that binds the flush path directly has no other; tests and bench.py use it too, so one
 * runtime owns every device pointer the encoder sees).  No reference counterpart: parquet-mr
 * keeps its buffers on the Java heap.  kpw_device_alloc returns NULL with *status set on
 * failure; the copies are synchronous and return a status. */
void *kpw_device_alloc(int device, uint64_t bytes, int *status);
void kpw_device_free(void *d_ptr);
int kpw_copy_h2d(int device, void *d_dst, const void *src, uint64_t bytes);
int kpw_copy_d2h(int device, void *dst, const void *d_src, uint64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* KPW_GPU_H */
