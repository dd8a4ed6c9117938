/*
 * kpw_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's Parquet write path, value by value, in the
 * order parquet-mr 1.10.1 executes it.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker/baseline — never as
 * the thing measured or shipped.
 *
 * Parity status: the reference is Java 8 + parquet-mr 1.10.1 + snappy-java (pom.xml:44-48),
 * none of which exists in this container (no JVM, no jars, no network).
 * The reference's own tests hold NO golden bytes.  This oracle is pinned by:
 *   (1) Parquet-spec known-answer vectors for the RLE/bit-packing hybrid and PLAIN
 *       (tests/golden/spec_vectors.json),
 *   (2) pyarrow 25 reading every file it writes back value-exact, and pyarrow's Snappy
 *       decoding every page it compresses,
 *   (3) the reference test's record-level assertions restated (round-trip multiset,
 *       getDataSize()/maxFileSize ratio, KafkaProtoParquetWriterTest.java:136-172).
 * Byte identity with parquet-mr itself is therefore "parity unpinned" (see DESIGN.md).
 */
#ifndef KPW_ORACLE_H
#define KPW_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/kpw_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kpwo_writer kpwo_writer;

/* ParquetFile(Path, Class<T>, ParquetProperties) — ParquetFile.java:36-54.  The file is
 * written to an in-memory buffer (the output stream is out of scope). */
kpwo_writer *kpwo_open(const kpw_schema *schema, const kpw_props *props, int *status);

/* parser.parseFrom(bytes) + ParquetFile.write(T) for one record
 * (KafkaProtoParquetWriter.java:268-277, ParquetFile.java:59-62).  Returns
 * KPW_ERR_INVALID_PROTO (record not written) for anything protobuf-java rejects. */
int kpwo_write(kpwo_writer *w, const uint8_t *rec, uint64_t len);

/* n consecutive kpwo_write calls; stops at the first invalid record. */
int kpwo_write_batch(kpwo_writer *w, const uint8_t *data, const uint64_t *offsets,
                     uint64_t n, uint64_t *n_written);

/* The WorkerThread loop restated (KafkaProtoParquetWriter.java:268-285): write records
 * one at a time and stop right after the first record for which
 * getDataSize() >= max_file_size.  *n_accepted = records written; *full = 1 if the
 * file became full. */
int kpwo_write_until_full(kpwo_writer *w, const uint8_t *data, const uint64_t *offsets,
                          uint64_t n, int64_t max_file_size, uint64_t *n_accepted, int *full);

int64_t kpwo_data_size(const kpwo_writer *w);      /* ParquetFile.getDataSize(), PF:77-79 */
int64_t kpwo_num_records(const kpwo_writer *w);    /* getNumWrittenRecords(), PF:81-83 */
int kpwo_close(kpwo_writer *w);                    /* ParquetFile.close(), PF:65-68 (idempotent) */
int kpwo_file_bytes(const kpwo_writer *w, const uint8_t **bytes, uint64_t *len);
int kpwo_num_row_groups(const kpwo_writer *w);
void kpwo_free(kpwo_writer *w);

/* ---- stand-alone primitives (known-answer tests) ---- */
/* RunLengthBitPackingHybridEncoder over n values of the given width; returns bytes
 * written or -1 if cap is too small. */
int64_t kpwo_rle_encode(const uint32_t *vals, uint64_t n, int bit_width, uint8_t *out, uint64_t cap);
/* DeltaBinaryPackingValuesWriterForInteger (is_long 0, low 32 bits of each value) /
 * ForLong (is_long 1) over n values, getBytes() of a fresh writer; -1 if cap too small. */
int64_t kpwo_delta_encode(const uint64_t *vals, uint64_t n, int is_long, uint8_t *out, uint64_t cap);
/* snappy::RawCompress, pinned algorithm (see oracle_snappy.c header). */
int64_t kpwo_snappy_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);
uint64_t kpwo_snappy_max_compressed_length(uint64_t n);
/* GZIP (oracle_deflate.c): zlib 1.2.11 level-6 raw deflate in java.util.zip.GZIPOutputStream
 * framing, one member per page; -1 if it does not fit `cap` */
int64_t kpwo_deflate_raw(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);
int64_t kpwo_gzip_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);
uint64_t kpwo_gzip_bound(uint64_t n);
uint32_t kpwo_crc32(uint32_t crc, const uint8_t *p, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
