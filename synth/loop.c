/* loop.c — the reference's per-record WorkerThread loop as a C caller (bench/test
 * infrastructure, not product code).
 *
 * KafkaProtoParquetWriter.java:268-285,306-308: for each polled record, parseFrom + write ONE
 * record into the current ParquetFile, then `currentFile.getDataSize() >= maxFileSize` decides
 * the rotation.  A JVM host bound to libkpw_gpu.so through FFM/JNI makes
 * exactly these two downcalls per record; driving them from C measures the library's cost per
 * record without Python's per-call overhead.  The function pointers are the C-ABI entry points
 * (kpw_writer_write / kpw_writer_data_size) or the oracle's (kpwo_write / kpwo_data_size).
 */
#include <stdint.h>

typedef int (*kpw_write_fn)(void *w, const uint8_t *data, const uint64_t *offsets, uint64_t n);
typedef int64_t (*kpw_ds_fn)(void *w);
typedef int (*kpwo_write_fn)(void *w, const uint8_t *rec, uint64_t len);

/* Records [0, n): write one, then getDataSize(); stops after the first record with
 * getDataSize() >= max_file_size (*full = 1) or at an error (*status).  Returns the records
 * written.  *last_size = the last getDataSize(). */
uint64_t loop_kpw(void *wfn, void *dfn, void *w, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                  int64_t max_file_size, int *full, int *status, int64_t *last_size)
{
    kpw_write_fn wr = (kpw_write_fn)wfn;
    kpw_ds_fn ds = (kpw_ds_fn)dfn;
    *full = 0;
    *status = 0;
    for (uint64_t i = 0; i < n; i++) {
        const int st = wr(w, data, offsets + i, 1);
        if (st) { *status = st; return i; }
        const int64_t s = ds(w);
        *last_size = s;
        if (s < 0) { *status = -100; return i + 1; }
        if (s >= max_file_size) { *full = 1; return i + 1; }
    }
    return n;
}

uint64_t loop_oracle(void *wfn, void *dfn, void *w, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                     int64_t max_file_size, int *full, int *status, int64_t *last_size)
{
    kpwo_write_fn wr = (kpwo_write_fn)wfn;
    kpw_ds_fn ds = (kpw_ds_fn)dfn;
    *full = 0;
    *status = 0;
    for (uint64_t i = 0; i < n; i++) {
        const int st = wr(w, data + offsets[i], offsets[i + 1] - offsets[i]);
        if (st) { *status = st; return i; }
        const int64_t s = ds(w);
        *last_size = s;
        if (s >= max_file_size) { *full = 1; return i + 1; }
    }
    return n;
}
