// sizemodel.h — exact host model of getDataSize() for the reference's per-record loop.
//
// The reference's WorkerThread writes ONE record and then asks ParquetFile.getDataSize()
// (KafkaProtoParquetWriter.java:277-285,306-308 -> ParquetFile.java:77-79), i.e. parquet-mr
// 1.10.1 InternalParquetRecordWriter.getDataSize() = lastRowGroupEndPos +
// columnStore.getBufferedSize().  Answering that from the GPU would re-encode the open row
// group per record, so the writer keeps this O(columns)-per-record model instead:
//
//   - a wire-length scan of each record (the K1 rules: field -> column, wire-type check, last
//     occurrence wins, unknown fields and groups skipped, 10-byte varints, missing required
//     -> invalid) giving presence and the raw (plain-equivalent) size of every column;
//   - per column ColumnWriterV1's buffered size: definition-level RunLengthBitPackingHybrid
//     encoder bytes emitted so far (counted, no bytes kept) + FallbackValuesWriter
//     rawDataByteSize / PlainValuesWriter size / BooleanPlainValuesWriter (count+7)/8, plus
//     ColumnChunkPageWriter.getMemSize(): the header + compressed bytes of the pages this
//     column already cut in the open row group;
//   - ColumnWriterV1.accountForValueWritten's sampled page check.  A page cut (pageSize <
//     blockSize) resets the column's page state here, and the cut page's header + compressed
//     size comes from the GPU (the writer encodes the open row group's prefix, Engine::
//     probe_pages) before the record's row-group check: add() returns PAGES and finish_pages()
//     completes the record with those sizes;
//   - InternalParquetRecordWriter.checkBlockSizeReached's sampled row-group check with Java's
//     float/long arithmetic.
//
// PARQUET_2_0 (an explicit opt-in; the reference never selects it, ParquetFile.java:42-50):
// ColumnWriteStoreV2.sizeCheck instead of the per-column page check (after the record, once
// rowCount reaches rowCountForNextSizeCheck: a column within 10% of pageSize writes its page),
// and BOOLEAN values counted as the RLE bytes of their RunLengthBitPackingHybridValuesWriter.
//
// It decides row-group cuts on the host for this loop; the GPU encodes exactly those records
// (the encoder's own planner plans the same cut, checked per row group).
#pragma once
#include <stdint.h>
#include <vector>

#include "engine.h"

namespace kpw {

// RunLengthBitPackingHybridEncoder(bitWidth 1) byte count: BytesInput size after each
// writeInt, without the bytes (the header byte of a bit-packed run is reserved when the run
// opens, as in writeOrAppendBitPackedRun).
struct RleCount {
    int64_t out = 0;
    uint32_t prev = 0;
    int32_t rc = 0;
    int32_t nbuf = 0;
    int32_t groups = 0;
    bool hdr_open = false;
    void write(uint32_t v);
};

class SizeModel {
public:
    enum { OK = 0, CUT = 1, PAGES = 2, INVALID = -1, MISMATCH = -3 };
    // false if the configuration is outside the model
    bool init(const std::vector<ColInfo> &cols, const kpw_props &props);
    // One record: OK, CUT (a row group ends with this record), INVALID (parseFrom would
    // throw; nothing changed), PAGES (at least one column cut a page with this record: call
    // finish_pages with the flushed page bytes before anything else).
    int add(const uint8_t *rec, uint64_t len);
    // Completes a PAGES record: per column the pages cut in the open row group so far and their
    // header + compressed bytes (from the GPU).  OK, CUT, or MISMATCH (page counts differ from
    // the model's: the two restatements disagree, a bug).
    // npages[c] < 0: column c was not probed (it cut no page since the last finish_pages, so
    // its flushed bytes are unchanged).
    int finish_pages(const std::vector<int32_t> &npages, const std::vector<int64_t> &flushed);
    // the columns that cut a page since the last finish_pages (the ones a probe must encode)
    void cut_columns(std::vector<char> &mask) const;
    // per column: the open row group's page cuts so far (a page ends before record cut_at[i])
    void page_cuts(std::vector<std::vector<int64_t>> &cuts) const;
    int64_t buffered() const;               // columnStore.getBufferedSize()
    int64_t record_count() const { return record_count_; }
    bool multi_page() const { return multi_; }
    // nextRowGroupSize for the open row group (HDFS alignment: set after each cut from the
    // file position; blockSize otherwise)
    void set_next_rg_size(int64_t t) { next_rg_size_ = t; }
    // a fresh row group (resynchronisation after the GPU planned the cuts)
    void restart(int64_t next_rg_size);

private:
    struct Col {
        int32_t field_number, wire_type, phys, optional, vsize;
        RleCount dl;
        int64_t data = 0;                   // raw bytes (non-boolean) or boolean values
        int64_t flushed = 0;                // pageWriter.getMemSize(): cut pages, header + compressed
        int32_t pages = 0;                  // pages cut in the open row group
        int32_t pages_known = 0;            // pages whose flushed bytes `flushed` holds
        std::vector<int64_t> cut_at;        // record count of the open row group at each page cut
        int32_t value_count = 0, next_check = 100;
        RleCount bv;                        // v2 BOOLEAN: RunLengthBitPackingHybridValuesWriter of the values
        int64_t rows_written = 0;           // v2: rowCount at this column's last page
        int64_t mem(bool v2) const;         // rl + dl + data buffered (the page check's memSize)
    };
    bool scan(const uint8_t *rec, uint64_t len);
    int block_check();                      // checkBlockSizeReached after a record: OK / CUT
    void reset_store();
    std::vector<Col> cols_;
    std::vector<int16_t> fmap_;             // field number (< 1024) -> column
    struct Wire {                           // what the scan reads per column, packed
        uint32_t wire_type, vsize, required;
    };
    std::vector<Wire> wire_;
    uint32_t nreq_ = 0;                     // required columns
    std::vector<uint32_t> seen_;            // == gen_: present in the record being scanned
    uint32_t gen_ = 0;
    std::vector<uint32_t> raw_;
    std::vector<uint8_t> bval_;             // BOOLEAN columns: the record's value (last occurrence)
    bool multi_ = false, v2_ = false;
    int64_t v2_next_check_ = 100;           // ColumnWriteStoreV2.rowCountForNextSizeCheck
    int64_t page_size_ = 0, block_size_ = 0, next_rg_size_ = 0;
    int64_t record_count_ = 0, next_mem_check_ = 100;
};

}  // namespace kpw
