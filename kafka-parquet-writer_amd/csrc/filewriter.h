// filewriter.h — host-side Parquet file assembly (what north_star keeps on the host):
// Thrift-compact page headers, column-chunk/row-group metadata and the footer, restating
// parquet-mr 1.10.1 ParquetFileWriter + ParquetMetadataConverter as driven by
// ColumnChunkPageWriteStore.flushToFileWriter (dictionary page first, then data pages).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <string>
#include <vector>

#include "engine.h"

namespace kpw {

struct StatsOut {
    int phys = 0;
    bool has = false;       // hasNonNullValue
    int64_t nulls = 0;
    std::string min, max;
};

struct ChunkMeta {
    int phys, codec;
    bool v2 = false;                              // EncodingStats.usesV2Pages
    std::vector<int> encodings;                   // insertion order, de-duplicated
    std::vector<std::pair<int, int>> dict_stats;  // (encoding, pages)
    std::vector<std::pair<int, int>> data_stats;
    int64_t num_values, total_uncomp, total_comp, data_page_offset;
    StatsOut stats;
};

struct RowGroupMeta {
    int64_t rows, total_bytes;
    std::vector<ChunkMeta> chunks;
};

// Thrift-compact PageHeader of one page exactly as write_row_group emits it
// (ParquetMetadataConverter.writeDataPageHeader / writeDataPageV2Header / dictionary page).
std::string page_header(const PageOut &pg, int phys);

// Host copy split over a few threads for large buffers (page faults and memcpy in parallel).
void par_copy(uint8_t *dst, const uint8_t *src, size_t n);

class FileWriter {
public:
    FileWriter(const std::vector<ColInfo> &cols, const std::string &message_name, const std::string &proto_class,
               const kpw_props &props);
    ~FileWriter();
    int open(const char *path);       // nullptr = memory
    // Appends one encoded row group; `pages` is host memory holding the batch's page bodies
    // (indexed by PageOut.offset relative to pages_base).  With d2h != nullptr (memory mode
    // only) `pages` is DEVICE memory: the bodies are copied straight into the in-memory file
    // on that stream (the caller synchronises it before the file is read).
    int write_row_group(const BatchOut &b, int rg, const uint8_t *pages, uint64_t pages_base, hipStream_t d2h = nullptr);
    bool memory_mode() const { return fp_ == nullptr; }
    // Bytes write_row_group would append for row group `rg` (page headers + compressed bodies).
    int64_t row_group_size(const BatchOut &b, int rg) const;
    int close();                      // footer + magic
    int64_t pos() const { return pos_; }
    // InternalParquetRecordWriter.nextRowGroupSize after the row groups written so far:
    // min(PaddingAlignment.nextRowGroupSize, blockSize); blockSize before the first one
    int64_t next_row_group_size() const;
    const uint8_t *memory_data();     // contiguous view (built on first use after close)
    size_t memory_size() const { return mem_len_; }
    const std::string &error() const { return err_; }
    // Memory mode, device assembly: while on, write_row_group (with `pages` = the DEVICE page
    // buffer) only records the job's bytes as segments — header / padding bytes into a host blob,
    // page bodies as device ranges — and takes their room in the in-memory file; take_asm()
    // hands them over with the file spans they fill.  The caller gathers them into one device
    // buffer and DMAs it straight into those spans (no host copy of the page bodies).
    struct AsmSeg { uint64_t dst; uint64_t src; uint32_t len; uint32_t dev; };   // dst: from the job's first byte
    void device_assembly(bool on) { dev_asm_ = on && fp_ == nullptr; }
    int take_asm(std::string &blob, std::vector<AsmSeg> &segs, uint64_t &total,
                 std::vector<std::pair<uint8_t *, size_t>> &spans);

private:
    int put(const void *p, size_t n);
    int put_device(const uint8_t *d, size_t n, hipStream_t s);
    int reserve(size_t n);            // arena room for n more bytes
    int align_for_row_group();        // PaddingAlignment.alignForRowGroup (startBlock)
    std::vector<ColInfo> cols_;
    std::string message_name_, proto_class_;
    kpw_props props_;
    FILE *fp_ = nullptr;
    // memory mode: pinned chunks (page bodies arrive by D2H straight into place); `flat_` is a
    // contiguous copy for memory_data() when there is more than one chunk
    std::vector<std::pair<uint8_t *, size_t>> chunks_;
    uint8_t *flat_ = nullptr;
    size_t mem_len_ = 0, mem_cap_ = 0;
    int64_t pos_ = 0;
    std::vector<RowGroupMeta> rgs_;
    std::string err_;
    bool closed_ = false;
    bool dev_asm_ = false;
    std::string asm_blob_;
    std::vector<AsmSeg> asm_segs_;
    uint64_t asm_start_ = 0, asm_len_ = 0;   // the job's range in the in-memory file
    int asm_put(const void *p, size_t n, bool dev);
};

}  // namespace kpw
