// filewriter.cpp — Thrift-compact serialisation + ParquetFileWriter restated (host side).
//
// Conventions of parquet-mr 1.10.1 this follows (unpinned byte-for-byte where the JVM is
// itself non-deterministic):
//  * data_page_offset = position at startColumn (points at the dictionary page when there is
//    one); dictionary_page_offset is assigned as a plain field by ParquetMetadataConverter
//    and therefore never serialised;
//  * page statistics = toParquetStatistics: legacy min/max only for SIGNED sort order or
//    min == max, min_value/max_value always, nothing if len(min)+len(max) >= 4096;
//  * ColumnMetaData.encodings: insertion order (the JVM HashSet<Encoding> order is identity-
//    hash based and not reproducible); key-value metadata in java.util.HashMap order;
//  * created_by "parquet-mr version 1.10.1 (build a89df8f9932b6ef6633d06069e50c9b7970bebd1)".
#include <thread>
#include <algorithm>
#include <cstdlib>
#include "filewriter.h"
#include "memcache.h"

#include <cstring>

namespace kpw {

namespace {

class TCompact {
public:
    explicit TCompact(std::string &b) : b_(b) { last_.push_back(0); }
    void varint(uint64_t v) { while (v >= 0x80) { b_.push_back((char)(v | 0x80)); v >>= 7; } b_.push_back((char)v); }
    static uint64_t zz(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }
    void field(int16_t id, uint8_t type)
    {
        const int16_t d = (int16_t)(id - last_.back());
        if (d > 0 && d <= 15) b_.push_back((char)((d << 4) | type));
        else { b_.push_back((char)type); varint(zz(id)); }
        last_.back() = id;
    }
    void i32(int16_t id, int32_t v) { field(id, 5); varint(zz(v)); }
    void i64(int16_t id, int64_t v) { field(id, 6); varint(zz(v)); }
    void bin(int16_t id, const std::string &s) { field(id, 8); raw_bin(s); }
    void raw_bin(const std::string &s) { varint(s.size()); b_.append(s); }
    void begin(int16_t id) { field(id, 12); last_.push_back(0); }
    void begin_elem() { last_.push_back(0); }
    void end() { b_.push_back(0); last_.pop_back(); }
    void list(int16_t id, uint8_t et, uint32_t n)
    {
        field(id, 9);
        if (n < 15) b_.push_back((char)((n << 4) | et));
        else { b_.push_back((char)(0xF0 | et)); varint(n); }
    }
    void stop() { b_.push_back(0); }

private:
    std::string &b_;
    std::vector<int16_t> last_;
};

bool stats_empty(const StatsOut &s) { return !s.has && s.nulls == 0; }

// ParquetMetadataConverter.toParquetStatistics (1.10.1)
void write_stats(TCompact &t, int16_t id, const StatsOut &s)
{
    t.begin(id);
    const bool smaller = !s.has || s.phys != KPW_BYTE_ARRAY || (s.min.size() + s.max.size()) < 4096;
    if (!stats_empty(s) && smaller) {
        if (s.has && (s.phys != KPW_BYTE_ARRAY || s.min == s.max)) { t.bin(1, s.max); t.bin(2, s.min); }
        t.i64(3, s.nulls);
        if (s.has) { t.bin(5, s.max); t.bin(6, s.min); }
    }
    t.end();
}

int java_cmp(int phys, const std::string &a, const std::string &b)
{
    auto u64 = [](const std::string &s) { uint64_t v = 0; for (size_t i = 0; i < s.size(); i++) v |= (uint64_t)(uint8_t)s[i] << (8 * i); return v; };
    if (phys == KPW_BYTE_ARRAY) {
        const size_t m = std::min(a.size(), b.size());
        for (size_t i = 0; i < m; i++)
            if (a[i] != b[i]) return (uint8_t)a[i] < (uint8_t)b[i] ? -1 : 1;
        return a.size() == b.size() ? 0 : (a.size() < b.size() ? -1 : 1);
    }
    const uint64_t x = u64(a), y = u64(b);
    switch (phys) {
    case KPW_INT32: { int32_t p = (int32_t)x, q = (int32_t)y; return p < q ? -1 : p > q; }
    case KPW_INT64: { int64_t p = (int64_t)x, q = (int64_t)y; return p < q ? -1 : p > q; }
    case KPW_BOOLEAN: return (int)x - (int)y;
    case KPW_FLOAT: {
        float p, q; uint32_t xp = (uint32_t)x, yq = (uint32_t)y; memcpy(&p, &xp, 4); memcpy(&q, &yq, 4);
        if (p < q) return -1; if (p > q) return 1;
        return (int32_t)xp == (int32_t)yq ? 0 : ((int32_t)xp < (int32_t)yq ? -1 : 1);
    }
    case KPW_DOUBLE: {
        double p, q; memcpy(&p, &x, 8); memcpy(&q, &y, 8);
        if (p < q) return -1; if (p > q) return 1;
        return (int64_t)x == (int64_t)y ? 0 : ((int64_t)x < (int64_t)y ? -1 : 1);
    }
    }
    return 0;
}

// Statistics.mergeStatistics
void merge_stats(StatsOut &dst, const StatsOut &src)
{
    if (src.has) {
        if (!dst.has) { dst.min = src.min; dst.max = src.max; dst.has = true; }
        else {
            if (java_cmp(dst.phys, dst.min, src.min) > 0) dst.min = src.min;
            if (java_cmp(dst.phys, dst.max, src.max) < 0) dst.max = src.max;
        }
    }
    dst.nulls += src.nulls;
}

void add_unique(std::vector<int> &v, int e)
{
    for (int x : v) if (x == e) return;
    v.push_back(e);
}
void add_count(std::vector<std::pair<int, int>> &v, int e)
{
    for (auto &p : v) if (p.first == e) { p.second++; return; }
    v.push_back({e, 1});
}

int32_t java_string_hash(const std::string &s)
{
    uint32_t h = 0;
    for (unsigned char c : s) h = 31 * h + c;
    return (int32_t)h;
}
uint32_t hm_spread(const std::string &s) { uint32_t h = (uint32_t)java_string_hash(s); return h ^ (h >> 16); }

const char *pt_name(int pt)
{
    static const char *n[] = {"", "TYPE_DOUBLE", "TYPE_FLOAT", "TYPE_INT64", "TYPE_UINT64", "TYPE_INT32", "TYPE_FIXED64",
                              "TYPE_FIXED32", "TYPE_BOOL", "TYPE_STRING", "TYPE_GROUP", "TYPE_MESSAGE", "TYPE_BYTES",
                              "TYPE_UINT32", "TYPE_ENUM", "TYPE_SFIXED32", "TYPE_SFIXED64", "TYPE_SINT32", "TYPE_SINT64"};
    return (pt > 0 && pt <= 18) ? n[pt] : "TYPE_UNKNOWN";
}

}  // namespace

std::string page_header(const PageOut &pg, int phys)
{
    std::string hdr;
    TCompact t(hdr);
    t.i32(1, pg.page_type);
    t.i32(2, (int32_t)pg.uncompressed_size);
    t.i32(3, (int32_t)pg.compressed_size);
    if (pg.page_type == KPW_DICTIONARY_PAGE) {
        t.begin(7);
        t.i32(1, pg.num_values);
        t.i32(2, pg.encoding);
        t.end();
    } else {
        StatsOut st;
        st.phys = phys;
        st.has = pg.has_min_max != 0;
        st.nulls = pg.null_count;
        st.min = pg.min;
        st.max = pg.max;
        if (pg.page_type == KPW_DATA_PAGE_V2) {
            // ParquetMetadataConverter.writeDataPageV2Header (is_compressed never set)
            t.begin(8);
            t.i32(1, pg.num_values);
            t.i32(2, (int32_t)pg.null_count);
            t.i32(3, pg.num_rows);
            t.i32(4, pg.encoding);
            t.i32(5, pg.dl_byte_length);
            t.i32(6, pg.rl_byte_length);
            if (!stats_empty(st)) write_stats(t, 8, st);
            t.end();
        } else {
            t.begin(5);
            t.i32(1, pg.num_values);
            t.i32(2, pg.encoding);
            t.i32(3, pg.dl_encoding);
            t.i32(4, pg.rl_encoding);
            if (!stats_empty(st)) write_stats(t, 5, st);
            t.end();
        }
    }
    t.stop();
    return hdr;
}

FileWriter::FileWriter(const std::vector<ColInfo> &cols, const std::string &message_name, const std::string &proto_class,
                       const kpw_props &props)
    : cols_(cols), message_name_(message_name), proto_class_(proto_class), props_(props) {}

FileWriter::~FileWriter()
{
    if (fp_) fclose(fp_);
    for (auto &c : chunks_) pin_free(c.first);
    free(flat_);
}

int FileWriter::reserve(size_t n)
{
    while (mem_len_ + n > mem_cap_) {
        const size_t c = std::max<size_t>(256ull << 20, std::min<size_t>(mem_cap_, 4ull << 30));
        uint8_t *q = (uint8_t *)pin_alloc(c);
        if (!q) { err_ = "out of pinned host memory"; return KPW_ERR_NOMEM; }
        chunks_.push_back({q, c});
        mem_cap_ += c;
    }
    return KPW_OK;
}

const uint8_t *FileWriter::memory_data()
{
    if (chunks_.empty()) return nullptr;
    if (chunks_.size() == 1) return chunks_[0].first;
    if (!flat_) {
        flat_ = (uint8_t *)malloc(mem_len_ ? mem_len_ : 1);
        if (!flat_) return nullptr;
        size_t at = 0;
        for (auto &c : chunks_) {
            const size_t k = std::min(c.second, mem_len_ - at);
            par_copy(flat_ + at, c.first, k);
            at += k;
            if (at == mem_len_) break;
        }
    }
    return flat_;
}

int FileWriter::put_device(const uint8_t *d, size_t n, hipStream_t s)
{
    if (!n) return KPW_OK;
    if (int st = reserve(n)) return st;
    size_t at = mem_len_, base = 0;
    for (auto &c : chunks_) {
        if (at < base + c.second) {
            const size_t off = at - base, k = std::min(n, c.second - off);
            if (hipMemcpyAsync(c.first + off, d, k, hipMemcpyDeviceToHost, s) != hipSuccess) {
                err_ = "D2H of a page failed";
                return KPW_ERR_DEVICE;
            }
            d += k;
            n -= k;
            at += k;
            mem_len_ += k;
            pos_ += (int64_t)k;
            if (!n) break;
        }
        base += c.second;
    }
    return KPW_OK;
}

void par_copy(uint8_t *dst, const uint8_t *src, size_t n)
{
    static const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    const size_t kMin = 4ull << 20;
    const unsigned t = (unsigned)std::min<size_t>(hw, n / kMin);
    if (t <= 1) { memcpy(dst, src, n); return; }
    std::vector<std::thread> th;
    th.reserve(t - 1);
    // ceil(n / t) rounded up to 4 KiB: the t chunks cover all n bytes (floor(n / t) lost the
    // last n % t bytes whenever it was already a multiple of 4 KiB: a C4 slot at 192 MiB kept 6
    // stale bytes, found by tests/test_gpu_fullsize.py)
    const size_t per = ((n + t - 1) / t + 4095) & ~(size_t)4095;
    for (unsigned i = 1; i < t; i++) {
        const size_t a = std::min(n, per * i), b = std::min(n, per * (i + 1));
        if (b > a) th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
    }
    memcpy(dst, src, std::min(n, per));
    for (auto &x : th) x.join();
}

int FileWriter::asm_put(const void *p, size_t n, bool dev)
{
    if (!n) return KPW_OK;
    if (asm_segs_.empty() && asm_len_ == 0) asm_start_ = mem_len_;
    if (dev) {
        asm_segs_.push_back({asm_len_, (uint64_t)(uintptr_t)p, (uint32_t)n, 1u});
    } else {
        asm_segs_.push_back({asm_len_, (uint64_t)asm_blob_.size(), (uint32_t)n, 0u});
        asm_blob_.append((const char *)p, n);
    }
    asm_len_ += n;
    if (int st = reserve(n)) return st;
    mem_len_ += n;
    pos_ += (int64_t)n;
    return KPW_OK;
}

int FileWriter::take_asm(std::string &blob, std::vector<AsmSeg> &segs, uint64_t &total,
                         std::vector<std::pair<uint8_t *, size_t>> &spans)
{
    blob.swap(asm_blob_);
    segs.swap(asm_segs_);
    total = asm_len_;
    spans.clear();
    size_t at = asm_start_, left = asm_len_, base = 0;
    for (auto &c : chunks_) {
        if (!left) break;
        if (at < base + c.second) {
            const size_t off = at - base, k = std::min(left, c.second - off);
            spans.push_back({c.first + off, k});
            at += k;
            left -= k;
        }
        base += c.second;
    }
    asm_blob_.clear();
    asm_segs_.clear();
    asm_len_ = 0;
    return left ? KPW_ERR_DEVICE : KPW_OK;
}

int FileWriter::put(const void *p, size_t n)
{
    if (!n) return KPW_OK;
    if (dev_asm_) return asm_put(p, n, false);
    if (fp_) {
        if (fwrite(p, 1, n, fp_) != n) { err_ = "short write"; return KPW_ERR_IO; }
    } else {
        if (int st = reserve(n)) return st;
        const uint8_t *src = (const uint8_t *)p;
        size_t base = 0, left = n;
        for (auto &c : chunks_) {
            if (mem_len_ < base + c.second) {
                const size_t off = mem_len_ - base, k = std::min(left, c.second - off);
                par_copy(c.first + off, src, k);
                src += k;
                left -= k;
                mem_len_ += k;
                if (!left) break;
            }
            base += c.second;
        }
    }
    pos_ += (int64_t)n;
    return KPW_OK;
}

int FileWriter::open(const char *path)
{
    if (path) {
        fp_ = fopen(path, "wb");  // Mode.OVERWRITE (ParquetFile.java:46)
        if (!fp_) { err_ = std::string("cannot create ") + path; return KPW_ERR_IO; }
    }
    return put("PAR1", 4);  // ParquetFileWriter.start()
}

// ParquetFileWriter 1.10.1 alignment: HadoopOutputFile.supportsBlockSize() (hdfs, webhdfs,
// viewfs) selects PaddingAlignment(max(dfs block size, rowGroupSize), rowGroupSize,
// maxPaddingSize); other file systems NoAlignment (dfs_block_size = 0).
static bool padding_alignment(const kpw_props &p) { return p.dfs_block_size > 0 && p.max_padding_size > 0; }
static int64_t dfs_block(const kpw_props &p) { return std::max<int64_t>(p.dfs_block_size, p.block_size); }

int64_t FileWriter::next_row_group_size() const
{
    if (rgs_.empty() || !padding_alignment(props_)) return props_.block_size;
    const int64_t bs = dfs_block(props_);
    const int64_t remaining = bs - pos_ % bs;
    if (remaining <= props_.max_padding_size) return props_.block_size;   // isPaddingNeeded: the next block starts fresh
    return std::min<int64_t>(remaining, props_.block_size);
}

int FileWriter::align_for_row_group()
{
    if (!padding_alignment(props_)) return KPW_OK;
    const int64_t bs = dfs_block(props_);
    int64_t remaining = bs - pos_ % bs;
    if (remaining > props_.max_padding_size) return KPW_OK;
    static const std::vector<uint8_t> zeros(1u << 20, 0);
    while (remaining > 0) {
        const size_t k = (size_t)std::min<int64_t>(remaining, (int64_t)zeros.size());
        if (int st = put(zeros.data(), k)) return st;
        remaining -= (int64_t)k;
    }
    return KPW_OK;
}

int FileWriter::write_row_group(const BatchOut &b, int rg, const uint8_t *pages, uint64_t pages_base, hipStream_t d2h)
{
    if (int st = align_for_row_group()) return st;   // startBlock
    const RowGroupOut &R = b.rgs[rg];
    RowGroupMeta rm;
    rm.rows = R.num_records;
    rm.total_bytes = 0;
    const int nc = (int)cols_.size();
    for (int c = 0; c < nc; c++) {
        const ChunkOut &co = b.chunks[R.first_chunk + c];
        ChunkMeta m;
        m.phys = cols_[c].phys;
        m.codec = props_.codec;
        m.num_values = co.num_values;
        m.data_page_offset = pos_;  // startColumn: currentChunkFirstDataPage
        m.stats.phys = m.phys;
        int64_t uncomp = 0, comp = 0;
        bool first_data = true;
        for (int p = co.first_page; p < co.first_page + co.num_pages; p++) {
            const PageOut &pg = b.pages[p];
            const std::string hdr = page_header(pg, m.phys);
            if (pg.page_type == KPW_DICTIONARY_PAGE) {
                add_count(m.dict_stats, pg.encoding);
                add_unique(m.encodings, pg.encoding);
            } else {
                StatsOut st;
                st.phys = m.phys;
                st.has = pg.has_min_max != 0;
                st.nulls = pg.null_count;
                st.min = pg.min;
                st.max = pg.max;
                if (pg.page_type == KPW_DATA_PAGE_V2) m.v2 = true;
                if (first_data) { m.stats = st; first_data = false; } else merge_stats(m.stats, st);
                add_count(m.data_stats, pg.encoding);
            }
            uncomp += pg.uncompressed_size + (int64_t)hdr.size();
            comp += pg.compressed_size + (int64_t)hdr.size();
            int st2 = put(hdr.data(), hdr.size());
            if (st2) return st2;
            st2 = dev_asm_ ? asm_put(pages + (pg.offset - pages_base), (size_t)pg.compressed_size, true)
                  : d2h && !fp_ ? put_device(pages + (pg.offset - pages_base), (size_t)pg.compressed_size, d2h)
                              : put(pages + (pg.offset - pages_base), (size_t)pg.compressed_size);
            if (st2) return st2;
        }
        // ColumnChunkPageWriter: rl encodings, dl encodings, data encodings (per page); v2
        // pages (writePageV2) record only their data encoding
        for (int p = co.first_page; p < co.first_page + co.num_pages; p++)
            if (b.pages[p].page_type == KPW_DATA_PAGE) add_unique(m.encodings, b.pages[p].rl_encoding);
        for (int p = co.first_page; p < co.first_page + co.num_pages; p++)
            if (b.pages[p].page_type == KPW_DATA_PAGE) add_unique(m.encodings, b.pages[p].dl_encoding);
        for (int p = co.first_page; p < co.first_page + co.num_pages; p++)
            if (b.pages[p].page_type != KPW_DICTIONARY_PAGE) add_unique(m.encodings, b.pages[p].encoding);
        m.total_uncomp = uncomp;
        m.total_comp = comp;
        rm.total_bytes += uncomp;
        rm.chunks.push_back(m);
    }
    rgs_.push_back(std::move(rm));
    return KPW_OK;
}

int64_t FileWriter::row_group_size(const BatchOut &b, int rg) const
{
    const RowGroupOut &R = b.rgs[rg];
    int64_t t = 0;
    for (int c = 0; c < (int)cols_.size(); c++) {
        const ChunkOut &co = b.chunks[R.first_chunk + c];
        for (int p = co.first_page; p < co.first_page + co.num_pages; p++)
            t += (int64_t)page_header(b.pages[p], cols_[c].phys).size() + b.pages[p].compressed_size;
    }
    return t;
}

int FileWriter::close()
{
    if (closed_) return KPW_OK;
    std::string f;
    TCompact t(f);
    int64_t num_rows = 0;
    for (auto &r : rgs_) num_rows += r.rows;
    t.i32(1, 1);
    t.list(2, 12, (uint32_t)cols_.size() + 1);
    t.begin_elem();
    t.bin(4, message_name_);
    t.i32(5, (int32_t)cols_.size());
    t.end();
    for (auto &c : cols_) {
        t.begin_elem();
        t.i32(1, c.phys);
        t.i32(3, c.optional ? 1 : 0);
        t.bin(4, c.name);
        if (c.utf8) t.i32(6, 0);
        t.i32(9, c.field_number);
        t.end();
    }
    t.i64(3, num_rows);
    t.list(4, 12, (uint32_t)rgs_.size());
    for (auto &r : rgs_) {
        t.begin_elem();
        t.list(1, 12, (uint32_t)r.chunks.size());
        for (size_t c = 0; c < r.chunks.size(); c++) {
            const ChunkMeta &m = r.chunks[c];
            t.begin_elem();
            t.i64(2, m.data_page_offset);
            t.begin(3);
            t.i32(1, m.phys);
            t.list(2, 5, (uint32_t)m.encodings.size());
            for (int e : m.encodings) t.varint(TCompact::zz(e));
            t.list(3, 8, 1);
            t.raw_bin(cols_[c].name);
            t.i32(4, m.codec);
            t.i64(5, m.num_values);
            t.i64(6, m.total_uncomp);
            t.i64(7, m.total_comp);
            t.i64(9, m.data_page_offset);
            if (!stats_empty(m.stats)) write_stats(t, 12, m.stats);
            t.list(13, 12, (uint32_t)(m.dict_stats.size() + m.data_stats.size()));
            for (auto &p : m.dict_stats) { t.begin_elem(); t.i32(1, KPW_DICTIONARY_PAGE); t.i32(2, p.first); t.i32(3, p.second); t.end(); }
            for (auto &p : m.data_stats) {   // EncodingStats.usesV2Pages -> DATA_PAGE_V2
                t.begin_elem(); t.i32(1, m.v2 ? KPW_DATA_PAGE_V2 : KPW_DATA_PAGE); t.i32(2, p.first); t.i32(3, p.second); t.end();
            }
            t.end();
            t.end();
        }
        t.i64(2, r.total_bytes);
        t.i64(3, r.rows);
        t.end();
    }
    // key/value metadata in java.util.HashMap order (ProtoWriteSupport.init + writer.model.name)
    {
        std::string desc;
        const size_t dot = message_name_.rfind('.');
        desc += "name: \"" + (dot == std::string::npos ? message_name_ : message_name_.substr(dot + 1)) + "\"\n";
        for (auto &c : cols_) {
            desc += "field {\n  name: \"" + c.name + "\"\n  number: " + std::to_string(c.field_number) + "\n  label: " +
                    (c.optional ? "LABEL_OPTIONAL" : "LABEL_REQUIRED") + "\n  type: " + pt_name(c.proto_type) + "\n}\n";
        }
        const std::string keys[3] = {"parquet.proto.class", "parquet.proto.descriptor", "writer.model.name"};
        const std::string vals[3] = {proto_class_, desc, "protobuf"};
        int src[2] = {0, 1};
        if ((hm_spread(keys[1]) & 15) < (hm_spread(keys[0]) & 15)) { src[0] = 1; src[1] = 0; }
        const int order[3] = {src[0], src[1], 2};
        std::vector<int> sorted;
        for (uint32_t bkt = 0; bkt < 4; bkt++)
            for (int i = 0; i < 3; i++) if ((hm_spread(keys[order[i]]) & 3) == bkt) sorted.push_back(order[i]);
        t.list(5, 12, 3);
        for (int k : sorted) { t.begin_elem(); t.bin(1, keys[k]); t.bin(2, vals[k]); t.end(); }
    }
    t.bin(6, "parquet-mr version 1.10.1 (build a89df8f9932b6ef6633d06069e50c9b7970bebd1)");
    t.list(7, 12, (uint32_t)cols_.size());
    for (size_t c = 0; c < cols_.size(); c++) { t.begin_elem(); t.begin(1); t.end(); t.end(); }
    t.stop();
    int st = put(f.data(), f.size());
    if (st) return st;
    const uint32_t fl = (uint32_t)f.size();
    const uint8_t le[4] = {(uint8_t)fl, (uint8_t)(fl >> 8), (uint8_t)(fl >> 16), (uint8_t)(fl >> 24)};
    st = put(le, 4);
    if (st) return st;
    st = put("PAR1", 4);
    if (st) return st;
    if (fp_) {
        if (fclose(fp_) != 0) { fp_ = nullptr; err_ = "close failed"; return KPW_ERR_IO; }
        fp_ = nullptr;
    }
    closed_ = true;
    return KPW_OK;
}

}  // namespace kpw
