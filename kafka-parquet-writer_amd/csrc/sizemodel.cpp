// sizemodel.cpp — host model of getDataSize() for the per-record loop (see sizemodel.h).
#include "sizemodel.h"

#include <climits>
#include <cstring>

namespace kpw {

namespace {

// Java (int)f / (long)f: NaN -> 0, saturating, truncation toward zero.
int32_t java_f2i(float f)
{
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}
int64_t java_f2l(float f)
{
    if (f != f) return 0;
    if (f >= 9223372036854775808.0f) return INT64_MAX;
    if (f <= -9223372036854775808.0f) return INT64_MIN;
    return (int64_t)f;
}
int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }   // Java long overflow

uint32_t varint_len(uint32_t v)
{
    uint32_t n = 1;
    while (v >= 0x80u) { v >>= 7; n++; }
    return n;
}

// CodedInputStream.readRawVarint64: at most 10 bytes
inline bool varint64(const uint8_t *d, uint64_t &pos, uint64_t end, uint64_t &out)
{
    if (pos < end && d[pos] < 0x80) {   // one byte: tags and small values
        out = d[pos++];
        return true;
    }
    uint64_t r = 0;
    for (int i = 0; i < 10; i++) {
        if (pos >= end) return false;
        const uint8_t b = d[pos++];
        r |= (uint64_t)(b & 0x7f) << (7 * i);
        if (!(b & 0x80)) { out = r; return true; }
    }
    return false;
}

// varint64 where 8 bytes can be read: the terminating byte found in one word (no per-byte
// branch: a 6-byte ts varint was 6 dependent compare-and-branch steps); longer ones and the
// last bytes of a record take varint64
inline bool varint64w(const uint8_t *d, uint64_t &pos, uint64_t end, uint64_t &out)
{
    if (end - pos >= 8) {
        uint64_t w;
        std::memcpy(&w, d + pos, 8);
        const uint64_t stop = ~w & 0x8080808080808080ull;
        if (stop) {
            const uint32_t nb = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;
            uint64_t v = 0;
            for (uint32_t i = 0; i < nb; i++) v |= ((w >> (8 * i)) & 0x7f) << (7 * i);
            out = v;
            pos += nb;
            return true;
        }
    }
    return varint64(d, pos, end, out);
}

// skipField for an unknown field whose tag was read (k_decode.hip skip_field rules)
bool skip_field(const uint8_t *d, uint64_t &pos, uint64_t end, uint32_t tag)
{
    uint64_t v;
    switch (tag & 7) {
    case 0: return varint64(d, pos, end, v);
    case 1: if (end - pos < 8) return false; pos += 8; return true;
    case 2:
        if (!varint64(d, pos, end, v) || (int32_t)(uint32_t)v < 0 || end - pos < (uint32_t)v) return false;
        pos += (uint32_t)v;
        return true;
    case 5: if (end - pos < 4) return false; pos += 4; return true;
    case 3: {
        uint32_t stack[100];
        int depth = 0;
        stack[depth++] = tag >> 3;
        while (depth > 0) {
            uint64_t t64;
            if (!varint64(d, pos, end, t64)) return false;
            const uint32_t t = (uint32_t)t64, w = t & 7;
            if ((t >> 3) == 0) return false;
            if (w == 4) {
                if ((t >> 3) != stack[depth - 1]) return false;
                depth--;
            } else if (w == 3) {
                if (depth >= 100) return false;
                stack[depth++] = t >> 3;
            } else if (w == 0) {
                if (!varint64(d, pos, end, v)) return false;
            } else if (w == 1) {
                if (end - pos < 8) return false;
                pos += 8;
            } else if (w == 5) {
                if (end - pos < 4) return false;
                pos += 4;
            } else if (w == 2) {
                if (!varint64(d, pos, end, v) || (int32_t)(uint32_t)v < 0 || end - pos < (uint32_t)v) return false;
                pos += (uint32_t)v;
            } else {
                return false;
            }
        }
        return true;
    }
    default: return false;   // END_GROUP at top level, wire types 6 / 7
    }
}

}  // namespace

// RunLengthBitPackingHybridEncoder.writeInt (bit width 1), sizes only
void RleCount::write(uint32_t v)
{
    // (written so that a random 0/1 stream costs no mispredicted branch on v == prev: the
    // repeat count is a select, and only the rare run ends and group ends branch)
    const bool same = v == prev;
    if (!same && rc >= 8) {                       // writeRleRun: endPreviousBitPackedRun + header + value
        hdr_open = false;
        groups = 0;
        out += varint_len((uint32_t)rc << 1) + 1;
        nbuf = 0;
    }
    rc = same ? rc + 1 : 1;
    prev = v;
    if (same && rc >= 8) return;                  // extends the RLE run
    if (++nbuf == 8) {                            // writeOrAppendBitPackedRun
        if (groups >= 63) { hdr_open = false; groups = 0; }
        if (!hdr_open) { out += 1; hdr_open = true; }
        out += 1;                                 // 8 values x 1 bit
        nbuf = 0;
        rc = 0;
        ++groups;
    }
}

int64_t SizeModel::Col::mem(bool v2) const
{
    // ColumnWriterV1: rl (DevNull) + dl + data buffered sizes; ColumnWriterV2: width-0 level
    // encoders emit nothing before toBytes, BOOLEAN values are RLE
    const int64_t d = phys != KPW_BOOLEAN ? data : v2 ? bv.out : (data + 7) / 8;
    return (optional ? dl.out : 0) + d;
}

bool SizeModel::init(const std::vector<ColInfo> &cols, const kpw_props &p)
{
    if (p.writer_version != 1 && p.writer_version != 2) return false;
    v2_ = p.writer_version == 2;
    // v2 cuts a page once a column is within 10% of pageSize, possible with pageSize >= blockSize
    // (the engine plans v2 pages below 2 x blockSize alike, Engine::init)
    multi_ = p.page_size < p.block_size || (v2_ && p.page_size / 2 < p.block_size);
    page_size_ = p.page_size;
    block_size_ = p.block_size;
    next_rg_size_ = p.block_size;
    fmap_.assign(FMAP_SIZE, -1);
    cols_.clear();
    wire_.clear();
    nreq_ = 0;
    for (size_t c = 0; c < cols.size(); c++) {
        Col k;
        k.field_number = cols[c].field_number;
        k.wire_type = cols[c].wire_type;
        k.phys = cols[c].phys;
        k.optional = cols[c].optional;
        k.vsize = cols[c].vsize;
        cols_.push_back(k);
        wire_.push_back(Wire{(uint32_t)cols[c].wire_type, (uint32_t)cols[c].vsize, cols[c].optional ? 0u : 1u});
        nreq_ += cols[c].optional ? 0u : 1u;
        if (cols[c].field_number < FMAP_SIZE) fmap_[cols[c].field_number] = (int16_t)c;
    }
    seen_.assign(cols_.size(), 0u);
    gen_ = 0;
    raw_.assign(cols_.size(), 0);
    bval_.assign(cols_.size(), 0);
    reset_store();
    next_mem_check_ = 100;
    return true;
}

void SizeModel::reset_store()
{
    for (Col &k : cols_) {
        k.dl = RleCount();
        k.data = 0;
        k.flushed = 0;
        k.pages = 0;
        k.pages_known = 0;
        k.cut_at.clear();
        k.value_count = 0;
        k.next_check = 100;   // props.getMinRowCountForPageSizeCheck()
        k.bv = RleCount();
        k.rows_written = 0;
    }
    record_count_ = 0;
    v2_next_check_ = 100;
}

void SizeModel::restart(int64_t next_rg_size)
{
    reset_store();
    next_mem_check_ = 100;
    next_rg_size_ = next_rg_size;
}

// parser.parseFrom(record.value()) validity + presence + raw sizes (K1's rules).  Presence is
// the record's generation number in seen_ (no clear per record); the required columns are
// counted as they first appear.
bool SizeModel::scan(const uint8_t *d, uint64_t len)
{
    if (++gen_ == 0) {   // wrapped: stale generations could match again
        std::fill(seen_.begin(), seen_.end(), 0u);
        gen_ = 1;
    }
    const uint32_t gen = gen_;
    uint32_t *seen = seen_.data();
    uint32_t *raw = raw_.data();
    uint8_t *bval = bval_.data();
    const int16_t *fmap = fmap_.data();
    const Wire *wire = wire_.data();
    uint32_t nreq = 0;
    uint64_t pos = 0;
    const uint64_t end = len;
    while (pos < end) {
        uint64_t t64;
        if (!varint64(d, pos, end, t64)) return false;
        const uint32_t tag = (uint32_t)t64, fno = tag >> 3, wt = tag & 7;
        if (fno == 0) return false;
        int c = -1;
        if (fno < (uint32_t)FMAP_SIZE) c = fmap[fno];
        else
            for (size_t k = 0; k < cols_.size(); k++)
                if ((uint32_t)cols_[k].field_number == fno) { c = (int)k; break; }
        if (c < 0 || wire[c].wire_type != wt) {
            if (!skip_field(d, pos, end, tag)) return false;
            continue;
        }
        uint64_t v;
        switch (wt) {
        case 0:
            if (!varint64w(d, pos, end, v)) return false;
            raw[c] = wire[c].vsize;
            bval[c] = v != 0;   // CodedInputStream.readBool
            break;
        case 1: if (end - pos < 8) return false; pos += 8; raw[c] = 8; break;
        case 5: if (end - pos < 4) return false; pos += 4; raw[c] = 4; break;
        default:   // 2: length-delimited (BYTE_ARRAY: 4-byte length + bytes)
            if (!varint64w(d, pos, end, v) || (int32_t)(uint32_t)v < 0 || end - pos < (uint32_t)v) return false;
            pos += (uint32_t)v;
            raw[c] = 4 + (uint32_t)v;
            break;
        }
        if (seen[c] != gen) {
            seen[c] = gen;
            nreq += wire[c].required;
        }
    }
    return nreq == nreq_;   // isInitialized: every required field present
}

int64_t SizeModel::buffered() const
{
    int64_t s = 0;
    for (const Col &k : cols_) s += k.mem(v2_) + k.flushed;
    return s;
}

int SizeModel::add(const uint8_t *rec, uint64_t len)
{
    if (!scan(rec, len)) return INVALID;
    bool cut = false;
    const uint32_t gen = gen_;
    for (size_t c = 0; c < cols_.size(); c++) {
        Col &k = cols_[c];
        const bool present = seen_[c] == gen;
        if (k.optional) k.dl.write(present ? 1u : 0u);
        if (k.phys != KPW_BOOLEAN) k.data += present ? raw_[c] : 0u;   // (a select: presence is random)
        else if (!v2_) k.data += present ? 1 : 0;
        else if (present) k.bv.write(bval_[c]);
        ++k.value_count;
        if (v2_) continue;   // ColumnWriteStoreV2 checks the store after the record
        // ColumnWriterV1.accountForValueWritten
        if (k.value_count > k.next_check) {
            const int64_t mem = k.mem(false);
            if (mem > page_size_) {
                // writePage inside the row group: the check restarts at half this page's
                // values; the page's header + compressed bytes join pageWriter.getMemSize()
                // (finish_pages, from the GPU)
                k.next_check = k.value_count / 2;
                k.value_count = 0;
                k.dl = RleCount();
                k.data = 0;
                k.pages++;
                k.cut_at.push_back(record_count_ + 1);   // the page ends after this record
                cut = true;
                continue;
            }
            float t = (float)k.value_count * (float)page_size_;
            t = t / (float)mem;
            k.next_check = java_f2i((float)k.value_count + t) / 2 + 1;
        }
    }
    ++record_count_;   // InternalParquetRecordWriter.recordCount = ColumnWriteStoreV2.rowCount
    if (v2_ && record_count_ >= v2_next_check_) {
        // ColumnWriteStoreV2.sizeCheck: thresholdTolerance = (long)(pageSize * 0.1f);
        // rowsToFillPage = (long)((float)rows) / usedMem * remainingMem
        const int64_t tol = (int64_t)((float)page_size_ * 0.1f);
        int64_t mn = INT64_MAX;
        for (Col &k : cols_) {
            const int64_t used = k.mem(true);
            const int64_t rows = record_count_ - k.rows_written;
            int64_t rem = page_size_ - used;
            if (rem <= tol) {   // ColumnWriterV2.writePage(rowCount)
                k.rows_written = record_count_;
                k.value_count = 0;
                k.dl = RleCount();
                k.bv = RleCount();
                k.data = 0;
                k.pages++;
                k.cut_at.push_back(record_count_);
                cut = true;
                rem = page_size_;
            }
            const int64_t fill = used == 0 ? 10000 : ((int64_t)(float)rows / used) * rem;
            if (fill < mn) mn = fill;
        }
        int64_t half = mn / 2;
        half = half < 100 ? 100 : (half > 10000 ? 10000 : half);
        v2_next_check_ = record_count_ + half;
    }
    return cut ? PAGES : block_check();
}

int SizeModel::finish_pages(const std::vector<int32_t> &npages, const std::vector<int64_t> &flushed)
{
    if (npages.size() != cols_.size() || flushed.size() != cols_.size()) return MISMATCH;
    for (size_t c = 0; c < cols_.size(); c++) {
        if (npages[c] < 0 ? cols_[c].pages != cols_[c].pages_known : npages[c] != cols_[c].pages) return MISMATCH;
    }
    for (size_t c = 0; c < cols_.size(); c++) {
        if (npages[c] >= 0) cols_[c].flushed = flushed[c];
        cols_[c].pages_known = cols_[c].pages;
    }
    return block_check();
}

void SizeModel::page_cuts(std::vector<std::vector<int64_t>> &cuts) const
{
    cuts.resize(cols_.size());
    for (size_t c = 0; c < cols_.size(); c++) cuts[c] = cols_[c].cut_at;
}

void SizeModel::cut_columns(std::vector<char> &mask) const
{
    mask.assign(cols_.size(), 0);
    for (size_t c = 0; c < cols_.size(); c++) mask[c] = cols_[c].pages != cols_[c].pages_known;
}

// InternalParquetRecordWriter.write -> checkBlockSizeReached
int SizeModel::block_check()
{
    if (record_count_ >= next_mem_check_) {
        const int64_t mem = buffered();
        const int64_t rec_size = mem / record_count_;
        if (mem > next_rg_size_ - 2 * rec_size) {
            reset_store();
            next_mem_check_ = 100;   // min(max(100, recordCount / 2), 10000) with recordCount reset to 0
            return CUT;
        }
        const int64_t est = jadd(record_count_, java_f2l((float)next_rg_size_ / (float)rec_size)) / 2;
        const int64_t a = est > 100 ? est : 100;
        const int64_t b = jadd(record_count_, 10000);
        next_mem_check_ = a < b ? a : b;
    }
    return OK;
}

}  // namespace kpw
