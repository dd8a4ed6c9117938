// model_check.cpp — test infrastructure (tests/test_size_model.py): the host size model
// (csrc/sizemodel.cpp) on synthetic Rec8 records, one record at a time as the per-record loop
// feeds it; prints the model's buffered size after each of the first `nb` records and the record
// count of every row group it cuts, for the test to compare with the CPU oracle.
//   model_check n seed block_size nb
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sizemodel.h"

extern "C" int synth_sizes(int kind, uint64_t seed, uint64_t start, uint64_t n, int param, uint32_t *sizes);
extern "C" int synth_fill(int kind, uint64_t seed, uint64_t start, uint64_t n, int param, const uint64_t *offsets,
                          uint8_t *out);

using namespace kpw;

int main(int argc, char **argv)
{
    if (argc < 5) return 2;
    const uint64_t n = strtoull(argv[1], nullptr, 10), seed = strtoull(argv[2], nullptr, 0);
    const int64_t block = strtoll(argv[3], nullptr, 10);
    const uint64_t nb = strtoull(argv[4], nullptr, 10);
    std::vector<uint32_t> sz(n);
    if (synth_sizes(1, seed, 0, n, 0, sz.data())) return 3;
    std::vector<uint64_t> off(n + 1, 0);
    for (uint64_t i = 0; i < n; i++) off[i + 1] = off[i] + sz[i];
    std::vector<uint8_t> data(off[n]);
    if (synth_fill(1, seed, 0, n, 0, off.data(), data.data())) return 3;
    // Rec8 (synth.REC8): ts, user_id, status?, price, score?, key16, region?, flag?
    struct { int fno, wt, phys, opt, vsize; } spec[8] = {
        {1, 0, KPW_INT64, 0, 8}, {2, 0, KPW_INT32, 0, 4}, {3, 0, KPW_INT32, 1, 4}, {4, 1, KPW_DOUBLE, 0, 8},
        {5, 1, KPW_DOUBLE, 1, 8}, {6, 2, KPW_BYTE_ARRAY, 0, 0}, {7, 2, KPW_BYTE_ARRAY, 1, 0}, {8, 0, KPW_BOOLEAN, 1, 1}};
    std::vector<ColInfo> cols(8);
    for (int c = 0; c < 8; c++) {
        cols[c].field_number = spec[c].fno;
        cols[c].wire_type = spec[c].wt;
        cols[c].phys = spec[c].phys;
        cols[c].optional = spec[c].opt;
        cols[c].vsize = spec[c].vsize;
    }
    kpw_props p{};
    p.block_size = block;
    p.page_size = (int32_t)(block < (1ll << 30) ? block : (1ll << 30));   // single-page regime
    p.dictionary_page_size = 1 << 20;
    p.enable_dictionary = 1;
    p.codec = 1;
    p.writer_version = 1;
    SizeModel m;
    if (!m.init(cols, p)) return 4;
    uint64_t rg_start = 0;
    for (uint64_t i = 0; i < n; i++) {
        const int r = m.add(data.data() + off[i], off[i + 1] - off[i]);
        if (r == SizeModel::INVALID || r == SizeModel::PAGES) return 5;
        if (i < nb) printf("B %llu %lld\n", (unsigned long long)i, (long long)m.buffered());
        if (r == SizeModel::CUT) {
            printf("CUT %llu\n", (unsigned long long)(i + 1 - rg_start));
            rg_start = i + 1;
            m.restart(block);
        }
    }
    printf("OPEN %llu\n", (unsigned long long)(n - rg_start));
    return 0;
}
