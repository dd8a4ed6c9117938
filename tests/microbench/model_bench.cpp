// model_bench.cpp — test infrastructure: host cost per record of the getDataSize() size model
// (csrc/sizemodel.cpp) on C2 Rec8 records, the per-record loop's CPU part, on this CPU (no GPU).
//   make -C tests/microbench build/model_bench && tests/microbench/build/model_bench [records]
#include <chrono>
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
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 2000000;
    std::vector<uint32_t> sz(n);
    if (synth_sizes(1, 0xC0FFEE02ull, 0, n, 0, sz.data())) return 2;   // kind 1: Rec8
    std::vector<uint64_t> off(n + 1, 0);
    for (uint64_t i = 0; i < n; i++) off[i + 1] = off[i] + sz[i];
    std::vector<uint8_t> data(off[n]);
    if (synth_fill(1, 0xC0FFEE02ull, 0, n, 0, off.data(), data.data())) return 2;
    // Rec8: ts, user_id, status?, price, score?, key16, region?, flag?
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
    for (int pass = 0; pass < 2; pass++) {
        const int32_t page = pass ? (1 << 20) : (128 << 20);
        kpw_props p{};
        p.block_size = 128ll << 20;
        p.page_size = page;
        p.dictionary_page_size = 1 << 20;
        p.enable_dictionary = 1;
        p.codec = 1;
        p.writer_version = 1;
        SizeModel m;
        if (!m.init(cols, p)) return 3;
        std::vector<int32_t> np(8, -1);
        std::vector<int64_t> fl(8, 0);
        volatile int64_t sink = 0;
        uint64_t cuts = 0, pages = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t i = 0; i < n; i++) {
            int r = m.add(data.data() + off[i], off[i + 1] - off[i]);
            if (r == SizeModel::PAGES) {   // flushed bytes as a probe would report them (sizes only)
                pages++;
                std::vector<std::vector<int64_t>> pc;
                m.page_cuts(pc);
                for (int c = 0; c < 8; c++) { np[c] = (int32_t)pc[c].size(); fl[c] = (int64_t)np[c] * 300000; }
                r = m.finish_pages(np, fl);
            }
            if (r == SizeModel::CUT) { cuts++; m.restart(p.block_size); }
            sink = sink + m.buffered();
        }
        const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / n;
        printf("page %9d: %.1f ns per record (add + buffered), %llu row groups, %llu page records\n", page, ns,
               (unsigned long long)cuts, (unsigned long long)pages);
    }
    return 0;
}
