// seg_bench.hip — test-infrastructure microbenchmark for K7's segment-parallel kernel.
//
// Reads page bodies (u64 length + bytes each, tests/microbench/dump_pages.py format), compresses
// them with (a) the sequential kernels alone and (b) k_snappy_seg + the sequential kernels on
// the fragments it hands on, checks every page byte-for-byte against the CPU oracle's pinned
// Snappy (oracle/oracle_snappy.c, linked as the checker only) and prints timings.
//   make -C tests/microbench build/seg_bench && tests/microbench/build/seg_bench pages.bin [reps]
#include "../../kafka-parquet-writer_amd/csrc/k_snappy.hip"
#include "../../kafka-parquet-writer_amd/csrc/k_snappy_seg.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include <unistd.h>

using namespace kpw;
extern "C" int64_t kpwo_snappy_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

int main(int argc, char **argv)
{
    if (argc < 2) { fprintf(stderr, "usage: seg_bench pages.bin [reps] [copies]\n"); return 2; }
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    const int copies = argc > 3 ? atoi(argv[3]) : 1;   // replicate the page set (more fragments per launch)
    std::vector<std::vector<uint8_t>> pages;
    {
        FILE *fp = fopen(argv[1], "rb");
        if (!fp) { fprintf(stderr, "cannot open %s\n", argv[1]); return 2; }
        uint64_t l;
        while (fread(&l, 8, 1, fp) == 1) {
            std::vector<uint8_t> b(l);
            if (l && fread(b.data(), 1, l, fp) != l) return 2;
            if (l) pages.push_back(std::move(b));
        }
        fclose(fp);
    }
    const size_t np0 = pages.size();
    for (int c = 1; c < copies; c++)
        for (size_t i = 0; i < np0; i++) pages.push_back(pages[i]);
    const size_t npages = pages.size();
    std::vector<uint8_t> host;
    std::vector<uint64_t> off, len;
    for (auto &pg : pages) {
        off.push_back(host.size()); len.push_back(pg.size());
        host.insert(host.end(), pg.begin(), pg.end());
        host.resize((host.size() + 255) & ~(size_t)255, 0);
    }
    host.resize(host.size() + 512, 0);
    std::vector<uint32_t> fpage, fidx;
    for (size_t p = 0; p < npages; p++)
        for (uint32_t k = 0; (uint64_t)k * SNAPPY_FRAG < len[p]; k++) { fpage.push_back((uint32_t)p); fidx.push_back(k); }
    const uint32_t nf = (uint32_t)fpage.size();
    uint64_t tot = 0;
    for (auto l : len) tot += l;
    printf("%zu pages, %u fragments, %.1f MB\n", npages, nf, tot / 1e6);
    uint8_t *d_in, *d_fout; uint64_t *d_off, *d_len; uint32_t *d_fp, *d_fi, *d_flen, *d_cnt; uint8_t *d_scr;
    CK(hipMalloc(&d_in, host.size())); CK(hipMemcpy(d_in, host.data(), host.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_off, npages * 8)); CK(hipMemcpy(d_off, off.data(), npages * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_len, npages * 8)); CK(hipMemcpy(d_len, len.data(), npages * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_fp, nf * 4)); CK(hipMemcpy(d_fp, fpage.data(), nf * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_fi, nf * 4)); CK(hipMemcpy(d_fi, fidx.data(), nf * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_fout, (size_t)nf * SNAPPY_FRAG_CAP)); CK(hipMalloc(&d_flen, nf * 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&d_scr, snappy_seg_scratch_bytes(cus))); CK(hipMalloc(&d_cnt, 64));
    uint64_t *d_ft; CK(hipMalloc(&d_ft, (size_t)nf * 16));
    // oracle: per page, compressed fragments (strip the varint length prefix)
    std::vector<std::vector<uint8_t>> want(npages);
    for (size_t p = 0; p < np0; p++) {
        want[p].resize(32 + len[p] + len[p] / 6);
        int64_t w = kpwo_snappy_compress(host.data() + off[p], len[p], want[p].data(), want[p].size());
        want[p].resize((size_t)w);
    }
    // per fragment: the oracle's output for the fragment alone (a fragment is compressed with
    // a fresh table: strip the varint length prefix), to name a mismatching fragment
    std::vector<std::vector<uint8_t>> wantf(nf);
    for (uint32_t f = 0; f < nf; f++) {
        if (fpage[f] >= np0) continue;
        const uint64_t o0 = (uint64_t)fidx[f] * SNAPPY_FRAG;
        const uint32_t fn = (uint32_t)std::min<uint64_t>(SNAPPY_FRAG, len[fpage[f]] - o0);
        std::vector<uint8_t> w(64 + fn + fn / 6);
        const int64_t wl = kpwo_snappy_compress(host.data() + off[fpage[f]] + o0, fn, w.data(), w.size());
        uint32_t pre = 1, v = fn;
        while (v >= 0x80) { v >>= 7; pre++; }
        wantf[f].assign(w.begin() + pre, w.begin() + wl);
    }
    auto check_frags = [&](const char *what) -> int {
        std::vector<uint32_t> fl(nf);
        CK(hipMemcpy(fl.data(), d_flen, nf * 4, hipMemcpyDeviceToHost));
        std::vector<uint8_t> fo((size_t)nf * SNAPPY_FRAG_CAP);
        CK(hipMemcpy(fo.data(), d_fout, fo.size(), hipMemcpyDeviceToHost));
        int nbad = 0;
        for (uint32_t f = 0; f < nf; f++) {
            if (fpage[f] >= np0) continue;
            const uint8_t *g = fo.data() + (size_t)f * SNAPPY_FRAG_CAP;
            const auto &w = wantf[f];
            if (fl[f] == w.size() && !memcmp(g, w.data(), w.size())) continue;
            uint32_t d = 0;
            while (d < fl[f] && d < w.size() && g[d] == w[d]) d++;
            if (nbad < 8)
                printf("FRAG MISMATCH [%s] frag %u (page %u idx %u): len %u want %zu, first diff at %u (got %02x want %02x)\n", what, f,
                       fpage[f], fidx[f], fl[f], w.size(), d, d < fl[f] ? g[d] : 0, d < w.size() ? w[d] : 0);
            if (nbad == 0 && getenv("SEG_DUMP_BAD")) {   // the fragment's input bytes, for the CPU model
                FILE *fp = fopen(getenv("SEG_DUMP_BAD"), "wb");
                const uint64_t o0 = (uint64_t)fidx[f] * SNAPPY_FRAG;
                const uint64_t fn = std::min<uint64_t>(SNAPPY_FRAG, len[fpage[f]] - o0);
                if (fp) { fwrite(&fn, 8, 1, fp); fwrite(host.data() + off[fpage[f]] + o0, 1, fn, fp); fclose(fp); }
            }
            nbad++;
        }
        if (nbad) printf("[%s] %d mismatching fragments\n", what, nbad);
        fflush(stdout);
        return nbad;
    };
    int bad = 0;
    for (int mode = 0; mode < 2; mode++) {
        SnappyArgs a{};
        a.in = d_in; a.page_off = d_off; a.page_len = d_len; a.npages = (uint32_t)npages; a.nfrags = nf;
        a.frag_page = d_fp; a.frag_idx = d_fi; a.frag_out = d_fout; a.frag_len = d_flen; a.ftime = d_ft;
        if (mode) { a.seg_scratch = d_scr; a.seg_counter = d_cnt; a.seg_grid = (uint32_t)cus; }
        CK(hipMemset(d_fout, 0, (size_t)nf * SNAPPY_FRAG_CAP));
        if (!(mode && getenv("SEG_DEBUG"))) {
            launch_snappy(a, 0);
            CK(hipDeviceSynchronize());
            bad += check_frags(mode ? "seg+v+s" : "v+s");
        }
        if (mode && getenv("SEG_DEBUG")) {   // watch k_snappy_seg alone through host-visible progress words
            uint32_t *dbg; CK(hipHostMalloc((void **)&dbg, (size_t)cus * 16, hipHostMallocCoherent | hipHostMallocMapped));
            memset(dbg, 0, (size_t)cus * 16);
            uint32_t *ddbg; CK(hipHostGetDevicePointer((void **)&ddbg, dbg, 0));
            uint64_t *d_prof; CK(hipMalloc(&d_prof, 128)); CK(hipMemset(d_prof, 0, 128));
            SnappyArgs c = a; c.seg_prof = d_prof; c.seg_dbg = ddbg;
            CK(hipMemset(d_cnt, 0, 4));
            CK(hipDeviceSynchronize());
            if (getenv("SEG_DEBUG")[0] == '2') hipLaunchKernelGGL(k_snappy_seg, dim3(cus), dim3(1024), 0, 0, c);
            else if (getenv("SEG_DEBUG")[0] == '3') { c.v_budget = 256; hipLaunchKernelGGL(k_snappy_v, dim3(nf), dim3(64), 0, 0, c); c.v_budget = 0; c.seg_only_marked = 1; hipLaunchKernelGGL(k_snappy_seg, dim3(cus), dim3(1024), 0, 0, c); }
            else hipLaunchKernelGGL(k_snappy_seg, dim3(cus), dim3(1024), 0, 0, c);
            for (int it = 0; it < 100; it++) {
                usleep(100000);
                int busy = 0;
                for (int b = 0; b < cus; b++) busy += !dbg[b * 4 + 3];
                if (!busy) break;
                if (it == 99 || it % 20 == 0) {
                    printf("t=%.1fs busy workgroups %d\n", it * 0.1, busy);
                    for (int b = 0; b < cus; b++)
                        if (!dbg[b * 4 + 3]) printf("  wg %d frag %u (page %u) round %u mark %u\n", b, dbg[b * 4], fpage[dbg[b * 4]], dbg[b * 4 + 1], dbg[b * 4 + 2]);
                    fflush(stdout);
                }
            }
            fflush(stdout);
            _exit(0);
        }
        if (mode) {   // how many fragments did the segment kernel hand on
            SnappyArgs b = a; b.seg_grid = (uint32_t)cus;
            CK(hipMemset(d_cnt, 0, 4));
            hipLaunchKernelGGL(k_snappy_seg, dim3(cus), dim3(1024), 0, 0, b);
            CK(hipDeviceSynchronize());
            std::vector<uint32_t> fl(nf);
            CK(hipMemcpy(fl.data(), d_flen, nf * 4, hipMemcpyDeviceToHost));
            uint32_t ho = 0;
            for (uint32_t f = 0; f < nf; f++) ho += fl[f] == SEG_ABORTED;
            hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0));
            for (int r = 0; r < reps; r++) { CK(hipMemset(d_cnt, 0, 4)); hipLaunchKernelGGL(k_snappy_seg, dim3(cus), dim3(1024), 0, 0, b); }
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            printf("k_snappy_seg alone: %.3f ms, handed on %u of %u fragments\n", ms / reps, ho, nf);
            {   // fragments k_snappy_seg finished itself must be exact
                std::vector<uint32_t> fl3(nf);
                CK(hipMemcpy(fl3.data(), d_flen, nf * 4, hipMemcpyDeviceToHost));
                std::vector<uint8_t> fo((size_t)nf * SNAPPY_FRAG_CAP);
                CK(hipMemcpy(fo.data(), d_fout, fo.size(), hipMemcpyDeviceToHost));
                int nb = 0;
                for (uint32_t f = 0; f < nf; f++) {
                    if (fpage[f] >= np0 || fl3[f] == SEG_ABORTED) continue;
                    const auto &w = wantf[f];
                    if (fl3[f] == w.size() && !memcmp(fo.data() + (size_t)f * SNAPPY_FRAG_CAP, w.data(), w.size())) continue;
                    if (nb++ < 8) printf("SEG-ALONE MISMATCH frag %u (page %u idx %u): len %u want %zu\n", f, fpage[f], fidx[f], fl3[f], w.size());
                }
                if (nb) { printf("[seg alone] %d mismatching fragments\n", nb); bad += nb; }
            }
            {   // phase profile of one launch (thread 0 of every workgroup, summed)
                uint64_t *d_prof; CK(hipMalloc(&d_prof, 128)); CK(hipMemset(d_prof, 0, 128));
                SnappyArgs c = b; c.seg_prof = d_prof;
                CK(hipMemset(d_cnt, 0, 4));
                hipLaunchKernelGGL(k_snappy_seg, dim3(cus), dim3(1024), 0, 0, c);
                CK(hipDeviceSynchronize());
                uint64_t pr[16]; CK(hipMemcpy(pr, d_prof, 128, hipMemcpyDeviceToHost));
                const double fr = pr[6] ? (double)pr[6] : 1;
                printf("per fragment (kcycles): setup %.1f scan %.1f parse %.1f check %.1f emit %.1f | rounds %.2f | frags %llu handed on %llu\n",
                       pr[0] / fr / 1e3, pr[1] / fr / 1e3, pr[2] / fr / 1e3, pr[3] / fr / 1e3, pr[4] / fr / 1e3, pr[5] / fr,
                       (unsigned long long)pr[6], (unsigned long long)pr[7]);
                printf("  setup: stage %.1f hist %.1f cscan %.1f scatter %.1f check %.1f | scan: pass1 %.1f carry %.1f pass2 %.1f (rest = final barrier)\n", pr[8] / fr / 1e3,
                       pr[9] / fr / 1e3, pr[10] / fr / 1e3, pr[11] / fr / 1e3, pr[12] / fr / 1e3, pr[13] / fr / 1e3, pr[14] / fr / 1e3, pr[15] / fr / 1e3);
                hipFree(d_prof);
            }
            launch_snappy(a, 0);
            CK(hipDeviceSynchronize());
        }
        std::vector<uint32_t> fl(nf);
        CK(hipMemcpy(fl.data(), d_flen, nf * 4, hipMemcpyDeviceToHost));
        {   // per page: mean / max fragment duration (us) of this mode's kernels
            std::vector<uint64_t> ft((size_t)nf * 2);
            CK(hipMemcpy(ft.data(), d_ft, ft.size() * 8, hipMemcpyDeviceToHost));
            for (size_t p = 0, f = 0; p < np0 && p < 40; p++) {
                double sum = 0, mx = 0; uint32_t c = 0;
                for (; f < nf && fpage[f] == p; f++) {
                    const double d = (double)((ft[2 * f + 1] & ~(1ull << 63)) - ft[2 * f]) / 100.0;   // 100 MHz wall clock
                    sum += d; mx = d > mx ? d : mx; c++;
                }
                printf("  mode %d page %2zu len %9llu frags %4u frag us mean %8.1f max %8.1f\n", mode, p, (unsigned long long)len[p], c, c ? sum / c : 0, mx);
            }
        }
        std::vector<uint8_t> fo((size_t)nf * SNAPPY_FRAG_CAP);
        CK(hipMemcpy(fo.data(), d_fout, fo.size(), hipMemcpyDeviceToHost));
        uint64_t comp = 0;
        int mism = 0;
        for (size_t p = 0, f = 0; p < npages; p++) {
            std::vector<uint8_t> got;
            uint32_t v = (uint32_t)len[p];
            while (v >= 0x80) { got.push_back((uint8_t)(v | 0x80)); v >>= 7; }
            got.push_back((uint8_t)v);
            for (; f < nf && fpage[f] == p; f++) {
                if (fl[f] > SNAPPY_FRAG_CAP) { printf("page %zu frag %zu: bad length %u\n", p, f, fl[f]); mism++; break; }
                got.insert(got.end(), fo.begin() + (size_t)f * SNAPPY_FRAG_CAP, fo.begin() + (size_t)f * SNAPPY_FRAG_CAP + fl[f]);
                comp += fl[f];
            }
            if (got != want[p % np0]) {
                if (mism < 5) {
                    size_t d = 0;
                    while (d < got.size() && d < want[p % np0].size() && got[d] == want[p % np0][d]) d++;
                    printf("MISMATCH mode=%d page=%zu len=%llu (got %zu want %zu, first diff at %zu)\n", mode, p,
                           (unsigned long long)len[p], got.size(), want[p % np0].size(), d);
                }
                mism++;
            }
        }
        bad += mism;
        if (mode) {   // the routed pipeline kernel by kernel (launch_snappy's sequence)
            hipEvent_t ev[5];
            for (auto &e : ev) CK(hipEventCreate(&e));
            SnappyArgs v = a; v.v_budget = getenv("KPW_SNAPPY_VBUDGET") ? (uint32_t)atoi(getenv("KPW_SNAPPY_VBUDGET")) : 256u;
            SnappyArgs g = a; g.seg_only_marked = v.v_budget ? 1 : 0;
            SnappyArgs b = a; b.v_only_handed_on = 1;
            SnappyArgs r = a; r.s_budget = getenv("KPW_SNAPPY_SBUDGET") ? (uint32_t)atoi(getenv("KPW_SNAPPY_SBUDGET")) : 128u;
            CK(hipEventRecord(ev[0]));
            hipLaunchKernelGGL(k_snappy_v, dim3(nf), dim3(64), 0, 0, v);
            if (v.v_budget && r.s_budget) hipLaunchKernelGGL(k_snappy_s_rest, dim3(nf), dim3(64), 0, 0, r);
            CK(hipEventRecord(ev[1]));
            CK(hipMemset(d_cnt, 0, 4));
            hipLaunchKernelGGL(k_snappy_seg, dim3(cus), dim3(1024), 0, 0, g);
            CK(hipEventRecord(ev[2]));
            hipLaunchKernelGGL(k_snappy_v, dim3(nf), dim3(64), 0, 0, b);
            CK(hipEventRecord(ev[3]));
            hipLaunchKernelGGL(k_snappy_s_rest, dim3(nf), dim3(64), 0, 0, a);
            CK(hipEventRecord(ev[4]));
            CK(hipEventSynchronize(ev[4]));
            float m[4];
            for (int i = 0; i < 4; i++) CK(hipEventElapsedTime(&m[i], ev[i], ev[i + 1]));
            std::vector<uint32_t> fl2(nf);
            CK(hipMemcpy(fl2.data(), d_flen, nf * 4, hipMemcpyDeviceToHost));
            printf("routed: v(budget %u) + s_rest(budget) %.3f ms | seg %.3f ms | v(rest) %.3f ms | s_rest %.3f ms\n", v.v_budget, m[0], m[1], m[2], m[3]);
        }
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) launch_snappy(a, 0);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%s: %.3f ms per launch (%.2f GB/s of pages), ratio %.3f, mismatching pages %d\n",
               mode ? "seg+v+s" : "v+s    ", ms / reps, tot / (ms / reps * 1e-3) / 1e9, (double)comp / tot, mism);
        fflush(stdout);
    }
    printf(bad ? "FAILED %d\n" : "ALL MATCH\n", bad);
    return bad ? 1 : 0;
}
