// snappy_bench.hip — test-infrastructure microbenchmark for K7 variants.
//
// Builds synthetic pages shaped like the C2 workload's columns, compresses them with each
// search variant (SEQ = sequential probes per literal search before 64-wide batches) and
// checks every output byte-for-byte against the CPU oracle's pinned Snappy
// (oracle/oracle_snappy.c, linked as the checker only).  Prints one line per (page, variant).
//   make -C tests/microbench && tests/microbench/build/snappy_bench
#include "../../kafka-parquet-writer_amd/csrc/k_snappy.hip"
#include "snappy_variants.hip"
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace kpw;
extern "C" int64_t kpwo_snappy_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

static uint64_t mix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; }

static std::vector<uint8_t> make_page(const std::string &kind, size_t target)
{
    std::vector<uint8_t> p;
    p.reserve(target + 64);
    uint64_t i = 0;
    auto put = [&](const void *v, size_t n) { const uint8_t *b = (const uint8_t *)v; p.insert(p.end(), b, b + n); };
    while (p.size() < target) {
        const uint64_t r = mix(i * 0x9E3779B97F4A7C15ull + 17);
        if (kind == "ts") { uint64_t v = 1700000000000ull + i + r % 1000; put(&v, 8); }
        else if (kind == "price") { double d = (double)(r >> 11) * (1.0 / 9007199254740992.0) * 1000.0; put(&d, 8); }
        else if (kind == "user_id") { uint32_t v = (uint32_t)(r & 0xFFFFF); put(&v, 4); }
        else if (kind == "ids14") { uint64_t v = r; put(&v, 7); }   // dense random bit-packed ids
        else if (kind == "key16") {   // PLAIN strings from 10k distinct 16-char keys
            static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
            uint64_t k = mix(0xA5A5 + r % 10000);
            uint32_t len = 16; put(&len, 4);
            for (int j = 0; j < 16; j++) { uint8_t c = (uint8_t)A[(k >> (j * 3 % 58)) % 62]; put(&c, 1); }
        } else if (kind == "json") {
            char buf[256];
            int n = snprintf(buf, sizeof buf, "{\"id\":%llu,\"event\":\"%s\",\"value\":%u,\"tags\":[\"a%u\",\"b%u\"]}",
                             (unsigned long long)i, (r & 1) ? "click" : "view", (unsigned)(r >> 40) % 100000,
                             (unsigned)(r >> 20) % 50, (unsigned)(r >> 30) % 7);
            uint32_t len = (uint32_t)n; put(&len, 4); put(buf, n);
        } else if (kind == "defl") {  // def-level RLE-ish bytes: short runs of a few symbols
            uint8_t b = (uint8_t)((r & 3) ? 0xFF : (r >> 8)); put(&b, 1);
        } else { fprintf(stderr, "kind?\n"); exit(2); }
        i++;
    }
    p.resize(target);
    return p;
}

template <int SEQ, int KIND>
static float run(const SnappyArgs &a, int reps)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto launch = [&]() {
        if (KIND == 1) hipLaunchKernelGGL(k_snappy_win<SEQ>, dim3(a.nfrags), dim3(64), 0, 0, a);
        else if (KIND == 2) hipLaunchKernelGGL(k_snappy_s<SEQ>, dim3(a.nfrags), dim3(64), 0, 0, a);
        else if (KIND == 3) hipLaunchKernelGGL(k_snappy_w<SEQ>, dim3(a.nfrags), dim3(64), 0, 0, a);
        else if (KIND == 4) {   // register-table kernel, batched LDS kernel for the fragments it gives up on
            hipLaunchKernelGGL(k_snappy_v, dim3(a.nfrags), dim3(64), 0, 0, a);
            hipLaunchKernelGGL(k_snappy_s_rest, dim3(a.nfrags), dim3(64), 0, 0, a);
        } else if (KIND == 5) hipLaunchKernelGGL(k_snappy_v, dim3(a.nfrags), dim3(64), 0, 0, a);
        else if (KIND == 9) hipLaunchKernelGGL(k_snappy_vns, dim3(a.nfrags), dim3(64), 0, 0, a);   // timing only
        else if (KIND == 7) {   // register-resident + scheduled fast path, then the batched LDS kernel
            hipLaunchKernelGGL(k_snappy_ra, dim3(a.nfrags), dim3(64), 0, 0, a);
            hipLaunchKernelGGL(k_snappy_s_rest, dim3(a.nfrags), dim3(64), 0, 0, a);
        }
        else if (KIND == 8) {   // windowed register-resident kernel, then the batched LDS kernel
            hipLaunchKernelGGL(k_snappy_w2, dim3(a.nfrags), dim3(64), 0, 0, a);
            hipLaunchKernelGGL(k_snappy_s_rest, dim3(a.nfrags), dim3(64), 0, 0, a);
        }
        else if (KIND == 6) {   // register-resident fragment kernel, then the batched LDS kernel
            hipLaunchKernelGGL(k_snappy_r, dim3(a.nfrags), dim3(64), 0, 0, a);
            hipLaunchKernelGGL(k_snappy_s_rest, dim3(a.nfrags), dim3(64), 0, 0, a);
        }
        else hipLaunchKernelGGL(k_snappy_frag<SEQ>, dim3(a.nfrags), dim3(64), 0, 0, a);
    };
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv)
{
    const size_t MB = 1 << 20;
    const size_t size = argc > 1 ? (size_t)atoll(argv[1]) * MB : 256 * MB;   // bytes per kind (many pages of 16 MiB)
    std::vector<std::string> kinds = {"ts", "price", "user_id", "ids14", "key16", "json", "defl"};
    // "@file": real pages dumped by dump_pages.py (u64 length + bytes each); every page of
    // at least 1 MiB becomes one kind "pageN", replicated to `size` bytes
    std::vector<std::vector<uint8_t>> file_pages;
    if (argc > 2 && argv[2][0] == '@') {
        kinds.clear();
        FILE *fp = fopen(argv[2] + 1, "rb");
        if (!fp) { fprintf(stderr, "cannot open %s\n", argv[2] + 1); return 2; }
        uint64_t l;
        for (int i = 0; fread(&l, 8, 1, fp) == 1; i++) {
            std::vector<uint8_t> b(l);
            if (fread(b.data(), 1, l, fp) != l) return 2;
            if (l >= MB) { kinds.push_back("page" + std::to_string(i)); file_pages.push_back(std::move(b)); }
        }
        fclose(fp);
    }
    int bad = 0;
    for (size_t ki = 0; ki < kinds.size(); ki++) {
        const char *kind = kinds[ki].c_str();
        if (argc > 2 && argv[2][0] != '@' && !strstr(argv[2], kind)) continue;   // optional kind filter, e.g. "ts,key16"
        if (argc > 3 && kinds[ki] != argv[3]) continue;                            // "@file pageN"
        // pages of 16 MiB (C2 pages are 2-17 MiB), or copies of the real page
        const size_t psz = file_pages.empty() ? 16 * MB : file_pages[ki].size();
        const size_t npages = (size + psz - 1) / psz;
        std::vector<uint8_t> host;
        std::vector<uint64_t> off, len;
        for (size_t p = 0; p < npages; p++) {
            std::vector<uint8_t> pg = file_pages.empty() ? make_page(kind, psz) : file_pages[ki];
            off.push_back(host.size()); len.push_back(pg.size());
            host.insert(host.end(), pg.begin(), pg.end());
        }
        host.resize(host.size() + 512, 0);   // K7 reads through 256-byte windows (the engine pads the same)
        std::vector<uint32_t> fpage, fidx;
        for (size_t p = 0; p < npages; p++)
            for (uint32_t k = 0; (uint64_t)k * SNAPPY_FRAG < len[p]; k++) { fpage.push_back((uint32_t)p); fidx.push_back(k); }
        const uint32_t nf = (uint32_t)fpage.size();
        uint8_t *d_in, *d_fout; uint64_t *d_off, *d_len; uint32_t *d_fp, *d_fi, *d_flen;
        CK(hipMalloc(&d_in, host.size())); CK(hipMemcpy(d_in, host.data(), host.size(), hipMemcpyHostToDevice));
        CK(hipMalloc(&d_off, npages * 8)); CK(hipMemcpy(d_off, off.data(), npages * 8, hipMemcpyHostToDevice));
        CK(hipMalloc(&d_len, npages * 8)); CK(hipMemcpy(d_len, len.data(), npages * 8, hipMemcpyHostToDevice));
        CK(hipMalloc(&d_fp, nf * 4)); CK(hipMemcpy(d_fp, fpage.data(), nf * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&d_fi, nf * 4)); CK(hipMemcpy(d_fi, fidx.data(), nf * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&d_fout, (size_t)nf * SNAPPY_FRAG_CAP)); CK(hipMalloc(&d_flen, nf * 4));
        SnappyArgs a{};
        a.in = d_in; a.page_off = d_off; a.page_len = d_len; a.npages = (uint32_t)npages; a.nfrags = nf;
        a.frag_page = d_fp; a.frag_idx = d_fi; a.frag_out = d_fout; a.frag_len = d_flen;
        // oracle output for page 0 (all pages of a kind share the generator, page 0 suffices + spot page last)
        std::vector<std::vector<uint8_t>> want(npages);
        for (size_t p : {(size_t)0, npages - 1}) {
            want[p].resize(32 + len[p] + len[p] / 6);
            int64_t w = kpwo_snappy_compress(host.data() + off[p], len[p], want[p].data(), want[p].size());
            want[p].resize((size_t)w);
        }
        auto check = [&](const char *var) {
            std::vector<uint32_t> fl(nf);
            CK(hipMemcpy(fl.data(), d_flen, nf * 4, hipMemcpyDeviceToHost));
            std::vector<uint8_t> fo((size_t)nf * SNAPPY_FRAG_CAP);
            CK(hipMemcpy(fo.data(), d_fout, fo.size(), hipMemcpyDeviceToHost));
            uint64_t comp = 0;
            for (uint32_t f = 0; f < nf; f++) comp += fl[f];
            for (size_t p : {(size_t)0, npages - 1}) {
                std::vector<uint8_t> got;
                uint32_t v = (uint32_t)len[p];
                while (v >= 0x80) { got.push_back((uint8_t)(v | 0x80)); v >>= 7; }
                got.push_back((uint8_t)v);
                for (uint32_t f = 0; f < nf; f++)
                    if (fpage[f] == p) got.insert(got.end(), fo.begin() + (size_t)f * SNAPPY_FRAG_CAP, fo.begin() + (size_t)f * SNAPPY_FRAG_CAP + fl[f]);
                if (got != want[p]) { printf("MISMATCH kind=%s variant=%s page=%zu (got %zu want %zu)\n", kind, var, p, got.size(), want[p].size()); bad++; }
            }
            return comp;
        };
        const double gb = (double)(npages * psz) / 1e9;
        struct V { const char *name; float (*fn)(const SnappyArgs &, int); };
        V vs[] = {{"s2", run<2, 2>}, {"v+s2", run<2, 4>}, {"r+s2", run<2, 6>}, {"ra+s2", run<2, 7>}, {"w2+s2", run<2, 8>}, {"x-vnostore", run<2, 9>}};
        {   // how many fragments the register-table kernel gives up on
            (void)run<2, 5>(a, 1);
            std::vector<uint32_t> fl(nf);
            CK(hipMemcpy(fl.data(), d_flen, nf * 4, hipMemcpyDeviceToHost));
            uint32_t ab = 0;
            for (uint32_t f = 0; f < nf; f++) ab += fl[f] == VT_ABORTED;
            printf("kind=%-8s v-kernel aborted %u of %u fragments\n", kind, ab, nf);
        }
        for (auto &v : vs) {
            CK(hipMemset(d_fout, 0, (size_t)nf * SNAPPY_FRAG_CAP));
            float ms = v.fn(a, 3);
            uint64_t comp = strncmp(v.name, "x-", 2) ? check(v.name) : 0;   // "x-" variants: timing only
            printf("kind=%-8s variant=%-7s frags=%6u ratio=%.3f ms=%8.3f GB/s=%7.2f\n", kind, v.name, nf,
                   (double)comp / (npages * psz), ms, gb / (ms * 1e-3));
            fflush(stdout);
        }
        hipFree(d_in); hipFree(d_off); hipFree(d_len); hipFree(d_fp); hipFree(d_fi); hipFree(d_fout); hipFree(d_flen);
    }
    printf(bad ? "FAILED %d\n" : "ALL MATCH\n", bad);
    return bad ? 1 : 0;
}
