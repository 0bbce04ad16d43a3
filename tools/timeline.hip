// timeline.hip -- diagnostic only (never shipped): the real engine built with GGP_TIMELINE, run on
// a synthetic forest with the path launch; prints, per launch phase, when the blocks reach it
// (constant 100 MHz clock, microseconds after the first block's entry): min / median / max.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//     -I gfp_gaussian_process_amd/csrc -o tools/timeline tools/timeline.hip \
//     -L gfp_gaussian_process_amd/lib -lggp_host -Wl,-rpath,'$ORIGIN/../gfp_gaussian_process_amd/lib'
//   tools/timeline TREES [ROWS_PER_TREE=200] [EVALS=5]    (TREES = 0: tools/timeline 0 input.csv EVALS csv_config)
#define GGP_TIMELINE
#include "ggp_engine.hip"
#include "ggp_host.h"

#include <algorithm>
#include <chrono>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char **argv)
{
    const int64_t trees = argc > 1 ? atoll(argv[1]) : 1000;
    const int64_t rows = trees > 0 && argc > 2 ? atoll(argv[2]) : 200;
    const int evals = argc > 3 ? atoi(argv[3]) : 5;
    ggp_host_forest *hf = nullptr;
    if (trees == 0) {   // TREES = 0: the CSV in ROWS_PER_TREE's place (the reference's example) with CONFIG in argv[4]
        ggp_csv_config *cfg = nullptr;
        ggp_dataset *ds = nullptr;
        if (ggp_csv_config_load(argc > 4 ? argv[4] : "", &cfg) != 0 || ggp_dataset_read(argv[2], cfg, &ds) != 0 ||
            ggp_forest_build(ds, -1, 1, 1, &hf) != 0) { fprintf(stderr, "csv: %s\n", ggp_host_last_error()); return 1; }
    } else if (ggp_synthetic_forest(trees, rows, 20261015ULL, 0, 1, 1, &hf) != 0) { fprintf(stderr, "synthetic failed\n"); return 1; }
    ggp_forest_desc d;
    ggp_host_forest_desc(hf, &d);
    ggp_forest *f = nullptr;
    if (ggp_forest_create(&d, &f) != GGP_OK) { fprintf(stderr, "create failed\n"); return 1; }
    const int nb = (int)f->shards[0]->n_paths;
    if (nb <= 0 || nb > 8192) { fprintf(stderr, "no path launch (%d paths)\n", nb); return 1; }
    const double P[11] = {2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04,
                          3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01};
    double ll;
    int64_t nc, nr;
    for (int k = 0; k < 3; ++k) ggp_total_loglik(f, P, &ll, &nc, &nr);
    const char *names[7] = {"entry", "dawson table in LDS", "lane constants", "first cell: steps begin",
                            "last cell: steps end", "last cell: state stored", "exit (after reduction)"};
    std::vector<unsigned long long> tl((size_t)nb * 8);
    for (int e = 0; e < evals; ++e) {
        unsigned long long z4[4] = {0, 0, 0, 0}, c4[4];
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_cnt), z4, sizeof z4);
        const auto h0 = std::chrono::steady_clock::now();
        ggp_total_loglik(f, P, &ll, &nc, &nr);
        (void)hipMemcpyFromSymbol(c4, HIP_SYMBOL(g_cnt), sizeof c4);
        printf("counts: steady steps %llu, with a stage-B rare branch %llu, dt-cache refreshes %llu, chunk loads %llu\n",
               c4[0], c4[1], c4[2], c4[3]);
        const auto h1 = std::chrono::steady_clock::now();
        (void)hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(g_tl), tl.size() * 8);
        unsigned long long t0 = ~0ull, tend = 0;
        for (int b = 0; b < nb; ++b) {
            t0 = std::min(t0, tl[(size_t)b * 8]);
            tend = std::max(tend, tl[(size_t)b * 8 + 6]);
        }
        printf("eval %d: trees=%lld rows/tree=%lld paths=%d host call %.1f us, first entry -> last exit %.1f us\n", e,
               (long long)trees, (long long)rows, nb, std::chrono::duration<double, std::micro>(h1 - h0).count(),
               (tend - t0) / 100.0);
        for (int k = 0; k < 7; ++k) {
            std::vector<double> v;
            for (int b = 0; b < nb; ++b) v.push_back((tl[(size_t)b * 8 + k] - t0) / 100.0);
            std::sort(v.begin(), v.end());
            printf("  %-28s min %8.2f  p10 %8.2f  med %8.2f  p90 %8.2f  max %8.2f us\n", names[k], v[0], v[v.size() / 10],
                   v[v.size() / 2], v[v.size() * 9 / 10], v.back());
        }
        // the hand-off to second daughters: the parent's publish -> the daughter's wait seeing it
        // -> its first step (blocks whose first cell waited: g_tlx set this evaluation)
        {
            std::vector<unsigned long long> tlx((size_t)nb * 2), tlc(1 << 16);
            (void)hipMemcpyFromSymbol(tlx.data(), HIP_SYMBOL(g_tlx), tlx.size() * 8);
            (void)hipMemcpyFromSymbol(tlc.data(), HIP_SYMBOL(g_tlc), tlc.size() * 8);
            std::vector<int32_t> pc((size_t)nb + 1), cells;
            const Shard *sh = f->shards[0];
            (void)hipMemcpy(pc.data(), sh->d_path_seq, pc.size() * 4, hipMemcpyDeviceToHost);
            cells.resize((size_t)pc[nb]);
            (void)hipMemcpy(cells.data(), sh->d_path_cells, cells.size() * 4, hipMemcpyDeviceToHost);
            std::vector<double> g1, g2;
            for (int b = 0; b < nb; ++b) {
                const int c = cells[(size_t)pc[b]];
                if (tlx[(size_t)b * 2] < t0 || tlx[(size_t)b * 2 + 1] < t0) continue;   // not a waiting block
                const int p = d.parent[c];
                if (p < 0 || p >= (1 << 16) || tlc[(size_t)p] < t0) continue;
                g1.push_back(((long long)tlx[(size_t)b * 2] - (long long)tlc[(size_t)p]) / 100.0);
                g2.push_back(((long long)tlx[(size_t)b * 2 + 1] - (long long)tlx[(size_t)b * 2]) / 100.0);
            }
            for (auto *v : {&g1, &g2}) std::sort(v->begin(), v->end());
            if (!g1.empty())
                printf("  hand-off (%zu second daughters): publish -> flag seen med %.2f p90 %.2f max %.2f us; "
                       "flag seen -> first step med %.2f p90 %.2f max %.2f us\n", g1.size(), g1[g1.size() / 2],
                       g1[g1.size() * 9 / 10], g1.back(), g2[g2.size() / 2], g2[g2.size() * 9 / 10], g2.back());
        }
        // per block phase durations (median over blocks)
        const char *dn[6] = {"table", "lane setup", "to first step", "steps (all cells)", "stores", "reduction"};
        printf("  per-block durations (median):");
        for (int k = 0; k < 6; ++k) {
            std::vector<double> v;
            for (int b = 0; b < nb; ++b) v.push_back(((long long)tl[(size_t)b * 8 + k + 1] - (long long)tl[(size_t)b * 8 + k]) / 100.0);
            std::sort(v.begin(), v.end());
            printf(" %s %.2f", dn[k], v[v.size() / 2]);
        }
        printf(" us\n");
    }
    // placement of the last evaluation's blocks: per SIMD (XCC, SE, SH, CU, SIMD) the number of
    // blocks and of root paths (steps begin within 20 us of the first entry: no wait), and the
    // blocks' end of steps by those counts
    {
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < nb; ++b) t0 = std::min(t0, tl[(size_t)b * 8]);
        std::map<unsigned long long, std::pair<int, int>> simd;   // key -> (blocks, roots)
        std::map<unsigned long long, int> cu;
        auto key_of = [&](int b, bool with_simd) {
            const unsigned long long h = tl[(size_t)b * 8 + 7];
            const unsigned lo = (unsigned)h, xcc = (unsigned)(h >> 32) & 0xf;
            const unsigned sm = (lo >> 4) & 3, c = (lo >> 8) & 15, sh = (lo >> 12) & 1, se = (lo >> 13) & 7;
            return ((unsigned long long)xcc << 32) | (se << 16) | (sh << 12) | (c << 4) | (with_simd ? sm : 0);
        };
        auto is_root = [&](int b) { return (tl[(size_t)b * 8 + 3] - t0) / 100.0 < 20.0; };
        for (int b = 0; b < nb; ++b) {
            auto &e = simd[key_of(b, true)];
            e.first++;
            e.second += is_root(b);
            cu[key_of(b, false)]++;
        }
        std::map<std::pair<int, int>, std::vector<double>> by;
        for (int b = 0; b < nb; ++b) {
            const auto e = simd[key_of(b, true)];
            by[{e.first, e.second}].push_back((tl[(size_t)b * 8 + 4] - t0) / 100.0);
        }
        std::map<int, int> cu_hist;
        for (auto &kv : cu) cu_hist[kv.second]++;
        printf("placement: %zu SIMDs used, %zu CUs used; blocks per CU:", simd.size(), cu.size());
        for (auto &kv : cu_hist) printf(" %d:%d", kv.first, kv.second);
        printf("\n  (blocks on the SIMD, root paths on the SIMD) -> blocks, steps-end mean / max us\n");
        for (auto &kv : by) {
            double m = 0, mx = 0;
            for (double v : kv.second) { m += v; mx = std::max(mx, v); }
            printf("  (%d, %d): %5zu blocks  end mean %8.2f  max %8.2f\n", kv.first.first, kv.first.second, kv.second.size(),
                   m / kv.second.size(), mx);
        }
    }
    ggp_forest_destroy(f);
    ggp_host_forest_free(hf);
    return 0;
}
