// stamp_group.hip -- diagnostic only (never shipped): the real engine built with GGP_STAMPS,
// run on a synthetic forest; prints s_memtime cycles per stage per step of k_loglik_group.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//     -I gfp_gaussian_process_amd/csrc -o tools/stamp_group tools/stamp_group.hip \
//     -L gfp_gaussian_process_amd/lib -lggp_host -Wl,-rpath,$PWD/gfp_gaussian_process_amd/lib
//   tools/stamp_group TREES [KERNEL=2] [ROWS_PER_TREE=200]
#define GGP_STAMPS
#include "ggp_engine.hip"
#include "ggp_host.h"

#include <cstdio>
#include <cstdlib>

int main(int argc, char **argv)
{
    const int64_t trees = argc > 1 ? atoll(argv[1]) : 1000;
    const int kernel = argc > 2 ? atoi(argv[2]) : GGP_KERNEL_GROUP;
    const int64_t rows = argc > 3 ? atoll(argv[3]) : 200;   // rows per tree (SURVEY 8(d) shape)
    ggp_host_forest *hf = nullptr;
    if (ggp_synthetic_forest(trees, rows, 20261015ULL, 0, 1, 1, &hf) != 0) { fprintf(stderr, "synthetic failed\n"); return 1; }
    ggp_forest_desc d;
    ggp_host_forest_desc(hf, &d);
    d.kernel = kernel;
    ggp_forest *f = nullptr;
    if (ggp_forest_create(&d, &f) != GGP_OK) { fprintf(stderr, "create: %s\n", ggp_strerror(GGP_EINVAL)); return 1; }
    const double P[11] = {2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04,
                          3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01};
    double ll;
    int64_t nc, nr;
    ggp_total_loglik(f, P, &ll, &nc, &nr);
    unsigned long long zero[64] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), zero, sizeof zero);
    const int reps = 5;
    for (int k = 0; k < reps; ++k) ggp_total_loglik(f, P, &ll, &nc, &nr);
    unsigned long long all[64];
    (void)hipMemcpyFromSymbol(all, HIP_SYMBOL(g_stamp), sizeof all);
    const char *gnames[8] = {"prefetch+step_init", "B exp/dawson/pow", "barrier 1", "C integrals",
                             "barrier 2", "D outputs+division", "update", "barrier 3"};
    // k_loglik_wave (ggp_wave.h): stamps 0..10
    const char *wnames[11] = {"scalars+monomials", "B exp/dawson", "barrier B", "C integrals",
                              "barrier C", "D output terms", "butterfly+OUT", "finish+innovation", "barrier+update",
                              "end step (flush/64)", "-"};
    for (int slot = 0; slot < 4; ++slot) {
        const unsigned long long *acc = all + 16 * slot;
        const double steps = (double)acc[15];
        if (steps == 0) continue;
        const bool wave = kernel == 3;
        const int ns = wave ? 11 : 8;
        unsigned long long tot = 0;
        for (int k = 0; k < ns; ++k) tot += acc[k];
        printf("trees=%lld %s ll=%.10g wave-steps=%.0f cycles/step=%.0f\n", (long long)trees,
               wave ? (slot == 3 ? "wave, levels <= 1024 cells" : "wave, levels > 1024 cells")
                    : (slot == 0 ? "G=64" : "G=32"), ll, steps, tot / steps);
        for (int k = 0; k < ns; ++k)
            printf("  %-22s %8.0f  (%4.1f%%)\n", wave ? wnames[k] : gnames[k], acc[k] / steps, 100.0 * acc[k] / tot);
    }
    if (kernel == 3) {
        unsigned long long ps[2][9];
        (void)hipMemcpyFromSymbol(ps, HIP_SYMBOL(g_pstamp), sizeof ps);
        const char *pn[8] = {"", "dawson table", "lane tasks+kappa", "cell prologue", "row chunk+barrier",
                             "first step", "steady steps", "state stores"};
        for (int s = 0; s < 2; ++s) {
            if (!ps[s][8]) continue;
            printf("launch phases, levels %s 1024 cells (%llu blocks), cycles per block:\n", s ? ">" : "<=", ps[s][8]);
            for (int k = 1; k < 8; ++k) printf("  %-20s %10.0f\n", pn[k], (double)ps[s][k] / ps[s][8]);
        }
    }
    ggp_forest_destroy(f);
    ggp_host_forest_free(hf);
    return 0;
}
