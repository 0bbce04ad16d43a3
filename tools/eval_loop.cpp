// eval_loop.cpp -- diagnostic only: back-to-back ggp_total_loglik calls from C++ on a synthetic
// forest (no Python in the loop), to split per-evaluation overhead into host and device parts.
//   hipcc -O2 -std=c++17 -I include -o tools/eval_loop tools/eval_loop.cpp \
//     -L gfp_gaussian_process_amd/lib -lggp -lggp_host -Wl,-rpath,$ORIGIN/../gfp_gaussian_process_amd/lib
//   tools/eval_loop TREES [KERNEL=0] [REPS=50]
#include "ggp.h"
#include "ggp_host.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>

int main(int argc, char **argv)
{
    const int64_t trees = argc > 1 ? atoll(argv[1]) : 1000;
    const int kernel = argc > 2 ? atoi(argv[2]) : GGP_KERNEL_AUTO;
    const int reps = argc > 3 ? atoi(argv[3]) : 50;
    ggp_host_forest *hf = nullptr;
    if (ggp_synthetic_forest(trees, 200, 20261015ULL, 0, 1, 1, &hf) != 0) return 1;
    ggp_forest_desc d;
    ggp_host_forest_desc(hf, &d);
    d.kernel = kernel;
    ggp_forest *f = nullptr;
    if (ggp_forest_create(&d, &f) != GGP_OK) return 1;
    const double P[11] = {2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04,
                          3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01};
    double ll = 0;
    int64_t nc, nr;
    for (int k = 0; k < 3; ++k) ggp_total_loglik(f, P, &ll, &nc, &nr);
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < reps; ++k) ggp_total_loglik(f, P, &ll, &nc, &nr);
    const auto t1 = std::chrono::steady_clock::now();
    printf("trees=%lld kernel=%d: %.4f ms/eval (C++ loop) ll=%.17g\n", (long long)trees, kernel,
           std::chrono::duration<double, std::milli>(t1 - t0).count() / reps, ll);
    // the host's own share: time inside ggp_total_loglik_async (enqueue) and inside
    // ggp_loglik_result (wait), and the kernel's device time (events)
    double t_enq = 0, t_wait = 0;
    float ms[16];
    int64_t rows[16];
    int32_t kk[16], nk = 0;
    ggp_last_launch_profile(f, ms, rows, kk, 16, &nk);   // switches the events on
    double t_dev = 0;
    for (int k = 0; k < reps; ++k) {
        const auto a = std::chrono::steady_clock::now();
        ggp_total_loglik_async(f, P);
        const auto b = std::chrono::steady_clock::now();
        ggp_loglik_result(f, &ll, &nc, &nr);
        const auto c = std::chrono::steady_clock::now();
        t_enq += std::chrono::duration<double, std::micro>(b - a).count();
        t_wait += std::chrono::duration<double, std::micro>(c - b).count();
        if (ggp_last_launch_profile(f, ms, rows, kk, 16, &nk) == GGP_OK)
            for (int i = 0; i < nk; ++i) t_dev += 1e3 * ms[i];
    }
    printf("  enqueue %.2f us, wait %.2f us, device (events) %.2f us per evaluation (profiled calls)\n", t_enq / reps,
           t_wait / reps, t_dev / reps);
    ggp_forest_destroy(f);
    ggp_host_forest_free(hf);
    return 0;
}
