// launch_latency.hip -- diagnostic: the host-side floor of one evaluation call.  Times (median of
// 2000 calls): an empty kernel + hipStreamSynchronize; a one-wave kernel that releases a sequence
// number into mapped host memory, which the host spins on (the engine's completion path,
// DESIGN.md "Completion"); ggp_total_loglik on a one-row forest (the engine's own call, minimal
// work); and the same call from Python/ctypes is in tools/launch_latency.py.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/launch_latency tools/launch_latency.hip \
//     -L gfp_gaussian_process_amd/lib -lggp -lggp_host -Wl,-rpath,'$ORIGIN/../gfp_gaussian_process_amd/lib'
#include <hip/hip_runtime.h>
#include "ggp.h"
#include "ggp_host.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}
__global__ void k_signal(int64_t *seq, int64_t v)
{
    if (threadIdx.x == 0) __hip_atomic_store(seq, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class F>
static double median_us(F &&f, int reps = 2000)
{
    std::vector<double> t(reps);
    for (int i = 0; i < 50; ++i) f(i);
    for (int i = 0; i < reps; ++i) {
        const auto a = std::chrono::steady_clock::now();
        f(i);
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main()
{
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int64_t *h = nullptr, *d = nullptr;
    (void)hipHostMalloc((void **)&h, 64, hipHostMallocMapped);
    (void)hipHostGetDevicePointer((void **)&d, h, 0);
    *h = 0;
    const double e = median_us([&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        (void)hipStreamSynchronize(s);
    });
    const double m = median_us([&](int i) {
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s, d, (int64_t)(i + 1000000));
        while (__atomic_load_n((volatile int64_t *)h, __ATOMIC_ACQUIRE) != i + 1000000) {
        }
    });
    const double l = median_us([&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); }, 200);
    (void)hipStreamSynchronize(s);
    ggp_host_forest *hf = nullptr;
    ggp_synthetic_forest(1, 4, 20261015ULL, 0, 1, 1, &hf);   // one tree: root 2 rows, daughters 1 + 1
    ggp_forest_desc dd;
    ggp_host_forest_desc(hf, &dd);
    ggp_forest *f = nullptr;
    ggp_forest_create(&dd, &f);
    const double P[11] = {2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04,
                          3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01};
    double ll;
    int64_t nc, nr;
    const double g = median_us([&](int) { ggp_total_loglik(f, P, &ll, &nc, &nr); });
    printf("empty kernel + hipStreamSynchronize   %7.2f us\n", e);
    printf("kernel + spin on a mapped seq slot    %7.2f us   (the engine's completion path)\n", m);
    printf("hipLaunchKernelGGL alone (enqueue)    %7.2f us\n", l);
    printf("ggp_total_loglik, 1 tree x 4 rows     %7.2f us   (4 cells' steps, setup, reduction)\n", g);
    ggp_forest_destroy(f);
    ggp_host_forest_free(hf);
    return 0;
}
