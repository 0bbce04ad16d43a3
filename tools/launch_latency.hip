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
struct BigArgs {
    double v[64];
};
template <int N>
struct Args {
    double v[N];
};
template <int N>
__global__ void k_args(Args<N> a, int64_t *seq, int64_t v)
{
    if (threadIdx.x == 0 && a.v[0] == 12345.0) __hip_atomic_store(seq, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int N>
static double enqueue_after_sync(hipStream_t s, int64_t *d)
{
    Args<N> a{};
    std::vector<double> t;
    for (int i = 0; i < 1050; ++i) {
        const auto x = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_args<N>, dim3(2000), dim3(64), 0, s, a, d, (int64_t)0);
        const auto y = std::chrono::steady_clock::now();
        (void)hipStreamSynchronize(s);
        if (i >= 50) t.push_back(std::chrono::duration<double, std::micro>(y - x).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}
__global__ void k_bigarg(BigArgs a, int64_t *seq, int64_t v)
{
    if (threadIdx.x == 0 && a.v[0] == 12345.0) __hip_atomic_store(seq, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
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
    // the enqueue of a launch with a 512-byte argument block (the path launch passes ~400 B), each
    // after the previous completed (as the engine's calls are)
    BigArgs ba{};
    std::vector<double> enq;
    for (int i = 0; i < 2050; ++i) {
        const auto a = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_bigarg, dim3(2000), dim3(64), 0, s, ba, d, (int64_t)0);
        const auto b = std::chrono::steady_clock::now();
        (void)hipStreamSynchronize(s);
        if (i >= 50) enq.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    std::sort(enq.begin(), enq.end());
    // the same with no arguments: does the argument block's size show in the enqueue?
    std::vector<double> enq0;
    for (int i = 0; i < 2050; ++i) {
        const auto a = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_empty, dim3(2000), dim3(64), 0, s);
        const auto b = std::chrono::steady_clock::now();
        (void)hipStreamSynchronize(s);
        if (i >= 50) enq0.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    std::sort(enq0.begin(), enq0.end());
    int dev = 0;
    const double gd = median_us([&](int) { (void)hipGetDevice(&dev); });
    const double sd = median_us([&](int) { (void)hipSetDevice(dev); });
    const double le = median_us([&](int) { (void)hipGetLastError(); });
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
    // C2 (1000 trees x 200): the call and its host split (ggp_call_trace), median of 500 calls
    ggp_host_forest *h2 = nullptr;
    ggp_synthetic_forest(1000, 200, 20261015ULL, 0, 1, 1, &h2);
    ggp_forest_desc d2;
    ggp_host_forest_desc(h2, &d2);
    ggp_forest *f2 = nullptr;
    ggp_forest_create(&d2, &f2);
    const double c2 = median_us([&](int) { ggp_total_loglik(f2, P, &ll, &nc, &nr); }, 500);
    std::vector<double> tr(6 * 500);
    int32_t ntr = 0;
    ggp_call_trace(f2, 500, tr.data(), &ntr);
    auto med = [&](int k) {
        std::vector<double> x;
        for (int i = 0; i < ntr; ++i) x.push_back(tr[6 * i + k]);
        std::sort(x.begin(), x.end());
        return x.empty() ? 0.0 : x[x.size() / 2];
    };
    printf("empty kernel + hipStreamSynchronize   %7.2f us\n", e);
    printf("kernel + spin on a mapped seq slot    %7.2f us   (the engine's completion path)\n", m);
    printf("hipLaunchKernelGGL alone (enqueue)    %7.2f us\n", l);
    printf("ggp_total_loglik, 1 tree x 4 rows     %7.2f us   (4 cells' steps, setup, reduction)\n", g);
    printf("enqueue of a 2000-block launch, 520 B of arguments  %7.2f us (median), %7.2f us (p90)\n",
           enq[enq.size() / 2], enq[enq.size() * 9 / 10]);
    printf("enqueue of a 2000-block launch, no arguments        %7.2f us (median)\n", enq0[enq0.size() / 2]);
    printf("enqueue by argument bytes (+16): 64 %.2f, 128 %.2f, 192 %.2f, 256 %.2f, 320 %.2f, 384 %.2f us\n",
           enqueue_after_sync<8>(s, d), enqueue_after_sync<16>(s, d), enqueue_after_sync<24>(s, d),
           enqueue_after_sync<32>(s, d), enqueue_after_sync<40>(s, d), enqueue_after_sync<48>(s, d));
    printf("hipGetDevice %7.3f us, hipSetDevice (same device) %7.3f us, hipGetLastError %7.3f us\n", gd, sd, le);
    printf("ggp_total_loglik C2 (1000 x 200)      %7.2f us: enqueue %.2f, wait %.2f (kernel %.2f), result %.2f\n",
           c2, med(0), med(1), med(3), med(2));
    ggp_forest_destroy(f2);
    ggp_host_forest_free(h2);
    ggp_forest_destroy(f);
    ggp_host_forest_free(hf);
    return 0;
}
