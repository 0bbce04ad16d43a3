// stamp_probe.hip -- diagnostic only (never shipped): cycles per stage of one propagation
// step in the group schedule (G = 64, one cell per wave), via s_memtime stamps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//         -I gfp_gaussian_process_amd/csrc -o tools/stamp_probe tools/stamp_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "ggp_device.h"
#include "ggp_prop.h"

#define STAMP(v)                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");    \
    __builtin_amdgcn_sched_barrier(0)

constexpr int kSlot = ggp::NX + ggp::ND + ggp::NPW + ggp::NI;
constexpr int kStageB = ggp::NXT + ggp::ND + 3;

__global__ __launch_bounds__(64) void probe(const double *m0, const double *C0, const double *pp, int steps,
                                            unsigned long long *out, double *sink)
{
    __shared__ double lds[kSlot];
    __shared__ double s_tab[GGP_DAWSON_NINT * GGP_DAWSON_NCOEF];
    for (int k = threadIdx.x; k < GGP_DAWSON_NINT * GGP_DAWSON_NCOEF; k += 64) s_tab[k] = ggp_dawson_coef[k];
    __syncthreads();
    double *Xl = lds, *Dl = Xl + ggp::NX, *Pl = Dl + ggp::ND, *Il = Pl + ggp::NPW;
    const int lg = threadIdx.x;
    double m[4], C[16];
    for (int k = 0; k < 4; ++k) m[k] = m0[k];
    for (int k = 0; k < 16; ++k) C[k] = C0[k];
    if (lg == 0) Xl[ggp::X_ONE] = 1.0;
    unsigned long long acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const double *p = pp;
    for (int s = 0; s < steps; ++s) {
        unsigned long long t0, t1, t2, t3, t4, t5;
        STAMP(t0);
        ggp::Step S;
        ggp::step_init(S, m, C, 1.0, ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]));
        STAMP(t1);
        unsigned long long u1, u2, u3;
        Xl[lg] = ggp::exp_task(S, lg);                        // exps 0..63
        __syncthreads();
        STAMP(u1);
        if (lg < 10) Xl[64 + lg] = ggp::exp_task(S, 64 + lg);  // exps 64..73
        __syncthreads();
        STAMP(u2);
        if (lg < ggp::ND) Dl[lg] = ggp::dawson_task(S, lg, s_tab);
        __syncthreads();
        STAMP(u3);
        if (lg < 3) { const double v = ggp::pow_task(S, lg); Pl[lg] = v; Pl[3 + lg] = 1.0 / v; }
        __syncthreads();
        STAMP(t2);
        acc[5] += u1 - t1; acc[6] += u2 - u1; acc[7] += u3 - u2; acc[8] += t2 - u3;
        for (int j = lg; j < ggp::NI; j += 64) Il[j] = ggp::tau_task(S, j, Xl, Dl, Pl);
        __syncthreads();
        STAMP(t3);
        ggp::outputs(S, Il, Xl, m, C);
        STAMP(t4);
        // a Kalman update to keep the state realistic
        ggp_innov v;
        const double x0 = 0.01, x1 = 5.0;
        ggp_innovation(m, C, p[7], p[8], 1, 0.0, v);
        double ll = ggp_ll_term(x0, x1, v, 3.67575413281869);
        ggp_posterior(m, C, x0, x1, v);
        __syncthreads();
        STAMP(t5);
        if (lg == 0) sink[0] += ll;
        acc[0] += t1 - t0; acc[1] += t2 - t1; acc[2] += t3 - t2; acc[3] += t4 - t3; acc[4] += t5 - t4;
    }
    if (lg == 0)
        for (int k = 0; k < 9; ++k) out[k] = acc[k];
    if (lg == 0) sink[1] = m[0] + C[5];
}

int main()
{
    // a realistic state: example root after a few steps
    double m[4] = {0.69, 3.18e4, 2.31e-3, 90.3};
    double C[16] = {0};
    C[0] = 8.4e-4; C[5] = 3.26e7; C[10] = 9.75e-8 / (2 * 4.36e-2); C[15] = 19.4 / (2 * 1.6e-2);
    C[1] = C[4] = 1.0;
    double p[11] = {2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01};
    double *dm, *dC, *dp, *sink;
    unsigned long long *dout;
    (void)hipMalloc(&dm, sizeof m); (void)hipMalloc(&dC, sizeof C); (void)hipMalloc(&dp, sizeof p);
    (void)hipMalloc(&dout, 16 * sizeof(unsigned long long)); (void)hipMalloc(&sink, 2 * sizeof(double));
    (void)hipMemcpy(dm, m, sizeof m, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, C, sizeof C, hipMemcpyHostToDevice);
    (void)hipMemcpy(dp, p, sizeof p, hipMemcpyHostToDevice);
    (void)hipMemset(sink, 0, 2 * sizeof(double));
    const int steps = 200;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dm, dC, dp, steps, dout, sink);
        (void)hipDeviceSynchronize();
    }
    unsigned long long out[16];
    (void)hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost);
    const char *names[5] = {"step_init", "B: exp/dawson/pow", "C: tauints", "D: outputs", "kalman update"};
    unsigned long long tot = 0;
    for (int k = 0; k < 5; ++k) tot += out[k];
    printf("s_memtime ticks per step (shader clock; %d steps, single wave):\n", steps);
    for (int k = 0; k < 5; ++k) printf("  %-22s %8.0f  (%4.1f%%)\n", names[k], (double)out[k] / steps, 100.0 * out[k] / tot);
    printf("  %-22s %8.0f\n", "total", (double)tot / steps);
    const char *sub[4] = {"B1 exps 0..63", "B2 exps 64..73", "B3 dawson x14", "B4 pow x3"};
    for (int k = 0; k < 4; ++k) printf("  %-22s %8.0f\n", sub[k], (double)out[5 + k] / steps);
    return 0;
}
