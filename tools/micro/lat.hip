// lat.hip -- diagnostic microbenchmark (never shipped): single-wave cycle costs of FP64 ops
// on gfx950 (dependent chain vs independent streams), exp(), LDS round trip, ds_bpermute.
#include <hip/hip_runtime.h>
#include <cstdio>

#define T0(v) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory")

__global__ void k(double *io, unsigned long long *out, int n)
{
    __shared__ double lds[256];
    const int l = threadIdx.x;
    double a = io[l], b = io[l + 64], c = io[l + 128], d = io[l + 192];
    lds[l] = a; lds[l + 64] = b;
    __syncthreads();
    unsigned long long t0, t1;
    // 1. dependent fma chain
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) a = __builtin_fma(a, b, c);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" :: "v"(a));
    T0(t1);
    out[0] = t1 - t0;
    // 2. four independent fma chains
    double e = a + 1, f = a + 2, g = a + 3;
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) { a = __builtin_fma(a, b, c); e = __builtin_fma(e, b, c); f = __builtin_fma(f, b, c); g = __builtin_fma(g, b, c); }
    asm volatile("" :: "v"(a), "v"(e), "v"(f), "v"(g));
    T0(t1);
    out[1] = t1 - t0;
    // 3. dependent exp chain
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) a = exp(a * 1e-3);
    asm volatile("" :: "v"(a));
    T0(t1);
    out[2] = t1 - t0;
    // 4. four independent exp chains
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) { a = exp(a * 1e-3); e = exp(e * 1e-3); f = exp(f * 1e-3); g = exp(g * 1e-3); }
    asm volatile("" :: "v"(a), "v"(e), "v"(f), "v"(g));
    T0(t1);
    out[3] = t1 - t0;
    // 5. dependent LDS read chain (address from value)
    int idx = l;
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) { double v = lds[idx]; idx = ((int)v & 63) + (l & 1); }
    asm volatile("" :: "v"(idx));
    T0(t1);
    out[4] = t1 - t0;
    // 6. dependent shfl_xor (ds_bpermute) chain on doubles
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) d = d + __shfl_xor(d, 1 << (i & 3));
    asm volatile("" :: "v"(d));
    T0(t1);
    out[5] = t1 - t0;
    // 7. dependent IEEE division chain
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) a = b / (a + 1.0);
    asm volatile("" :: "v"(a));
    T0(t1);
    out[6] = t1 - t0;
    // 8. dependent mul chain
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) a = a * b;
    asm volatile("" :: "v"(a));
    T0(t1);
    out[7] = t1 - t0;
    io[l] = a + d + e + f + g + (double)idx;
}

int main()
{
    double *io;
    unsigned long long *out, h[8];
    hipMalloc(&io, 256 * 8);
    hipMalloc(&out, 8 * 8);
    double hio[256];
    for (int i = 0; i < 256; ++i) hio[i] = 1.0 + 1e-3 * i;
    hipMemcpy(io, hio, sizeof hio, hipMemcpyHostToDevice);
    const int n = 1000;
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, io, out, n);
    hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    const char *names[8] = {"fma_f64 dependent", "fma_f64 4 indep chains (per iter)", "exp dependent", "exp 4 indep (per iter)",
                            "LDS read dependent", "shfl_xor f64 dependent", "IEEE div dependent", "mul_f64 dependent"};
    for (int i = 0; i < 8; ++i) printf("%-36s %8.1f cycles/iter\n", names[i], (double)h[i] / n);
    return 0;
}
