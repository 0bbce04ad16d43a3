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
    // 9. dependent f64 select chain (two v_cndmask_b32 per select)
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) { asm volatile("" : "+v"(a)); a = (l & (1 << (i & 3))) ? a : b; }
    asm volatile("" :: "v"(a));
    T0(t1);
    out[8] = t1 - t0;
    // 10. dependent v_rcp_f64 chain
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) a = __builtin_amdgcn_rcp(a);
    asm volatile("" :: "v"(a));
    T0(t1);
    out[9] = t1 - t0;
    // 11. dependent sqrt chain (ocml)
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) a = sqrt(a + 1.0);
    asm volatile("" :: "v"(a));
    T0(t1);
    out[10] = t1 - t0;
    // 12. dependent DPP row_shr:1 f64 add chain
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) {
        const long long bb = __double_as_longlong(d);
        const int lo = __builtin_amdgcn_mov_dpp((int)(bb & 0xffffffff), 0x111, 0xF, 0xF, true);
        const int hi = __builtin_amdgcn_mov_dpp((int)(bb >> 32), 0x111, 0xF, 0xF, true);
        d = d + __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
    }
    asm volatile("" :: "v"(d));
    T0(t1);
    out[11] = t1 - t0;
    // 13. LDS write then read of the same slot (stage handoff), dependent
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) { lds[l] = e; __builtin_amdgcn_s_waitcnt(0xc07f); e = lds[l ^ 1] + 1.0; }
    asm volatile("" :: "v"(e));
    T0(t1);
    out[12] = t1 - t0;
    // 14. dependent v_readlane broadcast of an f64 then fma
    T0(t0);
#pragma unroll 20
    for (int i = 0; i < n; ++i) {
        const long long bb = __double_as_longlong(f);
        const int lo = __builtin_amdgcn_readlane((int)(bb & 0xffffffff), 5);
        const int hi = __builtin_amdgcn_readlane((int)(bb >> 32), 5);
        f = __builtin_fma(__longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo)), b, c);
    }
    asm volatile("" :: "v"(f));
    T0(t1);
    out[13] = t1 - t0;
    io[l] = a + d + e + f + g + (double)idx;
}

int main()
{
    double *io;
    unsigned long long *out, h[14];
    hipMalloc(&io, 256 * 8);
    hipMalloc(&out, 14 * 8);
    double hio[256];
    for (int i = 0; i < 256; ++i) hio[i] = 1.0 + 1e-3 * i;
    hipMemcpy(io, hio, sizeof hio, hipMemcpyHostToDevice);
    const int n = 1000;
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, io, out, n);
    hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    const char *names[14] = {"fma_f64 dependent", "fma_f64 4 indep chains (per iter)", "exp dependent", "exp 4 indep (per iter)",
                            "LDS read dependent", "shfl_xor f64 dependent", "IEEE div dependent", "mul_f64 dependent",
                            "f64 select dependent", "v_rcp_f64 dependent", "sqrt (ocml) dependent", "DPP row_shr f64 add dependent",
                            "LDS write+read handoff dependent", "readlane bcast + fma dependent"};
    for (int i = 0; i < 14; ++i) printf("%-36s %8.1f cycles/iter\n", names[i], (double)h[i] / n);
    return 0;
}
