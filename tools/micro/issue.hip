// issue.hip -- diagnostic microbenchmark (never shipped): single-wave issue cost (s_memtime
// units per instruction) of the op classes the wave schedule uses, 4 independent chains each.
#include <hip/hip_runtime.h>
#include <cstdio>

#define T0(v) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory")
#define REP4(x) x x x x
#define BODY(name, idx, code)                                                     \
    T0(t0);                                                                       \
    for (int i = 0; i < n; ++i) { REP4(REP4(code)) }                              \
    asm volatile("" ::"v"(a), "v"(b), "v"(c), "v"(d));                            \
    T0(t1);                                                                       \
    out[idx] = t1 - t0;

__global__ void k(double *io, unsigned long long *out, int n)
{
    const int l = threadIdx.x;
    double a = io[l], b = io[l + 64], c = io[l + 128], d = io[l + 192];
    double x = io[l] * 0.5;
    int ia = l, ib = l + 1, ic = l + 2, id = l + 3;
    unsigned long long t0, t1;
    // 16 instructions x 4 chains per iteration -> 64 ops per iteration
    BODY("fma_f64", 0,
         asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x));)
    BODY("add_f64", 1,
         asm volatile("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x));)
    BODY("cndmask_b32", 2,
         asm volatile("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc" : "+v"(ia), "+v"(ib), "+v"(ic), "+v"(id) : "v"(l));)
    BODY("mov_b64", 3,
         asm volatile("v_mov_b64 %0, %4\n v_mov_b64 %1, %4\n v_mov_b64 %2, %4\n v_mov_b64 %3, %4" : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(x));)
    BODY("add_u32", 4,
         asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4" : "+v"(ia), "+v"(ib), "+v"(ic), "+v"(id) : "v"(l));)
    BODY("ldexp_f64", 5,
         asm volatile("v_ldexp_f64 %0, %0, %4\n v_ldexp_f64 %1, %1, %4\n v_ldexp_f64 %2, %2, %4\n v_ldexp_f64 %3, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(ia));)
    BODY("rcp_f64", 6,
         asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
    BODY("cvt_i32_f64", 7,
         asm volatile("v_cvt_i32_f64 %0, %4\n v_cvt_i32_f64 %1, %4\n v_cvt_i32_f64 %2, %4\n v_cvt_i32_f64 %3, %4" : "=v"(ia), "=v"(ib), "=v"(ic), "=v"(id) : "v"(x));)
    BODY("cmp_f64->vcc", 8,
         asm volatile("v_cmp_lt_f64 vcc, %0, %4\n v_cmp_lt_f64 vcc, %1, %4\n v_cmp_lt_f64 vcc, %2, %4\n v_cmp_lt_f64 vcc, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x) : "vcc");)
    BODY("rndne_f64", 9,
         asm volatile("v_rndne_f64 %0, %0\n v_rndne_f64 %1, %1\n v_rndne_f64 %2, %2\n v_rndne_f64 %3, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
    BODY("mul_lo_u32", 10,
         asm volatile("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4" : "+v"(ia), "+v"(ib), "+v"(ic), "+v"(id) : "v"(l));)
    BODY("readlane_b32", 11,
         asm volatile("v_readlane_b32 s40, %0, 0\n v_readlane_b32 s41, %1, 1\n v_readlane_b32 s42, %2, 2\n v_readlane_b32 s43, %3, 3" : "+v"(ia), "+v"(ib), "+v"(ic), "+v"(id) :: "s40", "s41", "s42", "s43");)
    BODY("mov_dpp_b32", 12,
         asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(ia), "+v"(ib), "+v"(ic), "+v"(id));)
    BODY("mul_f64", 13,
         asm volatile("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x));)
    BODY("pk_fma_f32", 14,
         asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x));)
    BODY("s_add_u32 (SALU)", 15,
         asm volatile("s_add_u32 s40, s40, 1\n s_add_u32 s41, s41, 1\n s_add_u32 s42, s42, 1\n s_add_u32 s43, s43, 1" ::: "s40", "s41", "s42", "s43", "scc");)
    io[l] = a + b + c + d + (double)(ia + ib + ic + id);
}

int main()
{
    double *io;
    unsigned long long *out, h[16];
    hipMalloc(&io, 256 * 8);
    hipMalloc(&out, 16 * 8);
    double hio[256];
    for (int i = 0; i < 256; ++i) hio[i] = 1.0 + 1e-3 * i;
    hipMemcpy(io, hio, sizeof hio, hipMemcpyHostToDevice);
    const int n = 200;
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, io, out, n);
    hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    const char *names[16] = {"v_fma_f64", "v_add_f64", "v_cndmask_b32", "v_mov_b64", "v_add_u32", "v_ldexp_f64",
                             "v_rcp_f64", "v_cvt_i32_f64", "v_cmp_lt_f64", "v_rndne_f64", "v_mul_lo_u32",
                             "v_readlane_b32", "v_mov_b32_dpp", "v_mul_f64", "v_pk_fma_f32", "s_add_u32"};
    for (int i = 0; i < 16; ++i) printf("%-16s %6.2f units/instr (4 independent chains)\n", names[i], (double)h[i] / (n * 64.0));
    return 0;
}
