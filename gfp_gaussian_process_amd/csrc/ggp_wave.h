// ggp_wave.h -- per-lane task bodies of the WAVE schedule (k_loglik_wave, ggp_engine.hip):
// one 64-lane wave per cell; in every stage of a step each lane runs ONE task:
//
//   stage B   lane l: exponential kXW[l] (64 state-dependent exponentials), Dawson value l
//             (l < 14), power l (l < 3); then lanes 0..3 form exp(c_B), exp(c_J), exp(c_G),
//             exp(c_I) as exp(c_A) times a cached exponential
//   stage C   lane l: integral l (l < 45)
//   per dt    exp(s t) (6) and the 18 exp-derived basis values of the outputs depend on the
//             parameters and dt only: formed when dt changes, kept in LDS
//
// Why separate bodies: the task kind differs between the lanes of one wave, and the
// compiler turns a per-kind ternary into divergent branches, sinking each candidate's
// arithmetic into its own branch -- the branches then issue one after another and their
// latency chains cannot overlap (measured: ~2.8k cycles for stage B).  Here
// every candidate is computed unconditionally and pinned (an empty asm keeps it at that
// point in the instruction stream) and a select picks the lane's value: one straight-line
// stream whose chains interleave.  Stores to a slot the lane does not own go to a per-lane
// dummy slot instead of being predicated (a predicated store would bring the branch back).
//
// The expressions are those of ggp_prop.h (bitwise the same value for every exponential,
// Dawson value, power and integral, given the same operands), except the four exp(c)
// products, which differ from exp(c) by ~1 ulp (DESIGN.md "Parity").
#pragma once
#include "ggp_outtab.h"
#include "ggp_prop.h"

namespace ggp {
namespace wave {

// keep x materialised here (no sinking into a select's branch); the value lives in VGPRs
GGP_DEV double pin(double x)
{
    asm volatile("" : "+v"(x));
    return x;
}

// the parameter-only constants in VGPRs: kept uniform they occupy ~40 SGPRs for the whole
// loop and push the kernel into SGPR spills (v_writelane / v_readlane traffic every step)
GGP_DEV OU pin_ou(OU P)
{
    P.ml = pin(P.ml); P.gl = pin(P.gl); P.sl2 = pin(P.sl2); P.mq = pin(P.mq); P.gq = pin(P.gq);
    P.sq2 = pin(P.sq2); P.b = pin(P.b); P.r_gl = pin(P.r_gl); P.r_gq = pin(P.r_gq); P.gq2 = pin(P.gq2);
    P.gqq2 = pin(P.gqq2); P.r_gq2 = pin(P.r_gq2); P.r_gqq2 = pin(P.r_gqq2); P.gl2 = pin(P.gl2);
    P.r_gl2 = pin(P.r_gl2); P.k_xl = pin(P.k_xl); P.k_xx = pin(P.k_xx); P.k_ll = pin(P.k_ll);
    P.k_qq = pin(P.k_qq);
    return P;
}

// ---- the per-step exponential list ----------------------------------------------------
constexpr bool x_cached(const int j)
{
    return j == XC_B || j == XC_J || j == XC_G || j == XC_I || (j >= XS_bt && j <= XS_gq);
}
struct XWList {
    unsigned char j[64];
    int n;
};
constexpr XWList make_xw()
{
    XWList L{};
    for (int j = 0; j < NXT; ++j)
        if (!x_cached(j)) L.j[L.n++] = (unsigned char)j;
    return L;
}
constexpr XWList kXW = make_xw();
static_assert(kXW.n == 64, "one state-dependent exponential per lane");
static_assert(kXW.j[0] == XC_A, "lane 0 holds exp(c_A) for the products");

// the B values as ((b + bl) + Cxl km) + gq ks (step_init's B0..B5, same rounding)
constexpr double kKm[6] = {1., 1., 2., 2., 1., 2.};
constexpr double kKs[6] = {0., -1., 0., -1., 1., 1.};

// ---- LDS layout (doubles) --------------------------------------------------------------
enum {
    L_X = 0,                  // exponentials (NX, incl. X_ONE = 1)
    L_D = L_X + NX,           // Dawson values
    L_P = L_D + ND,           // 4 a^1.5, 8 a^2.5, 16 a^3.5, reciprocals
    L_BV = L_P + NPW,         // outputs basis: 1, the 45 integrals, 18 exp-derived values
    L_V = L_BV + BV_N,        // outputs variables: 1, state, t
    L_OUT = L_V + V_N,        // the step's 14 outputs (block sums, written by the lead lanes)
    L_DUMMY = L_OUT + kOutN,  // one slot per lane for stores of lanes without a task
    kLds = L_DUMMY + 64
};

// ---- one lane's tasks (registers for the whole launch) ---------------------------------
struct LaneTasks {
    int x_dst, x_kind, x_ic, x_it;
    double x_km, x_ks;
    int d_dst, d_it;
    double d_km, d_ks;
    int p, p_dst0, p_dst1;
    int prod_dst, mult_off;
    ITask it;
    double i_km, i_ks;
    int i_dst;
    int sv, xs_dst, dv_dst;
    DTaskB dv;
    int out_dst;
};

GGP_DEV LaneTasks lane_tasks(const int lane)
{
    LaneTasks L;
    const int xj = kXW.j[lane];
    const XTask xt = kXT[xj];
    L.x_dst = L_X + xj;
    L.x_kind = xt.kind;
    L.x_ic = xt.ic;
    L.x_it = xt.it;
    L.x_km = kKm[xt.iB < 6 ? xt.iB : 0];
    L.x_ks = kKs[xt.iB < 6 ? xt.iB : 0];
    const DTask dk = kDT[lane < ND ? lane : 0];
    L.d_dst = lane < ND ? L_D + lane : L_DUMMY + lane;
    L.d_it = dk.it;
    L.d_km = kKm[dk.iB];
    L.d_ks = kKs[dk.iB];
    L.p = lane < 3 ? lane : 0;
    L.p_dst0 = lane < 3 ? L_P + lane : L_DUMMY + lane;
    L.p_dst1 = lane < 3 ? L_P + 3 + lane : L_DUMMY + lane;
    // exp(c_B) = exp(c_A) exp(-gl t), exp(c_J) = exp(c_I) = exp(c_A) exp(-gq t),
    // exp(c_G) = exp(c_A) / exp(b t)   (c_* of step_init)
    const int prod_slot = lane == 0 ? XC_B : lane == 1 ? XC_J : lane == 2 ? XC_G : XC_I;
    const int mult = lane == 0 ? L_X + XS_gl : lane == 2 ? L_BV + BV_R_EBT : L_X + XS_gq;
    L.prod_dst = lane < 4 ? L_X + prod_slot : L_DUMMY + lane;
    L.mult_off = lane < 4 ? mult : L_X + X_ONE;
    L.it = kIT[lane < NI ? lane : 0];
    L.i_km = kKm[L.it.iB];
    L.i_ks = kKs[L.it.iB];
    L.i_dst = lane < NI ? L_BV + BV_I + lane : L_DUMMY + lane;
    L.sv = lane < 6 ? lane : 0;
    L.xs_dst = lane < 6 ? L_X + XS_bt + lane : L_DUMMY + lane;
    L.dv = kDerived[lane < kNDerived ? lane : 0];
    L.dv_dst = lane < kNDerived ? L_BV + BV_R_EBT + lane : L_DUMMY + lane;
    // the lead lane of output k's block stores the block sum
    int out = L_DUMMY + lane;
#pragma unroll
    for (int k = 0; k < kOutN; ++k) out = kOutLead[k] == lane ? L_OUT + k : out;
    L.out_dst = out;
    return L;
}

// ---- operand selection from the step scalars (every lane holds the whole Step) ---------
GGP_DEV double bsel(const Step &S, const double km, const double ks)
{
    return ((S.b + S.bl) + S.Cxl * km) + S.gq * ks;
}

GGP_DEV double csel(const Step &S, const int ic)
{
    const double c0 = pin(S.c0), c1 = pin(S.c1), c2 = pin(S.c2), c3 = pin(S.c3), c4 = pin(S.c4);
    const double c5 = pin(S.c5), c6 = pin(S.c6), c7 = pin(S.c7), c8 = pin(S.c8), c9 = pin(S.c9);
    double c = c9;
    c = ic == 8 ? c8 : c;
    c = ic == 7 ? c7 : c;
    c = ic == 6 ? c6 : c;
    c = ic == 5 ? c5 : c;
    c = ic == 4 ? c4 : c;
    c = ic == 3 ? c3 : c;
    c = ic == 2 ? c2 : c;
    c = ic == 1 ? c1 : c;
    c = ic == 0 ? c0 : c;
    return c;
}

GGP_DEV double tsel(const Step &S, const int it)
{
    const double t = pin(S.t), t2 = pin(S.t2);
    return it == 0 ? 0.0 : it == 1 ? t : t2;
}

// the argument of exponential task x (exp_body, ggp_prop.h)
GGP_DEV double exp_arg(const Step &S, const LaneTasks &T)
{
    const double ti = tsel(S, T.x_it);
    const double B = pin(bsel(S, T.x_km, T.x_ks));
    const double c = csel(S, T.x_ic);
    const double n = pin(rdiv(-(B * B), S.four_a, S.r_four_a));
    const double zt = pin(B + S.two_a * ti);
    const double z = rdiv(T.x_it == 0 ? B : zt, S.two_sa, S.r_two_sa);
    const double argA = pin(ti * (B + S.a * ti));
    const double argE = pin(n + c + z * z);
    const double argZ = pin(S.a * (ti * ti) + B * ti + c);
    return T.x_kind == KX_C ? c : T.x_kind == KX_A ? argA : T.x_kind == KX_E ? argE : argZ;
}

// the argument of Dawson task d (zval, ggp_prop.h)
GGP_DEV double dawson_arg(const Step &S, const LaneTasks &T)
{
    const double B = pin(bsel(S, T.d_km, T.d_ks));
    const double zt = pin(B + S.two_a * tsel(S, T.d_it));
    return rdiv(T.d_it == 0 ? B : zt, S.two_sa, S.r_two_sa);
}

// exp(x) exactly as ocml's __ocml_exp_f64 computes it (the same constants, fma chain and
// ldexp; bitwise the same value), with every Horner step one VOP3 v_fma_f64: the compiler's own
// form is a v_mov_b64 of the loop-invariant coefficient plus a tied v_fmac_f64 per step
GGP_DEV double fma3(const double a, const double b, const double c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
#else
    return __builtin_fma(a, b, c);
#endif
}

GGP_DEV double exp_ocml(const double x)
{
    const double dn = __builtin_rint(x * 0x1.71547652b82fep+0);
    double t = __builtin_fma(-dn, 0x1.62e42fefa39efp-1, x);
    t = __builtin_fma(-dn, 0x1.abc9e3b39803fp-56, t);
    double p = fma3(t, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
    p = fma3(t, p, 0x1.71dee623fde64p-19);
    p = fma3(t, p, 0x1.a01997c89e6b0p-16);
    p = fma3(t, p, 0x1.a01a014761f6ep-13);
    p = fma3(t, p, 0x1.6c16c1852b7b0p-10);
    p = fma3(t, p, 0x1.1111111122322p-7);
    p = fma3(t, p, 0x1.55555555502a1p-5);
    p = fma3(t, p, 0x1.5555555555511p-3);
    p = fma3(t, p, 0x1.000000000000bp-1);
    p = __builtin_fma(t, p, 1.0);
    p = __builtin_fma(t, p, 1.0);
    const double r = __builtin_ldexp(p, (int)dn);
    const double o = x > 1024.0 ? __builtin_huge_val() : r;
    return x < -1075.0 ? 0.0 : o;
}

// ggp_dawson_tab without branches: one division for the continued fraction, a NaN falls
// through the polynomial (same values as ggp_dawson_tab).  tab: rows of kDawsonRow doubles
// (the 9 coefficients, zero-padded to 10), 16-B aligned: five 128-bit LDS reads per value;
// Horner with fused multiply-adds (<= 1 ulp from the separate-rounding form; the device
// Dawson stays within the reference's bound, tests/test_gpu_device_math.py)
constexpr int kDawsonRow = 10;
GGP_DEV double dawson_bf(const double x, const double *tab)
{
    const double ax = fabs(x);
    const double d1 = 1.0 + ax;
    const double y100 = rdiv(100.0, d1, frcp(d1));   // IEEE 100 / (1 + ax) for finite ax
    const double yk = y100 >= 0.0 ? y100 : 0.0;
    const int k = min((int)yk, GGP_DAWSON_NINT - 1);
    const double2 *c2 = reinterpret_cast<const double2 *>(tab + kDawsonRow * k);
    const double2 a01 = c2[0], a23 = c2[1], a45 = c2[2], a67 = c2[3], a89 = c2[4];
    const double t = 2.0 * y100 - (double)(2 * k + 1);
    double h = __builtin_fma(a89.x, t, a67.y);
    h = __builtin_fma(h, t, a67.x);
    h = __builtin_fma(h, t, a45.y);
    h = __builtin_fma(h, t, a45.x);
    h = __builtin_fma(h, t, a23.y);
    h = __builtin_fma(h, t, a23.x);
    h = __builtin_fma(h, t, a01.y);
    const double poly = pin(__builtin_fma(h, t, a01.x));
    // the Taylor and continued-fraction branches are rare (|x| < ~0.03, |x| > 45): formed only
    // when some lane of the wave needs them (a wave-uniform branch; NaN takes neither)
    const bool use_taylor = y100 >= (double)GGP_DAWSON_NINT, use_cf = ax > 45.0;
    double taylor = 0.0, cf = 0.0;
    if (__builtin_amdgcn_ballot_w64(use_taylor)) {
        const double x2 = ax * ax;
        const double *tc = ggp_dawson_taylor;
        taylor = pin(ax * (tc[0] - x2 * (tc[1] - x2 * (tc[2] - x2 * (tc[3] - x2 * tc[4])))));
    }
    if (__builtin_amdgcn_ballot_w64(use_cf)) {
        const bool far = ax > 5e7;
        const double num = far ? GGP_ISPI : pin(GGP_ISPI * ((ax * ax) * (ax * ax - 4.5) + 2));
        const double den = far ? ax : pin(ax * ((ax * ax) * (ax * ax - 5) + 3.75));
        cf = pin(num / den);
    }
    const double w = use_cf ? cf : (use_taylor ? taylor : poly);
    return GGP_SPI2 * (x < 0.0 ? -w : w);
}

// pow_task without branches
GGP_DEV double pow_bf(const Step &S, const int p)
{
    const double sa = S.two_sa * 0.5, a = S.a;
    const double p0 = pin(4. * (a * sa)), p1 = pin(8. * ((a * a) * sa)), p2 = pin(16. * (((a * a) * a) * sa));
    return p == 0 ? p0 : p == 1 ? p1 : p2;
}

// reciprocals of the powers from the step's 1/(4a) and 1/(2 sqrt a): 1/(4 a^1.5) =
// 2 r4a r2sa, then each next power one factor 2 r4a = 1/(2a) more.  They only seed rdiv
// (q = x r, then one residual correction against the exact divisor), whose quotient does not
// depend on a few ulp in r: one division per step less than 1.0 / pow.
GGP_DEV double rpow_bf(const Step &S, const int p)
{
    const double r0 = pin(2. * (S.r_four_a * S.r_two_sa));
    const double r1 = pin(2. * (S.r_four_a * r0));
    const double r2 = pin(2. * (S.r_four_a * r1));
    return p == 0 ? r0 : p == 1 ? r1 : r2;
}

// tau_unified without branches (X, Dw, PW: the LDS arrays)
GGP_DEV double tau_bf(const Step &S, const ITask T, const double km, const double ks, const double *X,
                      const double *Dw, const double *PW)
{
    const double D0 = Dw[T.d0], D1 = Dw[T.d1];
    const double E0 = X[T.x0], E1 = X[T.x1];
    const double ec = X[T.xc], ea0 = X[T.xa0], ea1 = X[T.xa1];
    const int k = T.k;
    const int kk = k == 0 ? 0 : k - 1;
    const double pd = PW[kk], pr = PW[3 + kk];
    const double B = pin(bsel(S, km, ks));
    const double t0 = tsel(S, T.it0), t1 = tsel(S, T.it1);
    const double BB = pin(B * B);
    const double al3 = pin(BB - 2. * S.two_a);
    const double al = k == 1 ? 1.0 : k == 2 ? B : al3;
    const double be2 = pin(-S.two_a), be3 = pin(-S.two_a * B);
    const double be = k == 1 ? 0.0 : k == 2 ? be2 : be3;
    const double ga = k == 3 ? S.four_aa : 0.0;
    const double P0 = al + t0 * (be + ga * t0), P1 = al + t1 * (be + ga * t1);
    const double q1 = pin(B * 2.), q2 = pin((S.two_a - BB) * 2.), q3 = pin(B * (-6. * S.a + BB) * 2.);
    const double Q = k == 0 ? -2.0 : k == 1 ? q1 : k == 2 ? q2 : q3;
    const double S1 = k == 2 ? S.two_sa : S.m2sa;
    const double dterm = pin(Q * (E0 * D0 - E1 * D1));
    const double xfull = pin(S1 * ec * (ea0 * P0 - ea1 * P1) + dterm);
    const double x = k == 0 ? dterm : xfull;
    const double den = k == 0 ? S.two_sa : pd, rden = k == 0 ? S.r_two_sa : pr;
    return rdiv(x, den, rden);
}

// ggp_posterior with the lower triangle of C formed only on the cell's last row: on every
// other row the next propagation reads the upper triangle (step_init) and then overwrites
// all of C (out_store), so those six entries are dead.  Same expressions, same bits.
GGP_DEV void posterior(double *m, double *C, const double x0, const double x1, const ggp_innov &v, const bool last)
{
    double K[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) K[i] = C[i];
    double KS0[4], KS1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        KS0[i] = K[i] * v.si00 + K[4 + i] * v.si10;
        KS1[i] = K[i] * v.si01 + K[4 + i] * v.si11;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = m[i] + (KS0[i] * x0 + KS1[i] * x1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) C[4 * i + j] = C[4 * i + j] - (KS0[i] * K[j] + KS1[i] * K[4 + j]);
    if (last) {   // wave-uniform (one cell per wave)
#pragma unroll
        for (int i = 1; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) C[4 * i + j] = C[4 * i + j] - (KS0[i] * K[j] + KS1[i] * K[4 + j]);
    }
}

// the outputs' variables V (ggp_outtab.h): lane 0 stores them, stage D reads them
GGP_DEV void store_v(const Step &S, double *V)
{
    const double v[V_N - 1] = {S.bx,  S.bg,  S.bl - S.ml, S.bq - S.mq, S.Cxx, S.Cxg, S.Cxl, S.Cxq,
                               S.Cgg, S.Cgl, S.Cgq,       S.Cll,       S.Clq, S.Cqq, S.t};
#pragma unroll
    for (int k = 0; k < V_N - 1; ++k) V[1 + k] = v[k];
}

}  // namespace wave
}  // namespace ggp
