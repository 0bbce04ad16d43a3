// ggp_wave.h -- per-lane task bodies of the WAVE schedule (k_loglik_wave, ggp_engine.hip):
// one 64-lane wave per cell; in every stage of a step each lane runs ONE task:
//
//   stage B   lane l: exponential kXW[l] (64 state-dependent exponentials), Dawson value l
//             (l < 14); lane 0 stores the tauint denominators and their reciprocals; then
//             lanes 0..3 form exp(c_B), exp(c_J), exp(c_G), exp(c_I) as exp(c_A) times a
//             cached exponential
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
    L_P = L_D + ND,           // tauint denominators 2 sqrt a, 4 a^1.5, 8 a^2.5, 16 a^3.5, then reciprocals
    L_BV = L_P + 8,           // outputs basis: 1, the 45 integrals, 18 exp-derived values
    L_V = L_BV + BV_N,        // outputs variables: 1, state, t
    L_OUT = L_V + V_N,        // the step's 14 outputs (block sums, written by the lead lanes)
    L_DUMMY = L_OUT + kOutN,  // one slot per lane for stores of lanes without a task
    kLds = L_DUMMY + 64
};

// ---- the step scalars every lane holds (wave-uniform values, formed from the state) ------
// Only what the lanes' tasks read: a = Cll/2 and its roots and reciprocals, b + bl, Cxl, and
// the two bases of the c values.  sqrt(a) is ocml's own iteration (bitwise its value for
// a >= 2^-767, where ocml does not rescale); its Goldschmidt half-reciprocal is the rdiv
// seed 1/(2 sqrt a), and its square the seed 1/(4a) (seeds only: rdiv's residual correction
// makes the quotient independent of an ulp in them).
struct WStep {
    double t, a, two_a, four_a, four_aa, two_sa, m2sa, r_two_sa, r_four_a, bbl, Cxl, bx, Cxx;
};

GGP_DEV WStep wstep(const double *m, const double *C, const double t, const double b)
{
    WStep S;
    S.t = t;
    const double a = C[10] / 2.;
    S.a = a;
#if defined(__HIP_DEVICE_COMPILE__)
    const double r = __builtin_amdgcn_rsq(a);
#else
    const double r = 1.0 / sqrt(a);
#endif
    double h = 0.5 * r, s = a * r;
    const double e = __builtin_fma(-h, s, 0.5);
    s = __builtin_fma(s, e, s);
    h = __builtin_fma(h, e, h);
    double d = __builtin_fma(-s, s, a);
    s = __builtin_fma(d, h, s);
    d = __builtin_fma(-s, s, a);
    s = __builtin_fma(d, h, s);
    s = (a == 0.0 || a == __builtin_huge_val()) ? a : s;   // ocml: sqrt(+-0, +inf) = the input
    S.two_sa = 2. * s;
    S.m2sa = -2. * s;
    S.r_two_sa = h;
    S.r_four_a = h * h;
    S.two_a = 2. * a;
    S.four_a = 4. * a;
    S.four_aa = 4 * (a * a);
    S.bbl = b + m[2];
    S.Cxl = C[2];
    S.bx = m[0];
    S.Cxx = C[0];
    return S;
}

// ---- one lane's tasks (registers for the whole launch) ---------------------------------
// Operands are formed from lane constants instead of select chains:
//   B  = fma(Cxl, km, b + bl) + gq ks   (km in {1, 2} makes the fma exact: step_init's B bitwise)
//   ti = t * tau                        (tau in {0, 1, 2}: 0, t, 2t exactly)
//   c  = fma(kc, t, fma(Cxx, m2, bx m1)) (m1, m2 = 1, 1/2 or 2, 2: the base bx + Cxx/2 or
//        2 (bx + Cxx) exactly; kc t folds step_init's -b t - gl t ... into one rounding)
struct LaneTasks {
    int x_dst, x_isE, x_isA;
    double x_tau, x_km, x_gqks, x_m1, x_m2, x_kc;
    int d_dst;
    double d_tau, d_km, d_gqks;
    int prod_dst, mult_off;
    ITask it;
    double i_tau0, i_tau1, i_km, i_gqks, i_s1;
    int i_dst;
    int out_dst;
};

// kc of c value ic (step_init's c0..c9 as base + kc t)
GGP_DEV double c_slope(const int ic, const OU &P)
{
    const double b = P.b, gl = P.gl, gq = P.gq;
    switch (ic) {
    case cA: return -b;
    case cB: return -b - gl;
    case cJ: return -b - gq;
    case cG: return -2 * b;
    case cC: return -2 * b;
    case cD: return -(2 * b + gq);
    case cE: return -2 * b;
    case cF: return -2 * b + gq;
    case cI: return -b - gq;
    default: return -2 * b - 2 * gq;   // cH
    }
}

GGP_DEV LaneTasks lane_tasks(const int lane, const OU &P)
{
    LaneTasks L;
    const int xj = kXW.j[lane];
    const XTask xt = kXT[xj];
    L.x_dst = L_X + xj;
    L.x_isE = xt.kind == KX_E;
    L.x_isA = xt.kind == KX_A;
    L.x_tau = (double)xt.it;
    const int xb = xt.iB < 6 ? xt.iB : 0;
    L.x_km = kKm[xb];
    L.x_gqks = P.gq * kKs[xb];
    const bool half = xt.ic == cA || xt.ic == cB || xt.ic == cJ || xt.ic == cG || xt.ic == cI;
    L.x_m1 = half ? 1.0 : 2.0;
    L.x_m2 = half ? 0.5 : 2.0;
    L.x_kc = c_slope(xt.ic, P);
    const DTask dk = kDT[lane < ND ? lane : 0];
    L.d_dst = lane < ND ? L_D + lane : L_DUMMY + lane;
    L.d_tau = (double)dk.it;
    L.d_km = kKm[dk.iB];
    L.d_gqks = P.gq * kKs[dk.iB];
    // exp(c_B) = exp(c_A) exp(-gl t), exp(c_J) = exp(c_I) = exp(c_A) exp(-gq t),
    // exp(c_G) = exp(c_A) / exp(b t)   (c_* of step_init)
    const int prod_slot = lane == 0 ? XC_B : lane == 1 ? XC_J : lane == 2 ? XC_G : XC_I;
    const int mult = lane == 0 ? L_X + XS_gl : lane == 2 ? L_BV + BV_R_EBT : L_X + XS_gq;
    L.prod_dst = lane < 4 ? L_X + prod_slot : L_DUMMY + lane;
    L.mult_off = lane < 4 ? mult : L_X + X_ONE;
    L.it = kIT[lane < NI ? lane : 0];
    L.i_s1 = L.it.k == 2 ? 1.0 : -1.0;
    L.i_tau0 = (double)L.it.it0;
    L.i_tau1 = (double)L.it.it1;
    L.i_km = kKm[L.it.iB];
    L.i_gqks = P.gq * kKs[L.it.iB];
    L.i_dst = lane < NI ? L_BV + BV_I + lane : L_DUMMY + lane;
    // the lead lane of output k's block stores the block sum
    int out = L_DUMMY + lane;
#pragma unroll
    for (int k = 0; k < kOutN; ++k) out = kOutLead[k] == lane ? L_OUT + k : out;
    L.out_dst = out;
    return L;
}

// The per-dt block (exp(s t) and the exp-derived basis of the outputs, formed when dt changes):
// its lane tasks are formed there from the lane number, not kept in registers for the launch
GGP_DEV int xs_dst_of(const int lane) { return lane < 6 ? L_X + XS_bt + lane : L_DUMMY + lane; }
GGP_DEV int dv_dst_of(const int lane) { return lane < kNDerived ? L_BV + BV_R_EBT + lane : L_DUMMY + lane; }
GGP_DEV DTaskB dv_of(const int lane) { return kDerived[lane < kNDerived ? lane : 0]; }

// the exponents s of exp(s t) (pickSV, ggp_prop.h)
GGP_DEV double sv_of(const OU &P, const int s)
{
    return s == 0 ? P.b : s == 1 ? P.b + P.gl : s == 2 ? 2 * P.b : s == 3 ? P.b + P.gq : s == 4 ? -P.gl : -P.gq;
}

GGP_DEV double bval(const WStep &S, const double km, const double gqks)
{
    return __builtin_fma(S.Cxl, km, S.bbl) + gqks;
}

// the argument of exponential task x (exp_body, ggp_prop.h): exp(c) is the Z form at ti = 0
// (a 0 + B 0 + c == c)
GGP_DEV double exp_arg(const WStep &S, const LaneTasks &T)
{
    const double ti = S.t * T.x_tau;
    const double B = pin(bval(S, T.x_km, T.x_gqks));
    const double c = pin(__builtin_fma(T.x_kc, S.t, __builtin_fma(S.Cxx, T.x_m2, S.bx * T.x_m1)));
    const double n = pin(rdiv(-(B * B), S.four_a, S.r_four_a));
    const double z = rdiv(B + S.two_a * ti, S.two_sa, S.r_two_sa);
    const double argA = pin(ti * (B + S.a * ti));
    const double argE = pin(n + c + z * z);
    const double argZ = pin(S.a * (ti * ti) + B * ti + c);
    return T.x_isE ? argE : T.x_isA ? argA : argZ;
}

// the argument of Dawson task d (zval, ggp_prop.h; ti = 0: B + 0 == B)
GGP_DEV double dawson_arg(const WStep &S, const LaneTasks &T)
{
    const double B = bval(S, T.d_km, T.d_gqks);
    return rdiv(B + S.two_a * (S.t * T.d_tau), S.two_sa, S.r_two_sa);
}

// exp_ocml: ggp_prop.h (shared with the lane schedule)

// ggp_dawson_tab without branches: one division for the continued fraction, a NaN falls
// through the polynomial (same values as ggp_dawson_tab).  tab: rows of kDawsonRow doubles
// (the 9 coefficients, zero-padded to 10), 16-B aligned: five 128-bit LDS reads per value;
// Horner with fused multiply-adds (<= 1 ulp from the separate-rounding form; the device
// Dawson stays within the reference's bound, tests/test_gpu_device_math.py)
constexpr int kDawsonRow = 10;
#ifndef GGP_HOST_SIM
GGP_DEV double dawson_bf(const double x, const double *tab)
{
    const double ax = fabs(x);
    const double d1 = 1.0 + ax;
    const double y100 = rdiv(100.0, d1, frcp(d1));   // IEEE 100 / (1 + ax) for finite ax
#if defined(__HIP_DEVICE_COMPILE__)
    int kt;   // v_cvt_i32_f64: NaN -> 0 (then t and the value are NaN), no guard needed
    asm("v_cvt_i32_f64 %0, %1" : "=v"(kt) : "v"(y100));
    const int k = min(kt, GGP_DAWSON_NINT - 1);
    const double2 *c2 = reinterpret_cast<const double2 *>(tab + __mul24(k, kDawsonRow));
#else
    const int k = min((int)(y100 >= 0.0 ? y100 : 0.0), GGP_DAWSON_NINT - 1);
    const double2 *c2 = reinterpret_cast<const double2 *>(tab + kDawsonRow * k);
#endif
    const double2 a01 = c2[0], a23 = c2[1], a45 = c2[2], a67 = c2[3], a89 = c2[4];
    const double t = 2.0 * y100 - (double)(2 * k + 1);
    double h = __builtin_fma(a89.x, t, a67.y);
    h = __builtin_fma(h, t, a67.x);
    h = __builtin_fma(h, t, a45.y);
    h = __builtin_fma(h, t, a45.x);
    h = __builtin_fma(h, t, a23.y);
    h = __builtin_fma(h, t, a23.x);
    h = __builtin_fma(h, t, a01.y);
    double w = pin(__builtin_fma(h, t, a01.x));
    // the Taylor and continued-fraction branches are rare (|x| < ~0.03, |x| > 45; exclusive):
    // formed, and selected, only when some lane of the wave needs them (a wave-uniform branch;
    // NaN takes neither)
    const bool use_taylor = y100 >= (double)GGP_DAWSON_NINT, use_cf = ax > 45.0;
    if (__builtin_amdgcn_ballot_w64(use_taylor)) {
        const double x2 = ax * ax;
        const double *tc = ggp_dawson_taylor;
        const double taylor = pin(ax * (tc[0] - x2 * (tc[1] - x2 * (tc[2] - x2 * (tc[3] - x2 * tc[4])))));
        w = use_taylor ? taylor : w;
    }
    if (__builtin_amdgcn_ballot_w64(use_cf)) {
        const bool far = ax > 5e7;
        const double num = far ? GGP_ISPI : pin(GGP_ISPI * ((ax * ax) * (ax * ax - 4.5) + 2));
        const double den = far ? ax : pin(ax * ((ax * ax) * (ax * ax - 5) + 3.75));
        const double cf = pin(num / den);
        w = use_cf ? cf : w;
    }
    return GGP_SPI2 * (x < 0.0 ? -w : w);
}

#endif  // GGP_HOST_SIM

// The tauint denominators of k = 0..3 (2 sqrt a, then pow_task's 4 a^1.5, 8 a^2.5, 16 a^3.5)
// and their rdiv seeds (r_two_sa, then 1/(4 a^1.5) = 2 r4a r2sa and each next power one factor
// 2 r4a = 1/(2a) more: seeds only, rdiv's residual correction makes the quotient independent of
// a few ulp in them).  Uniform values: lane 0 stores them (no per-lane select).
GGP_DEV void store_pw(const WStep &S, double *PW)
{
    const double sa = S.two_sa * 0.5, a = S.a;   // sqrt(a) exactly
    const double r0 = 2. * (S.r_four_a * S.r_two_sa);
    const double r1 = 2. * (S.r_four_a * r0);
    const double r2 = 2. * (S.r_four_a * r1);
    PW[0] = S.two_sa;
    PW[1] = 4. * (a * sa);
    PW[2] = 8. * ((a * a) * sa);
    PW[3] = 16. * (((a * a) * a) * sa);
    PW[4] = S.r_two_sa;
    PW[5] = r0;
    PW[6] = r1;
    PW[7] = r2;
}

// tau_unified without branches (X, Dw, PW: the LDS arrays)
GGP_DEV double tau_bf(const WStep &S, const LaneTasks &L, const double *X, const double *Dw, const double *PW)
{
    const ITask T = L.it;
    const double D0 = Dw[T.d0], D1 = Dw[T.d1];
    const double E0 = X[T.x0], E1 = X[T.x1];
    const double ec = X[T.xc], ea0 = X[T.xa0], ea1 = X[T.xa1];
    const int k = T.k;
    const double den = PW[k], rden = PW[4 + k];
    const double B = pin(bval(S, L.i_km, L.i_gqks));
    const double t0 = S.t * L.i_tau0, t1 = S.t * L.i_tau1;
    const double BB = pin(B * B);
    const double al3 = pin(BB - 2. * S.two_a);
    const double al = k == 1 ? 1.0 : k == 2 ? B : al3;
    const double be2 = pin(-S.two_a), be3 = pin(-S.two_a * B);
    const double be = k == 1 ? 0.0 : k == 2 ? be2 : be3;
    const double ga = k == 3 ? S.four_aa : 0.0;
    const double P0 = al + t0 * (be + ga * t0), P1 = al + t1 * (be + ga * t1);
    const double q1 = pin(B * 2.), q2 = pin((S.two_a - BB) * 2.), q3 = pin(B * (-6. * S.a + BB) * 2.);
    const double Q = k == 0 ? -2.0 : k == 1 ? q1 : k == 2 ? q2 : q3;
    const double S1 = S.two_sa * L.i_s1;   // 2 sqrt a (k = 2) or -2 sqrt a
    const double dterm = pin(Q * (E0 * D0 - E1 * D1));
    const double xfull = pin(S1 * ec * (ea0 * P0 - ea1 * P1) + dterm);
    const double x = k == 0 ? dterm : xfull;
    return rdiv(x, den, rden);
}

// The measurement step of the wave schedule (ggp_innovation + ggp_posterior, likelihood.h:53-69,
// predictions.h:84-89) with fused multiply-adds in the gain and the update: C_ij - (a + b)
// keeps the reference's association (a + b by one fma), so the posterior agrees with the
// lane schedule's to the last bits of each entry (the wave schedule is not bitwise equal to
// it anyway, DESIGN.md "Parity").  S10 == S01 here (out_store writes C[4] = C[1]), so
// si10 == si01.  The lower triangle of C is formed only on the cell's last row: on every
// other row the next propagation reads the upper triangle and overwrites all of C.
struct WInnov {
    double S00, S01, S11, si00, si01, si11;
};

GGP_DEV WInnov innovation(const double *m, const double *C, const double var_x, const double var_g, const int scaled,
                          const double fp_auto)
{
    WInnov v;
    const double d11 = scaled ? var_g * (m[1] + fp_auto) : var_g;
    v.S00 = C[0] + var_x;
    v.S01 = C[1] + 0.0;
    v.S11 = C[5] + d11;
    const double det = v.S00 * v.S11 - v.S01 * v.S01;   // Eigen fixed 2x2 determinant (S10 == S01)
    const double invdet = 1.0 / det;
    v.si00 = v.S11 * invdet;
    v.si01 = -v.S01 * invdet;
    v.si11 = v.S00 * invdet;
    return v;
}

GGP_DEV void posterior(double *m, double *C, const double x0, const double x1, const WInnov &v, const bool last)
{
    double K[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) K[i] = C[i];
    double KS0[4], KS1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        KS0[i] = __builtin_fma(K[4 + i], v.si01, K[i] * v.si00);
        KS1[i] = __builtin_fma(K[4 + i], v.si11, K[i] * v.si01);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = m[i] + __builtin_fma(KS1[i], x1, KS0[i] * x0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) C[4 * i + j] = C[4 * i + j] - __builtin_fma(KS1[i], K[4 + j], KS0[i] * K[j]);
    if (last) {   // wave-uniform (one cell per wave)
#pragma unroll
        for (int i = 1; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) C[4 * i + j] = C[4 * i + j] - __builtin_fma(KS1[i], K[4 + j], KS0[i] * K[j]);
    }
}

// the ll term's quadratic form (ggp_ll_term's q, likelihood.h:26-32) from the ring's row values
GGP_DEV double ll_quad(const double x0, const double x1, const double S00, const double S01, const double S11)
{
    const double det = S00 * S11 - S01 * S01;
    const double invdet = 1.0 / det;
    const double si00 = S11 * invdet, si01 = -S01 * invdet, si11 = S00 * invdet;
    const double h0 = -0.5 * x0, h1 = -0.5 * x1;
    return (h0 * si00 + h1 * si01) * x0 + (h0 * si01 + h1 * si11) * x1;
}

// the outputs' variables V (ggp_outtab.h): lane 0 stores them, stage D reads them
GGP_DEV void store_v(const double *m, const double *C, const double t, const OU &P, double *V)
{
    const double v[V_N - 1] = {m[0], m[1], m[2] - P.ml, m[3] - P.mq, C[0], C[1], C[2], C[3],
                               C[5], C[6], C[7], C[10], C[11], C[15], t};
#pragma unroll
    for (int k = 0; k < V_N - 1; ++k) V[1 + k] = v[k];
}

}  // namespace wave
}  // namespace ggp
