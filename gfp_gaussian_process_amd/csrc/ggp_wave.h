// ggp_wave.h -- task tables and per-lane bodies of the WAVE schedule (k_loglik_wave,
// ggp_engine.hip): one 64-lane wave per cell, every stage of a step one task per lane.
//
// A step (one row, likelihood.h:53-102 with mean_cov_model.h:211-274 in between) is five
// stages separated by LDS hand-offs inside the wave:
//
//   B   lanes 0-45: one of the 46 exponentials that depend on the state (the other 28 of the
//       step's 74 are exp(s t) cached per dt, or products exp(c) * exp(k t) of a computed one
//       and a cached one: argument O(1), no cancellation, <= 2 ulp); lanes 46-59: one of the
//       14 Dawson values.  Both kinds run ONE instruction stream: a reduction (exp: rint,
//       two fma; Dawson: y = 100 / (1 + |x|), interval, Chebyshev variable), then one 11-step
//       Horner over a 12-coefficient LDS row (the exp row holds ocml's constants, a Dawson row
//       its interval's polynomial with three leading zeros: bitwise the same Horner), then
//       ldexp / sign.  The rare branches (exp beyond 2^50, Dawson Taylor / continued fraction)
//       only when a lane needs them (one ballot).
//   C   lanes 0-44: one of the 45 tauint integrals; the four kinds (k = 0..3) in one stream, the
//       per-kind operands formed by fused multiply-adds with 0/1 lane constants (no selects);
//       the product exponentials multiplied in as they are read.
//   D   the outputs' sparse trilinear form (ggp_outtab.h): 4 terms per lane over 60 state
//       monomials formed once per step (one per lane), a DPP butterfly per output block.
//   F   finish: lane e forms state entry e of the propagated prior (the covariances' sum -
//       nm_i nm_j), and lanes 20 and 24 -x0 = m0 - y_l, -x1 = m1 - y_f.
//   U   update (ggp_innovation + ggp_posterior): the 2x2 innovation in every lane (uniform),
//       then lane e forms posterior entry e (4 means, 16 covariances) from five LDS reads:
//       the 20-double state is DISTRIBUTED over the lanes, never held whole in registers.
//
// The first step of a cell (no propagation for a root's first row, the division map for a
// daughter's) runs the update uniformly in every lane (ggp_wave.h innovation / posterior,
// the same expressions) and scatters the state to the lanes.
//
// Everything here compiles for the host too (GGP_HOST_SIM: tools/hostsim.cpp emulates the
// 64 lanes stage by stage to measure the numerics against the oracle).
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

// the B values as ((b + bl) + Cxl km) + gq ks (step_init's B0..B5, same rounding)
constexpr double kKm[6] = {1., 1., 2., 2., 1., 2.};
constexpr double kKs[6] = {0., -1., 0., -1., 1., 1.};

// ---- the step scalars every lane holds, and the measurement step -------------------------------
// ---- the step scalars every lane holds (wave-uniform values, formed from the state) ------
// Only what the lanes' tasks read: a = Cll/2 and its roots and reciprocals, b + bl, Cxl, and
// the two bases of the c values.  sqrt(a) is ocml's own iteration (bitwise its value for
// a >= 2^-767, where ocml does not rescale); its Goldschmidt half-reciprocal is the rdiv
// seed 1/(2 sqrt a), and its square the seed 1/(4a) (seeds only: rdiv's residual correction
// makes the quotient independent of an ulp in them).
struct WStep {
    double t, a, two_a, four_a, four_aa, two_sa, m2sa, r_two_sa, r_four_a, bbl, Cxl, bx, Cxx;
    double r_two_sa0;   // the unrefined seed 0.5 rsq(a) of r_two_sa (stage B's table row only)
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
    S.r_two_sa0 = h;
    const double e = __builtin_fma(-h, s, 0.5);
    s = __builtin_fma(s, e, s);
    h = __builtin_fma(h, e, h);
    // one residual correction (ocml takes two: its result can differ in the last bit, which moves
    // the step's values by an ulp -- the wave schedule is not bitwise the lane schedule anyway)
    const double d = __builtin_fma(-s, s, a);
    s = __builtin_fma(d, h, s);
    // (ocml's sqrt returns a itself for a = 0 and +inf; here a step with such an a gives NaN either
    // way: the Dawson argument B / (2 sqrt a) and the integrals divide by sqrt a)
    S.two_sa = 2. * s;
    S.m2sa = -2. * s;
    S.r_two_sa = h;
    S.r_four_a = h * h;
    S.two_a = 2. * a;
    S.four_a = 4. * a;
    S.four_aa = S.two_a * S.two_a;   // 4 (a a): scaling by 4 is exact, one multiply
    S.bbl = b + m[2];
    S.Cxl = C[2];
    S.bx = m[0];
    S.Cxx = C[0];
    return S;
}

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

// the exponents s of exp(s t) (pickSV, ggp_prop.h)
GGP_DEV double sv_of(const OU &P, const int s)
{
    return s == 0 ? P.b : s == 1 ? P.b + P.gl : s == 2 ? 2 * P.b : s == 3 ? P.b + P.gq : s == 4 ? -P.gl : -P.gq;
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


// ---- exponentials: computed in stage B, cached per dt, or products ----------------------
// factor kinds of a product exponential X[j] = X[rep] * factor
enum { F_ONE = 0, F_EGL, F_EGQ, F_REBT, F_EPGQ };
struct XMap {
    unsigned char rep, fac;
};
// c_B = c_A - gl t, c_J = c_I = c_A - gq t, c_G = c_A - b t (half base); c_E = c_C,
// c_D = c_C - gq t, c_F = c_C + gq t (double base): exp(c + ...) = exp(c_rep + ...) exp(+-k t)
constexpr XMap xmap(const int j)
{
    switch (j) {
    case XC_B: return {XC_A, F_EGL};
    case XC_J: return {XC_A, F_EGQ};
    case XC_G: return {XC_A, F_REBT};
    case XC_I: return {XC_A, F_EGQ};
    case XC_D: return {XC_C, F_EGQ};
    case XC_E: return {XC_C, F_ONE};
    case XC_F: return {XC_C, F_EPGQ};
    case XZ_1Bt: return {XZ_1At, F_EGL};
    case XZ_1Jt: return {XZ_1At, F_EGQ};
    case XZ_1Gt: return {XZ_1At, F_REBT};
    case XZ_2Bt: return {XZ_2At, F_EGL};
    case XZ_2Jt: return {XZ_2At, F_EGQ};
    case XZ_2It: return {XZ_2At, F_EGQ};
    case XZ_2Gt: return {XZ_2At, F_REBT};
    case XZ_3Et: return {XZ_3Ct, F_ONE};
    case XZ_3Dt: return {XZ_3Ct, F_EGQ};
    case XZ_4Et: return {XZ_4Ct, F_ONE};
    case XZ_4Ft: return {XZ_4Ct, F_EPGQ};
    case XZ_3E2: return {XZ_3C2, F_ONE};
    case XZ_3D2: return {XZ_3C2, F_EGQ};
    case XZ_4E2: return {XZ_4C2, F_ONE};
    case XZ_4F2: return {XZ_4C2, F_EPGQ};
    default: return {(unsigned char)j, F_ONE};
    }
}
constexpr bool x_computed(const int j)
{
    return j < NXT && !(j >= XS_bt && j <= XS_gq) && xmap(j).rep == j;
}

constexpr int kNExp = 46, kNDaw = ND, kLaneD0 = kNExp;   // lanes 46..59: Dawson values
struct XList {
    unsigned char j[kNExp];
    int n;
};
constexpr XList make_xlist()
{
    XList L{};
    for (int j = 0; j < NXT; ++j)
        if (x_computed(j)) L.j[L.n++] = (unsigned char)j;
    return L;
}
constexpr XList kXL = make_xlist();
static_assert(kXL.n == kNExp, "46 state-dependent exponentials are computed per step");
static_assert(kNExp + kNDaw <= 64, "stage B: one task per lane");

// ---- the outputs' state monomials (stage D): V[v1] V[v2] V[v3] of every term, deduplicated --
struct MonoList {
    unsigned char v[64][3];
    unsigned char term[64][kOutL];   // monomial index of lane l's term q
    int n;
};
constexpr MonoList make_monos()
{
    MonoList M{};
    for (int l = 0; l < 64; ++l)
        for (int q = 0; q < kOutL; ++q) {
            const OutTerm T = kOutTerm[l][q];
            int f = -1;
            for (int i = 0; i < M.n; ++i)
                if (M.v[i][0] == T.v1 && M.v[i][1] == T.v2 && M.v[i][2] == T.v3) f = i;
            if (f < 0) {
                f = M.n++;
                M.v[f][0] = T.v1;
                M.v[f][1] = T.v2;
                M.v[f][2] = T.v3;
            }
            M.term[l][q] = (unsigned char)f;
        }
    return M;
}
constexpr MonoList kMono = make_monos();
static_assert(kMono.n <= 64, "one monomial per lane");

// ---- LDS layout (doubles, one array) --------------------------------------------------
constexpr int kTabRow = 12;                       // Horner coefficients per row (exp row: ocml's)
constexpr int kTabRows = GGP_DAWSON_NINT + 1;     // Dawson rows 0..96, then the exp row
constexpr int kExpRow = GGP_DAWSON_NINT;
enum {
    L_TAB = 0,                                    // 16-B aligned rows
    L_X = L_TAB + kTabRows * kTabRow,             // exponentials (NX slots: X_ONE = 1), then exp(+gq t)
    L_XPGQ = L_X + NX,
    L_D = L_XPGQ + 1,                             // Dawson values
    L_BV = L_D + ND,                              // outputs basis: 1, the 45 integrals, 18 exp-derived
    L_V = L_BV + BV_N,                            // outputs variables: 1, state, t
    L_MONO = L_V + V_N,                           // the step's state monomials
    L_OUT = L_MONO + 64,                          // the 14 raw outputs (block sums)
    L_ZERO = L_OUT + kOutN,                       // 0.0 and 1.0 for the finish fma
    L_ONE1 = L_ZERO + 1,
    L_ST = L_ONE1 + 1,                            // prior: m[4], C[16], -x0 at 20, -x1 at 24
    L_POST = L_ST + 28,                           // posterior: m[4], C[16]
    L_RX0 = L_POST + 20,                          // ll ring: prior m0, m1, S00, S01, S11 per row
    L_RX1 = L_RX0 + 64,
    L_RS0 = L_RX1 + 64,
    L_RS1 = L_RS0 + 64,
    L_RS2 = L_RS1 + 64,
    L_RT = L_RS2 + 64,                            // ll terms of the chunk
    L_ROWL = L_RT + 64,                           // this 64-row chunk's data (+ next time)
    L_ROWF = L_ROWL + 64,
    L_ROWT = L_ROWF + 64,
    L_DUMMY = L_ROWT + 66,                        // one slot per lane for stores without a task
    L_RED = L_DUMMY + 64,                         // the in-launch reduction's prefetched tables
    L_DTK = L_RED + 68,                           // the dt cache: kDtWays keys (dt's bits), then
    L_DTC = L_DTK + 8,                            // per way the kDtVals values that depend on dt only
    kLds = L_DTC + 8 * 25
};
// the dt cache: the values a step reads that depend on the parameters and dt only (the six
// exp(s t), exp(+gq t) and the 18 exp-derived basis values), kept for the last kDtWays distinct
// dt of the block (a cell's times are floats: the example's dt = 1 comes in 13 bit patterns,
// alternating, so one entry missed 36% of its steps)
constexpr int kDtWays = 8, kDtVals = 7 + kNDerived;
static_assert(kDtVals == 25, "the cache way layout holds 25 values");
// the working slot of cached value v (lane v copies it)
constexpr int dt_slot(const int v) { return v < 6 ? L_X + XS_bt + v : v == 6 ? L_XPGQ : L_BV + BV_R_EBT + (v - 7); }
static_assert(L_X % 2 == 0 && L_TAB == 0, "128-bit table rows");
static_assert(L_RT % 2 == 0, "128-bit ll-term reads");

// the exp row: ocml's exp polynomial (ggp_prop.h exp_ocml), Horner from the top, the two
// trailing fma(t, p, 1.0) steps as coefficients 1.0
constexpr double kExpCoef[kTabRow] = {0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22, 0x1.71dee623fde64p-19,
                                      0x1.a01997c89e6b0p-16, 0x1.a01a014761f6ep-13, 0x1.6c16c1852b7b0p-10,
                                      0x1.1111111122322p-7,  0x1.55555555502a1p-5,  0x1.5555555555511p-3,
                                      0x1.000000000000bp-1,  1.0,                   1.0};
// table entry k of the LDS copy: Dawson row r = [0, 0, 0, c8 .. c0] (three leading zeros keep
// the 8-step Horner bitwise: fma(0, t, 0) = 0, fma(0, t, c8) = c8), then the exp row
GGP_DEV double tab_entry(const int k)
{
    const int r = k / kTabRow, i = k % kTabRow;
    if (r == kExpRow) return kExpCoef[i];
    return i < 3 ? 0.0 : ggp_dawson_coef[GGP_DAWSON_NCOEF * r + (kTabRow - 1 - i)];
}

#if !defined(GGP_HOST_SIM)
// The LDS image of the table (tab_entry for k = 0 .. kTabRows * kTabRow - 1), laid out in global
// memory exactly as the launch copies it: each lane moves contiguous 16-byte pieces (10 coalesced
// loads per lane instead of 19 gathers through tab_entry's row / column arithmetic).  The
// coefficients come from a constexpr copy of the same dawson_table.inc.
namespace cx {
#pragma push_macro("GGP_DAWSON_TABLE_QUALIFIER")
#undef GGP_DAWSON_TABLE_QUALIFIER
#define GGP_DAWSON_TABLE_QUALIFIER constexpr
#include "dawson_table.inc"
#pragma pop_macro("GGP_DAWSON_TABLE_QUALIFIER")
}  // namespace cx
struct TabImg {
    double v[kTabRows * kTabRow];
};
constexpr TabImg make_tab_img()
{
    TabImg T{};
    for (int k = 0; k < kTabRows * kTabRow; ++k) {
        const int r = k / kTabRow, i = k % kTabRow;
        T.v[k] = r == kExpRow ? kExpCoef[i] : i < 3 ? 0.0 : cx::ggp_dawson_coef[GGP_DAWSON_NCOEF * r + (kTabRow - 1 - i)];
    }
    return T;
}
static_assert((kTabRows * kTabRow) % 2 == 0, "the image moves in 16-byte pieces");
__constant__ __attribute__((aligned(16))) const TabImg kTabImg = make_tab_img();
#endif

// ---- lane constants -------------------------------------------------------------------------
// LaneC: everything that does not depend on the parameters, a compile-time table (kLaneTab, one
// row per lane, loaded once per launch); Lane: the registers the step reads, completed from
// the row and the parameters (lane_from).  Slots are indices into the one LDS array.
struct LaneC {
    // stage B: argument forms (ggp_wave.h exp_arg); Dawson lanes use z only.  The c slope is
    // kb b + kgl gl + kgq gq (c_slope's value: the integer coefficients are exact)
    double b_tau, b_km, b_ks, b_m1, b_m2, b_kb, b_kgl, b_kgq, b_mult, b_zc;
    int b_isE, b_isA, b_isD, b_exmask, b_sgn, b_dst;
    // stage C: the integral (tau_unified) with 0/1 selectors
    double i_tau0, i_tau1, i_km, i_ks, i_u0, i_u1, i_u2, i_w2, i_w3, i_g, i_s0, i_s1, i_s2, i_s3, i_S1;
    int i_d0, i_d1, i_e0r, i_e0f, i_e1r, i_e1f, i_ecr, i_ecf, i_a0, i_a1, i_dst;
    // stage D: monomial task, terms (kappa index; 255 = padding)
    int mo_v0, mo_v1, mo_v2, mo_dst;
    int d_mono[kOutL], d_basis[kOutL], d_kap[kOutL];
    int d_bs, d_out;
    // finish / update (vshift = fml ml + fmq mq)
    int f_src, f_na, f_nb, f_row, f_dst;
    int u_ub, u_wb, u_c, u_post, u_v;
    double u_fml, u_fmq;
};

struct Lane {
    double b_tau, b_km, b_gqks, b_m1, b_m2, b_kc, b_mult, b_zc;
    int b_isE, b_isA, b_isD, b_exmask, b_sgn, b_dst;
    double i_tau0, i_tau1, i_km, i_gqks, i_u0, i_u1, i_u2, i_w2, i_w3, i_g, i_s0, i_s1, i_s2, i_s3, i_S1;
    int i_d0, i_d1, i_e0r, i_e0f, i_e1r, i_e1f, i_ecr, i_ecf, i_a0, i_a1, i_dst;
    int mo_v0, mo_v1, mo_v2, mo_dst;
    int d_mono[kOutL], d_basis[kOutL];
    double d_kap[kOutL];
    int d_bs, d_out;
    int f_src, f_na, f_nb, f_row, f_dst;
    int u_ub, u_wb, u_c, u_post, u_v;
    double u_vshift;
    double c_sv;   // the per-dt block: exp(c_sv t) for lanes 0-6 (exp(s t) of pickSV, then exp(+gq t))
};

// c_slope (ggp_wave.h) as integer coefficients of (b, gl, gq)
constexpr void c_coef(const int ic, double &kb, double &kgl, double &kgq)
{
    kb = (ic == cA || ic == cB || ic == cJ || ic == cI) ? -1.0 : -2.0;
    kgl = ic == cB ? -1.0 : 0.0;
    kgq = (ic == cJ || ic == cI || ic == cD) ? -1.0 : ic == cF ? 1.0 : ic == cH ? -2.0 : 0.0;
}

constexpr int fac_slot(const int f)
{
    return f == F_EGL ? L_X + XS_gl : f == F_EGQ ? L_X + XS_gq : f == F_REBT ? L_BV + BV_R_EBT : f == F_EPGQ ? L_XPGQ : L_X + X_ONE;
}

constexpr LaneC make_lane_c(const int lane)
{
    LaneC L{};
    // ---- stage B
    {
        const bool isD = lane >= kLaneD0 && lane < kLaneD0 + kNDaw;
        const bool isX = lane < kNExp;
        const int xj = kXL.j[isX ? lane : 0];
        const XTask xt = kXT[xj];
        if (isD) {
            const DTask dk = kDT[lane - kLaneD0];
            L.b_tau = (double)dk.it;
            L.b_km = wave::kKm[dk.iB];
            L.b_ks = wave::kKs[dk.iB];
            L.b_m1 = 1.0;
            L.b_m2 = 0.5;
            L.b_isD = 1;
            L.b_exmask = 0;
            L.b_mult = GGP_SPI2;
            L.b_sgn = (int)0x80000000u;   // z's sign onto the value (Dawson is odd)
            L.b_dst = L_D + (lane - kLaneD0);
        } else {
            const int xb = xt.iB < 6 ? xt.iB : 0;
            L.b_tau = (double)xt.it;
            L.b_km = wave::kKm[xb];
            L.b_ks = wave::kKs[xb];
            const bool half = xt.ic == cA || xt.ic == cB || xt.ic == cJ || xt.ic == cG || xt.ic == cI;
            L.b_m1 = half ? 1.0 : 2.0;
            L.b_m2 = half ? 0.5 : 2.0;
            c_coef(xt.ic, L.b_kb, L.b_kgl, L.b_kgq);
            L.b_isE = xt.kind == KX_E;
            L.b_isA = xt.kind == KX_A;
            // c enters the Z kind's argument (and the C kind's: t = 0 there), not the A kind's
            L.b_zc = xt.kind == KX_A ? 0.0 : 1.0;
            L.b_exmask = -1;
            L.b_mult = 1.0;
            L.b_sgn = 0;
            L.b_dst = isX ? L_X + xj : L_DUMMY + lane;
        }
    }
    // ---- stage C
    {
        const bool has = lane < NI;
        const ITask T = kIT[has ? lane : 0];
        L.i_tau0 = (double)T.it0;
        L.i_tau1 = (double)T.it1;
        L.i_km = wave::kKm[T.iB];
        L.i_ks = wave::kKs[T.iB];
        const int k = T.k;
        L.i_u0 = k == 1 ? 1.0 : 0.0;
        L.i_u1 = k == 2 ? 1.0 : 0.0;
        L.i_u2 = k == 3 ? 1.0 : 0.0;
        L.i_w2 = k == 2 ? 1.0 : 0.0;
        L.i_w3 = k == 3 ? 1.0 : 0.0;
        L.i_g = k == 3 ? 1.0 : 0.0;
        L.i_s0 = k == 0 ? -2.0 : 0.0;
        L.i_s1 = k == 1 ? 1.0 : 0.0;
        L.i_s2 = k == 2 ? 1.0 : 0.0;
        L.i_s3 = k == 3 ? 1.0 : 0.0;
        L.i_S1 = k == 0 ? 0.0 : k == 2 ? 1.0 : -1.0;
        L.i_d0 = L_D + T.d0;
        L.i_d1 = L_D + T.d1;
        L.i_e0r = L_X + xmap(T.x0).rep;
        L.i_e0f = fac_slot(xmap(T.x0).fac);
        L.i_e1r = L_X + xmap(T.x1).rep;
        L.i_e1f = fac_slot(xmap(T.x1).fac);
        L.i_ecr = L_X + xmap(T.xc).rep;
        L.i_ecf = fac_slot(xmap(T.xc).fac);
        L.i_a0 = L_X + T.xa0;
        L.i_a1 = L_X + T.xa1;
        L.i_dst = has ? L_BV + BV_I + lane : L_DUMMY + lane;
    }
    // ---- stage D
    {
        const bool mo = lane < kMono.n;
        L.mo_v0 = L_V + kMono.v[mo ? lane : 0][0];
        L.mo_v1 = L_V + kMono.v[mo ? lane : 0][1];
        L.mo_v2 = L_V + kMono.v[mo ? lane : 0][2];
        L.mo_dst = mo ? L_MONO + lane : L_DUMMY + lane;
        for (int q = 0; q < kOutL; ++q) {
            const OutTerm T = kOutTerm[lane][q];
            L.d_mono[q] = L_MONO + kMono.term[lane][q];
            L.d_basis[q] = L_BV + T.basis;
            L.d_kap[q] = T.kap;
        }
        L.d_bs = kOutBlock[lane];
        int out = L_DUMMY + lane;
        for (int k = 0; k < kOutN; ++k) out = kOutLead[k] == lane ? L_OUT + k : out;
        L.d_out = out;
    }
    // ---- finish (lane e: prior entry e) and update (posterior entry e)
    {
        // output index of each C entry (out_store)
        constexpr int kCo[16] = {4, 5, 6, 7, 5, 8, 9, 10, 6, 9, 11, 12, 7, 10, 12, 13};
        const int e = lane;
        L.f_row = 0;
        if (e < 4) {
            L.f_src = L_OUT + e;
            L.f_na = L_ZERO;
            L.f_nb = L_ZERO;
            L.f_dst = L_ST + e;
        } else if (e < 20) {
            const int o = kCo[e - 4];
            L.f_src = L_OUT + o;
            L.f_na = kOutNm[o][0] >= 0 ? L_OUT + kOutNm[o][0] : L_ZERO;
            L.f_nb = kOutNm[o][0] >= 0 ? L_OUT + kOutNm[o][1] : L_ZERO;
            L.f_dst = L_ST + e;
        } else if (e == 20 || e == 24) {   // -x0 = m0 - y_l, -x1 = m1 - y_f (the row slot added per step)
            L.f_src = L_OUT + (e == 20 ? 0 : 1);
            L.f_na = L_ONE1;
            L.f_nb = e == 20 ? L_ROWL : L_ROWF;
            L.f_row = 1;
            L.f_dst = L_ST + e;
        } else {
            L.f_src = L_ZERO;
            L.f_na = L_ZERO;
            L.f_nb = L_ZERO;
            L.f_dst = L_DUMMY + lane;
        }
        // posterior entry e: c - fma(KS1[i], z, KS0[i] * w), KS from u = C[0][i], v = C[1][i]
        // (u, v at ST[4 + i], ST[8 + i]); w, z = C[0][j], C[1][j] for a covariance, -x0, -x1 for a mean
        if (e < 20) {
            const int i = e < 4 ? e : (e - 4) / 4, j = e < 4 ? -1 : (e - 4) % 4;
            L.u_ub = L_ST + 4 + i;
            L.u_wb = j < 0 ? L_ST + 20 : L_ST + 4 + j;
            L.u_c = L_ST + e;
            L.u_post = L_POST + e;
            // stage D's variables: the means (bl - ml, bq - mq) and the upper triangle
            constexpr int kCv[16] = {V_CXX, V_CXG, V_CXL, V_CXQ, -1, V_CGG, V_CGL, V_CGQ, -1, -1, V_CLL, V_CLQ, -1, -1, -1, V_CQQ};
            const int vs = e < 4 ? V_BX + e : kCv[e - 4];
            L.u_v = vs >= 0 ? L_V + vs : L_DUMMY + lane;
            L.u_fml = e == 2 ? 1.0 : 0.0;
            L.u_fmq = e == 3 ? 1.0 : 0.0;
        } else {
            L.u_ub = L_ST + 4;
            L.u_wb = L_ST + 4;
            L.u_c = L_ST;
            L.u_post = L_DUMMY + lane;
            L.u_v = L_DUMMY + lane;
        }
    }
    return L;
}

struct LaneTab {
    LaneC l[64];
};
constexpr LaneTab make_lane_tab()
{
    LaneTab T{};
    for (int l = 0; l < 64; ++l) T.l[l] = make_lane_c(l);
    return T;
}
constexpr LaneTab kLaneTab = make_lane_tab();

// The table's row in packed form: every LaneC double is a small multiple of 1/2 (stored doubled,
// in a signed byte) or, for b_mult, one of two constants (a flag); every slot an LDS index below
// 2^15 (a short).  100 bytes per lane instead of 400: each block's setup reads 6.4 KB of lane
// constants instead of 25.6 KB (the launch timeline's "table" phase).
// unpack_lane(pack_lane(row)) == row for every lane (static_assert below), so the registers the
// step reads are bitwise the unpacked table's.
enum { LP_ISE = 1, LP_ISA = 2, LP_ISD = 4, LP_EXMASK = 8, LP_SGN = 16, LP_FROW = 32 };
struct LaneP {
    signed char b_tau, b_km, b_ks, b_m1, b_m2, b_kb, b_kgl, b_kgq, b_zc;
    signed char i_tau0, i_tau1, i_km, i_ks, i_u0, i_u1, i_u2, i_w2, i_w3, i_g, i_s0, i_s1, i_s2, i_s3, i_S1;
    signed char u_fml, u_fmq;
    unsigned char flags, d_bs;
    unsigned char d_kap[kOutL];
    short b_dst, i_d0, i_d1, i_e0r, i_e0f, i_e1r, i_e1f, i_ecr, i_ecf, i_a0, i_a1, i_dst;
    short mo_v0, mo_v1, mo_v2, mo_dst;
    short d_mono[kOutL], d_basis[kOutL];
    short d_out, f_src, f_na, f_nb, f_dst, u_ub, u_wb, u_c, u_post, u_v;
};
constexpr signed char half2(const double v) { return (signed char)(int)(2.0 * v); }
constexpr LaneP pack_lane(const LaneC &C)
{
    LaneP P{};
    P.b_tau = half2(C.b_tau); P.b_km = half2(C.b_km); P.b_ks = half2(C.b_ks); P.b_m1 = half2(C.b_m1);
    P.b_m2 = half2(C.b_m2); P.b_kb = half2(C.b_kb); P.b_kgl = half2(C.b_kgl); P.b_kgq = half2(C.b_kgq);
    P.b_zc = half2(C.b_zc);
    P.i_tau0 = half2(C.i_tau0); P.i_tau1 = half2(C.i_tau1); P.i_km = half2(C.i_km); P.i_ks = half2(C.i_ks);
    P.i_u0 = half2(C.i_u0); P.i_u1 = half2(C.i_u1); P.i_u2 = half2(C.i_u2); P.i_w2 = half2(C.i_w2);
    P.i_w3 = half2(C.i_w3); P.i_g = half2(C.i_g); P.i_s0 = half2(C.i_s0); P.i_s1 = half2(C.i_s1);
    P.i_s2 = half2(C.i_s2); P.i_s3 = half2(C.i_s3); P.i_S1 = half2(C.i_S1);
    P.u_fml = half2(C.u_fml); P.u_fmq = half2(C.u_fmq);
    P.flags = (unsigned char)((C.b_isE ? LP_ISE : 0) | (C.b_isA ? LP_ISA : 0) | (C.b_isD ? LP_ISD : 0) |
                              (C.b_exmask ? LP_EXMASK : 0) | (C.b_sgn ? LP_SGN : 0) | (C.f_row ? LP_FROW : 0));
    P.d_bs = (unsigned char)C.d_bs;
    for (int q = 0; q < kOutL; ++q) {
        P.d_kap[q] = (unsigned char)C.d_kap[q];
        P.d_mono[q] = (short)C.d_mono[q];
        P.d_basis[q] = (short)C.d_basis[q];
    }
    P.b_dst = (short)C.b_dst; P.i_d0 = (short)C.i_d0; P.i_d1 = (short)C.i_d1; P.i_e0r = (short)C.i_e0r;
    P.i_e0f = (short)C.i_e0f; P.i_e1r = (short)C.i_e1r; P.i_e1f = (short)C.i_e1f; P.i_ecr = (short)C.i_ecr;
    P.i_ecf = (short)C.i_ecf; P.i_a0 = (short)C.i_a0; P.i_a1 = (short)C.i_a1; P.i_dst = (short)C.i_dst;
    P.mo_v0 = (short)C.mo_v0; P.mo_v1 = (short)C.mo_v1; P.mo_v2 = (short)C.mo_v2; P.mo_dst = (short)C.mo_dst;
    P.d_out = (short)C.d_out; P.f_src = (short)C.f_src; P.f_na = (short)C.f_na; P.f_nb = (short)C.f_nb;
    P.f_dst = (short)C.f_dst; P.u_ub = (short)C.u_ub; P.u_wb = (short)C.u_wb; P.u_c = (short)C.u_c;
    P.u_post = (short)C.u_post; P.u_v = (short)C.u_v;
    return P;
}
GGP_DEV constexpr LaneC unpack_lane(const LaneP &P)
{
    LaneC C{};
    C.b_tau = 0.5 * P.b_tau; C.b_km = 0.5 * P.b_km; C.b_ks = 0.5 * P.b_ks; C.b_m1 = 0.5 * P.b_m1;
    C.b_m2 = 0.5 * P.b_m2; C.b_kb = 0.5 * P.b_kb; C.b_kgl = 0.5 * P.b_kgl; C.b_kgq = 0.5 * P.b_kgq;
    C.b_zc = 0.5 * P.b_zc;
    C.b_isE = (P.flags & LP_ISE) ? 1 : 0; C.b_isA = (P.flags & LP_ISA) ? 1 : 0; C.b_isD = (P.flags & LP_ISD) ? 1 : 0;
    C.b_exmask = (P.flags & LP_EXMASK) ? -1 : 0;
    C.b_sgn = (P.flags & LP_SGN) ? (int)0x80000000u : 0;
    C.b_mult = C.b_isD ? GGP_SPI2 : 1.0;
    C.b_dst = P.b_dst;
    C.i_tau0 = 0.5 * P.i_tau0; C.i_tau1 = 0.5 * P.i_tau1; C.i_km = 0.5 * P.i_km; C.i_ks = 0.5 * P.i_ks;
    C.i_u0 = 0.5 * P.i_u0; C.i_u1 = 0.5 * P.i_u1; C.i_u2 = 0.5 * P.i_u2; C.i_w2 = 0.5 * P.i_w2;
    C.i_w3 = 0.5 * P.i_w3; C.i_g = 0.5 * P.i_g; C.i_s0 = 0.5 * P.i_s0; C.i_s1 = 0.5 * P.i_s1;
    C.i_s2 = 0.5 * P.i_s2; C.i_s3 = 0.5 * P.i_s3; C.i_S1 = 0.5 * P.i_S1;
    C.i_d0 = P.i_d0; C.i_d1 = P.i_d1; C.i_e0r = P.i_e0r; C.i_e0f = P.i_e0f; C.i_e1r = P.i_e1r; C.i_e1f = P.i_e1f;
    C.i_ecr = P.i_ecr; C.i_ecf = P.i_ecf; C.i_a0 = P.i_a0; C.i_a1 = P.i_a1; C.i_dst = P.i_dst;
    C.mo_v0 = P.mo_v0; C.mo_v1 = P.mo_v1; C.mo_v2 = P.mo_v2; C.mo_dst = P.mo_dst;
    for (int q = 0; q < kOutL; ++q) {
        C.d_mono[q] = P.d_mono[q];
        C.d_basis[q] = P.d_basis[q];
        C.d_kap[q] = P.d_kap[q];
    }
    C.d_bs = P.d_bs; C.d_out = P.d_out;
    C.f_src = P.f_src; C.f_na = P.f_na; C.f_nb = P.f_nb; C.f_row = (P.flags & LP_FROW) ? 1 : 0; C.f_dst = P.f_dst;
    C.u_ub = P.u_ub; C.u_wb = P.u_wb; C.u_c = P.u_c; C.u_post = P.u_post; C.u_v = P.u_v;
    C.u_fml = 0.5 * P.u_fml; C.u_fmq = 0.5 * P.u_fmq;
    return C;
}
constexpr bool same_lane(const LaneC &a, const LaneC &b)
{
    bool ok = a.b_tau == b.b_tau && a.b_km == b.b_km && a.b_ks == b.b_ks && a.b_m1 == b.b_m1 && a.b_m2 == b.b_m2 &&
              a.b_kb == b.b_kb && a.b_kgl == b.b_kgl && a.b_kgq == b.b_kgq && a.b_mult == b.b_mult && a.b_zc == b.b_zc &&
              a.b_isE == b.b_isE && a.b_isA == b.b_isA && a.b_isD == b.b_isD && a.b_exmask == b.b_exmask &&
              a.b_sgn == b.b_sgn && a.b_dst == b.b_dst && a.i_tau0 == b.i_tau0 && a.i_tau1 == b.i_tau1 &&
              a.i_km == b.i_km && a.i_ks == b.i_ks && a.i_u0 == b.i_u0 && a.i_u1 == b.i_u1 && a.i_u2 == b.i_u2 &&
              a.i_w2 == b.i_w2 && a.i_w3 == b.i_w3 && a.i_g == b.i_g && a.i_s0 == b.i_s0 && a.i_s1 == b.i_s1 &&
              a.i_s2 == b.i_s2 && a.i_s3 == b.i_s3 && a.i_S1 == b.i_S1 && a.i_d0 == b.i_d0 && a.i_d1 == b.i_d1 &&
              a.i_e0r == b.i_e0r && a.i_e0f == b.i_e0f && a.i_e1r == b.i_e1r && a.i_e1f == b.i_e1f &&
              a.i_ecr == b.i_ecr && a.i_ecf == b.i_ecf && a.i_a0 == b.i_a0 && a.i_a1 == b.i_a1 && a.i_dst == b.i_dst &&
              a.mo_v0 == b.mo_v0 && a.mo_v1 == b.mo_v1 && a.mo_v2 == b.mo_v2 && a.mo_dst == b.mo_dst &&
              a.d_bs == b.d_bs && a.d_out == b.d_out && a.f_src == b.f_src && a.f_na == b.f_na && a.f_nb == b.f_nb &&
              a.f_row == b.f_row && a.f_dst == b.f_dst && a.u_ub == b.u_ub && a.u_wb == b.u_wb && a.u_c == b.u_c &&
              a.u_post == b.u_post && a.u_v == b.u_v && a.u_fml == b.u_fml && a.u_fmq == b.u_fmq;
    for (int q = 0; q < kOutL; ++q)
        ok = ok && a.d_mono[q] == b.d_mono[q] && a.d_basis[q] == b.d_basis[q] && a.d_kap[q] == b.d_kap[q];
    return ok;
}
struct LanePTab {
    LaneP l[64];
};
constexpr LanePTab make_lane_ptab()
{
    LanePTab T{};
    for (int l = 0; l < 64; ++l) T.l[l] = pack_lane(kLaneTab.l[l]);
    return T;
}
constexpr LanePTab kLanePTab = make_lane_ptab();
constexpr bool check_lane_ptab()
{
    for (int l = 0; l < 64; ++l)
        if (!same_lane(unpack_lane(kLanePTab.l[l]), kLaneTab.l[l])) return false;
    return true;
}
static_assert(check_lane_ptab(), "the packed lane table unpacks to the lane table, field for field");

// the lane's registers from its row and the parameters; kap: the 33 kappas (LDS, lane_kappa)
GGP_DEV Lane lane_from(const int lane, const LaneC &C, const OU &P, const double *kap)
{
    Lane L;
    L.b_tau = C.b_tau; L.b_km = C.b_km; L.b_gqks = P.gq * C.b_ks; L.b_m1 = C.b_m1; L.b_m2 = C.b_m2;
    L.b_kc = __builtin_fma(C.b_kgq, P.gq, __builtin_fma(C.b_kgl, P.gl, C.b_kb * P.b));
    L.b_mult = C.b_mult;
    L.b_zc = C.b_zc;
    L.b_isE = C.b_isE; L.b_isA = C.b_isA; L.b_isD = C.b_isD; L.b_exmask = C.b_exmask; L.b_sgn = C.b_sgn;
    L.b_dst = C.b_dst;
    L.i_tau0 = C.i_tau0; L.i_tau1 = C.i_tau1; L.i_km = C.i_km; L.i_gqks = P.gq * C.i_ks;
    L.i_u0 = C.i_u0; L.i_u1 = C.i_u1; L.i_u2 = C.i_u2; L.i_w2 = C.i_w2; L.i_w3 = C.i_w3; L.i_g = C.i_g;
    L.i_s0 = C.i_s0; L.i_s1 = C.i_s1; L.i_s2 = C.i_s2; L.i_s3 = C.i_s3; L.i_S1 = C.i_S1;
    L.i_d0 = C.i_d0; L.i_d1 = C.i_d1; L.i_e0r = C.i_e0r; L.i_e0f = C.i_e0f; L.i_e1r = C.i_e1r; L.i_e1f = C.i_e1f;
    L.i_ecr = C.i_ecr; L.i_ecf = C.i_ecf; L.i_a0 = C.i_a0; L.i_a1 = C.i_a1; L.i_dst = C.i_dst;
    L.mo_v0 = C.mo_v0; L.mo_v1 = C.mo_v1; L.mo_v2 = C.mo_v2; L.mo_dst = C.mo_dst;
#pragma unroll
    for (int q = 0; q < kOutL; ++q) {
        L.d_mono[q] = C.d_mono[q];
        L.d_basis[q] = C.d_basis[q];
        L.d_kap[q] = C.d_kap[q] == 255 ? 0.0 : kap[C.d_kap[q]];
    }
    L.d_bs = C.d_bs; L.d_out = C.d_out;
    L.f_src = C.f_src; L.f_na = C.f_na; L.f_nb = C.f_nb; L.f_row = C.f_row; L.f_dst = C.f_dst;
    L.u_ub = C.u_ub; L.u_wb = C.u_wb; L.u_c = C.u_c; L.u_post = C.u_post; L.u_v = C.u_v;
    L.u_vshift = __builtin_fma(C.u_fmq, P.mq, C.u_fml * P.ml);
    L.c_sv = lane < 6 ? wave::sv_of(P, lane) : P.gq;
    return L;
}

// kappa k of the outputs (out_kappa's value) for lanes k < kOutNK: one per lane instead of four
GGP_DEV double lane_kappa(const int lane, const OU &P) { return out_kappa(P, lane < kOutNK ? lane : 0); }

// ---- step scalars from the posterior (every lane the same values) --------------------------
// bx, bl, Cxx, Cxl, Cll as stored by the update (POST[0], [2], [4], [6], [14])
GGP_DEV wave::WStep wstep2(const double bx, const double bl, const double Cxx, const double Cxl, const double Cll,
                           const double t, const double b)
{
    double m[4] = {bx, 0.0, bl, 0.0}, C[16] = {};
    C[0] = Cxx;
    C[2] = Cxl;
    C[10] = Cll;
    return wave::wstep(m, C, t, b);
}

// 1/d: v_rcp_f64 and one Newton step -- an rdiv seed (the residual step makes the quotient
// independent of an ulp or two in it)
GGP_DEV double rcp1(const double d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const double r = __builtin_amdgcn_rcp(d);
    return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
#else
    return 1.0 / d;
#endif
}

// 1/d from v_rcp_f64 alone (a seed: a few 1e-8 relative)
GGP_DEV double rcp0(const double d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcp(d);
#else
    return 1.0 / d;
#endif
}

// 1/d: v_rcp_f64 and two Newton steps (within an ulp: the update's 1/det)
GGP_DEV double rcp2(const double d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
#else
    return 1.0 / d;
#endif
}

GGP_DEV int mul24(const int a, const int b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __mul24(a, b);   // v_mul_i32_i24: full rate (v_mul_lo_u32 is quarter rate)
#else
    return a * b;
#endif
}

GGP_DEV int cvt_i32(const double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int k;   // v_cvt_i32_f64: NaN -> 0, saturating
    asm("v_cvt_i32_f64 %0, %1" : "=v"(k) : "v"(x));
    return k;
#else
    if (x != x) return 0;
    return x >= 2147483647.0 ? 2147483647 : x <= -2147483648.0 ? (-2147483647 - 1) : (int)x;
#endif
}

// the high 32 bits of a double, and a double with its high word replaced
GGP_DEV int hi32(const double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __double2hiint(x);
#else
    long long b;
    __builtin_memcpy(&b, &x, 8);
    return (int)(b >> 32);
#endif
}
GGP_DEV double with_hi(const double x, const int hi)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __hiloint2double(hi, __double2loint(x));
#else
    unsigned long long b;
    __builtin_memcpy(&b, &x, 8);
    b = (b & 0xffffffffULL) | ((unsigned long long)(unsigned)hi << 32);
    double y;
    __builtin_memcpy(&y, &b, 8);
    return y;
#endif
}

// ---- stage B: one transcendental per lane ---------------------------------------------------
// the rare branches: exp beyond 2^50 (ocml's exp), Dawson Taylor (y100 >= 97) and continued
// fraction (|x| > 45), as ggp_wave.h dawson_bf
GGP_DEV double stageB_rare(const bool isD, const double arg, const double z, const double v)
{
    if (!isD) return fabs(arg) < kExpFastMax ? v : exp(arg);
    const double ax = fabs(z);
    const double y100 = 100.0 / (1.0 + ax);
    double w;
    if (ax > 45.0) {
        const bool far = ax > 5e7;
        const double num = far ? GGP_ISPI : GGP_ISPI * ((ax * ax) * (ax * ax - 4.5) + 2);
        const double den = far ? ax : ax * ((ax * ax) * (ax * ax - 5) + 3.75);
        w = num / den;
    } else if (y100 >= (double)GGP_DAWSON_NINT) {
        const double x2 = ax * ax;
        const double *tc = ggp_dawson_taylor;
        w = ax * (tc[0] - x2 * (tc[1] - x2 * (tc[2] - x2 * (tc[3] - x2 * tc[4]))));
    } else {
        return v;
    }
    return GGP_SPI2 * (z < 0.0 ? -w : w);
}

struct BOut {
    double v, arg, z;
    bool rare;
};

GGP_DEV void sched_fence()
{
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}

GGP_DEV BOut stageB(const wave::WStep &S, const Lane &L, const double *lds)
{
    // z first, then the Dawson interval from 1 / (1 + |z|) -- the reciprocal td needs anyway (v_rcp_f64
    // and one Newton step): the quotient biased up by 2^-22 makes k floor(y100) -- on an interval
    // boundary too (x = 24: y100 = 4) -- or, for y100 within 2.4e-5 below the next integer, that
    // integer, where td lies within 5e-5 below -1 (the row's polynomial holds there).  The table
    // row's six 128-bit LDS reads are then in flight while the exponential's argument and
    // reduction are formed (exp lanes read the exp row).
    const double ti = S.t * L.b_tau;
    const double B = wave::pin(__builtin_fma(S.Cxl, L.b_km, S.bbl) + L.b_gqks);
    const double xz = __builtin_fma(S.two_a, ti, B);
    const double z = rdiv(xz, S.two_sa, S.r_two_sa);
    const double ax = fabs(z);
    const double d1 = 1.0 + ax;
    const double r1 = rcp1(d1);
    const double ya = (100.0 * (1.0 + 0x1p-22)) * r1;
    const int kraw = cvt_i32(ya);
    const int k = min(kraw, GGP_DAWSON_NINT - 1);
    const int row = L.b_isD ? mul24(k, kTabRow) : kExpRow * kTabRow;
    const double *A = lds + L_TAB + row;
    double a[kTabRow];
#pragma unroll
    for (int i = 0; i < kTabRow; ++i) a[i] = A[i];
    sched_fence();
    // td = 2 y100 - (2k + 1) as (200 - (2k + 1) d1) / d1: the numerator by one fma (exact before
    // its rounding), so td is within ~2 ulp of itself, not of y100 (near small |z| an ulp of y100
    // is tens of ulp of the value: dx/dy ~ 1e-2, x ~ 0.05)
    const double td = __builtin_fma(-(double)(2 * k + 1), d1, 200.0) * r1;
    const double c = wave::pin(__builtin_fma(L.b_kc, S.t, __builtin_fma(S.Cxx, L.b_m2, S.bx * L.b_m1)));
    const double n = wave::pin(rdiv(-(B * B), S.four_a, S.r_four_a));
    // the A and Z kinds in one form: argZ = a ti^2 + B ti + c, argA = the same without c (c times
    // the lane's 0/1 constant), then one select against the E kind
    const double argE = wave::pin(__builtin_fma(z, z, n + c));
    const double argAZ = wave::pin(__builtin_fma(S.a, ti * ti, __builtin_fma(B, ti, c * L.b_zc)));
    const double arg = L.b_isE ? argE : argAZ;
    // exp reduction (exp_ocml)
    const double dn = __builtin_rint(arg * 0x1.71547652b82fep+0);
    double r = __builtin_fma(-dn, 0x1.62e42fefa39efp-1, arg);
    r = __builtin_fma(-dn, 0x1.abc9e3b39803fp-56, r);
    const double tv = L.b_isD ? td : r;
    double h = __builtin_fma(a[0], tv, a[1]);
#pragma unroll
    for (int i = 2; i < kTabRow; ++i) h = __builtin_fma(h, tv, a[i]);
    // no branches below: the exponent masked to 0 on Dawson lanes, z's sign bit onto a Dawson
    // value's (two 32-bit operations on the high word; an exp lane's mask is 0), the rare flags
    // by bitwise ops
    double v = __builtin_ldexp(h * L.b_mult, cvt_i32(dn) & L.b_exmask);
    v = with_hi(v, hi32(v) ^ (hi32(z) & L.b_sgn));
    BOut o;
    o.v = v;
    o.arg = arg;
    o.z = z;
    // Taylor (y100 >= 97) flagged from the biased quotient's integer part (it is >= the exact
    // y100, so no Taylor case is missed): stageB_rare decides on the exact quotient and returns
    // the table value when neither branch applies
    const bool rare_d = (kraw >= GGP_DAWSON_NINT) | (ax > 45.0);
    const bool rare_e = !(fabs(arg) < kExpFastMax);
    o.rare = ((L.b_isD != 0) & rare_d) | ((L.b_isD == 0) & rare_e);
    return o;
}

// ---- stage C: one integral per lane (tau_unified; mean_cov_model.h:9-67) --------------------
GGP_DEV double stageC(const wave::WStep &S, const Lane &L, const double *lds)
{
    const double D0 = lds[L.i_d0], D1 = lds[L.i_d1];
    const double E0 = lds[L.i_e0r] * lds[L.i_e0f];
    const double E1 = lds[L.i_e1r] * lds[L.i_e1f];
    const double ec = lds[L.i_ecr] * lds[L.i_ecf];
    const double ea0 = lds[L.i_a0], ea1 = lds[L.i_a1];
    const double B = wave::pin(__builtin_fma(S.Cxl, L.i_km, S.bbl) + L.i_gqks);
    const double t0 = S.t * L.i_tau0, t1 = S.t * L.i_tau1;
    const double BB = wave::pin(B * B);
    const double al3 = BB - S.four_a;
    const double al = __builtin_fma(L.i_u2, al3, __builtin_fma(L.i_u1, B, L.i_u0));
    const double be = -S.two_a * __builtin_fma(L.i_w3, B, L.i_w2);
    const double ga = L.i_g * S.four_aa;
    const double P0 = __builtin_fma(t0, __builtin_fma(ga, t0, be), al), P1 = __builtin_fma(t1, __builtin_fma(ga, t1, be), al);
    // Q = s0 + s1 2B + s2 2(2a - BB) + s3 2B(BB - 6a): one selector is nonzero (tau kind k), so
    // the factor 2 applied once to the selected term gives the same bits as applying it per term
    const double q2 = S.two_a - BB, q3 = B * __builtin_fma(-6., S.a, BB);
    const double Q = __builtin_fma(2., __builtin_fma(L.i_s3, q3, __builtin_fma(L.i_s2, q2, L.i_s1 * B)), L.i_s0);
    const double S1 = S.two_sa * L.i_S1;
    const double dterm = wave::pin(Q * __builtin_fma(E0, D0, -(E1 * D1)));
    const double x = __builtin_fma(S1 * ec, __builtin_fma(ea0, P0, -(ea1 * P1)), dterm);
    // the denominator 2^(k+1) a^k sqrt(a) as two_sa (2a)^k: the products of store_pw's
    // denominators (scaling by powers of two is exact), and an rdiv seed from v_rcp_f64
    const double p1 = S.two_a, p2 = p1 * p1, p3 = p2 * p1;
    const double qk = __builtin_fma(L.i_s3, p3, __builtin_fma(L.i_s2, p2, __builtin_fma(L.i_s1, p1, -0.5 * L.i_s0)));
    const double den = S.two_sa * qk;
    // rdiv's residual step on the v_rcp_f64 seed alone (relative error e ~ 1e-8): the quotient
    // within e^2 + its roundings, an ulp or two -- no Newton step on the seed
    return rdiv(x, den, rcp0(den));
}

// ---- stage D: the lane's output terms over the step's monomials ------------------------------
GGP_DEV double stageD(const Lane &L, const double *lds)
{
    double kv[kOutL], bv[kOutL];
#pragma unroll
    for (int q = 0; q < kOutL; ++q) {
        kv[q] = L.d_kap[q] * lds[L.d_mono[q]];
        bv[q] = lds[L.d_basis[q]];
    }
    double acc = kv[0] * bv[0];
#pragma unroll
    for (int q = 1; q < kOutL; ++q) acc = __builtin_fma(kv[q], bv[q], acc);
    return acc;
}

GGP_DEV double mono(const Lane &L, const double *lds) { return (lds[L.mo_v0] * lds[L.mo_v1]) * lds[L.mo_v2]; }

// ---- finish and update ------------------------------------------------------------------------
GGP_DEV double finish(const Lane &L, const double *lds, const int slot)
{
    return __builtin_fma(-lds[L.f_na], lds[L.f_nb + mul24(slot, L.f_row)], lds[L.f_src]);   // f_row: 0 or 1
}
// the same with the row's slot as a byte offset held in a vector register (the step loop's sv)
GGP_DEV double finish_sv(const Lane &L, const double *lds, const int sv)
{
    const double *row = reinterpret_cast<const double *>(reinterpret_cast<const char *>(lds + L.f_nb) + mul24(sv, L.f_row));
    return __builtin_fma(-lds[L.f_na], *row, lds[L.f_src]);
}

struct UInnov {
    double S00, S01, S11, invdet;
};
// the innovation covariance S from the prior's C00, C01, C11 and m1 (ggp_wave.h innovation's
// expressions) and 1/det S by rcp2 (its Newton steps run while the update's operands load).
// D11 = var_g (m1 + fp_auto) under the scaled noise model, var_g otherwise, as one fma on the
// launch constants g_sc = scaled ? var_g : 0, g_0 = scaled ? 0 : var_g (the same value, no select);
// S01 = C01 (the reference's C01 + 0 differs only in the sign of a zero, which no later product
// or sum with a nonzero value can show)
GGP_DEV UInnov uinnov(const double m1, const double C00, const double C01, const double C11, const double var_x,
                      const double g_sc, const double g_0, const double fp_auto)
{
    UInnov v;
    const double d11 = __builtin_fma(g_sc, m1 + fp_auto, g_0);
    v.S00 = C00 + var_x;
    v.S01 = C01;
    v.S11 = C11 + d11;
    const double det = __builtin_fma(v.S00, v.S11, -(v.S01 * v.S01));
    v.invdet = rcp2(det);
    return v;
}

// the update's operands of lane e: u = C[0][i], v = C[1][i] and w, z = C[0][j], C[1][j] (a
// covariance) or -x0, -x1 (a mean); its own prior entry c is the lane's finish value
struct UOps {
    double u, vv, w, z;
};
GGP_DEV UOps upost_load(const Lane &L, const double *lds)
{
    UOps q;
    q.u = lds[L.u_ub];
    q.vv = lds[L.u_ub + 4];
    q.w = lds[L.u_wb];
    q.z = lds[L.u_wb + 4];
    return q;
}

// posterior entry of lane e, C_ij - (KS1_i C1j + KS0_i C0j) with K S^-1 = K adj(S) / det S: the
// adjugate products first, the reciprocal determinant applied once by the last fma (ggp_wave.h
// posterior's terms; m_i + (KS1_i x1 + KS0_i x0) == m_i - (KS1_i (-x1) + KS0_i (-x0)))
GGP_DEV double upost(const UOps &q, const double c, const UInnov &v)
{
    const double A0 = __builtin_fma(q.vv, -v.S01, q.u * v.S11);
    const double A1 = __builtin_fma(q.vv, v.S00, q.u * -v.S01);
    return __builtin_fma(-__builtin_fma(A1, q.z, A0 * q.w), v.invdet, c);
}

#ifdef GGP_HOST_SIM
// ---- host emulation of one propagation + update step over the 64 lanes -----------------------
// lds: the wave's LDS (table filled), state in POST / V; dt cache filled for t.  Returns the
// posterior in lds POST.  Used by tools/hostsim.cpp to compare against the oracle.
struct HostWave {
    double lds[kLds];
    Lane L[64];
    OU P;
    double b, t_cached = -1.0;
    HostWave(const double *p)
    {
        P = make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
        b = P.b;
        for (int i = 0; i < kLds; ++i) lds[i] = 0.0;
        for (int k = 0; k < kTabRows * kTabRow; ++k) lds[L_TAB + k] = tab_entry(k);
        double kap[kOutNK];
        for (int k = 0; k < kOutNK; ++k) kap[k] = lane_kappa(k, P);
        for (int l = 0; l < 64; ++l) L[l] = lane_from(l, kLaneTab.l[l], P, kap);
        lds[L_X + X_ONE] = 1.0;
        lds[L_BV + BV_ONE] = 1.0;
        lds[L_V + V_ONE] = 1.0;
        lds[L_ONE1] = 1.0;
        lds[L_ZERO] = 0.0;
    }
    void dt_cache(const double t)
    {
        if (t == t_cached) return;
        for (int s = 0; s < 6; ++s) lds[L_X + XS_bt + s] = exp(wave::sv_of(P, s) * t);
        lds[L_XPGQ] = exp(P.gq * t);
        double X[NX];
        for (int k = 0; k < NX; ++k) X[k] = lds[L_X + k];
        for (int j = 0; j < kNDerived; ++j) lds[L_BV + BV_R_EBT + j] = derived_generic(kDerived[j], X, P.gl, t);
        lds[L_V + V_T] = t;
        t_cached = t;
    }
    // propagate the state in POST over t: raw outputs to OUT
    void propagate(const double t)
    {
        dt_cache(t);
        const double *po = lds + L_POST;
        const wave::WStep S = wstep2(po[0], po[2], po[4], po[6], po[14], t, b);
        for (int l = 0; l < 64; ++l) lds[L[l].mo_dst] = mono(L[l], lds);
        double vb[64];
        for (int l = 0; l < 64; ++l) {
            const BOut o = stageB(S, L[l], lds);
            vb[l] = o.rare ? stageB_rare(L[l].b_isD, o.arg, o.z, o.v) : o.v;
        }
        for (int l = 0; l < 64; ++l) lds[L[l].b_dst] = vb[l];
        double vc[64];
        for (int l = 0; l < 64; ++l) vc[l] = stageC(S, L[l], lds);
        for (int l = 0; l < 64; ++l) lds[L[l].i_dst] = vc[l];
        double part[64];
        for (int l = 0; l < 64; ++l) part[l] = stageD(L[l], lds);
        for (int st = 0; st < 4; ++st) {
            double nx[64];
            for (int l = 0; l < 64; ++l) nx[l] = kOutBlock[l] > (1 << st) ? part[l] + part[out_partner(l, st)] : part[l];
            for (int l = 0; l < 64; ++l) part[l] = nx[l];
        }
        for (int l = 0; l < 64; ++l) lds[L[l].d_out] = part[l];
    }
    // finish + distributed update with row data (y_l, y_f) at slot 0; returns the ll ring inputs
    void update(const double y_l, const double y_f, const double var_x, const double var_g, const int scaled,
                const double fp_auto, double *ring5)
    {
        lds[L_ROWL] = y_l;
        lds[L_ROWF] = y_f;
        double f[64];
        for (int l = 0; l < 64; ++l) f[l] = finish(L[l], lds, 0);
        for (int l = 0; l < 64; ++l) lds[L[l].f_dst] = f[l];
        const double *st = lds + L_ST;
        const UInnov v = uinnov(st[1], st[4], st[5], st[9], var_x, scaled ? var_g : 0.0, scaled ? 0.0 : var_g, fp_auto);
        double u[64];
        for (int l = 0; l < 64; ++l) u[l] = upost(upost_load(L[l], lds), f[l], v);
        for (int l = 0; l < 64; ++l) {
            lds[L[l].u_post] = u[l];
            lds[L[l].u_v] = u[l] - L[l].u_vshift;
        }
        ring5[0] = st[20];
        ring5[1] = st[24];
        ring5[2] = v.S00;
        ring5[3] = v.S01;
        ring5[4] = v.S11;
    }
};
#endif

}  // namespace wave
}  // namespace ggp
