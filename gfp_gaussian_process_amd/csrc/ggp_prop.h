// ggp_prop.h -- the propagation step mean_cov_model (mean_cov_model.h:211-274) as a set of
// data-parallel TASKS over one step's shared scalars, so that two schedules can run it:
//
//   lane kernel  : one lane owns a cell; every task index is a compile-time constant
//                  (unrolled), arrays live in registers;
//   group kernel : G lanes own a cell; lane l runs tasks l, l+G, ...; arrays live in LDS.
//
// Both schedules (and the lane-pair, batch and smoother kernels) execute the SAME expression
// for every value, so they are bitwise equal (tests/test_gpu_parity.py).  The expressions are
// the reference's, term by term, with two departures that all these kernels share: a*b + c
// inside one expression is one fma (GGP_CONTRACT), and 22 of the 74 exponentials are products
// of two others (kXP below).  The 59 tauint calls of one step dedupe to 45 distinct integrals
// over 74 distinct exponentials (54 computed) and 14 Dawson values.
//
// Division: x/d for a denominator used several times per step is evaluated as
// q = x*r, e = fma(-q,d,x), q' = fma(e,r,q) with r = 1/d correctly rounded (Markstein):
// correctly rounded, i.e. bitwise equal to IEEE x/d for finite normal operands (checked on
// 2e8 random pairs); 3 instructions instead of ~11.
#pragma once
#include <utility>

#include "ggp_device.h"

#ifndef GGP_EXP_TABLE_DEFINED
#define GGP_EXP_TABLE_DEFINED
#ifdef GGP_HOST_SIM
#define GGP_EXP_TABLE_QUALIFIER static const
#else
#define GGP_EXP_TABLE_QUALIFIER static __constant__ const
#endif
#include "exp_table.inc"
#endif

namespace ggp {

// GGP_EXACT: the propagator in the oracle's arithmetic, step for step (DESIGN.md §2 "Exact
// arithmetic"): glibc's exp (exp_glibc), every one of the 74 exponentials computed from its own
// argument (no products), no fma contraction.  The default build keeps the fast forms.
#ifdef GGP_EXACT
constexpr bool kExact = true;
#else
constexpr bool kExact = false;
#endif

// the propagator's LDS table: the Dawson coefficients (GGP_DAWSON_NINT x NCOEF doubles), one pad
// double, then glibc's exp table (2^(k/128), 256 64-bit words, 16-byte aligned)
constexpr int kDawsonTabN = GGP_DAWSON_NINT * GGP_DAWSON_NCOEF;
constexpr int kExpTabOff = (kDawsonTabN + 1) & ~1;
constexpr int kPropTabN = kExpTabOff + GGP_EXP_TAB_N;
static_assert(kExpTabOff % 2 == 0, "16-byte aligned exp table rows");
GGP_DEV const uint64_t *exp_tab_of(const double *tab) { return reinterpret_cast<const uint64_t *>(tab + kExpTabOff); }
// entry k of the combined table (a fill loop's source)
GGP_DEV double prop_tab_entry(const int k)
{
    return k < kDawsonTabN ? ggp_dawson_coef[k] : k < kExpTabOff ? 0.0 : __builtin_bit_cast(double, ggp_exp_tab[k - kExpTabOff]);
}
#ifdef GGP_HOST_SIM
// the combined table on the host (diagnostic builds)
inline const double *host_prop_tab()
{
    static double t[kPropTabN];
    static bool done = false;
    if (!done) {
        for (int k = 0; k < kPropTabN; ++k) t[k] = prop_tab_entry(k);
        done = true;
    }
    return t;
}
#endif

GGP_DEV double rdiv(double x, double d, double r)
{
    const double q = x * r;
    const double e = __builtin_fma(-q, d, x);
    return __builtin_fma(e, r, q);
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
    // ocml's range checks (x > 1024 -> inf, x < -1075 -> 0) are left out.  For |x| < 2^50,
    // dn = rint(x log2 e) is within 0.7 of x log2 e, so |t| < 0.6 and p is finite: v_ldexp_f64
    // then overflows to inf / underflows to 0 exactly where ocml's checks would (the int
    // conversion saturates), and the value is ocml's bitwise.  Beyond 2^50 (+-inf included) t
    // is not reduced and the value is not ocml's: callers bound |x| (kExpFastMax)
    return __builtin_ldexp(p, (int)dn);
}

constexpr double kExpFastMax = 0x1p50;   // exp_ocml is ocml's exp for |x| below this

// exp(x) for the lane schedules: exp_ocml's sequence with the compiler's own operand choice (SGPR
// coefficients, no inline asm) and without ocml's per-call range checks (two compares and four
// selects); the check becomes one compare folded into the lane's flag `big`.  A lane whose flag is
// set recomputes its exponentials with ocml's exp (lane_exps' cold path), so every value is ocml's
// bitwise: exp_ocml's for |x| < kExpFastMax, ocml's own beyond
GGP_DEV double exp_lane(const double x, bool &big)
{
    big = big | !(__builtin_fabs(x) < kExpFastMax);
    const double dn = __builtin_rint(x * 0x1.71547652b82fep+0);
    double t = __builtin_fma(-dn, 0x1.62e42fefa39efp-1, x);
    t = __builtin_fma(-dn, 0x1.abc9e3b39803fp-56, t);
    double p = __builtin_fma(t, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
    p = __builtin_fma(t, p, 0x1.71dee623fde64p-19);
    p = __builtin_fma(t, p, 0x1.a01997c89e6b0p-16);
    p = __builtin_fma(t, p, 0x1.a01a014761f6ep-13);
    p = __builtin_fma(t, p, 0x1.6c16c1852b7b0p-10);
    p = __builtin_fma(t, p, 0x1.1111111122322p-7);
    p = __builtin_fma(t, p, 0x1.55555555502a1p-5);
    p = __builtin_fma(t, p, 0x1.5555555555511p-3);
    p = __builtin_fma(t, p, 0x1.000000000000bp-1);
    p = __builtin_fma(t, p, 1.0);
    p = __builtin_fma(t, p, 1.0);
    return __builtin_ldexp(p, (int)dn);
}

// exp(x) as the reference's libm computes it: glibc's table-driven exp (sysdeps/ieee754/dbl-64/
// e_exp.c), in the build an x86-64 CPU with FMA runs (the reference is built for plain x86-64,
// src/Makefile:2, and its exp() call resolves to glibc's FMA variant at run time).  The same
// operations in the same order, with fma exactly where that build has one (its machine code:
// kd, both reduction steps, both polynomial halves and the last scale step), so the value is
// glibc's bitwise (tests/test_exp_glibc.py: every double of several ranges against this
// process's libm).  x = k ln2/128 + r; exp(x) = 2^(k/128) (1 + tail) exp(r); tab = exp_table.inc
// (LDS on the device: one 16-byte read per call).  |x| < 2^-54, |x| >= 512, inf and NaN take
// glibc's special paths (exp_glibc_special).
// Provenance and licence: the algorithm and the constants below are Szabolcs Nagy's exp from Arm's
// optimized-routines (math/exp.c, math/exp_data.c; MIT OR Apache-2.0 WITH LLVM-exception), which
// glibc ships as e_exp.c / e_exp_data.c (LGPL-2.1-or-later).  The code here is a restatement of
// that published algorithm, not its source text; the 2^(k/128) table is computed by
// tools/gen_exp_table.py (checked bitwise against this process's libm), and the eight constants
// are the numeric values the bitwise result requires.
constexpr double kGInvLn2N = 0x1.71547652b82fep0 * 128, kGShift = 0x1.8p52;
constexpr double kGNegLn2hiN = -0x1.62e42fefa0000p-8, kGNegLn2loN = -0x1.cf79abc9e3b3ap-47;
constexpr double kGC2 = 0x1.ffffffffffdbdp-2, kGC3 = 0x1.555555555543cp-3;
constexpr double kGC4 = 0x1.55555cf172b91p-5, kGC5 = 0x1.1111167a4d017p-7;

GGP_DEV double bits_to_double(const uint64_t u) { return __builtin_bit_cast(double, u); }
GGP_DEV uint64_t double_to_bits(const double d) { return __builtin_bit_cast(uint64_t, d); }

// the main path's reduction and polynomial: returns tmp, sets sbits and ki
GGP_DEV double exp_glibc_core(const double x, const uint64_t *tab, uint64_t &sbits, uint64_t &ki)
{
    double kd = __builtin_fma(x, kGInvLn2N, kGShift);
    ki = double_to_bits(kd);
    kd = kd - kGShift;
    double r = __builtin_fma(kd, kGNegLn2hiN, x);
    r = __builtin_fma(kd, kGNegLn2loN, r);
    const uint32_t idx = 2u * (uint32_t)(ki & 127u);
    const double tail = bits_to_double(tab[idx]);
    sbits = tab[idx + 1] + (ki << 45);
    const double r2 = r * r;
    const double p1 = __builtin_fma(r, kGC3, kGC2);
    const double p2 = __builtin_fma(r, kGC5, kGC4);
    const double acc = __builtin_fma(p1, r2, r + tail);
    return __builtin_fma(r2 * r2, p2, acc);
}

// glibc's paths outside 2^-54 <= |x| < 512 (e_exp.c specialcase and the top12 checks); the lane
// kernels reach them only through their cold paths (propagate_lane_cold, the lane-pair share loop)
GGP_DEV double exp_glibc_special(const double x, const uint64_t *tab)
{
    const uint64_t ix = double_to_bits(x);
    const uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ffu;
    if (abstop < 0x3c9u) return x + 1.0;                       // |x| < 2^-54 (and +-0)
    if (abstop >= 0x409u) {                                     // |x| >= 1024, inf, NaN
        if (ix == 0xfff0000000000000ull) return 0.0;           // -inf
        if (abstop == 0x7ffu) return x + 1.0;                  // +inf, NaN
        return (ix >> 63) ? 0.0 : __builtin_inf();             // underflow / overflow
    }
    uint64_t sbits, ki;
    const double tmp = exp_glibc_core(x, tab, sbits, ki);
    if ((ki & 0x80000000ull) == 0) {                            // k > 0: scale may overflow
        const double scale = bits_to_double(sbits - (1009ull << 52));
        return 0x1p1009 * __builtin_fma(scale, tmp, scale);
    }
    const double scale = bits_to_double(sbits + (1022ull << 52));  // k < 0: the subnormal range
    const double st = scale * tmp;
    double y = scale + st;
    if (y < 1.0) {
        const double hi = y + 1.0;
        double lo = (scale - y) + st;
        lo = ((1.0 - hi) + y) + lo;
        y = (lo + hi) - 1.0;
        if (y == 0.0) y = 0.0;
    }
    return 0x1p-1022 * y;
}

// the main path only, branch-free (no special-path test per call): `big` collects whether x lies
// outside 2^-54 <= |x| < 512, where the caller must recompute with exp_glibc.  Any x (inf, NaN
// included) reads a table entry in range, so the unchecked value is harmless before that
GGP_DEV double exp_glibc_main(const double x, const uint64_t *tab, bool &big)
{
    const uint32_t abstop = (uint32_t)(double_to_bits(x) >> 52) & 0x7ffu;
    big = big | (abstop - 0x3c9u >= 0x3fu);
    uint64_t sbits, ki;
    const double tmp = exp_glibc_core(x, tab, sbits, ki);
    const double scale = bits_to_double(sbits);
    double y = __builtin_fma(scale, tmp, scale);
#if defined(__HIP_DEVICE_COMPILE__)
    // materialised here: left to the optimiser, the polynomial sinks to the value's uses and the
    // table words stay live instead (the lane kernels spill ~400 registers)
    asm volatile("" : "+v"(y));
#endif
    return y;
}

GGP_DEV double exp_glibc(const double x, const uint64_t *tab)
{
    const uint32_t abstop = (uint32_t)(double_to_bits(x) >> 52) & 0x7ffu;
    if (__builtin_expect(abstop - 0x3c9u >= 0x3fu, 0)) return exp_glibc_special(x, tab);
    uint64_t sbits, ki;
    const double tmp = exp_glibc_core(x, tab, sbits, ki);
    const double scale = bits_to_double(sbits);
    return __builtin_fma(scale, tmp, scale);
}

// 1/d for finite nonzero d as v_rcp_f64 and two Newton steps (5 instructions against the ~11 of
// the IEEE sequence).  Used where the value only seeds rdiv, whose residual correction makes
// the quotient independent of an ulp in the seed.  d = 0 or inf gives NaN (IEEE: inf, 0);
// at such d the seeded quotients are NaN in both forms.
GGP_DEV double frcp(double d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
#else
    return 1.0 / d;
#endif
}

// ---- indices -------------------------------------------------------------------------
// b values (tauint 2nd argument)            B1..B6  -> 0..5
// c values (tauint 3rd argument)            cA cB cJ cG cC cD cE cF cI cH -> 0..9
// time points                               0, t, 2t -> 0..2
enum { cA = 0, cB, cJ, cG, cC, cD, cE, cF, cI, cH };
enum { KX_C = 0, KX_A, KX_S, KX_E, KX_Z };      // exp kinds

// exponential slots
enum {
    XC_A = 0, XC_B, XC_J, XC_G, XC_C, XC_D, XC_E, XC_F, XC_I,                 // exp(c)
    XA_1t, XA_2t, XA_3t, XA_4t, XA_32, XA_42,                                  // exp(ti (B + a ti))
    XS_bt, XS_bglt, XS_2bt, XS_bgqt, XS_gl, XS_gq,                             // exp(s t)
    XE_2A0, XE_2At, XE_1A0, XE_1At, XE_1B0, XE_1Bt, XE_2B0, XE_2Bt, XE_1J0, XE_1Jt,
    XE_2J0, XE_2Jt, XE_1G0, XE_1Gt, XE_2G0, XE_2Gt, XE_3C0, XE_3Ct, XE_3C2, XE_4C0,
    XE_4Ct, XE_4C2, XE_3Dt, XE_3D2, XE_4E0, XE_4Et, XE_4E2, XE_4Ft, XE_4F2,    // exp(-B^2/4a + c + z^2)
    XZ_1At, XZ_2At, XZ_1Bt, XZ_2Bt, XZ_1Jt, XZ_2Jt, XZ_2It, XZ_5It, XZ_1Gt, XZ_2Gt,
    XZ_3Ct, XZ_4Ct, XZ_3Et, XZ_4Et, XZ_3E2, XZ_3C2, XZ_3Dt, XZ_3D2, XZ_4E2, XZ_4C2,
    XZ_4Ft, XZ_4F2, XZ_6Ht, XZ_6H2,                                            // exp(a ti^2 + B ti + c)
    X_ONE,                                                                     // 1.0 (t0 = 0)
    NX
};
constexpr int NXT = X_ONE;   // 74 exponentials to compute

struct XTask { unsigned char kind, iB, ic, it; };
// kind, B (or s for KX_S), c, t
constexpr XTask kXT[NXT] = {
    {KX_C, 0, cA, 0}, {KX_C, 0, cB, 0}, {KX_C, 0, cJ, 0}, {KX_C, 0, cG, 0}, {KX_C, 0, cC, 0},
    {KX_C, 0, cD, 0}, {KX_C, 0, cE, 0}, {KX_C, 0, cF, 0}, {KX_C, 0, cI, 0},
    {KX_A, 0, 0, 1}, {KX_A, 1, 0, 1}, {KX_A, 2, 0, 1}, {KX_A, 3, 0, 1}, {KX_A, 2, 0, 2}, {KX_A, 3, 0, 2},
    {KX_S, 0, 0, 0}, {KX_S, 1, 0, 0}, {KX_S, 2, 0, 0}, {KX_S, 3, 0, 0}, {KX_S, 4, 0, 0}, {KX_S, 5, 0, 0},
    {KX_E, 1, cA, 0}, {KX_E, 1, cA, 1}, {KX_E, 0, cA, 0}, {KX_E, 0, cA, 1}, {KX_E, 0, cB, 0},
    {KX_E, 0, cB, 1}, {KX_E, 1, cB, 0}, {KX_E, 1, cB, 1}, {KX_E, 0, cJ, 0}, {KX_E, 0, cJ, 1},
    {KX_E, 1, cJ, 0}, {KX_E, 1, cJ, 1}, {KX_E, 0, cG, 0}, {KX_E, 0, cG, 1}, {KX_E, 1, cG, 0},
    {KX_E, 1, cG, 1}, {KX_E, 2, cC, 0}, {KX_E, 2, cC, 1}, {KX_E, 2, cC, 2}, {KX_E, 3, cC, 0},
    {KX_E, 3, cC, 1}, {KX_E, 3, cC, 2}, {KX_E, 2, cD, 1}, {KX_E, 2, cD, 2}, {KX_E, 3, cE, 0},
    {KX_E, 3, cE, 1}, {KX_E, 3, cE, 2}, {KX_E, 3, cF, 1}, {KX_E, 3, cF, 2},
    {KX_Z, 0, cA, 1}, {KX_Z, 1, cA, 1}, {KX_Z, 0, cB, 1}, {KX_Z, 1, cB, 1}, {KX_Z, 0, cJ, 1},
    {KX_Z, 1, cJ, 1}, {KX_Z, 1, cI, 1}, {KX_Z, 4, cI, 1}, {KX_Z, 0, cG, 1}, {KX_Z, 1, cG, 1},
    {KX_Z, 2, cC, 1}, {KX_Z, 3, cC, 1}, {KX_Z, 2, cE, 1}, {KX_Z, 3, cE, 1}, {KX_Z, 2, cE, 2},
    {KX_Z, 2, cC, 2}, {KX_Z, 2, cD, 1}, {KX_Z, 2, cD, 2}, {KX_Z, 3, cE, 2}, {KX_Z, 3, cC, 2},
    {KX_Z, 3, cF, 1}, {KX_Z, 3, cF, 2}, {KX_Z, 5, cH, 1}, {KX_Z, 5, cH, 2},
};

// ---- the lane schedules' exponentials: 54 computed, 22 products ------------------------------
// Several c values differ by a multiple of t: c_B = c_A - gl t, c_J = c_I = c_A - gq t,
// c_G = c_A - b t, c_E = c_C, c_D = c_C - gq t, c_F = c_C + gq t.  So 22 of the 74 slots are
// exp(c_rep + ...) exp(+-k t): the product of a computed exponential and one of exp(-gl t),
// exp(-gq t) (slots XS_gl, XS_gq), exp(-b t) or exp(gq t) (two more exponentials, slots XF_MBT
// and XF_PGQ past NX), or a copy (factor X_ONE = 1).  The argument of a product's factors is O(1)
// with no cancellation, so a product is within ~2 ulp of the direct exponential (ggp_wave.h
// forms the same products).  The lane, lane-pair, group, batch and smoother kernels all take the
// products, so they stay bitwise equal to one another.
enum { XF_MBT = NX, XF_PGQ, NXE };   // slots of the lane schedules' X arrays (NXE doubles)
constexpr XTask kXF[2] = {{KX_S, 6, 0, 0}, {KX_S, 7, 0, 0}};   // exp(-b t), exp(gq t): pickSV 6, 7

struct XProd { unsigned char j, rep, fac; };   // X[j] = X[rep] * X[fac]
// the lane schedules take the products unless GGP_EXACT (then all 74 are computed, kXCN below)
constexpr XProd kXP[] = {
    {XC_B, XC_A, XS_gl},     {XC_J, XC_A, XS_gq},     {XC_G, XC_A, XF_MBT},    {XC_I, XC_A, XS_gq},
    {XC_D, XC_C, XS_gq},     {XC_E, XC_C, X_ONE},     {XC_F, XC_C, XF_PGQ},
    {XZ_1Bt, XZ_1At, XS_gl}, {XZ_1Jt, XZ_1At, XS_gq}, {XZ_1Gt, XZ_1At, XF_MBT},
    {XZ_2Bt, XZ_2At, XS_gl}, {XZ_2Jt, XZ_2At, XS_gq}, {XZ_2It, XZ_2At, XS_gq}, {XZ_2Gt, XZ_2At, XF_MBT},
    {XZ_3Et, XZ_3Ct, X_ONE}, {XZ_3Dt, XZ_3Ct, XS_gq}, {XZ_4Et, XZ_4Ct, X_ONE}, {XZ_4Ft, XZ_4Ct, XF_PGQ},
    {XZ_3E2, XZ_3C2, X_ONE}, {XZ_3D2, XZ_3C2, XS_gq}, {XZ_4E2, XZ_4C2, X_ONE}, {XZ_4F2, XZ_4C2, XF_PGQ},
};
constexpr int NXP = sizeof(kXP) / sizeof(kXP[0]);
constexpr int NXPU = kExact ? 0 : NXP;          // products the lane schedules form
constexpr int NXC = kExact ? NXT : NXT - NXP + 2;   // exponentials computed per step

constexpr bool x_is_product(const int j)
{
    for (int p = 0; p < NXPU; ++p)
        if (kXP[p].j == j) return true;
    return false;
}
struct XCList {
    unsigned char j[NXC];   // destination slot
    XTask T[NXC];
};
constexpr XCList make_xc()
{
    XCList L{};
    int n = 0;
    for (int j = 0; j < NXT; ++j)
        if (!x_is_product(j)) { L.j[n] = (unsigned char)j; L.T[n] = kXT[j]; ++n; }
    if (!kExact) {
        L.j[n] = XF_MBT; L.T[n] = kXF[0]; ++n;
        L.j[n] = XF_PGQ; L.T[n] = kXF[1]; ++n;
    }
    return L;
}
constexpr XCList kXC = make_xc();
static_assert(NXP == 22 && NXC == (kExact ? 74 : 54), "54 computed exponentials, 22 products (74, none: exact)");
constexpr bool check_products()
{
    for (int p = 0; p < NXPU; ++p)   // every operand is a computed slot
        if (x_is_product(kXP[p].rep) || x_is_product(kXP[p].fac)) return false;
    return true;
}
static_assert(check_products(), "a product's operands are computed exponentials");

// Dawson slots D(B, t_i)
enum { D_1_0 = 0, D_1_t, D_2_0, D_2_t, D_3_0, D_3_t, D_3_2, D_4_0, D_4_t, D_4_2, D_5_0, D_5_t,
       D_6_t, D_6_2, ND };
struct DTask { unsigned char iB, it; };
constexpr DTask kDT[ND] = {{0, 0}, {0, 1}, {1, 0}, {1, 1}, {2, 0}, {2, 1}, {2, 2},
                           {3, 0}, {3, 1}, {3, 2}, {4, 0}, {4, 1}, {5, 1}, {5, 2}};

// tauint slots (k = 1 first, then k = 0, 2, 3)
enum {
    O_2A = 0, O_1A, O_1B, O_2B, O_1J, O_2J, O_1G, O_2G, O_3C, O_4C, O_3C2, O_3D2, O_4E, O_4E2,
    O_4C2, O_4F2,
    Z_1A, Z_2A, Z_1B, Z_2B, Z_1J, Z_2J, Z_2I, Z_5I, Z_1G, Z_2G, Z_3C, Z_4C, Z_3E, Z_4E, Z_3E2,
    Z_3C2, Z_3D2, Z_4E2, Z_4C2, Z_4F2, Z_6H2,
    T_2A, T_2B, T_2J, T_2G, T_4C, T_4C2,
    H_4C, H_4C2,
    NI
};
struct ITask { unsigned char k, iB, it0, it1, xc, x0, x1, xa0, xa1, d0, d1; };
constexpr ITask kIT[NI] = {
    // k = 1: ec, E0, E1, ea0, ea1, D0, D1
    {1, 1, 0, 1, XC_A, XE_2A0, XE_2At, X_ONE, XA_2t, D_2_0, D_2_t},
    {1, 0, 0, 1, XC_A, XE_1A0, XE_1At, X_ONE, XA_1t, D_1_0, D_1_t},
    {1, 0, 0, 1, XC_B, XE_1B0, XE_1Bt, X_ONE, XA_1t, D_1_0, D_1_t},
    {1, 1, 0, 1, XC_B, XE_2B0, XE_2Bt, X_ONE, XA_2t, D_2_0, D_2_t},
    {1, 0, 0, 1, XC_J, XE_1J0, XE_1Jt, X_ONE, XA_1t, D_1_0, D_1_t},
    {1, 1, 0, 1, XC_J, XE_2J0, XE_2Jt, X_ONE, XA_2t, D_2_0, D_2_t},
    {1, 0, 0, 1, XC_G, XE_1G0, XE_1Gt, X_ONE, XA_1t, D_1_0, D_1_t},
    {1, 1, 0, 1, XC_G, XE_2G0, XE_2Gt, X_ONE, XA_2t, D_2_0, D_2_t},
    {1, 2, 0, 1, XC_C, XE_3C0, XE_3Ct, X_ONE, XA_3t, D_3_0, D_3_t},
    {1, 3, 0, 1, XC_C, XE_4C0, XE_4Ct, X_ONE, XA_4t, D_4_0, D_4_t},
    {1, 2, 1, 2, XC_C, XE_3Ct, XE_3C2, XA_3t, XA_32, D_3_t, D_3_2},
    {1, 2, 1, 2, XC_D, XE_3Dt, XE_3D2, XA_3t, XA_32, D_3_t, D_3_2},
    {1, 3, 0, 1, XC_E, XE_4E0, XE_4Et, X_ONE, XA_4t, D_4_0, D_4_t},
    {1, 3, 1, 2, XC_E, XE_4Et, XE_4E2, XA_4t, XA_42, D_4_t, D_4_2},
    {1, 3, 1, 2, XC_C, XE_4Ct, XE_4C2, XA_4t, XA_42, D_4_t, D_4_2},
    {1, 3, 1, 2, XC_F, XE_4Ft, XE_4F2, XA_4t, XA_42, D_4_t, D_4_2},
    // k = 0: Z0 (lower limit, = exp(c) at t0 = 0), Z1, D0, D1
    {0, 0, 0, 1, 0, XC_A, XZ_1At, 0, 0, D_1_0, D_1_t},
    {0, 1, 0, 1, 0, XC_A, XZ_2At, 0, 0, D_2_0, D_2_t},
    {0, 0, 0, 1, 0, XC_B, XZ_1Bt, 0, 0, D_1_0, D_1_t},
    {0, 1, 0, 1, 0, XC_B, XZ_2Bt, 0, 0, D_2_0, D_2_t},
    {0, 0, 0, 1, 0, XC_J, XZ_1Jt, 0, 0, D_1_0, D_1_t},
    {0, 1, 0, 1, 0, XC_J, XZ_2Jt, 0, 0, D_2_0, D_2_t},
    {0, 1, 0, 1, 0, XC_I, XZ_2It, 0, 0, D_2_0, D_2_t},
    {0, 4, 0, 1, 0, XC_I, XZ_5It, 0, 0, D_5_0, D_5_t},
    {0, 0, 0, 1, 0, XC_G, XZ_1Gt, 0, 0, D_1_0, D_1_t},
    {0, 1, 0, 1, 0, XC_G, XZ_2Gt, 0, 0, D_2_0, D_2_t},
    {0, 2, 0, 1, 0, XC_C, XZ_3Ct, 0, 0, D_3_0, D_3_t},
    {0, 3, 0, 1, 0, XC_C, XZ_4Ct, 0, 0, D_4_0, D_4_t},
    {0, 2, 0, 1, 0, XC_E, XZ_3Et, 0, 0, D_3_0, D_3_t},
    {0, 3, 0, 1, 0, XC_E, XZ_4Et, 0, 0, D_4_0, D_4_t},
    {0, 2, 1, 2, 0, XZ_3Et, XZ_3E2, 0, 0, D_3_t, D_3_2},
    {0, 2, 1, 2, 0, XZ_3Ct, XZ_3C2, 0, 0, D_3_t, D_3_2},
    {0, 2, 1, 2, 0, XZ_3Dt, XZ_3D2, 0, 0, D_3_t, D_3_2},
    {0, 3, 1, 2, 0, XZ_4Et, XZ_4E2, 0, 0, D_4_t, D_4_2},
    {0, 3, 1, 2, 0, XZ_4Ct, XZ_4C2, 0, 0, D_4_t, D_4_2},
    {0, 3, 1, 2, 0, XZ_4Ft, XZ_4F2, 0, 0, D_4_t, D_4_2},
    {0, 5, 1, 2, 0, XZ_6Ht, XZ_6H2, 0, 0, D_6_t, D_6_2},
    // k = 2
    {2, 1, 0, 1, XC_A, XE_2A0, XE_2At, X_ONE, XA_2t, D_2_0, D_2_t},
    {2, 1, 0, 1, XC_B, XE_2B0, XE_2Bt, X_ONE, XA_2t, D_2_0, D_2_t},
    {2, 1, 0, 1, XC_J, XE_2J0, XE_2Jt, X_ONE, XA_2t, D_2_0, D_2_t},
    {2, 1, 0, 1, XC_G, XE_2G0, XE_2Gt, X_ONE, XA_2t, D_2_0, D_2_t},
    {2, 3, 0, 1, XC_C, XE_4C0, XE_4Ct, X_ONE, XA_4t, D_4_0, D_4_t},
    {2, 3, 1, 2, XC_C, XE_4Ct, XE_4C2, XA_4t, XA_42, D_4_t, D_4_2},
    // k = 3
    {3, 3, 0, 1, XC_C, XE_4C0, XE_4Ct, X_ONE, XA_4t, D_4_0, D_4_t},
    {3, 3, 1, 2, XC_C, XE_4Ct, XE_4C2, XA_4t, XA_42, D_4_t, D_4_2},
};

// ---- OU parameters and the parameter-only constants of one step -----------------------
// Everything here depends on the 7 propagator parameters only, so a kernel forms it once
// instead of once per step (values identical: the same expressions).
struct OU {
    double ml, gl, sl2, mq, gq, sq2, b;
    double r_gl, r_gq, gq2, gqq2, r_gq2, r_gqq2, gl2, r_gl2;
    double k_xl, k_xx, k_ll, k_qq;   // the sl2 / sq2 prefactors of cov_xl, cov_xx, cov_ll, cov_qq
};

// x^3 correctly rounded (but for ties within ~2^-100 relative): the exact square and cube as
// double-doubles (fma residuals), one rounding at the end.  pow(x, 3) in the reference
// (mean_cov_model.h:95) is glibc's pow, itself correctly rounded but for ~1e-3 of arguments
GGP_DEV double cube_cr(const double x)
{
    const double p = x * x, e1 = __builtin_fma(x, x, -p);
    const double q = p * x, e2 = __builtin_fma(p, x, -q);
    return q + __builtin_fma(e1, x, e2);
}

// a^k sqrt(a), k = 1..3, correctly rounded in the same sense: sqrt(a) = s + ds (s correctly
// rounded, ds from the exact residual a - s^2), a^k as a double-double, the product's error
// terms summed, one rounding.  GGP_EXACT's form of pow(a, k + 1/2) (mean_cov_model.h:33, 48, 66)
GGP_DEV double pow_half_cr(const double a, const int k)
{
    const double s = sqrt(a);
    const double ds = __builtin_fma(-s, s, a) * (0.5 / s);
    double h = a, l = 0.0;
    if (k >= 2) {
        const double p = a * a;
        l = __builtin_fma(a, a, -p);
        h = p;
    }
    if (k >= 3) {
        const double p = h * a;
        l = __builtin_fma(h, a, -p) + l * a;
        h = p;
    }
    const double P = h * s;
    return P + (__builtin_fma(h, s, -P) + (l * s + h * ds));
}

GGP_DEV OU make_ou(const double ml, const double gl, const double sl2, const double mq, const double gq,
                   const double sq2, const double b)
{
    OU P;
    P.ml = ml; P.gl = gl; P.sl2 = sl2; P.mq = mq; P.gq = gq; P.sq2 = sq2; P.b = b;
    P.r_gl = 1.0 / gl;
    P.r_gq = 1.0 / gq;
    P.gq2 = 2. * gq;
    P.gqq2 = 2. * (gq * gq);
    P.r_gq2 = 1.0 / P.gq2;
    P.r_gqq2 = 1.0 / P.gqq2;
    P.gl2 = gl * gl;
    P.r_gl2 = 1.0 / P.gl2;
    P.k_xl = sl2 / (2 * (gl * gl));
    P.k_xx = sl2 / (2 * cube_cr(gl));
    P.k_ll = sl2 / (2 * gl);
    P.k_qq = rdiv(sq2, 2 * gq, P.r_gq2);
    return P;
}

// ---- per-step scalars ------------------------------------------------------------------
struct Step {
    // z(t0) state (mean_cov_model.h:221-235) and OU parameters (already sign-flipped for _r)
    double bx, bg, bl, bq, Cxx, Cxg, Cxl, Cxq, Cgg, Cgl, Cgq, Cll, Clq, Cqq;
    double ml, gl, sl2, mq, gq, sq2, b, t, t2;
    // derived
    double a, two_sa, m2sa, two_a, four_a, four_aa;
    double B0, B1, B2, B3, B4, B5;                     // B1..B6
    double c0, c1, c2, c3, c4, c5, c6, c7, c8, c9;     // cA cB cJ cG cC cD cE cF cI cH
    double r_two_sa, r_four_a, r_gl, r_gq;
    double gq2, gqq2, r_gq2, r_gqq2, gl2, r_gl2, k_xl, k_xx, k_ll, k_qq;
    // indexed operands of the tasks (selects: no dynamic register indexing)
    GGP_DEV double Bv(int i) const;
    GGP_DEV double Cv(int i) const;
    GGP_DEV double Tv(int i) const;
    GGP_DEV double SVv(int s) const;
};

GGP_DEV void step_init(Step &S, const double *m, const double *C, const double t, const OU &P)
{
    GGP_CONTRACT
    const double ml = P.ml, gl = P.gl, gq = P.gq, b = P.b;
    S.bx = m[0]; S.bg = m[1]; S.bl = m[2]; S.bq = m[3];
    S.Cxx = C[0]; S.Cxg = C[1]; S.Cxl = C[2]; S.Cxq = C[3];
    S.Cgg = C[5]; S.Cgl = C[6]; S.Cgq = C[7];
    S.Cll = C[10]; S.Clq = C[11]; S.Cqq = C[15];
    S.ml = ml; S.gl = gl; S.sl2 = P.sl2; S.mq = P.mq; S.gq = gq; S.sq2 = P.sq2; S.b = b;
    S.r_gl = P.r_gl; S.r_gq = P.r_gq;
    S.gq2 = P.gq2; S.gqq2 = P.gqq2; S.r_gq2 = P.r_gq2; S.r_gqq2 = P.r_gqq2;
    S.gl2 = P.gl2; S.r_gl2 = P.r_gl2;
    S.k_xl = P.k_xl; S.k_xx = P.k_xx; S.k_ll = P.k_ll; S.k_qq = P.k_qq;
    S.t = t;
    S.t2 = 2 * t;
    const double a = S.Cll / 2.;
    const double sa = sqrt(a);
    S.a = a;
    S.two_sa = 2. * sa;
    S.m2sa = -2. * sa;
    S.two_a = 2. * a;
    S.four_a = 4. * a;
    S.four_aa = 4 * (a * a);
    const double bx = S.bx, Cxx = S.Cxx, bl = S.bl, Cxl = S.Cxl;
    S.B0 = b + bl + Cxl;
    S.B1 = b + bl + Cxl - gq;
    S.B2 = b + bl + 2 * Cxl;
    S.B3 = b + bl + 2 * Cxl - gq;
    S.B4 = b + bl + Cxl + gq;
    S.B5 = b + bl + 2 * Cxl + gq;
    S.c0 = bx + Cxx / 2. - b * t;                  // cA
    S.c1 = bx + Cxx / 2. - b * t - gl * t;         // cB
    S.c2 = bx + Cxx / 2. - b * t - gq * t;         // cJ
    S.c3 = bx + Cxx / 2. - 2 * b * t;              // cG
    S.c4 = 2 * (bx + Cxx - b * t);                 // cC
    S.c5 = 2 * bx + 2 * Cxx - (2 * b + gq) * t;    // cD
    S.c6 = 2 * bx + 2 * Cxx - 2 * b * t;           // cE
    S.c7 = 2 * bx + 2 * Cxx - 2 * b * t + gq * t;  // cF
    S.c8 = -b * t + bx + Cxx / 2. - gq * t;        // cI
    S.c9 = 2 * bx + 2 * Cxx - 2 * b * t - 2 * gq * t;  // cH
    S.r_two_sa = frcp(S.two_sa);   // rdiv seeds only
    S.r_four_a = frcp(S.four_a);
}

// select without dynamic register indexing (compile-time index folds to one operand)
GGP_DEV double pickB(const Step &S, int i)
{
    return i == 0 ? S.B0 : i == 1 ? S.B1 : i == 2 ? S.B2 : i == 3 ? S.B3 : i == 4 ? S.B4 : S.B5;
}
GGP_DEV double pickC(const Step &S, int i)
{
    return i == 0 ? S.c0 : i == 1 ? S.c1 : i == 2 ? S.c2 : i == 3 ? S.c3 : i == 4 ? S.c4
         : i == 5 ? S.c5 : i == 6 ? S.c6 : i == 7 ? S.c7 : i == 8 ? S.c8 : S.c9;
}
GGP_DEV double pickT(const Step &S, int i) { return i == 0 ? 0.0 : i == 1 ? S.t : S.t2; }
// the exponents s of exp(s t) (mean_cov_model.h: b, b + gl, 2b, b + gq, -gl, -gq; then the
// product factors' -b, gq)
constexpr int NSV = 8;
GGP_DEV double pickSV(const Step &S, int s)
{
    return s == 0 ? S.b : s == 1 ? S.b + S.gl : s == 2 ? 2 * S.b : s == 3 ? S.b + S.gq : s == 4 ? -S.gl
         : s == 5 ? -S.gq : s == 6 ? -S.b : S.gq;
}
GGP_DEV double Step::Bv(int i) const { return pickB(*this, i); }
GGP_DEV double Step::Cv(int i) const { return pickC(*this, i); }
GGP_DEV double Step::Tv(int i) const { return pickT(*this, i); }
GGP_DEV double Step::SVv(int s) const { return pickSV(*this, s); }

// ---- the step block in LDS (group schedule) ----------------------------------------------
// One lane forms the Step and stores it; the task lanes read their operands by index (one
// LDS load instead of a select chain) and the Step does not stay live in registers across
// the task stages.  Values are copies, so results are bitwise those of the register form.
enum {
    SB_B = 0, SB_C = SB_B + 6, SB_T = SB_C + 10, SB_SV = SB_T + 3,
    SB_A = SB_SV + NSV, SB_TWO_A, SB_FOUR_A, SB_R_FOUR_A, SB_TWO_SA, SB_R_TWO_SA, SB_M2SA, SB_FOUR_AA,
    SB_STATE,                         // bx bg bl bq Cxx Cxg Cxl Cxq Cgg Cgl Cgq Cll Clq Cqq
    SB_N = SB_STATE + 14
};
enum { OU_N = 19 };                   // the OU struct, once per workgroup

GGP_DEV void store_ou(const OU &P, double *o)
{
    const double v[OU_N] = {P.ml, P.gl, P.sl2, P.mq, P.gq, P.sq2, P.b, P.r_gl, P.r_gq, P.gq2, P.gqq2,
                            P.r_gq2, P.r_gqq2, P.gl2, P.r_gl2, P.k_xl, P.k_xx, P.k_ll, P.k_qq};
#pragma unroll
    for (int k = 0; k < OU_N; ++k) o[k] = v[k];
}

GGP_DEV OU load_ou(const double *o)
{
    OU P;
    P.ml = o[0]; P.gl = o[1]; P.sl2 = o[2]; P.mq = o[3]; P.gq = o[4]; P.sq2 = o[5]; P.b = o[6];
    P.r_gl = o[7]; P.r_gq = o[8]; P.gq2 = o[9]; P.gqq2 = o[10]; P.r_gq2 = o[11]; P.r_gqq2 = o[12];
    P.gl2 = o[13]; P.r_gl2 = o[14]; P.k_xl = o[15]; P.k_xx = o[16]; P.k_ll = o[17]; P.k_qq = o[18];
    return P;
}

GGP_DEV void store_step(const Step &S, double *sb)
{
#pragma unroll
    for (int i = 0; i < 6; ++i) sb[SB_B + i] = pickB(S, i);
#pragma unroll
    for (int i = 0; i < 10; ++i) sb[SB_C + i] = pickC(S, i);
#pragma unroll
    for (int i = 0; i < 3; ++i) sb[SB_T + i] = pickT(S, i);
#pragma unroll
    for (int i = 0; i < NSV; ++i) sb[SB_SV + i] = pickSV(S, i);
    sb[SB_A] = S.a; sb[SB_TWO_A] = S.two_a; sb[SB_FOUR_A] = S.four_a; sb[SB_R_FOUR_A] = S.r_four_a;
    sb[SB_TWO_SA] = S.two_sa; sb[SB_R_TWO_SA] = S.r_two_sa; sb[SB_M2SA] = S.m2sa; sb[SB_FOUR_AA] = S.four_aa;
    const double st[14] = {S.bx, S.bg, S.bl, S.bq, S.Cxx, S.Cxg, S.Cxl, S.Cxq, S.Cgg, S.Cgl, S.Cgq, S.Cll, S.Clq, S.Cqq};
#pragma unroll
    for (int k = 0; k < 14; ++k) sb[SB_STATE + k] = st[k];
}

// the full Step back from the block (the outputs stage); unused fields are dead loads
GGP_DEV void load_step(Step &S, const double *sb, const double *ou)
{
    const OU P = load_ou(ou);
    S.ml = P.ml; S.gl = P.gl; S.sl2 = P.sl2; S.mq = P.mq; S.gq = P.gq; S.sq2 = P.sq2; S.b = P.b;
    S.r_gl = P.r_gl; S.r_gq = P.r_gq;
    S.gq2 = P.gq2; S.gqq2 = P.gqq2; S.r_gq2 = P.r_gq2; S.r_gqq2 = P.r_gqq2;
    S.gl2 = P.gl2; S.r_gl2 = P.r_gl2;
    S.k_xl = P.k_xl; S.k_xx = P.k_xx; S.k_ll = P.k_ll; S.k_qq = P.k_qq;
    S.B0 = sb[SB_B]; S.B1 = sb[SB_B + 1]; S.B2 = sb[SB_B + 2]; S.B3 = sb[SB_B + 3]; S.B4 = sb[SB_B + 4];
    S.B5 = sb[SB_B + 5];
    S.c0 = sb[SB_C]; S.c1 = sb[SB_C + 1]; S.c2 = sb[SB_C + 2]; S.c3 = sb[SB_C + 3]; S.c4 = sb[SB_C + 4];
    S.c5 = sb[SB_C + 5]; S.c6 = sb[SB_C + 6]; S.c7 = sb[SB_C + 7]; S.c8 = sb[SB_C + 8]; S.c9 = sb[SB_C + 9];
    S.t = sb[SB_T + 1]; S.t2 = sb[SB_T + 2];
    S.a = sb[SB_A]; S.two_a = sb[SB_TWO_A]; S.four_a = sb[SB_FOUR_A]; S.r_four_a = sb[SB_R_FOUR_A];
    S.two_sa = sb[SB_TWO_SA]; S.r_two_sa = sb[SB_R_TWO_SA]; S.m2sa = sb[SB_M2SA]; S.four_aa = sb[SB_FOUR_AA];
    S.bx = sb[SB_STATE]; S.bg = sb[SB_STATE + 1]; S.bl = sb[SB_STATE + 2]; S.bq = sb[SB_STATE + 3];
    S.Cxx = sb[SB_STATE + 4]; S.Cxg = sb[SB_STATE + 5]; S.Cxl = sb[SB_STATE + 6]; S.Cxq = sb[SB_STATE + 7];
    S.Cgg = sb[SB_STATE + 8]; S.Cgl = sb[SB_STATE + 9]; S.Cgq = sb[SB_STATE + 10]; S.Cll = sb[SB_STATE + 11];
    S.Clq = sb[SB_STATE + 12]; S.Cqq = sb[SB_STATE + 13];
}

// task operand view of the block: the members the task bodies use, indexed loads for the rest
struct StepL {
    const double *sb;
    double a, two_a, four_a, r_four_a, two_sa, r_two_sa, m2sa, four_aa, t;
    GGP_DEV explicit StepL(const double *p)
        : sb(p), a(p[SB_A]), two_a(p[SB_TWO_A]), four_a(p[SB_FOUR_A]), r_four_a(p[SB_R_FOUR_A]),
          two_sa(p[SB_TWO_SA]), r_two_sa(p[SB_R_TWO_SA]), m2sa(p[SB_M2SA]), four_aa(p[SB_FOUR_AA]),
          t(p[SB_T + 1]) {}
    GGP_DEV double Bv(int i) const { return sb[SB_B + i]; }
    GGP_DEV double Cv(int i) const { return sb[SB_C + i]; }
    GGP_DEV double Tv(int i) const { return sb[SB_T + i]; }
    GGP_DEV double SVv(int s) const { return sb[SB_SV + s]; }
};

// z = (B + 2a t_i) / (2 sqrt a)  (t_i = 0: B / (2 sqrt a)).  ST = Step (registers) or StepL.
template <class ST>
GGP_DEV double zval(const ST &S, int iB, int it)
{
    GGP_CONTRACT
    const double B = S.Bv(iB);
    const double num = it == 0 ? B : B + S.two_a * S.Tv(it);
    return rdiv(num, S.two_sa, S.r_two_sa);
}

template <class ST>
GGP_DEV double exp_arg_body(const ST &S, const XTask T)
{
    GGP_CONTRACT
    // branch-free: every candidate argument is formed from selected operands and the kind
    // picks one, so lanes holding different kinds do not serialise (group schedule)
    const double ti = S.Tv(T.it);
    const double B = S.Bv(T.iB);
    const double c = S.Cv(T.ic);
    const double sv = S.SVv(T.iB);
    const double n = rdiv(-(B * B), S.four_a, S.r_four_a);
    const double zn = T.it == 0 ? B : B + S.two_a * ti;
    const double z = rdiv(zn, S.two_sa, S.r_two_sa);
    const double argA = ti * (B + S.a * ti);
    const double argS = sv * S.t;
    const double argE = n + c + z * z;
    const double argZ = S.a * (ti * ti) + B * ti + c;
    return T.kind == KX_C ? c : T.kind == KX_A ? argA : T.kind == KX_S ? argS
         : T.kind == KX_E ? argE : argZ;
}

#ifdef GGP_HOST_SIM
// diagnostic hooks (tools/parity_attrib.cpp): the exponential the lane bodies take (glibc's, or
// exp_ocml's emulation), and pow(a, k + 1/2) as the reference forms it instead of a^k sqrt(a)
extern double (*ggp_hs_exp)(double);
extern int ggp_hs_pow_libm;
#endif
#if defined(GGP_EXACT)
#define GGP_LANE_EXP(v, tab) exp_glibc((v), exp_tab_of(tab))
#elif defined(GGP_HOST_SIM)
#define GGP_LANE_EXP(v, tab) ggp_hs_exp(v)
#else
#define GGP_LANE_EXP(v, tab) exp(v)
#endif

// tab: the propagator's table (kPropTabN doubles: the Dawson rows, then the exp table)
template <class ST>
GGP_DEV double exp_body(const ST &S, const XTask T, const double *tab)
{
    (void)tab;
    return GGP_LANE_EXP(exp_arg_body(S, T), tab);
}

GGP_DEV double exp_task(const Step &S, int j, const double *tab) { return exp_body(S, kXT[j], tab); }

template <class ST>
GGP_DEV double dawson_body(const ST &S, const DTask T, const double *tab)
{
    return ggp_dawson_tab(zval(S, T.iB, T.it), tab);
}

GGP_DEV double dawson_task(const Step &S, int d, const double *tab) { return dawson_body(S, kDT[d], tab); }

// the computed list's task descriptors, packed (pack_x's layout), for runtime-indexed loops
struct PackedXC {
    uint32_t w[NXC];
};
constexpr PackedXC make_packed_xc()
{
    PackedXC p{};
    for (int k = 0; k < NXC; ++k)
        p.w[k] = (uint32_t)kXC.T[k].kind | (uint32_t)kXC.T[k].iB << 8 | (uint32_t)kXC.T[k].ic << 16 |
                 (uint32_t)kXC.T[k].it << 24;
    return p;
}
#if defined(GGP_HOST_SIM)
static const PackedXC kXCPacked = make_packed_xc();
#else
static __constant__ const PackedXC kXCPacked = make_packed_xc();
#endif

// task descriptors packed in one register word (group schedule: loaded once per kernel)
GGP_DEV uint32_t pack_x(const XTask T) { return T.kind | T.iB << 8 | T.ic << 16 | (uint32_t)T.it << 24; }
GGP_DEV XTask unpack_x(const uint32_t w)
{
    return XTask{(unsigned char)(w & 0xff), (unsigned char)(w >> 8 & 0xff), (unsigned char)(w >> 16 & 0xff),
                 (unsigned char)(w >> 24)};
}
GGP_DEV uint32_t pack_d(const DTask T) { return T.iB | T.it << 8; }
GGP_DEV DTask unpack_d(const uint32_t w) { return DTask{(unsigned char)(w & 0xff), (unsigned char)(w >> 8 & 0xff)}; }

// the three tauint denominators 4 a^1.5, 8 a^2.5, 16 a^3.5.  pow(a, k + 1/2) is formed as
// a^k * sqrt(a) (sqrt correctly rounded, <= 2 ulp from glibc's pow; the total
// log-likelihood moves by ~1e-11 relative, DESIGN.md "Parity") -- ~10x cheaper than ocml pow.
template <class ST>
GGP_DEV double pow_task(const ST &S, int p)
{
    const double sa = S.two_sa * 0.5;           // sqrt(a), exact
    const double a = S.a;
#ifdef GGP_HOST_SIM
    if (ggp_hs_pow_libm) return p == 0 ? 4. * pow(a, 1.5) : p == 1 ? 8. * pow(a, 2.5) : 16. * pow(a, 3.5);
#endif
    if constexpr (kExact) return p == 0 ? 4. * pow_half_cr(a, 1) : p == 1 ? 8. * pow_half_cr(a, 2) : 16. * pow_half_cr(a, 3);
    return p == 0 ? 4. * (a * sa) : p == 1 ? 8. * ((a * a) * sa) : 16. * (((a * a) * a) * sa);
}
constexpr int NPW = 6;   // 3 denominators + 3 reciprocals

// ---- tauint from its pieces (mean_cov_model.h:9-67) ----------------------------------
// PW = {4 a^1.5, 8 a^2.5, 16 a^3.5, and their reciprocals}
template <class ST, class XA, class DA, class PA>
GGP_DEV double tau_body(const ST &S, const ITask T, const XA &X, const DA &Dw, const PA &PW)
{
    GGP_CONTRACT
    const double D0 = Dw[T.d0], D1 = Dw[T.d1];
    if (T.k == 0) {   // zerotauint
        const double Z0 = X[T.x0], Z1 = X[T.x1];
        const double x = 2. * (-Z0 * D0 + Z1 * (D1));
        return rdiv(x, S.two_sa, S.r_two_sa);
    }
    const double B = S.Bv(T.iB);
    const double ec = X[T.xc], E0 = X[T.x0], E1 = X[T.x1], ea0 = X[T.xa0], ea1 = X[T.xa1];
    if (T.k == 1) {   // onetauint
        const double x = (S.m2sa * ec * (ea0 - ea1) + B * 2. * (E0 * D0 - E1 * D1));
        return rdiv(x, PW[0], PW[3]);
    }
    const double t0 = S.Tv(T.it0), t1 = S.Tv(T.it1);
    if (T.k == 2) {   // twotauint
        const double x = (S.two_sa * ec * (ea0 * (B - S.two_a * t0) - ea1 * (B - S.two_a * t1))
                          + (E0 * (S.two_a - B * B) * 2. * D0 + E1 * (-S.two_a + B * B) * 2. * D1));
        return rdiv(x, PW[1], PW[4]);
    }
    // treetauint
    const double a = S.a;
    const double x = (S.m2sa * ec
                      * ((B * B) * (ea0 - ea1) - S.two_a * ea0 * (2. + B * t0) + S.two_a * ea1 * (2 + B * t1)
                         + S.four_aa * (ea0 * (t0 * t0) - ea1 * (t1 * t1))))
                     + E0 * B * (-6. * a + B * B) * 2. * D0
                     - E1 * B * (-6 * a + B * B) * 2. * D1;
    return rdiv(x, PW[2], PW[5]);
}

// One expression for all four tauint kinds (the wave schedule: no divergence between k):
//   x = S1 * ec * (ea0 P(t0) - ea1 P(t1)) + Q (E0 D0 - E1 D1),  I = x / den_k
//   k=0: S1 = 0, Q = -2, den = 2 sqrt a   (E = Z slots)   == 2 (-Z0 D0 + Z1 D1) bitwise
//   k=1: S1 = -2 sqrt a, P = 1, Q = 2 B                  == tau_body bitwise
//   k=2: S1 = 2 sqrt a, P = B - 2a t, Q = 2 (2a - B^2)   (E-term grouping differs: ulps)
//   k=3: S1 = -2 sqrt a, P = B^2 - 4a - 2aB t + 4a^2 t^2, Q = 2 B (B^2 - 6a)  (ulps)
template <class ST, class XA, class DA, class PA>
GGP_DEV double tau_unified(const ST &S, const ITask T, const XA &X, const DA &Dw, const PA &PW)
{
    const double D0 = Dw[T.d0], D1 = Dw[T.d1];
    const double E0 = X[T.x0], E1 = X[T.x1];
    const double B = S.Bv(T.iB);
    const double t0 = S.Tv(T.it0), t1 = S.Tv(T.it1);
    const int k = T.k;
    const double BB = B * B;
    const double al = k == 1 ? 1.0 : k == 2 ? B : BB - 2. * S.two_a;
    const double be = k == 1 ? 0.0 : k == 2 ? -S.two_a : -S.two_a * B;
    const double ga = k == 3 ? S.four_aa : 0.0;
    const double P0 = al + t0 * (be + ga * t0), P1 = al + t1 * (be + ga * t1);
    const double Q = k == 0 ? -2.0 : k == 1 ? B * 2. : k == 2 ? (S.two_a - BB) * 2. : B * (-6. * S.a + BB) * 2.;
    const double S1 = k == 2 ? S.two_sa : S.m2sa;
    const double ec = X[T.xc], ea0 = X[T.xa0], ea1 = X[T.xa1];
    const double dterm = Q * (E0 * D0 - E1 * D1);
    const double x = k == 0 ? dterm : S1 * ec * (ea0 * P0 - ea1 * P1) + dterm;
    const double den = k == 0 ? S.two_sa : PW[k - 1], rden = k == 0 ? S.r_two_sa : PW[k + 2];
    return rdiv(x, den, rden);
}

template <class XA, class DA, class PA>
GGP_DEV double tau_task(const Step &S, int j, const XA &X, const DA &Dw, const PA &PW)
{
    return tau_body(S, kIT[j], X, Dw, PW);
}

// ---- the outputs: new mean and covariance (mean_cov_model.h:73-208) -------------------
// PARTS selects the output groups a caller forms (the lane-pair schedule splits them over its
// waves): 1 = cov_xg; 2 = cov_xl, cov_xq, cov_gl, cov_xx, cov_ll; 4 = cov_gq, cov_lq, cov_qq;
// 8 = cov_gg; the means always.  Outputs of a group not formed are left 0.
template <int PARTS = 15, class IA, class XA>
GGP_DEV void outputs(const Step &S, const IA &I, const XA &X, double *m, double *C)
{
    GGP_CONTRACT
    const double t = S.t, bx = S.bx, bg = S.bg, bl = S.bl, bq = S.bq;
    const double Cxx = S.Cxx, Cxg = S.Cxg, Cxl = S.Cxl, Cxq = S.Cxq, Cgg = S.Cgg, Cgl = S.Cgl;
    const double Cgq = S.Cgq, Cll = S.Cll, Clq = S.Clq, Cqq = S.Cqq;
    const double ml = S.ml, gl = S.gl, mq = S.mq, gq = S.gq, sq2 = S.sq2;
    const double rgl = S.r_gl, rgq = S.r_gq;
    const double ebt = X[XS_bt], ebglt = X[XS_bglt], e2bt = X[XS_2bt], ebgqt = X[XS_bgqt];
    const double egl = X[XS_gl], egq = X[XS_gq];
    // rdiv seeds only (frcp)
    const double r_ebt = frcp(ebt), r_ebglt = frcp(ebglt), r_ebgqt = frcp(ebgqt);
    const double ebt_gl = ebt * gl, ebglt_gl = ebglt * gl;
    const double r_ebt_gl = frcp(ebt_gl), r_ebglt_gl = frcp(ebglt_gl);
    const double gq2 = S.gq2, gqq2 = S.gqq2;
    const double r_gq2 = S.r_gq2, r_gqq2 = S.r_gqq2;
#define DGL(x) rdiv((x), gl, rgl)
#define DGQ(x) rdiv((x), gq, rgq)

    double nm[4];
    nm[0] = bx + ml * t + DGL((bl - ml) * (1 - egl));
    nm[1] = rdiv(bg, ebt, r_ebt) + Clq * I[O_2A] + mq * I[Z_1A] + (bq + Cxq - mq) * I[Z_2A];
    nm[2] = ml + (bl - ml) * egl;
    nm[3] = mq + (bq - mq) * egq;

    double nxg = 0, nxl = 0, nxq = 0, ngl = 0, nxx = 0, nll = 0, ngq = 0, ngg = 0, nlq = 0, nqq = 0;
    if constexpr ((PARTS & 1) != 0) {
    // cov_xg (mean_cov_model.h:97-115)
    nxg =
        rdiv(bg * bx, ebt, r_ebt) + rdiv(Cxg, ebt, r_ebt) + rdiv(bg * bl, ebt_gl, r_ebt_gl)
        + rdiv(Cgl, ebt_gl, r_ebt_gl) - rdiv(bg * bl, ebglt_gl, r_ebglt_gl) - rdiv(Cgl, ebglt_gl, r_ebglt_gl)
        - rdiv(bg * ml, ebt_gl, r_ebt_gl) + rdiv(bg * ml, ebglt_gl, r_ebglt_gl) + rdiv(bg * ml * t, ebt, r_ebt)
        + (Cxl * mq + DGL(Cll * mq)) * I[O_1A]
        - DGL(Cll * mq * I[O_1B])
        + (bx * Clq + bq * Cxl + Cxl * Cxq + Clq * Cxx + DGL(bq * Cll) + DGL(bl * Clq) + DGL(Clq * Cxl)
           + DGL(Cll * Cxq) - DGL(Clq * ml) - Cxl * mq - DGL(Cll * mq) + Clq * ml * t) * I[O_2A]
        + (-(DGL(bq * Cll)) - DGL(bl * Clq) - DGL(Clq * Cxl) - DGL(Cll * Cxq) + DGL(Clq * ml)
           + DGL(Cll * mq)) * I[O_2B]
        + (Clq * Cxl + DGL(Cll * Clq)) * I[T_2A]
        - DGL(Cll * Clq * I[T_2B])
        + (bx * mq + Cxx * mq + DGL(bl * mq) + DGL(Cxl * mq) - DGL(ml * mq) + ml * mq * t) * I[Z_1A]
        + (-(DGL(bl * mq)) - DGL(Cxl * mq) + DGL(ml * mq)) * I[Z_1B]
        + (bq * bx + Cxq + bx * Cxq + bq * Cxx + Cxq * Cxx + DGL(bl * bq) + DGL(Clq) + DGL(bq * Cxl)
           + DGL(bl * Cxq) + DGL(Cxl * Cxq) - DGL(bq * ml) - DGL(Cxq * ml) - bx * mq - Cxx * mq
           - DGL(bl * mq) - DGL(Cxl * mq) + DGL(ml * mq) + bq * ml * t + Cxq * ml * t - ml * mq * t) * I[Z_2A]
        + (-(DGL(bl * bq)) - DGL(Clq) - DGL(bq * Cxl) - DGL(bl * Cxq) - DGL(Cxl * Cxq) + DGL(bq * ml)
           + DGL(Cxq * ml) + DGL(bl * mq) + DGL(Cxl * mq) - DGL(ml * mq)) * I[Z_2B]
        - nm[1] * nm[0];
    }
    if constexpr ((PARTS & 2) != 0) {
    // cov_xl, cov_xq (mean_cov_model.h:117-123)
    nxl = S.k_xl * ((1 - egl) * (1 - egl))
                       + DGL(Cll * egl * (1 - egl)) + Cxl * egl;
    nxq = DGL(Clq * (1 - egl) * egq) + Cxq * egq;

    // cov_gl (mean_cov_model.h:172-181)
    ngl =
        rdiv(bg * bl, ebglt, r_ebglt) + rdiv(Cgl, ebglt, r_ebglt) + rdiv(bg * ml, ebt, r_ebt)
        - rdiv(bg * ml, ebglt, r_ebglt)
        + Cll * mq * I[O_1B] + Clq * ml * I[O_2A]
        + (bq * Cll + bl * Clq + Clq * Cxl + Cll * Cxq - Clq * ml - Cll * mq) * I[O_2B]
        + Cll * Clq * I[T_2B] + ml * mq * I[Z_1A]
        + (bl * mq + Cxl * mq - ml * mq) * I[Z_1B]
        + (bq * ml + Cxq * ml - ml * mq) * I[Z_2A]
        + (bl * bq + Clq + bq * Cxl + bl * Cxq + Cxl * Cxq - bq * ml - Cxq * ml - bl * mq - Cxl * mq
           + ml * mq) * I[Z_2B]
        - nm[1] * nm[2];

    // cov_xx, cov_ll (mean_cov_model.h:93-95, 198-200)
    nxx = rdiv(Cll * ((1 - egl) * (1 - egl)), S.gl2, S.r_gl2) + rdiv(2 * Cxl * (1 - egl), gl, rgl) + Cxx
          + S.k_xx * (2 * gl * t - 3 + 4 * egl - (egl * egl));
    nll = Cll * (egl * egl) + S.k_ll * (1 - (egl * egl));
    }
    if constexpr ((PARTS & 4) != 0) {
    // cov_gq (mean_cov_model.h:183-196)
    ngq =
        rdiv(bg * bq, ebgqt, r_ebgqt) + rdiv(Cgq, ebgqt, r_ebgqt) + rdiv(bg * mq, ebt, r_ebt)
        - rdiv(bg * mq, ebgqt, r_ebgqt)
        + Clq * mq * I[O_1J] + Clq * mq * I[O_2A]
        + (2 * bq * Clq + 2 * Clq * Cxq - 2 * Clq * mq) * I[O_2J]
        + (Clq * Clq) * I[T_2J] + (mq * mq) * I[Z_1A]
        + (bq * mq + Cxq * mq - (mq * mq)) * I[Z_1J]
        + (bq * mq + Cxq * mq - (mq * mq)) * I[Z_2A]
        - rdiv(sq2 * I[Z_2I], gq2, r_gq2)
        + ((bq * bq) + Cqq + 2 * bq * Cxq + (Cxq * Cxq) - 2 * bq * mq - 2 * Cxq * mq + (mq * mq)) * I[Z_2J]
        + rdiv(sq2 * I[Z_5I], gq2, r_gq2)
        - nm[1] * nm[3];

    // cov_lq, cov_qq (mean_cov_model.h:202-208)
    nlq = Clq * egl * egq;
    nqq = S.k_qq * (1 - (egq * egq)) + Cqq * (egq * egq);
    }
    if constexpr ((PARTS & 8) != 0) {
    // cov_gg (mean_cov_model.h:125-170)
    const double k17 = DGQ(2 * bq * mq) + DGQ(4 * Cxq * mq) - DGQ(2 * (mq * mq));
    const double k19 = DGQ(-2 * bq * mq) - DGQ(4 * Cxq * mq) + DGQ(2 * (mq * mq));
    ngg =
        ((bg * bg) + Cgg) / e2bt
        + 2 * Cgl * mq * I[O_1G]
        + DGQ(mq * (2 * Clq + gq * mq) * I[O_3C])
        + 2 * (bq * Cgl + bg * Clq + Clq * Cxg + Cgl * Cxq - Cgl * mq) * I[O_2G]
        + DGQ(((bq * bq) * gq + Cqq * gq + 4 * bq * Cxq * gq + 4 * (Cxq * Cxq) * gq - 2 * Clq * mq
               - 2 * bq * gq * mq - 4 * Cxq * gq * mq + gq * (mq * mq)) * I[O_4C])
        - (mq * mq) * I[O_3C2]
        - DGQ(2 * Clq * mq * I[O_3D2])
        - rdiv(sq2 * I[O_4E], gq2, r_gq2)
        + rdiv(sq2 * I[O_4E2], gq2, r_gq2)
        + (-(bq * bq) - Cqq - 4 * bq * Cxq - 4 * (Cxq * Cxq) + 2 * bq * mq + 4 * Cxq * mq - (mq * mq)
           + 4 * bq * Clq * t + 8 * Clq * Cxq * t - 4 * Clq * mq * t) * I[O_4C2]
        + DGQ(2 * Clq * mq * I[O_4F2])
        + (Clq * Clq) * I[H_4C]
        - (Clq * Clq) * I[H_4C2]
        + 2 * Cgl * Clq * I[T_2G]
        + (2 * bq * Clq + 4 * Clq * Cxq - 2 * Clq * mq) * I[T_4C]
        + (-2 * bq * Clq - 4 * Clq * Cxq + 2 * Clq * mq + 2 * (Clq * Clq) * t) * I[T_4C2]
        + (2 * bg * mq + 2 * Cxg * mq) * I[Z_1G]
        + k17 * I[Z_3C]
        + (2 * bg * bq + 2 * Cgq + 2 * bq * Cxg + 2 * bg * Cxq + 2 * Cxg * Cxq - 2 * bg * mq
           - 2 * Cxg * mq) * I[Z_2G]
        + k19 * I[Z_4C]
        + rdiv(sq2 * I[Z_3E], gqq2, r_gqq2)
        + rdiv(sq2 * I[Z_3E2], gqq2, r_gqq2)
        + 2 * (mq * mq) * t * I[Z_3C2]
        + k19 * I[Z_3D2]
        - rdiv(sq2 * I[Z_4E], gqq2, r_gqq2)
        - DGQ(sq2 * t * I[Z_4E2])
        + (2 * (bq * bq) * t + 2 * Cqq * t + 8 * bq * Cxq * t + 8 * (Cxq * Cxq) * t - 4 * bq * mq * t
           - 8 * Cxq * mq * t + 2 * (mq * mq) * t) * I[Z_4C2]
        + k17 * I[Z_4F2]
        - rdiv(sq2 * I[Z_6H2], gqq2, r_gqq2)
        - (nm[1] * nm[1]);
    }

#undef DGL
#undef DGQ
    m[0] = nm[0]; m[1] = nm[1]; m[2] = nm[2]; m[3] = nm[3];
    C[0] = nxx;  C[1] = nxg;  C[2] = nxl;  C[3] = nxq;
    C[4] = nxg;  C[5] = ngg;  C[6] = ngl;  C[7] = ngq;
    C[8] = nxl;  C[9] = ngl;  C[10] = nll; C[11] = nlq;
    C[12] = nxq; C[13] = ngq; C[14] = nlq; C[15] = nqq;
}

// ---- cross_cov_model (mean_cov_model.h:380-432): K_{n+1,n} from the same step's integrals
// (its I0/I1/I2 calls are the O_1A, O_2A, T_2A, Z_1A, Z_2A integrals of mean_cov_model) ----
template <class IA, class XA>
GGP_DEV void cross_outputs(const Step &S, const IA &I, const XA &X, double *K)
{
    GGP_CONTRACT
    const double bx = S.bx, bg = S.bg, bl = S.bl, bq = S.bq;
    const double Cxx = S.Cxx, Cxg = S.Cxg, Cxl = S.Cxl, Cxq = S.Cxq, Cgg = S.Cgg, Cgl = S.Cgl;
    const double Cgq = S.Cgq, Cll = S.Cll, Clq = S.Clq, Cqq = S.Cqq;
    const double gl = S.gl, mq = S.mq, rgl = S.r_gl;
    const double ebt = X[XS_bt], egl = X[XS_gl], egq = X[XS_gq];
    const double r_ebt = frcp(ebt);   // rdiv seed
    // nm(1): mean_g at the end of the step, the same expression as outputs()
    const double nm1 = rdiv(bg, ebt, r_ebt) + Clq * I[O_2A] + mq * I[Z_1A] + (bq + Cxq - mq) * I[Z_2A];
    K[0] = Cxx + rdiv(Cxl * (1 - egl), gl, rgl);
    K[1] = Cxg + rdiv(Cgl * (1 - egl), gl, rgl);
    K[2] = Cxl + rdiv(Cll * (1 - egl), gl, rgl);
    K[3] = Cxq + rdiv(Clq * (1 - egl), gl, rgl);
    K[4] = rdiv(bg * bx, ebt, r_ebt) + rdiv(Cxg, ebt, r_ebt) + Cxl * mq * I[O_1A]
           + (bx * Clq + bq * Cxl + Cxl * Cxq + Clq * Cxx - Cxl * mq) * I[O_2A] + Clq * Cxl * I[T_2A]
           + (bx * mq + Cxx * mq) * I[Z_1A]
           + (bq * bx + Cxq + bx * Cxq + bq * Cxx + Cxq * Cxx - bx * mq - Cxx * mq) * I[Z_2A] - nm1 * bx;
    K[5] = rdiv(bg * bg, ebt, r_ebt) + rdiv(Cgg, ebt, r_ebt) + Cgl * mq * I[O_1A]
           + (bq * Cgl + bg * Clq + Clq * Cxg + Cgl * Cxq - Cgl * mq) * I[O_2A] + Cgl * Clq * I[T_2A]
           + (bg * mq + Cxg * mq) * I[Z_1A]
           + (bg * bq + Cgq + bq * Cxg + bg * Cxq + Cxg * Cxq - bg * mq - Cxg * mq) * I[Z_2A] - nm1 * bg;
    K[6] = rdiv(bg * bl, ebt, r_ebt) + rdiv(Cgl, ebt, r_ebt) + Cll * mq * I[O_1A]
           + (bq * Cll + bl * Clq + Clq * Cxl + Cll * Cxq - Cll * mq) * I[O_2A] + Cll * Clq * I[T_2A]
           + (bl * mq + Cxl * mq) * I[Z_1A]
           + (bl * bq + Clq + bq * Cxl + bl * Cxq + Cxl * Cxq - bl * mq - Cxl * mq) * I[Z_2A] - nm1 * bl;
    K[7] = rdiv(bg * bq, ebt, r_ebt) + rdiv(Cgq, ebt, r_ebt) + Clq * mq * I[O_1A]
           + (2 * bq * Clq + 2 * Clq * Cxq - Clq * mq) * I[O_2A] + (Clq * Clq) * I[T_2A]
           + (bq * mq + Cxq * mq) * I[Z_1A]
           + ((bq * bq) + Cqq + 2 * bq * Cxq + (Cxq * Cxq) - bq * mq - Cxq * mq) * I[Z_2A] - nm1 * bq;
    K[8] = Cxl * egl;  K[9] = Cgl * egl;  K[10] = Cll * egl; K[11] = Clq * egl;
    K[12] = Cxq * egq; K[13] = Cgq * egq; K[14] = Clq * egq; K[15] = Cqq * egq;
}

// ---- lane schedule: one lane runs every task of its own cell; the task descriptors are
// constexpr template arguments, so every array index is a compile-time constant and the
// arrays stay in registers.
template <size_t... J>
GGP_DEV void lane_exps(const Step &S, double *X, const double *tab, std::index_sequence<J...>)
{
    ((X[J] = exp_body(S, XTask{kXT[J].kind, kXT[J].iB, kXT[J].ic, kXT[J].it}, tab)), ...);
}
// GGP_EXACT's exponentials of the computed list, tasks [OFF, OFF + N): exp_glibc's main path in
// blocks of kExpBlock behind a scheduling barrier each (left free, the scheduler issues every
// table read of the step first and the lane kernels spill ~1300 registers), `big` collected
#ifndef GGP_EXP_BLOCK
#define GGP_EXP_BLOCK 8
#endif
constexpr int kExpBlock = GGP_EXP_BLOCK;
template <size_t B, size_t... K>
GGP_DEV void glibc_exp_block(const Step &S, double *Xc, const uint64_t *et, bool &big, std::index_sequence<K...>)
{
    ((Xc[B + K] = exp_glibc_main(exp_arg_body(S, XTask{kXC.T[B + K].kind, kXC.T[B + K].iB, kXC.T[B + K].ic,
                                                       kXC.T[B + K].it}), et, big)), ...);
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}
template <size_t OFF, size_t N, size_t... Bi>
GGP_DEV void glibc_exps(const Step &S, double *Xc, const uint64_t *et, bool &big, std::index_sequence<Bi...>)
{
    (glibc_exp_block<OFF + Bi * kExpBlock>(
         S, Xc, et, big, std::make_index_sequence<(N - Bi * kExpBlock < (size_t)kExpBlock ? N - Bi * kExpBlock : kExpBlock)>{}),
     ...);
}
template <size_t OFF, size_t N>
GGP_DEV void glibc_exps_all(const Step &S, double *Xc, const double *tab, bool &big)
{
    glibc_exps<OFF, N>(S, Xc, exp_tab_of(tab), big, std::make_index_sequence<(N + kExpBlock - 1) / kExpBlock>{});
}

// the computed exponentials kXC, tasks K: Xc[K] (the list's order; lane_expand puts them in
// their slots)
template <size_t... K>
GGP_DEV void lane_exps_c(const Step &S, double *Xc, const double *tab, std::index_sequence<K...>)
{
    ((Xc[K] = exp_body(S, XTask{kXC.T[K].kind, kXC.T[K].iB, kXC.T[K].ic, kXC.T[K].it}, tab)), ...);
}
// the same values with exp_lane (one compare per exponential instead of ocml's checks): faster
// where registers allow (the lane-pair schedule's share of the tasks: C4 shard 0.81 -> 0.79 ms),
// slower in the one-wave lane and smoother kernels, which keep lane_exps_c (tools/lane_ab.py)
// GGP_EXACT: exp_glibc's main path only; `cold` is set when an argument lies outside it (the
// caller then redoes the lane's step through propagate_lane_cold)
template <size_t OFF, size_t... K>
GGP_DEV void lane_exps_flagged(const Step &S, double *Xc, const double *tab, std::index_sequence<K...>, bool &cold)
{
    if constexpr (kExact) {
        glibc_exps_all<OFF, sizeof...(K)>(S, Xc, tab, cold);
        return;
    }
    bool big = false;
    ((Xc[OFF + K] = exp_lane(exp_arg_body(S, XTask{kXC.T[OFF + K].kind, kXC.T[OFF + K].iB, kXC.T[OFF + K].ic,
                                                    kXC.T[OFF + K].it}), big)), ...);
    if (big)   // an argument beyond kExpFastMax (inf / NaN states): ocml's exp for this lane's set
        ((Xc[OFF + K] = exp_body(S, XTask{kXC.T[OFF + K].kind, kXC.T[OFF + K].iB, kXC.T[OFF + K].ic,
                                          kXC.T[OFF + K].it}, tab)), ...);
}
// Xc (the computed list) into the slots of X [NXE], X_ONE, then the 22 products
template <size_t... K, size_t... P>
GGP_DEV void lane_expand(const double *Xc, double *X, std::index_sequence<K...>, std::index_sequence<P...>)
{
    ((X[kXC.j[K]] = Xc[K]), ...);
    X[X_ONE] = 1.0;
    ((X[kXP[P].j] = X[kXP[P].rep] * X[kXP[P].fac]), ...);
}
// the computed exponentials into their slots and X_ONE, no products (XView forms them at their reads)
template <size_t... K>
GGP_DEV void lane_slots(const double *Xc, double *X, std::index_sequence<K...>)
{
    ((X[kXC.j[K]] = Xc[K]), ...);
    X[X_ONE] = 1.0;
}
GGP_DEV void lane_expand(const double *Xc, double *X)
{
    lane_expand(Xc, X, std::make_index_sequence<NXC>{}, std::make_index_sequence<NXPU>{});
}
// A product's factor is exp(-gl t), exp(-gq t), exp(-b t) or exp(gq t): beyond |k t| ~ 700 it
// under- or overflows while the direct exponential of the sum may not (0 x inf = NaN where the
// reference is finite).  Such a step (rare: a dt of weeks at the example's rates, where the
// reference's own integrals stop being finite first, tests/test_gpu_parity.py long-dt test) forms
// the 22 slots from their own arguments instead
GGP_DEV bool products_risky(const Step &S)
{
    const double m = fmax(fabs(S.gl * S.t), fmax(fabs(S.gq * S.t), fabs(S.b * S.t)));
    return !(m <= 700.0);
}
template <size_t... P>
GGP_DEV void lane_direct_products(const Step &S, double *X, const double *tab, std::index_sequence<P...>)
{
    ((X[kXP[P].j] = exp_body(S, kXT[kXP[P].j], tab)), ...);
}
GGP_DEV void lane_guard_products(const Step &S, double *X, const double *tab)
{
    if constexpr (NXPU > 0) {
        if (__builtin_expect(products_risky(S), 0)) lane_direct_products(S, X, tab, std::make_index_sequence<NXPU>{});
    }
}
template <size_t... J>
GGP_DEV void lane_dawsons(const Step &S, double *Dw, const double *tab, std::index_sequence<J...>)
{
    ((Dw[J] = ggp_dawson_tab(zval(S, kDT[J].iB, kDT[J].it), tab)), ...);
}
template <int J, class XA, class DA, class PA>
GGP_DEV double lane_tau(const Step &S, const XA &X, const DA &Dw, const PA &PW)
{
    constexpr ITask T = kIT[J];
    return tau_body(S, T, X, Dw, PW);
}
template <class XA, class DA, class PA, size_t... J>
GGP_DEV void lane_taus(const Step &S, const XA &X, const DA &Dw, const PA &PW, double *I,
                       std::index_sequence<J...>)
{
    ((I[J] = lane_tau<(int)J>(S, X, Dw, PW)), ...);
}

// the lane schedule's exponentials as the integrals read them: a product slot is formed at its
// read (the same X[rep] * X[fac], bitwise lane_expand's), so the 22 products are never all live
struct XView {
    const double *X;
    GGP_DEV double operator[](const int j) const
    {
        for (int p = 0; p < NXPU; ++p)
            if (kXP[p].j == j) return X[kXP[p].rep] * X[kXP[p].fac];
        return X[j];
    }
};
// ---- lane schedule: one lane runs every task of its own cell
// K (optional, 16): cross_cov_model of the same step (the -j path)
// MAT: the 22 products materialised in X (and replaced by their direct exponentials where
// lane_guard_products finds the step risky); otherwise formed where the integrals read them
template <bool COLD, bool MAT = true>
GGP_DEV void propagate_lane_body(double *m, double *C, const double t, const OU &P, const double *tab, double *K);

// GGP_EXACT's cold step: an exponential argument outside exp_glibc's main path (|x| >= 512, inf,
// NaN) somewhere in this lane's step -- the whole step again with every exponential through
// exp_glibc's special paths.  Out of line on the device: the hot step keeps its registers
#if defined(GGP_HOST_SIM)
inline
#else
__device__ __attribute__((noinline))
#endif
void propagate_lane_cold(double *m, double *C, const double t, const OU &P, const double *tab, double *K)
{
    propagate_lane_body<true>(m, C, t, P, tab, K);
}

template <bool COLD, bool MAT>
GGP_DEV void propagate_lane_body(double *m, double *C, const double t, const OU &P, const double *tab, double *K)
{
    Step S;
    step_init(S, m, C, t, P);
    double Xc[NXC], X[NXE];
    if constexpr (kExact && !COLD) {
        bool big = false;
        glibc_exps_all<0, NXC>(S, Xc, tab, big);
        if (__builtin_expect(big, 0)) {   // m, C are untouched so far
            propagate_lane_cold(m, C, t, P, tab, K);
            return;
        }
    } else {
#ifdef GGP_LANE_FLAGGED
        bool cold = false;
        lane_exps_flagged<0>(S, Xc, tab, std::make_index_sequence<NXC>{}, cold);
#else
        lane_exps_c(S, Xc, tab, std::make_index_sequence<NXC>{});
#endif
    }
    if constexpr (MAT) {
        lane_expand(Xc, X);
        lane_guard_products(S, X, tab);
    } else {
        lane_slots(Xc, X, std::make_index_sequence<NXC>{});
    }
    double Dw[ND];
    lane_dawsons(S, Dw, tab, std::make_index_sequence<ND>{});
    double PW[NPW];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        PW[p] = pow_task(S, p);
        PW[3 + p] = frcp(PW[p]);   // rdiv seeds
    }
    double I[NI];
    if constexpr (MAT)
        lane_taus(S, X, Dw, PW, I, std::make_index_sequence<NI>{});
    else
        lane_taus(S, XView{X}, Dw, PW, I, std::make_index_sequence<NI>{});
    if (K) cross_outputs(S, I, X, K);
#ifdef GGP_STUB_OUT   // diagnostic probe only (tools/gpu_r4g.sh): the outputs stage left out
    for (int j = 0; j < NI; ++j) C[j & 15] += 1e-300 * (I[j] * X[XS_bt + (j % 6)]);
#else
    outputs(S, I, X, m, C);
#endif
}

// products_risky from the step's inputs alone (the same test on the same values)
GGP_DEV bool products_risky_t(const double t, const OU &P)
{
    const double m = fmax(fabs(P.gl * t), fmax(fabs(P.gq * t), fabs(P.b * t)));
    return !(m <= 700.0);
}

// The lane step with its products formed at the integrals' reads: 22 values fewer live across the
// integrals (k_loglik_level 342 -> 296 registers, C4/C5 lane levels ~2% faster, bitwise the same).
// A step where some lane of the wave is risky (products_risky) takes the materialised form, whose
// guard replaces the products by their direct exponentials -- a wave-uniform branch, so a lane
// never runs both forms (the exact engine has no products and one form)
GGP_DEV void propagate_lane(double *m, double *C, const double t, const OU &P, const double *tab, double *K = nullptr)
{
    if constexpr (NXPU > 0) {
#if defined(__HIP_DEVICE_COMPILE__)
        const bool mat = __builtin_amdgcn_ballot_w64(products_risky_t(t, P)) != 0;
#else
        const bool mat = products_risky_t(t, P);
#endif
        if (__builtin_expect(mat, 0))
            propagate_lane_body<false, true>(m, C, t, P, tab, K);
        else
            propagate_lane_body<false, false>(m, C, t, P, tab, K);
    } else {
        propagate_lane_body<false>(m, C, t, P, tab, K);
    }
}

// division map of mean_cov_after_division (predictions.h:40-60), after the propagation
GGP_DEV void division_map(double *m, double *C, const double var_dx, const double var_dg,
                          const int binomial, const double log2)
{
    if (binomial) {
        C[0] += var_dx;
        C[1] = C[4] = m[1] / 2. * var_dx + C[1];
        C[5] = var_dx * (m[1] * m[1] + C[5]) / 2. + var_dg * m[1] / 4. * (1 - var_dx) + C[5] / 4.;
        C[9] /= 2; C[6] /= 2;
        C[13] /= 2; C[7] /= 2;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) { C[4 + j] *= 0.5; C[4 * j + 1] *= 0.5; }
        C[0] = var_dx + C[0];
        C[5] = var_dg + C[5];
    }
    m[0] = m[0] + -log2;
    m[1] = 0.5 * m[1];
}

}  // namespace ggp
