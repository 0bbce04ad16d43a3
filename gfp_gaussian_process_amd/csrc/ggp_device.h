// ggp_device.h -- FP64 device math of the lineage-tree likelihood path (gfx950).
//
// What is here, and the reference it restates:
//   ggp_dawson          Faddeeva::Dawson / w_im / w_im_y100  Faddeeva.cc:467-471, 1458-1888
//   ggp_innovation,     S = C[0:2,0:2] + D, S^-1, ll term,    likelihood.h:26-32, 53-69
//   ggp_ll_term,        posterior                             predictions.h:84-89
//   ggp_posterior
// The propagator (mean_cov_model.h) is in ggp_prop.h.
//
// Evaluation order follows the reference expression by expression.  The library is built with
// -ffp-contract=off; the bodies the lane schedules run fuse a*b + c within one expression
// (GGP_CONTRACT below).  Rounding at that level, like ocml's exp against glibc's (<= 1 ulp),
// moves the total log-likelihood by ~1e-10 relative at most (measured, DESIGN.md "Parity").
#pragma once
#include <math.h>

#ifdef GGP_HOST_SIM
// host simulation of the device math (tools/hostsim.cpp, g++): the same source, glibc libm.
// Diagnostic builds only; the shipped library is always the gfx950 code object.
#include <algorithm>
#include <cstdint>
using std::min;
#define GGP_DEV inline
#define GGP_DAWSON_TABLE_QUALIFIER static const
#include "dawson_table.inc"
#else
#include <hip/hip_runtime.h>
#ifndef GGP_DEVICE_TABLE_DEFINED
#define GGP_DEVICE_TABLE_DEFINED
#define GGP_DAWSON_TABLE_QUALIFIER static __constant__ const
#include "dawson_table.inc"
#endif
#define GGP_DEV __device__ __forceinline__
#endif

// GGP_CONTRACT, first statement of a lane-schedule body: FMA contraction within each source
// expression of that body (clang's "on": a*b + c of one expression becomes one fma; nothing is
// fused across statements).  What fuses is decided by the expression alone, so the lane, group,
// lane-pair, batch and smoother kernels, which all run these bodies, stay bitwise equal to one
// another.  The wave schedule (ggp_wave.h) and the oracle keep their own forms.  -DGGP_NO_CONTRACT
// builds the uncontracted bodies (A/B, DESIGN.md "Parity").  A host simulation built by clang
// with -DGGP_HOST_CONTRACT -mfma contracts exactly as the device does (tools/parity_attrib.cpp).
#if defined(GGP_NO_CONTRACT) || defined(GGP_EXACT) || (defined(GGP_HOST_SIM) && !defined(GGP_HOST_CONTRACT))
#define GGP_CONTRACT
#else
#define GGP_CONTRACT _Pragma("clang fp contract(on)")
#endif

// ------------------------------------------------------------------------------------------
// Dawson: w_im on y = 1/(1+|x|) with 97 polynomial pieces (degree 6..8, zero-padded to 9),
// Taylor for y100 >= 97, continued fraction for |x| > 45.
// ------------------------------------------------------------------------------------------
// branch-free on |x| <= 45 so that the 14 Dawson values of a step overlap their table loads;
// `tab` is the coefficient table (constant memory, or an LDS copy in the group schedule)
// x / d for d >= 1 (finite): v_rcp_f64, two Newton steps, one Markstein correction -- the
// IEEE quotient in practice (the A/B totals are bitwise unchanged) at ~6 instructions against
// the ~11 of the IEEE sequence; 14 per step in the lane and group schedules
GGP_DEV double ggp_div_ge1(const double x, const double d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    const double q = x * r;
    return fma(fma(-q, d, x), r, q);
#else
    return x / d;
#endif
}

GGP_DEV double ggp_w_im_abs(double ax, const double *tab)
{
    GGP_CONTRACT
    const double y100 = ggp_div_ge1(100.0, 1.0 + ax);
    const int k = min((int)y100, GGP_DAWSON_NINT - 1);
    const double *c = tab + GGP_DAWSON_NCOEF * k;
    const double t = 2.0 * y100 - (double)(2 * k + 1);
    const double poly = c[0] + (c[1] + (c[2] + (c[3] + (c[4] + (c[5] + (c[6] + (c[7] + c[8] * t) * t) * t) * t) * t) * t) * t) * t;
    const double x2 = ax * ax;
    const double *tc = ggp_dawson_taylor;
    const double taylor = ax * (tc[0] - x2 * (tc[1] - x2 * (tc[2] - x2 * (tc[3] - x2 * tc[4]))));
    // the continued fraction (|x| > 45) is rare: its divisions only when some lane needs them
    double cf = 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_amdgcn_ballot_w64(ax > 45.0))
#endif
        cf = ax > 5e7 ? GGP_ISPI / ax
                      : GGP_ISPI * ((ax * ax) * (ax * ax - 4.5) + 2) / (ax * ((ax * ax) * (ax * ax - 5) + 3.75));
    return ax > 45.0 ? cf : (y100 >= (double)GGP_DAWSON_NINT ? taylor : poly);
}

#ifdef GGP_HOST_SIM
// diagnostic hook (tools/parity_attrib.cpp): every Dawson value from another implementation
extern double (*ggp_hs_dawson)(double);
#endif

GGP_DEV double ggp_dawson_tab(double x, const double *tab)
{
#ifdef GGP_HOST_SIM
    if (ggp_hs_dawson) return ggp_hs_dawson(x);
#endif
    if (x != x) return x;
    const double w = ggp_w_im_abs(fabs(x), tab);
    return GGP_SPI2 * (x < 0.0 ? -w : w);
}

GGP_DEV double ggp_dawson(double x) { return ggp_dawson_tab(x, ggp_dawson_coef); }

// ------------------------------------------------------------------------------------------
// Parameters and state
// ------------------------------------------------------------------------------------------
struct ggp_params {           // Parameters.h:175 order
    double p[11];
};

// ------------------------------------------------------------------------------------------
// Kalman measurement step (likelihood.h:53-95, predictions.h:84-89)
// ------------------------------------------------------------------------------------------
struct ggp_innov {
    double S00, S01, S10, S11, si00, si01, si10, si11;
};

GGP_DEV void ggp_innovation(const double *m, const double *C, const double var_x, const double var_g,
                            const int scaled, const double fp_auto, ggp_innov &v)
{
    GGP_CONTRACT
    const double d11 = scaled ? var_g * (m[1] + fp_auto) : var_g;
    v.S00 = C[0] + var_x;
    v.S01 = C[1] + 0.0;
    v.S10 = C[4] + 0.0;
    v.S11 = C[5] + d11;
    const double det = v.S00 * v.S11 - v.S10 * v.S01;        // Eigen fixed 2x2 determinant
    const double invdet = 1.0 / det;
    v.si00 = v.S11 * invdet;
    v.si10 = -v.S10 * invdet;
    v.si01 = -v.S01 * invdet;
    v.si11 = v.S00 * invdet;
}

// log(S.determinant()) on a dynamic 2x2: Eigen PartialPivLU (first max |a_i0| pivot)
GGP_DEV double ggp_det_pplu(double s00, double s01, double s10, double s11)
{
    double sign = 1.0;
    if (fabs(s10) > fabs(s00)) {
        double t0 = s00, t1 = s01;
        s00 = s10; s01 = s11; s10 = t0; s11 = t1;
        sign = -1.0;
    }
    if (s00 != 0.0) {
        s10 = s10 / s00;
        s11 = s11 - s10 * s01;
    }
    return sign * (s00 * s11);
}

// log_likelihood (likelihood.h:26-32). two_log_2pi is 2*log(2*M_PI) as the host folds it.
GGP_DEV double ggp_ll_term(const double x0, const double x1, const ggp_innov &v, const double two_log_2pi)
{
    GGP_CONTRACT
    const double h0 = -0.5 * x0, h1 = -0.5 * x1;
    const double r0 = h0 * v.si00 + h1 * v.si10;
    const double r1 = h0 * v.si01 + h1 * v.si11;
    const double q = r0 * x0 + r1 * x1;
    return q - 0.5 * log(ggp_det_pplu(v.S00, v.S01, v.S10, v.S11)) - two_log_2pi;
}

GGP_DEV void ggp_posterior(double *m, double *C, const double x0, const double x1, const ggp_innov &v)
{
    GGP_CONTRACT
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
        for (int j = 0; j < 4; ++j) C[4 * i + j] = C[4 * i + j] - (KS0[i] * K[j] + KS1[i] * K[4 + j]);
}

