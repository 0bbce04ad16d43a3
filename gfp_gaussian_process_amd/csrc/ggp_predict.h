// ggp_predict.h -- the -p smoother on the device (predictions.h:93-499).
//
//   k_fwd_level   prediction_forward / sc_prediction_forward  predictions.h:93-173
//                 (per-row segment parameters; the posterior of every row is stored)
//   k_bwd_level   prediction_backward / sc_prediction_backward predictions.h:368-444
//                 (reverse time: ml, mq, beta negated; leaves start on top of the forward
//                 pass's final state, internal cells fuse both daughters)
//   k_combine     combine_predictions                          predictions.h:466-499
//                 (forward x backward, divided by the stationary prior; 5 dense 4x4
//                 inverses per row by partial-pivot LU, one lane per row)
// Levels are processed top-down for the forward pass and bottom-up for the backward pass;
// every row of the combine is independent.
#pragma once
#include "ggp_device.h"
#include "ggp_prop.h"

namespace ggp {

// dense 4x4 inverse by partial-pivot LU (first max |a| pivot, unit-lower L), solved column by
// column against the identity -- the algorithm of oracle/ggp_oracle.c inv4.  FAST (the combine
// only, DESIGN.md "Smoother"): divide by each pivot through its reciprocal (4 divisions instead
// of 22, one more rounding per quotient).  (Solving only the lower triangle of each column and
// mirroring it, A being symmetric, saved 5% more but moved the combined rows 10x further from
// the exact combine: 1.1e-10 against 1.2e-11.)
template <bool FAST = false>
GGP_DEV void inv4(const double *A, double *R)
{
    double lu[16], rd[4];
    int perm[4] = {0, 1, 2, 3};
#pragma unroll
    for (int i = 0; i < 16; ++i) lu[i] = A[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int piv = k;
        double big = fabs(lu[4 * k + k]);
#pragma unroll
        for (int i = k + 1; i < 4; ++i) {
            const double v = fabs(lu[4 * i + k]);
            if (v > big) { big = v; piv = i; }
        }
        if (piv != k) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // swap rows k and piv without dynamic register indexing
                double rk = lu[4 * k + j], rp = 0.0;
#pragma unroll
                for (int i = k + 1; i < 4; ++i) rp = (i == piv) ? lu[4 * i + j] : rp;
                lu[4 * k + j] = rp;
#pragma unroll
                for (int i = k + 1; i < 4; ++i) lu[4 * i + j] = (i == piv) ? rk : lu[4 * i + j];
            }
            int pk = perm[k], pp = 0;
#pragma unroll
            for (int i = k + 1; i < 4; ++i) pp = (i == piv) ? perm[i] : pp;
            perm[k] = pp;
#pragma unroll
            for (int i = k + 1; i < 4; ++i) perm[i] = (i == piv) ? pk : perm[i];
        }
        if constexpr (FAST) rd[k] = 1.0 / lu[4 * k + k];
        if (big != 0.0) {
#pragma unroll
            for (int i = k + 1; i < 4; ++i) {
                if constexpr (FAST) lu[4 * i + k] *= rd[k];
                else lu[4 * i + k] /= lu[4 * k + k];
            }
#pragma unroll
            for (int i = k + 1; i < 4; ++i)
#pragma unroll
                for (int j = k + 1; j < 4; ++j) lu[4 * i + j] -= lu[4 * i + k] * lu[4 * k + j];
        }
    }
#pragma unroll
    for (int col = 0; col < 4; ++col) {
        double y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = (perm[i] == col) ? 1.0 : 0.0;
#pragma unroll
        for (int i = 1; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) y[i] -= lu[4 * i + j] * y[j];
#pragma unroll
        for (int i = 3; i >= 0; --i) {
#pragma unroll
            for (int j = i + 1; j < 4; ++j) y[i] -= lu[4 * i + j] * y[j];
            if constexpr (FAST) y[i] *= rd[i];
            else y[i] /= lu[4 * i + i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) R[4 * i + col] = y[i];
    }
}

GGP_DEV void mm4(const double *A, const double *B, double *R)
{
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double s = A[4 * i] * B[j];
#pragma unroll
            for (int k = 1; k < 4; ++k) s = s + A[4 * i + k] * B[4 * k + j];
            R[4 * i + j] = s;
        }
}

GGP_DEV void mv4(const double *A, const double *v, double *r)
{
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double s = A[4 * i] * v[0];
#pragma unroll
        for (int k = 1; k < 4; ++k) s = s + A[4 * i + k] * v[k];
        r[i] = s;
    }
}

// multiply_gaussian (predictions.h:183-188): in place on (m1, c1).  FAST: the mean as
// nc (i1 m1 + i2 m2), three matrix-vector products instead of two 4x4 products and two
// matrix-vector ones
template <bool FAST = false>
GGP_DEV void mult_gauss(double *m1, double *c1, const double *m2, const double *c2)
{
    double i1[16], i2[16], sum[16], nc[16], t1[16], t2[16], v1[4], v2[4];
    inv4<FAST>(c1, i1);
    inv4<FAST>(c2, i2);
#pragma unroll
    for (int k = 0; k < 16; ++k) sum[k] = i1[k] + i2[k];
    inv4<FAST>(sum, nc);
    if constexpr (FAST) {
        mv4(i1, m1, v1);
        mv4(i2, m2, v2);
#pragma unroll
        for (int k = 0; k < 4; ++k) v1[k] = v1[k] + v2[k];
        mv4(nc, v1, m1);
#pragma unroll
        for (int k = 0; k < 16; ++k) c1[k] = nc[k];
        return;
    }
    mm4(nc, i1, t1);
    mm4(nc, i2, t2);
    mv4(t1, m1, v1);
    mv4(t2, m2, v2);
#pragma unroll
    for (int k = 0; k < 4; ++k) m1[k] = v1[k] + v2[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) c1[k] = nc[k];
}

// divide_by_prior (predictions.h:446-463).  FAST: the prior precision's product with its mean
// formed from its two nonzero entries (the same values up to the sign of a zero)
template <bool FAST = false>
GGP_DEV void divide_prior(double *m, double *c, const double *p)
{
    const double mp[4] = {0, 0, p[0], p[3]};
    double ip[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) ip[k] = 0.0;
    ip[10] = (2. * p[1]) / p[2];
    ip[15] = (2. * p[4]) / p[5];
    double ic[16], d[16], nc[16], a[4], bv[4], r[4];
    inv4<FAST>(c, ic);
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = ic[k] - ip[k];
    inv4<FAST>(d, nc);
    mv4(ic, m, a);
    if constexpr (FAST) {
        bv[0] = bv[1] = 0.0;
        bv[2] = ip[10] * mp[2];
        bv[3] = ip[15] * mp[3];
    } else {
        mv4(ip, mp, bv);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = a[k] - bv[k];
    mv4(nc, r, m);
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = nc[k];
}

// combine_predictions' row (predictions.h:466-499) in information form (the combine's FAST form):
// multiply_gaussian forms nc = (i1 + i2)^-1 and divide_by_prior inverts it back, ic = nc^-1,
// before subtracting the prior precision ip -- ic is i1 + i2 up to rounding, and ic nc (i1 m1 +
// i2 m2) is i1 m1 + i2 m2.  So the row is (i1 + i2 - ip)^-1 (i1 m1 + i2 m2 - ip mp): three 4x4
// inverses instead of five.  On the example every combined row stays within 1.5e-11 of the
// oracle's five-inverse combine in the smoother tests' normalisation (median 4e-14), 1e5 x below
// the oracle's own movement under +-1 ulp exp() noise (tests/test_gpu_parity.py
// test_predict_every_row_within_the_oracles_own_noise, test_combine_fast_form_vs_exact).
GGP_DEV void combine_info(double *m, double *C, const double *mb, const double *Cb, const double *p)
{
    double i1[16], i2[16], d[16], nc[16], v1[4], v2[4];
    inv4<true>(C, i1);
    inv4<true>(Cb, i2);
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = i1[k] + i2[k];
    const double ip10 = (2. * p[1]) / p[2], ip15 = (2. * p[4]) / p[5];   // divide_by_prior's ip
    d[10] = d[10] - ip10;
    d[15] = d[15] - ip15;
    mv4(i1, m, v1);
    mv4(i2, mb, v2);
#pragma unroll
    for (int k = 0; k < 4; ++k) v1[k] = v1[k] + v2[k];
    v1[2] = v1[2] - ip10 * p[0];
    v1[3] = v1[3] - ip15 * p[3];
    inv4<true>(d, nc);
    mv4(nc, v1, m);
#pragma unroll
    for (int k = 0; k < 16; ++k) C[k] = nc[k];
}

// reverse_mean / reverse_cov (predictions.h:278-301)
GGP_DEV void reverse_state(double *m, double *C)
{
    m[2] = -m[2]; m[3] = -m[3];
    C[2] = -C[2]; C[8] = -C[8]; C[3] = -C[3]; C[12] = -C[12];
    C[6] = -C[6]; C[9] = -C[9]; C[7] = -C[7]; C[13] = -C[13];
}

// the per-daughter map of mean_cov_after_division_r (predictions.h:214-237)
GGP_DEV void division_map_r(double *m, double *C, const double var_dx, const double var_dg,
                            const int binomial, const double log2)
{
    if (binomial) {
        C[0] += var_dx;
        C[5] = 8. * var_dx * (m[1] * m[1] + C[5]) + 2. * var_dg * m[1] + 8. * C[5];
        C[1] = C[4] = 2. * m[1] * var_dx + 4. * C[1];
        C[9] *= 2; C[6] *= 2; C[13] *= 2; C[7] *= 2;
        m[0] += log2;
        m[1] *= 2;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) { C[4 + j] *= 2.0; C[4 * j + 1] *= 2.0; }
        C[0] = var_dx + C[0];
        C[5] = var_dg + C[5];
        m[0] = m[0] + log2;
        m[1] = 2.0 * m[1];
    }
}

}  // namespace ggp
