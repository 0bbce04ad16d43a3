// ggp_joints.h -- the -j path on the device (src/correlation_tree.h:132-651 over the Gaussian
// algebra of src/Gaussians.h:42-157).  Same operations, in the same order, as the CPU oracle
// oracle/ggp_oracle_joints.c; row-major matrices, chained products left to right.
//
//   k_joint_rows   per row, independent of the start: the backward factor divided by the prior
//                  (incorporate_backward_prob :420-447), the step conditional P(z_r+1 | z_r)
//                  (consecutive_conditional[_cell_division] :234-356) and the start joint
//                  P(z_r+1, z_r) (consecutive_joint[_cell_division] :158-318)
//   k_joint_walk   per start row: the walk of sc_joint_distributions / joint_distributions_recr
//                  / calc_joint_distributions (:464-600) through the subtree, depth first
//                  (daughter1 before daughter2) with an explicit stack, counting or emitting
#pragma once
#include "ggp_predict.h"
#include "ggp_prop.h"

namespace ggp {

template <int N, int K, int M>
GGP_DEV void jmm(const double *A, const double *B, double *R)
{   // R[N x M] = A[N x K] B[K x M]
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < M; ++j) {
            double s = A[i * K] * B[j];
#pragma unroll
            for (int l = 1; l < K; ++l) s += A[i * K + l] * B[l * M + j];
            R[i * M + j] = s;
        }
}

template <int N, int M>
GGP_DEV void jt(const double *A, double *R)
{
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < M; ++j) R[j * N + i] = A[i * M + j];
}

// 2x2 partial-pivot LU inverse (the dynamic MatrixXd of include_measurement)
GGP_DEV void inv2(const double *A, double *R)
{
    double a00 = A[0], a01 = A[1], a10 = A[2], a11 = A[3];
    const bool sw = fabs(a10) > fabs(a00);
    const double u00 = sw ? a10 : a00, u01 = sw ? a11 : a01, l0 = sw ? a00 : a10, l1 = sw ? a01 : a11;
    double l = l0, u11 = l1;
    if (u00 != 0.0) {
        l = l0 / u00;
        u11 = l1 - l * u01;
    }
    // columns of the identity permuted: perm = sw ? {1, 0} : {0, 1}
#pragma unroll
    for (int col = 0; col < 2; ++col) {
        double y0 = (sw ? 1 : 0) == col ? 1.0 : 0.0;
        double y1 = (sw ? 0 : 1) == col ? 1.0 : 0.0;
        y1 -= l * y0;
        y1 /= u11;
        y0 -= u01 * y1;
        y0 /= u00;
        R[col] = y0;
        R[2 + col] = y1;
    }
}

struct G4 { double m[4], C[16]; };
struct G8 { double m[8], C[64]; };
struct A4 { double a[4], F[16], A[16]; };

GGP_DEV void jblk(const double *C8, int r0, int c0, double *out)
{
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) out[4 * i + j] = C8[8 * (r0 + i) + c0 + j];
}

GGP_DEV void jput(double *C8, int r0, int c0, const double *b)
{
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) C8[8 * (r0 + i) + c0 + j] = b[4 * i + j];
}

GGP_DEV G4 g_multiply(const G4 &n1, const G4 &n2)
{
    double s[16], si[16], t1[16], t2[16], v1[4], v2[4];
    G4 r;
#pragma unroll
    for (int k = 0; k < 16; ++k) s[k] = n1.C[k] + n2.C[k];
    inv4(s, si);
    jmm<4, 4, 4>(n2.C, si, t1);
    jmm<4, 4, 1>(t1, n1.m, v1);
    jmm<4, 4, 4>(n1.C, si, t2);
    jmm<4, 4, 1>(t2, n2.m, v2);
#pragma unroll
    for (int k = 0; k < 4; ++k) r.m[k] = v1[k] + v2[k];
    jmm<4, 4, 4>(t2, n2.C, r.C);
    return r;
}

GGP_DEV A4 a_transform(const A4 &g)
{
    double Fi[16], t[16], Fit[16], nFi[16];
    A4 r;
    inv4(g.F, Fi);
#pragma unroll
    for (int k = 0; k < 16; ++k) nFi[k] = -Fi[k];
    jmm<4, 4, 1>(nFi, g.a, r.a);
#pragma unroll
    for (int k = 0; k < 16; ++k) r.F[k] = Fi[k];
    jmm<4, 4, 4>(Fi, g.A, t);
    jt<4, 4>(Fi, Fit);
    jmm<4, 4, 4>(t, Fit, r.A);
    return r;
}

GGP_DEV G4 a_transform_at(const A4 &g, const double *y)
{
    double Fi[16], t[16], Fit[16], d[4];
    G4 r;
    inv4(g.F, Fi);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = y[k] - g.a[k];
    jmm<4, 4, 1>(Fi, d, r.m);
    jmm<4, 4, 4>(Fi, g.A, t);
    jt<4, 4>(Fi, Fit);
    jmm<4, 4, 4>(t, Fit, r.C);
    return r;
}

GGP_DEV G8 to_joint(const G4 &mg, const A4 &cd)
{
    G8 j;
    double Fm[4], Ct[16], Ft[16], X[16], B[16];
    jmm<4, 4, 1>(cd.F, mg.m, Fm);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        j.m[k] = mg.m[k];
        j.m[4 + k] = cd.a[k] + Fm[k];
    }
    jt<4, 4>(mg.C, Ct);
    jt<4, 4>(cd.F, Ft);
    jput(j.C, 0, 0, mg.C);
    jmm<4, 4, 4>(Ct, Ft, X);
    jput(j.C, 0, 4, X);
    jmm<4, 4, 4>(cd.F, mg.C, X);
    jput(j.C, 4, 0, X);
    double FCt[16];
    jmm<4, 4, 4>(cd.F, Ct, FCt);
    jmm<4, 4, 4>(FCt, Ft, X);
#pragma unroll
    for (int k = 0; k < 16; ++k) B[k] = cd.A[k] + X[k];
    jput(j.C, 4, 4, B);
    return j;
}

GGP_DEV void separate(const G8 &j, G4 &mg, A4 &cd)
{
    double B[16], K[16], A[16], Ai[16], Kt[16], KtAi[16], v[4], KtAiK[16];
    jblk(j.C, 4, 4, B);
    jblk(j.C, 0, 4, K);
    jblk(j.C, 0, 0, A);
    inv4(A, Ai);
    jt<4, 4>(K, Kt);
    jmm<4, 4, 4>(Kt, Ai, KtAi);
    jmm<4, 4, 1>(KtAi, j.m, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        mg.m[k] = j.m[k];
        cd.a[k] = j.m[4 + k] - v[k];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mg.C[k] = A[k];
        cd.F[k] = KtAi[k];
    }
    jmm<4, 4, 4>(KtAi, K, KtAiK);
#pragma unroll
    for (int k = 0; k < 16; ++k) cd.A[k] = B[k] - KtAiK[k];
}

GGP_DEV G8 flip_xy(const G8 &g)
{
    G8 r;
    double b[16], bt[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        r.m[k] = g.m[4 + k];
        r.m[4 + k] = g.m[k];
    }
    jblk(g.C, 4, 4, b); jput(r.C, 0, 0, b);
    jblk(g.C, 0, 4, b); jt<4, 4>(b, bt); jput(r.C, 0, 4, bt);
    jblk(g.C, 4, 0, b); jt<4, 4>(b, bt); jput(r.C, 4, 0, bt);
    jblk(g.C, 0, 0, b); jput(r.C, 4, 4, b);
    return r;
}

GGP_DEV void include_measurement(G8 &j, const double *D, const double x, const double g)
{
    const double S[4] = {j.C[0] + D[0], j.C[1] + D[1], j.C[8] + D[2], j.C[9] + D[3]};
    double Si[4], K[16], Kt[16], KtSi[16], d[8];
    const double xg[2] = {x - j.m[0], g - j.m[1]};
    inv2(S, Si);
#pragma unroll
    for (int k = 0; k < 16; ++k) K[k] = j.C[k];   // rows 0-1 of the 8x8
    jt<2, 8>(K, Kt);
    jmm<8, 2, 2>(Kt, Si, KtSi);
    jmm<8, 2, 1>(KtSi, xg, d);
    double dC[64];
    jmm<8, 2, 8>(KtSi, K, dC);
#pragma unroll
    for (int k = 0; k < 8; ++k) j.m[k] = j.m[k] + d[k];
#pragma unroll
    for (int k = 0; k < 64; ++k) j.C[k] = j.C[k] - dC[k];
}

GGP_DEV void join8(const double *m_top, const double *m_bot, const double *C11, const double *C12,
                   const double *C21, const double *C22, G8 &j)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        j.m[k] = m_top[k];
        j.m[4 + k] = m_bot[k];
    }
    jput(j.C, 0, 0, C11);
    jput(j.C, 0, 4, C12);
    jput(j.C, 4, 0, C21);
    jput(j.C, 4, 4, C22);
}

// the backward factor of row r divided by the prior (the first half of incorporate_backward_prob)
GGP_DEV G4 backward_over_prior(const double *bwd_r, const double *p)
{
    const double mp[4] = {0, 0, p[0], p[3]};
    double ip[16], bi[16], d[16], nc[16], a[4], b[4], r[4];
#pragma unroll
    for (int k = 0; k < 16; ++k) ip[k] = 0.0;
    ip[10] = (2. * p[1]) / p[2];
    ip[15] = (2. * p[4]) / p[5];
    inv4(bwd_r + 4, bi);
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = bi[k] - ip[k];
    inv4(d, nc);
    jmm<4, 4, 1>(bi, bwd_r, a);
    jmm<4, 4, 1>(ip, mp, b);
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = a[k] - b[k];
    G4 back;
    jmm<4, 4, 1>(nc, r, back.m);
#pragma unroll
    for (int k = 0; k < 16; ++k) back.C[k] = nc[k];
    return back;
}

GGP_DEV bool cross_small(const G8 &j, const double tol)
{
    bool small = true;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 4; k < 8; ++k) small = small && !(fabs(j.C[8 * i + k] / (j.m[i] * j.m[k])) > tol);
    return small;
}

GGP_DEV G8 next_joint(const G8 &joint, const A4 &cond)
{
    G4 mg;
    A4 sc;
    separate(joint, mg, sc);
    double s[16], si[16], t1[16], t2[16], v1[4], v2[4];
#pragma unroll
    for (int k = 0; k < 16; ++k) s[k] = mg.C[k] + cond.A[k];
    inv4(s, si);
    A4 NX;
    jmm<4, 4, 4>(cond.A, si, t1);
    jmm<4, 4, 1>(t1, mg.m, v1);
    jmm<4, 4, 4>(mg.C, si, t2);
    jmm<4, 4, 1>(t2, cond.a, v2);
#pragma unroll
    for (int k = 0; k < 4; ++k) NX.a[k] = v1[k] + v2[k];
    jmm<4, 4, 4>(t2, cond.F, NX.F);
    jmm<4, 4, 4>(t2, cond.A, NX.A);
    A4 G;
#pragma unroll
    for (int k = 0; k < 4; ++k) G.a[k] = cond.a[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        G.F[k] = cond.F[k];
        G.A[k] = mg.C[k] + cond.A[k];
    }
    const G4 next_marginal = a_transform_at(G, mg.m);
    A4 nc;
    double Fa[4], FA[16], Ft[16], FAFt[16];
    jmm<4, 4, 1>(sc.F, NX.a, Fa);
#pragma unroll
    for (int k = 0; k < 4; ++k) nc.a[k] = sc.a[k] + Fa[k];
    jmm<4, 4, 4>(sc.F, NX.F, nc.F);
    jmm<4, 4, 4>(sc.F, NX.A, FA);
    jt<4, 4>(sc.F, Ft);
    jmm<4, 4, 4>(FA, Ft, FAFt);
#pragma unroll
    for (int k = 0; k < 16; ++k) nc.A[k] = sc.A[k] + FAFt[k];
    return to_joint(next_marginal, nc);
}

// the binomial division of consecutive_{joint,conditional}_cell_division (:170-202) on the
// forward posterior fwd_t propagated over dt (m2, C2) and its cross block
GGP_DEV void division_binomial_j(const double *p, const double *m2in, const double *C2in, const double *fwd_t,
                                 double *m2, double *C2, double *cross)
{
    const double var_dx = p[9], var_dg = p[10];
#pragma unroll
    for (int k = 0; k < 4; ++k) m2[k] = m2in[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) C2[k] = C2in[k];
    C2[0] += var_dx;
    C2[1] = C2[4] = m2[1] / 2. * var_dx + C2[1];
    C2[5] = var_dx * (m2[1] * m2[1] + C2[5]) / 2. + var_dg * m2[1] / 4. * (1 - var_dx) + C2[5] / 4.;
    C2[9] /= 2; C2[6] /= 2;
    C2[13] /= 2; C2[7] /= 2;
    const double F[16] = {1, 0, 0, 0, 0, 0.5, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    double Fm[4];
    jmm<4, 4, 1>(F, m2, Fm);
    m2[0] = Fm[0] + -log(2.);
    m2[1] = Fm[1] + 0.0;
    m2[2] = Fm[2] + 0.0;
    m2[3] = Fm[3] + 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) cross[k] = fwd_t[4 + k];
#pragma unroll
    for (int j = 0; j < 4; ++j) cross[4 + j] /= 2.;
}

GGP_DEV A4 division_affine(const double *p)
{
    A4 g;
#pragma unroll
    for (int k = 0; k < 4; ++k) g.a[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) g.F[k] = g.A[k] = 0.0;
    g.a[0] = -log(2.);
    g.F[0] = 1; g.F[5] = 0.5; g.F[10] = 1; g.F[15] = 1;
    g.A[0] = p[9];
    g.A[5] = p[10];
    return g;
}

}  // namespace ggp
