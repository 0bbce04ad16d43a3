/* ggp_oracle_joints.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's -j path
 * (src/correlation_tree.h:132-651 over the Gaussian algebra of src/Gaussians.h:42-157).
 *
 * Checker for the GPU joints; never linked into the product.  Matrices are row-major.
 * Eigen evaluates chained products left to right ((A*B)*C); that order is kept.  Dynamic
 * MatrixXd inverses are partial-pivot LU (Eigen PartialPivLU); Eigen's blocked/vectorised
 * GEMM may sum inner products in another order, so results can differ from a reference
 * binary in the last bits ("parity unpinned": no reference run is possible here).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ggp_oracle.h"

/* ---- small dense algebra ------------------------------------------------------------ */
static void mat_mul(int n, int k, int m, const double *A, const double *B, double *R)
{   /* R[n x m] = A[n x k] B[k x m] */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            double s = A[i * k] * B[j];
            for (int l = 1; l < k; ++l) s += A[i * k + l] * B[l * m + j];
            R[i * m + j] = s;
        }
}

static void mat_t(int n, int m, const double *A, double *R)
{   /* R[m x n] = A^T */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) R[j * n + i] = A[i * m + j];
}

static void inv_n(int n, const double *A, double *R)
{   /* partial-pivot LU (first max |a|, unit-lower L), solved against the identity */
    double lu[64];
    int perm[8];
    memcpy(lu, A, sizeof(double) * n * n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    for (int k = 0; k < n; ++k) {
        int piv = k;
        double big = fabs(lu[k * n + k]);
        for (int i = k + 1; i < n; ++i)
            if (fabs(lu[i * n + k]) > big) { big = fabs(lu[i * n + k]); piv = i; }
        if (piv != k) {
            for (int j = 0; j < n; ++j) { double t = lu[k * n + j]; lu[k * n + j] = lu[piv * n + j]; lu[piv * n + j] = t; }
            int t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
        }
        if (big != 0.0) {
            for (int i = k + 1; i < n; ++i) lu[i * n + k] /= lu[k * n + k];
            for (int i = k + 1; i < n; ++i)
                for (int j = k + 1; j < n; ++j) lu[i * n + j] -= lu[i * n + k] * lu[k * n + j];
        }
    }
    for (int col = 0; col < n; ++col) {
        double y[8];
        for (int i = 0; i < n; ++i) y[i] = (perm[i] == col) ? 1.0 : 0.0;
        for (int i = 1; i < n; ++i)
            for (int j = 0; j < i; ++j) y[i] -= lu[i * n + j] * y[j];
        for (int i = n - 1; i >= 0; --i) {
            for (int j = i + 1; j < n; ++j) y[i] -= lu[i * n + j] * y[j];
            y[i] /= lu[i * n + i];
        }
        for (int i = 0; i < n; ++i) R[i * n + col] = y[i];
    }
}

/* ---- Gaussians.h ---------------------------------------------------------------------- */
typedef struct { double m[8], C[64]; } gauss8;           /* joint over [first 4; last 4] */
typedef struct { double m[4], C[16]; } gauss4;
typedef struct { double a[4], F[16], A[16]; } affine4;   /* N(y | a + F x, A) */

static void blk(const double *C8, int r0, int c0, double *out)
{   /* 4x4 block of an 8x8 matrix */
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = C8[8 * (r0 + i) + c0 + j];
}

static void put_blk(double *C8, int r0, int c0, const double *b)
{
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) C8[8 * (r0 + i) + c0 + j] = b[4 * i + j];
}

/* Gaussian::multiply (Gaussians.h:42-49): (n2.C (n1.C+n2.C)^-1) n1.m + (n1.C (..)^-1) n2.m,
 * C = (n1.C (..)^-1) n2.C */
static gauss4 g_multiply(const gauss4 *n1, const gauss4 *n2)
{
    double s[16], si[16], t1[16], t2[16], v1[4], v2[4];
    gauss4 r;
    for (int k = 0; k < 16; ++k) s[k] = n1->C[k] + n2->C[k];
    inv_n(4, s, si);
    mat_mul(4, 4, 4, n2->C, si, t1);
    mat_mul(4, 4, 1, t1, n1->m, v1);
    mat_mul(4, 4, 4, n1->C, si, t2);
    mat_mul(4, 4, 1, t2, n2->m, v2);
    for (int k = 0; k < 4; ++k) r.m[k] = v1[k] + v2[k];
    mat_mul(4, 4, 4, t2, n2->C, r.C);
    return r;
}

/* Affine_gaussian::transform() (Gaussians.h:70-80) */
static affine4 a_transform(const affine4 *g)
{
    double Fi[16], t[16], Fit[16], nFi[16];
    affine4 r;
    inv_n(4, g->F, Fi);
    for (int k = 0; k < 16; ++k) nFi[k] = -Fi[k];
    mat_mul(4, 4, 1, nFi, g->a, r.a);
    memcpy(r.F, Fi, sizeof Fi);
    mat_mul(4, 4, 4, Fi, g->A, t);
    mat_t(4, 4, Fi, Fit);
    mat_mul(4, 4, 4, t, Fit, r.A);
    return r;
}

/* Affine_gaussian::transform(y) (Gaussians.h:82-86) */
static gauss4 a_transform_at(const affine4 *g, const double *y)
{
    double Fi[16], t[16], Fit[16], d[4];
    gauss4 r;
    inv_n(4, g->F, Fi);
    for (int k = 0; k < 4; ++k) d[k] = y[k] - g->a[k];
    mat_mul(4, 4, 1, Fi, d, r.m);
    mat_mul(4, 4, 4, Fi, g->A, t);
    mat_t(4, 4, Fi, Fit);
    mat_mul(4, 4, 4, t, Fit, r.C);
    return r;
}

/* Seperated_gaussian::to_joint (Gaussians.h:105-121) */
static gauss8 to_joint(const gauss4 *mg, const affine4 *cd)
{
    gauss8 j;
    double Fm[4], Ct[16], Ft[16], CtFt[16], FC[16], FCt[16], FCtFt[16], B[16];
    mat_mul(4, 4, 1, cd->F, mg->m, Fm);
    for (int k = 0; k < 4; ++k) { j.m[k] = mg->m[k]; j.m[4 + k] = cd->a[k] + Fm[k]; }
    mat_t(4, 4, mg->C, Ct);
    mat_t(4, 4, cd->F, Ft);
    mat_mul(4, 4, 4, Ct, Ft, CtFt);
    mat_mul(4, 4, 4, cd->F, mg->C, FC);
    mat_mul(4, 4, 4, cd->F, Ct, FCt);
    mat_mul(4, 4, 4, FCt, Ft, FCtFt);
    for (int k = 0; k < 16; ++k) B[k] = cd->A[k] + FCtFt[k];
    put_blk(j.C, 0, 0, mg->C);
    put_blk(j.C, 0, 4, CtFt);
    put_blk(j.C, 4, 0, FC);
    put_blk(j.C, 4, 4, B);
    return j;
}

/* seperate_gaussian (Gaussians.h:124-143) */
static void separate(const gauss8 *j, gauss4 *mg, affine4 *cd)
{
    double B[16], K[16], A[16], Ai[16], Kt[16], KtAi[16], v[4], KtAiK[16];
    blk(j->C, 4, 4, B);
    blk(j->C, 0, 4, K);
    blk(j->C, 0, 0, A);
    inv_n(4, A, Ai);
    mat_t(4, 4, K, Kt);
    mat_mul(4, 4, 4, Kt, Ai, KtAi);
    mat_mul(4, 4, 1, KtAi, j->m, v);
    for (int k = 0; k < 4; ++k) { mg->m[k] = j->m[k]; cd->a[k] = j->m[4 + k] - v[k]; }
    memcpy(mg->C, A, sizeof A);
    memcpy(cd->F, KtAi, sizeof KtAi);
    mat_mul(4, 4, 4, KtAi, K, KtAiK);
    for (int k = 0; k < 16; ++k) cd->A[k] = B[k] - KtAiK[k];
}

/* Gaussian::flip_xy (Gaussians.h:145-157) */
static gauss8 flip_xy(const gauss8 *g)
{
    gauss8 r;
    double b[16], bt[16];
    for (int k = 0; k < 4; ++k) { r.m[k] = g->m[4 + k]; r.m[4 + k] = g->m[k]; }
    blk(g->C, 4, 4, b); put_blk(r.C, 0, 0, b);
    blk(g->C, 0, 4, b); mat_t(4, 4, b, bt); put_blk(r.C, 0, 4, bt);
    blk(g->C, 4, 0, b); mat_t(4, 4, b, bt); put_blk(r.C, 4, 0, bt);
    blk(g->C, 0, 0, b); put_blk(r.C, 4, 4, b);
    return r;
}

/* ---- correlation_tree.h ------------------------------------------------------------------ */
/* include_measurement (:132-154): Si of the dynamic 2x2 by partial-pivot LU */
static gauss8 include_measurement(const gauss8 *j, const double *D, double x, double g)
{
    double S[4] = {j->C[0] + D[0], j->C[1] + D[1], j->C[8] + D[2], j->C[9] + D[3]}, Si[4];
    double xg[2] = {x - j->m[0], g - j->m[1]};
    double K[16], Kt[16], KtSi[16], d[8], dC[64];
    gauss8 r;
    inv_n(2, S, Si);
    for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 8; ++k) K[i * 8 + k] = j->C[i * 8 + k];
    mat_t(2, 8, K, Kt);
    mat_mul(8, 2, 2, Kt, Si, KtSi);
    mat_mul(8, 2, 1, KtSi, xg, d);
    mat_mul(8, 2, 8, KtSi, K, dC);
    for (int k = 0; k < 8; ++k) r.m[k] = j->m[k] + d[k];
    for (int k = 0; k < 64; ++k) r.C[k] = j->C[k] - dC[k];
    return r;
}

static void join8(const double *m_top, const double *m_bot, const double *C11, const double *C12, const double *C21,
                  const double *C22, gauss8 *j)
{
    for (int k = 0; k < 4; ++k) { j->m[k] = m_top[k]; j->m[4 + k] = m_bot[k]; }
    put_blk(j->C, 0, 0, C11);
    put_blk(j->C, 0, 4, C12);
    put_blk(j->C, 4, 0, C21);
    put_blk(j->C, 4, 4, C22);
}

/* consecutive_joint (:285-318): [z_n+1, z_n] from the forward posterior at t */
static gauss8 consecutive_joint(const double *p, const double *fwd_t, double dt)
{
    double m1[4], C1[16], m2[4], C2[16], cross[16], crossT[16];
    gauss8 j;
    memcpy(m1, fwd_t, sizeof m1);
    memcpy(C1, fwd_t + 4, sizeof C1);
    ora_cross_cov_model(m1, C1, dt, p, cross);
    memcpy(m2, m1, sizeof m2);
    memcpy(C2, C1, sizeof C2);
    ora_mean_cov_model(m2, C2, dt, p);
    mat_t(4, 4, cross, crossT);
    join8(m2, m1, C2, cross, crossT, C1, &j);
    return j;
}

/* consecutive_conditional (:321-356) */
static affine4 consecutive_conditional(const double *p, const double *fwd_t, double dt)
{
    double m1[4], C1[16], m2[4], C2[16], cross[16], crossT[16];
    gauss8 j;
    gauss4 mg;
    affine4 cd;
    memcpy(m1, fwd_t, sizeof m1);
    memcpy(C1, fwd_t + 4, sizeof C1);
    ora_cross_cov_model(m1, C1, dt, p, cross);
    memcpy(m2, m1, sizeof m2);
    memcpy(C2, C1, sizeof C2);
    ora_mean_cov_model(m2, C2, dt, p);
    mat_t(4, 4, cross, crossT);
    join8(m1, m2, C1, crossT, cross, C2, &j);
    separate(&j, &mg, &cd);
    return a_transform(&cd);
}

/* the binomial branch shared by consecutive_{joint,conditional}_cell_division (:170-202) */
static void division_binomial(const double *p, const double *fwd_t, double dt, double *m2, double *C2, double *cross)
{
    const double var_dx = p[9], var_dg = p[10];
    memcpy(m2, fwd_t, 4 * sizeof(double));
    memcpy(C2, fwd_t + 4, 16 * sizeof(double));
    ora_mean_cov_model(m2, C2, dt, p);
    C2[0] += var_dx;
    C2[1] = C2[4] = m2[1] / 2. * var_dx + C2[1];
    C2[5] = var_dx * (m2[1] * m2[1] + C2[5]) / 2. + var_dg * m2[1] / 4. * (1 - var_dx) + C2[5] / 4.;
    C2[9] /= 2; C2[6] /= 2;
    C2[13] /= 2; C2[7] /= 2;
    {   /* mean = F mean + f, F = diag(1, 1/2, 1, 1), f = (-log 2, 0, 0, 0) */
        const double F[16] = {1, 0, 0, 0, 0, 0.5, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        double Fm[4];
        mat_mul(4, 4, 1, F, m2, Fm);
        m2[0] = Fm[0] + -log(2.);
        m2[1] = Fm[1] + 0.0;
        m2[2] = Fm[2] + 0.0;
        m2[3] = Fm[3] + 0.0;
    }
    memcpy(cross, fwd_t + 4, 16 * sizeof(double));
    for (int j = 0; j < 4; ++j) cross[4 + j] /= 2.;
}

static void division_affine(const double *p, affine4 *g)
{
    memset(g, 0, sizeof *g);
    g->a[0] = -log(2.);
    g->F[0] = 1; g->F[5] = 0.5; g->F[10] = 1; g->F[15] = 1;
    g->A[0] = p[9];
    g->A[5] = p[10];
}

/* consecutive_joint_cell_division (:158-231) */
static gauss8 consecutive_joint_cell_division(const double *p, const double *fwd_t, double dt, int binomial)
{
    gauss8 j;
    if (binomial) {
        double m2[4], C2[16], cross[16], crossT[16];
        division_binomial(p, fwd_t, dt, m2, C2, cross);
        mat_t(4, 4, cross, crossT);
        join8(m2, fwd_t, C2, cross, crossT, fwd_t + 4, &j);
        return j;
    }
    /* gauss: the joint of the forward marginal and the division map (the propagation over
     * dt computed by the reference in this branch is not used by it) */
    gauss4 mg;
    affine4 cd;
    memcpy(mg.m, fwd_t, sizeof mg.m);
    memcpy(mg.C, fwd_t + 4, sizeof mg.C);
    division_affine(p, &cd);
    j = to_joint(&mg, &cd);
    return flip_xy(&j);
}

/* consecutive_conditional_cell_division (:234-283) */
static affine4 consecutive_conditional_cell_division(const double *p, const double *fwd_t, double dt, int binomial)
{
    affine4 cd;
    if (binomial) {
        double m2[4], C2[16], cross[16], crossT[16];
        gauss8 j;
        gauss4 mg;
        division_binomial(p, fwd_t, dt, m2, C2, cross);
        mat_t(4, 4, cross, crossT);
        join8(fwd_t, m2, fwd_t + 4, crossT, cross, C2, &j);
        separate(&j, &mg, &cd);
        return a_transform(&cd);
    }
    division_affine(p, &cd);
    return a_transform(&cd);
}

/* next_joint (:384-418) with calc_x / calc_X / calc_Y (:363-375) and propagation (:379-384) */
static gauss8 next_joint(const gauss8 *joint, const affine4 *cond)
{
    gauss4 mg;
    affine4 sc;
    separate(joint, &mg, &sc);
    double s[16], si[16], t1[16], t2[16], v1[4], v2[4];
    for (int k = 0; k < 16; ++k) s[k] = mg.C[k] + cond->A[k];
    inv_n(4, s, si);
    affine4 NX;
    mat_mul(4, 4, 4, cond->A, si, t1);
    mat_mul(4, 4, 1, t1, mg.m, v1);
    mat_mul(4, 4, 4, mg.C, si, t2);
    mat_mul(4, 4, 1, t2, cond->a, v2);
    for (int k = 0; k < 4; ++k) NX.a[k] = v1[k] + v2[k];
    mat_mul(4, 4, 4, t2, cond->F, NX.F);
    mat_mul(4, 4, 4, t2, cond->A, NX.A);
    affine4 G;
    memcpy(G.a, cond->a, sizeof G.a);
    memcpy(G.F, cond->F, sizeof G.F);
    for (int k = 0; k < 16; ++k) G.A[k] = mg.C[k] + cond->A[k];
    gauss4 next_marginal = a_transform_at(&G, mg.m);
    /* propagation(sc, NX): (a.a + a.F x.a, a.F x.F, a.A + (a.F x.A) a.F^T) */
    affine4 nc;
    double Fa[4], FA[16], FAFt[16], Ft[16];
    mat_mul(4, 4, 1, sc.F, NX.a, Fa);
    for (int k = 0; k < 4; ++k) nc.a[k] = sc.a[k] + Fa[k];
    mat_mul(4, 4, 4, sc.F, NX.F, nc.F);
    mat_mul(4, 4, 4, sc.F, NX.A, FA);
    mat_t(4, 4, sc.F, Ft);
    mat_mul(4, 4, 4, FA, Ft, FAFt);
    for (int k = 0; k < 16; ++k) nc.A[k] = sc.A[k] + FAFt[k];
    return to_joint(&next_marginal, &nc);
}

/* incorporate_backward_prob (:420-447) */
static gauss8 incorporate_backward(const gauss8 *joint, const double *bwd_r, const double *p)
{
    gauss4 mg;
    affine4 cd;
    separate(joint, &mg, &cd);
    const double mp[4] = {0, 0, p[0], p[3]};
    double ip[16] = {0}, bi[16], d[16], nc[16], a[4], b[4], r[4];
    ip[10] = (2. * p[1]) / p[2];
    ip[15] = (2. * p[4]) / p[5];
    inv_n(4, bwd_r + 4, bi);
    for (int k = 0; k < 16; ++k) d[k] = bi[k] - ip[k];
    inv_n(4, d, nc);
    mat_mul(4, 4, 1, bi, bwd_r, a);
    mat_mul(4, 4, 1, ip, mp, b);
    for (int k = 0; k < 4; ++k) r[k] = a[k] - b[k];
    gauss4 back;
    mat_mul(4, 4, 1, nc, r, back.m);
    memcpy(back.C, nc, sizeof nc);
    gauss4 marginal = g_multiply(&mg, &back);
    return to_joint(&marginal, &cd);
}

/* crosscovariance_is_small (:449-458); abs() on a double resolves to fabs through <math.h> */
static int cross_small(const gauss8 *j, double tol)
{
    for (int i = 0; i < 4; ++i)
        for (int k = 4; k < 8; ++k)
            if (fabs(j->C[8 * i + k] / (j->m[i] * j->m[k])) > tol) return 0;
    return 1;
}

/* ---- the walk ---------------------------------------------------------------------------- */
typedef struct {
    const ora_forest *f;
    const double *params, *fwd, *bwd, *bstate;
    int n_seg;
    double tol;
    int64_t start, cap, count;
    int64_t *out_idx;
    double *out_val;
    gauss8 *joint;   /* per cell: MOMAdata::joint */
} walk_t;

static const double *segp(const walk_t *w, int64_t r)
{
    int s = w->f->segment ? w->f->segment[r] : 0;
    if (s < 0 || s >= w->n_seg) s = 0;
    return w->params + 11 * s;
}

static void emit(walk_t *w, int64_t target, const gauss8 *j)
{
    if (w->count < w->cap) {
        w->out_idx[2 * w->count] = w->start;
        w->out_idx[2 * w->count + 1] = target;
        memcpy(w->out_val + 72 * w->count, j->m, 8 * sizeof(double));
        memcpy(w->out_val + 72 * w->count + 8, j->C, 64 * sizeof(double));
    }
    w->count++;
}

/* calc_joint_distributions (:464-524); returns 1 when the cross-covariance became small */
static int calc_joints(walk_t *w, int64_t c, int64_t n)
{
    const ora_forest *f = w->f;
    const int64_t r0 = f->row_off[c], rows = f->row_off[c + 1] - r0;
    /* cell.mean(1): the cell's state after the -p run (the backward pass's final state) */
    const double mean1 = w->bstate[(size_t)ORA_STATE * c + 1];
    for (int64_t m = 1; n + m < rows; ++m) {
        const int64_t r = r0 + n + m;
        const double *p = segp(w, r);
        double D[4] = {p[7], 0, 0, f->noise_scaled ? p[8] * (mean1 + f->fp_auto) : p[8]};
        w->joint[c] = include_measurement(&w->joint[c], D, f->log_length[r], f->fp[r]);
        gauss8 comb = incorporate_backward(&w->joint[c], w->bwd + (size_t)ORA_STATE * r, p);
        if (cross_small(&comb, w->tol)) return 1;
        emit(w, r, &comb);
        if (n + m < rows - 1) {
            affine4 cd = consecutive_conditional(p, w->fwd + (size_t)ORA_STATE * r, f->time[r + 1] - f->time[r]);
            w->joint[c] = next_joint(&w->joint[c], &cd);
        } else {
            if (f->d1[c] >= 0) {
                const int64_t d1 = f->d1[c];
                affine4 cd = consecutive_conditional_cell_division(
                    segp(w, r0 + rows - 1), w->fwd + (size_t)ORA_STATE * r, f->time[f->row_off[d1]] - f->time[r],
                    f->div_binomial);
                w->joint[c] = next_joint(&w->joint[c], &cd);
                w->joint[d1] = w->joint[c];
            }
            if (f->d2[c] >= 0) w->joint[f->d2[c]] = w->joint[c];
        }
    }
    return 0;
}

/* joint_distributions_recr (:531-552) */
static void walk_recr(walk_t *w, int64_t c, int64_t n, int at_division)
{
    if (c < 0) return;
    if (!at_division && calc_joints(w, c, n)) return;
    walk_recr(w, w->f->d1[c], -1, 0);
    walk_recr(w, w->f->d2[c], -1, 0);
}

int64_t ora_joints(const ora_forest *f, const double *params, int n_seg, const double *fwd, const double *bwd,
                   const double *bstate, double tol, int64_t r_lo, int64_t r_hi, int64_t cap, int64_t *out_idx,
                   double *out_val)
{
    walk_t w = {f, params, fwd, bwd, bstate, n_seg, tol, 0, cap, 0, out_idx, out_val, NULL};
    w.joint = (gauss8 *)calloc((size_t)(f->n_cells > 0 ? f->n_cells : 1), sizeof(gauss8));
    /* sc_joint_distributions (:557-600) for every start row in [r_lo, r_hi) */
    for (int64_t c = 0; c < f->n_cells; ++c) {
        const int64_t r0 = f->row_off[c], rows = f->row_off[c + 1] - r0;
        for (int64_t n = 0; n < rows; ++n) {
            const int64_t r = r0 + n;
            if (r < r_lo || r >= r_hi) continue;
            w.start = r;
            const double *p = segp(&w, r);
            if (n < rows - 1) {
                w.joint[c] = consecutive_joint(p, fwd + (size_t)ORA_STATE * r, f->time[r + 1] - f->time[r]);
                walk_recr(&w, c, n, 0);
            } else {
                if (f->d1[c] >= 0) {
                    const int64_t d1 = f->d1[c];
                    w.joint[c] = consecutive_joint_cell_division(p, fwd + (size_t)ORA_STATE * r,
                                                                 f->time[f->row_off[d1]] - f->time[r], f->div_binomial);
                    w.joint[d1] = w.joint[c];
                }
                if (f->d2[c] >= 0) w.joint[f->d2[c]] = w.joint[c];
                walk_recr(&w, c, n, 1);
            }
        }
    }
    free(w.joint);
    return w.count;
}
