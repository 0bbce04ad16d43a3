/*
 * ggp_oracle.h -- CPU restatement of the reference's lineage-tree likelihood path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gfp_gaussian_process_amd/, the
 * libggp C-ABI) links, loads or calls this code.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg use it, as the checker / the timed CPU baseline.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - Dawson: pinned.  Compared with the reference's own Faddeeva.cc compiled in place
 *     into oracle/_ref (tests/golden/dawson_ref.json) and with the Maple values of the
 *     Faddeeva self-test (tests/golden/dawson_maple.json).
 *   - Propagator / likelihood / smoother: restated expression-by-expression from the
 *     reference source (file:line cited per function).  The reference cannot be executed
 *     here (it needs Eigen 3.3.7, absent from this image, and the task forbids shimming
 *     it), so these are "parity unpinned" against a reference execution; the tauint
 *     integrals are additionally checked against their defining quadrature.
 *
 * Cell layout: cells in input order, rows of cell c are row_off[c] .. row_off[c+1]-1.
 * State per cell: 20 doubles = mean[4] then cov[16] row-major (the reference keeps a
 * full, possibly bitwise-asymmetric Eigen::MatrixXd, src/moma_input.h:57-58).
 */
#ifndef GGP_ORACLE_H
#define GGP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_STATE 20

typedef struct {
    int64_t n_cells;
    int64_t n_rows;
    const int64_t *row_off;     /* [n_cells+1]                                   */
    const int32_t *parent;      /* [n_cells] -1 = root                           */
    const int32_t *d1;          /* [n_cells] first daughter in input order, -1   */
    const int32_t *d2;          /* [n_cells] second daughter, -1                 */
    const double *time;         /* [n_rows] already divided by rescale_time      */
    const double *log_length;   /* [n_rows]                                      */
    const double *fp;           /* [n_rows]                                      */
    const int32_t *segment;     /* [n_rows] or NULL (all segment 0)              */
    double root_mean_xg[2], root_var_xg[2];   /* init_cells_f, moma_input.h:675-704 */
    double leaf_mean_xg[2], leaf_var_xg[2];   /* init_cells_r, moma_input.h:706-735 */
    int noise_scaled;           /* 1 = "scaled" (default), 0 = "const"           */
    int div_binomial;           /* 1 = "binomial" (default), 0 = "gauss"         */
    double fp_auto;
} ora_forest;

/* Faddeeva::Dawson restated (Faddeeva.cc:467-471, w_im :1864-1888, w_im_y100 :1458-1862) */
double ora_dawson(double x);
/* zerotauint..treetauint (mean_cov_model.h:9-67): k = 0..3 */
double ora_tauint(int k, double a, double b, double c, double t1, double t0);
/* mean_cov_model (mean_cov_model.h:211-274): in-place on m[4], C[16];
 * p = {ml, gl, sl2, mq, gq, sq2, beta} */
void ora_mean_cov_model(double *m, double *C, double t, const double *p);
/* cross_cov_model (mean_cov_model.h:380-432): out[16] row-major */
void ora_cross_cov_model(const double *m, const double *C, double t, const double *p, double *out);

/* total_likelihood 2-arg form (likelihood.h:170-174, :125-159): returns +ll.
 * state: [n_cells*ORA_STATE], carried across calls exactly like MOMAdata.mean/cov.
 * On NaN: returns NaN and sets nan_cell, nan_row to the first NaN in reference order
 * (root order, DFS pre-order, row).  cell_ll (optional) gets per-cell partial sums. */
double ora_total_loglik(const ora_forest *f, const double *params, double *state,
                        int64_t *nan_cell, int64_t *nan_row, double *cell_ll);

/* -p: prediction_forward / prediction_backward / combine_predictions
 * (predictions.h:93-173, :183-444, :446-499).  params: n_seg*11.
 * state: [n_cells*ORA_STATE] (fresh cells = zeros, main.cpp:435).
 * fwd/bwd/comb: [n_rows*ORA_STATE] each (mean[4], cov[16]) or NULL. */
int ora_predict(const ora_forest *f, const double *params, int n_seg, double *state,
                double *fwd, double *bwd, double *comb);

/* -j: collect_joint_distributions (correlation_tree.h:464-651), compute only.  For every
 * start row r in [r_lo, r_hi) (input order) the joints P(z_target, z_r | D) the reference
 * adds to its Joint_vector, in the order it adds them: out_idx[2k] = start row,
 * out_idx[2k+1] = target row, out_val[72k..] = mean[8], cov[64] (row-major).  fwd/bwd are
 * ora_predict's outputs and bstate the state buffer it leaves (MOMAdata::mean/cov after -p).
 * Returns the number of joints (only the first cap are stored). */
int64_t ora_joints(const ora_forest *f, const double *params, int n_seg, const double *fwd,
                   const double *bwd, const double *bstate, double tol, int64_t r_lo,
                   int64_t r_hi, int64_t cap, int64_t *out_idx, double *out_val);

#ifdef ORA_EXPERIMENT
/* sensitivity experiments only: replace exp() on the propagator path */
extern double (*ora_exp_hook)(double);
extern double (*ora_dawson_hook)(double);
extern void (*ora_mcm_hook)(double *, double *, double, const double *);
#endif

#ifdef __cplusplus
}
#endif
#endif
