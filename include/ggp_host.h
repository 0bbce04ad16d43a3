/*
 * ggp_host.h -- C-ABI of the host-side forest ingest (libggp_host.so, plain C++17).
 *
 * Host half of the drop-in: it re-implements the reference's data-model layer with the
 * same semantics so that a forest handed to libggp is index-for-index the reference's
 * std::vector<MOMAdata>:
 *
 *   ggp_csv_config_load    CSVconfig::CSVconfig          CSVconfig.h:26-98
 *   ggp_param_file_load    Parameter_set::Parameter_set  Parameters.h:133-176 (+ :50-85)
 *   ggp_dataset_read       read_data                     moma_input.h:401-527
 *                          get_cell_id / remove_last_decimal            :320-355
 *   ggp_dataset_segments   get_segment_indices           moma_input.h:538-570
 *   ggp_forest_build       get_segment + build_cell_genealogy + init_cells
 *                                                        moma_input.h:580-620, 125-151, 675-741
 *
 * build_cell_genealogy is O(N^2) string compares in the reference; here it is a hash map
 * with identical outcomes (parent = LAST cell in vector order with a matching id, every
 * matching cell gets the child as daughter1 then daughter2, a third child is an error).
 */
#ifndef GGP_HOST_H
#define GGP_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "ggp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ggp_csv_config ggp_csv_config;
typedef struct ggp_dataset ggp_dataset;
typedef struct ggp_host_forest ggp_host_forest;

/* Parameter file (Parameters.h).  kind: 0 fixed, 1 free, 2 bound (Parameter::fixed/free/bound) */
typedef struct {
    char name[GGP_N_PARAMS][16];
    int32_t kind[GGP_N_PARAMS];
    int32_t set[GGP_N_PARAMS];
    double init[GGP_N_PARAMS], step[GGP_N_PARAMS], lower[GGP_N_PARAMS], upper[GGP_N_PARAMS];
} ggp_param_set;

/* error text of the last failing call on this thread */
const char *ggp_host_last_error(void);

int ggp_csv_config_load(const char *path /* NULL or "" = defaults */, ggp_csv_config **out);
void ggp_csv_config_free(ggp_csv_config *c);
/* accessors used by tests: key in {time_col, length_col, fp_col, delm, segment_col,
 * filter_col, rescale_time, fp_auto, length_islog, cell_tags, parent_tags} */
int ggp_csv_config_get(const ggp_csv_config *c, const char *key, char *buf, size_t buflen);

/* returns GGP_OK; GGP_EINVAL (message via ggp_host_last_error) on a malformed file or an
 * incomplete one when check_complete != 0 (Parameter_set::check_if_complete) */
int ggp_param_file_load(const char *path, int32_t check_complete, ggp_param_set *out);

int ggp_dataset_read(const char *infile, const ggp_csv_config *cfg, ggp_dataset **out);
void ggp_dataset_free(ggp_dataset *d);
int64_t ggp_dataset_n_cells(const ggp_dataset *d);
int64_t ggp_dataset_n_rows(const ggp_dataset *d);
/* Binary dataset: read_data's output (cells in input order, time already
 * rescaled, length already log'd, segment per row, ids) as structure-of-arrays, magic
 * "GGPD0001" (layout in ggp_host.cpp).  Loads at disk speed where the CSV parser would take
 * minutes (C4/C5 sizes); everything downstream (segments, get_segment, genealogy) is the same.
 * ggp_dataset_is_binary: 1 if the file starts with the magic.  ggp_dataset_create: a dataset
 * from arrays (e.g. a synthetic forest) to save. */
int ggp_dataset_is_binary(const char *path);
int ggp_dataset_save(const ggp_dataset *d, const char *path);
int ggp_dataset_load(const char *path, ggp_dataset **out);
int ggp_dataset_create(int64_t n_cells, const int64_t *row_offset, const double *time, const double *log_length,
                       const double *fp, const int32_t *segment, const char *const *ids,
                       const char *const *parent_ids, double fp_auto, ggp_dataset **out);
/* A dataset as the reference's input CSV (the example's column layout: an index column,
 * cell_id, time_min, parent_id, log_length, gfp[, segment]) plus the csv_config that reads it
 * back (length_islog = true, rescale_time = 1): values in %.17g, so ggp_dataset_read of the
 * pair gives the dataset bit for bit -- a synthetic forest the reference binary can read
 * (SURVEY §8(d)).  Ids are written verbatim; an id read_data would renormalise (all digits and
 * dots, last part zeros: moma_input.h:320-338) is refused (GGP_EINVAL). */
int ggp_dataset_write_csv(const ggp_dataset *d, const char *csv_path, const char *config_path);

/* segment indices in order of first occurrence; *n receives the count (<= cap copied) */
int ggp_dataset_segments(const ggp_dataset *d, int32_t *out, int32_t cap, int32_t *n);

/* segment < 0: the whole dataset (-p / -j path, main.cpp:434-443)
 * segment >= 0: get_segment copy (-m / -s path, main.cpp:402-432) */
int ggp_forest_build(const ggp_dataset *d, int32_t segment, int32_t noise_scaled,
                     int32_t division_binomial, ggp_host_forest **out);
void ggp_host_forest_free(ggp_host_forest *f);
/* fills every field of desc except device/kernel; pointers stay owned by f */
int ggp_host_forest_desc(const ggp_host_forest *f, ggp_forest_desc *desc);
const char *ggp_host_forest_cell_id(const ggp_host_forest *f, int64_t i);
const char *ggp_host_forest_parent_id(const ggp_host_forest *f, int64_t i);
int64_t ggp_host_forest_n_roots(const ggp_host_forest *f);

/* Synthetic forests (BASELINE.md / SURVEY.md §8d): n_trees trees of P rows each, a root
 * of P/2 rows and two daughters of P/4 rows (P=200: 100+50+50), dt = 1, data simulated
 * from the model SDE with the example parameters, Philox4x32 keyed by (seed, tree).
 * Deterministic and independent of how trees are split: tree k of a forest built with
 * first_tree = k0 is tree k0+k of the full forest. */
int ggp_synthetic_forest(int64_t n_trees, int64_t rows_per_tree, uint64_t seed,
                         int64_t first_tree, int32_t noise_scaled, int32_t division_binomial,
                         ggp_host_forest **out);

/* ---- -m / error-bar numerics (CPU; the objective is a callback) ------------------------
 * The objective returns 0 and writes *value, or non-zero to stop the run (the reference's
 * objective throws std::domain_error on a NaN likelihood, likelihood.h:71-93). */
typedef int (*ggp_objective_fn)(const double *x, double *value, void *data);

/* NLopt 2.7.1 LN_NELDERMEAD as minimizer_nlopt.h:112-215 configures it (bounds, initial
 * step, ftol_abs; maxeval <= 0: none).  Returns the nlopt_result code (3 FTOL_REACHED,
 * 4 XTOL_REACHED, 5 MAXEVAL_REACHED, -1 FAILURE, -2 INVALID_ARGS, -5 FORCED_STOP); x is
 * the best point seen, *minf its value.  Restatement: csrc/host/ggp_nelder_mead.h. */
int ggp_nldrmd_minimize(int32_t n, ggp_objective_fn f, void *data, const double *lb, const double *ub,
                        double *x, const double *dx, double ftol_abs, int64_t maxeval, double *minf,
                        int64_t *nevals);

/* ggp_nldrmd_minimize with the lookahead (csrc/host/ggp_nelder_mead.h Lookahead), for an
 * objective whose calls carry state: need(x, data) returns non-zero when the objective cannot
 * serve the call x from what it evaluated ahead; tree(x, pred, n_pts, data) then receives the
 * run's possible next calls (n_pts points, n doubles each; pred[i] = the point whose state point i
 * starts from, -1 = the next call) to evaluate ahead, e.g. with ggp_total_loglik_tree.  depth /
 * max_nodes bound the tree (<= 0: 2 / 40).  The calls made, and the result, are those of
 * ggp_nldrmd_minimize. */
typedef int (*ggp_ahead_need_fn)(const double *x, void *data);
typedef void (*ggp_ahead_tree_fn)(const double *x, const int32_t *pred, int32_t n_pts, void *data);
int ggp_nldrmd_minimize_ahead(int32_t n, ggp_objective_fn f, ggp_ahead_need_fn need, ggp_ahead_tree_fn tree,
                              void *data, const double *lb, const double *ub, double *x, const double *dx,
                              double ftol_abs, int64_t maxeval, double *minf, int64_t *nevals, int32_t depth,
                              int32_t max_nodes);

/* num_hessian_ll (likelihood.h:211-258): central 4-point differences over the parameters
 * idx[0..k-1] of x, h_i = max(x_i * epsilon, 1e-12), evaluated in the reference's order
 * (i, j, then ++ +- -+ --).  out: k*k row-major.  Returns 0, or the callback's stop. */
int ggp_num_hessian(int32_t n, ggp_objective_fn f, void *data, const double *x, const int32_t *idx, int32_t k,
                    double epsilon, double *out);

/* Eigen 3.3 MatrixXd::inverse(): partial-pivot LU (first max |a|), solved against the
 * identity.  a, out: k*k row-major. */
int ggp_inverse_pplu(int32_t k, const double *a, double *out);

#ifdef __cplusplus
}
#endif
#endif
