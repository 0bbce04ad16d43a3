/*
 * ggp.h -- C-ABI of the MI355X lineage-tree likelihood engine (libggp.so).
 *
 * This is the drop-in boundary for the reference's hot path.  The reference is one C++
 * translation unit with no plugin/FFI layer; the seam it replaces is the
 * C++ call boundary below the optimiser / scan / Hessian / smoother drivers:
 *
 *   ggp_total_loglik  replaces  total_likelihood(params, cells)      likelihood.h:170-174
 *                               (and the NLopt vfunc form            likelihood.h:125-159,
 *                                total_likelihood_log_params         likelihood.h:161-167:
 *                                the caller negates / exponentiates)
 *                               incl. likelihood_recr / sc_likelihood likelihood.h:36-122
 *   ggp_total_loglik_chain  a known sequence of total_likelihood calls, each from the state
 *                               the previous left: num_hessian_ll's 4k^2  likelihood.h:211-258
 *                               calls, the -s scan's                      main.cpp:80-114
 *   ggp_total_loglik_batch  the 4k^2 objective calls of num_hessian_ll   likelihood.h:211-258
 *                               (opt-in: points independent, not chained)
 *   ggp_joints        replaces  collect_joint_distributions (compute) correlation_tree.h:464-651
 *   ggp_predict       replaces  prediction_forward                   predictions.h:166-173
 *                               prediction_backward                  predictions.h:438-444
 *                               combine_predictions                  predictions.h:466-499
 *   ggp_forest_create replaces  the in-memory std::vector<MOMAdata> after
 *                               build_cell_genealogy + init_cells    moma_input.h:125-151,738-741
 *                               (sharded over the devices of the descriptor)
 *   ggp_predict_rows  replaces  the row loop of write_predictions_to_file predictions.h:563-602
 *
 * Plain pointers and sizes only; no HIP or torch types.  The library copies its inputs.
 *
 * Carried state: the reference's objective is stateful -- a root cell's covariance
 * off-diagonals survive from one total_likelihood call to the next (predictions.h:63-78
 * resets only the mean and the diagonal).  A ggp_forest keeps that state on the device
 * and carries it across ggp_total_loglik calls exactly like the MOMAdata vector does;
 * ggp_reset_state() restores the "fresh cells" (all zero) state of read_data().
 * ggp_predict always starts from fresh cells, as main.cpp:434-438 does.
 *
 * Errors: return codes instead of C++ exceptions.  GGP_ENAN corresponds to the
 * std::domain_error("Likelihood is Nan") of likelihood.h:71-93; the first NaN in
 * reference order (roots in input order, DFS pre-order, row) is reported.  After GGP_ENAN
 * the carried state is unspecified (the reference terminates there; which cells the failed
 * call updated depends on the schedule): ggp_reset_state or ggp_set_state before the next
 * evaluation.  Not re-entrant: one host thread per handle.
 */
#ifndef GGP_H
#define GGP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGP_OK 0
#define GGP_EINVAL 1   /* bad descriptor / argument                              */
#define GGP_ENAN 2     /* log-likelihood is NaN (likelihood.h:71-93)             */
#define GGP_EDEV 3     /* HIP runtime / device error                             */
#define GGP_ENOMEM 4   /* device allocation failed                               */
#define GGP_ETIMEOUT 5 /* a wait inside one evaluation timed out: a daughter cell's
                          wait for its parent (a scheduling stall, never a model NaN),
                          or a peer rank that never reached the collective; the carried
                          state is unspecified afterwards, as after GGP_ENAN          */

#define GGP_N_PARAMS 11      /* Parameters.h:175 order                           */
#define GGP_STATE_DOUBLES 20 /* per cell/row: mean[4] then cov[16] row-major     */

typedef struct ggp_forest ggp_forest;

#define GGP_ALL_DEVICES (-1) /* ggp_forest_desc.n_devices: every visible device     */

typedef struct {
    int64_t n_cells;             /* cells in input order (read_data order)           */
    int64_t n_rows;              /* data points (count_data_points)                  */
    const int64_t *row_offset;   /* [n_cells+1]                                      */
    const int32_t *parent;       /* [n_cells] -1 = root   (MOMAdata::parent)         */
    const int32_t *daughter1;    /* [n_cells] -1 = none   (MOMAdata::daughter1)      */
    const int32_t *daughter2;    /* [n_cells] -1 = none   (MOMAdata::daughter2)      */
    const int32_t *segment;      /* [n_rows] segment index per row, or NULL (all 0)  */
    const double *time;          /* [n_rows] time / rescale_time                     */
    const double *log_length;    /* [n_rows]                                         */
    const double *fp;            /* [n_rows]                                         */
    double root_mean_xg[2];      /* init_cells_f: mean of first x, g                 */
    double root_var_xg[2];       /*               population variance                */
    double leaf_mean_xg[2];      /* init_cells_r: mean of last x, g                  */
    double leaf_var_xg[2];
    int32_t noise_scaled;        /* 1 = "scaled" (default), 0 = "const"              */
    int32_t division_binomial;   /* 1 = "binomial" (default), 0 = "gauss"            */
    double fp_auto;              /* CSVconfig::fp_auto                               */
    int32_t n_devices;           /* shard the forest over these devices; 0 = device 0
                                    only (a zero-filled descriptor), GGP_ALL_DEVICES
                                    (-1) = every visible device                      */
    int32_t kernel;              /* GGP_KERNEL_*: scheduling policy (see below)         */
    const int32_t *devices;      /* [n_devices] HIP ordinals or NULL (= 0..n_devices-1);
                                    an ordinal may repeat: logical shards on one device */
    int64_t max_shard_rows;      /* 0: one shard per device entry; > 0: as many shards
                                    (chunks) as it takes for each to hold at most this
                                    many rows (a reduction block is never split), dealt
                                    round-robin over the devices, so the -p workspace
                                    of a device holds one chunk at a time              */
} ggp_forest_desc;

/* Sharding.  Trees are independent (likelihood.h:125-159 has no term across
 * trees), so the handle splits the forest into shards of whole trees -- whole reduction blocks
 * of B consecutive trees in root order, B a function of the tree count only -- by LPT on row
 * counts, one shard per device entry (or more, see max_shard_rows).  One host thread enqueues
 * every device, then sums: each block's trees in a fixed order on its device, the block sums in
 * a fixed pairwise tree on the host.  So every result (total, NaN location, -p rows, joints,
 * carried state) has the same bits for any device list -- 8 GPUs, or N logical shards on one. */

#define GGP_KERNEL_AUTO 0     /* per level: WAVE up to 5 cells per SIMD, PAIR up to
                                 2 x 64 cells per CU, LANE above (measured crossovers,
                                 DESIGN.md); GGP_AUTO_SMALL=group: GROUP, GROUP, PAIR,
                                 LANE -- every schedule bitwise equal to LANE         */
#define GGP_KERNEL_LANE 1     /* one lane per cell (throughput)                      */
#define GGP_KERNEL_GROUP 2    /* G lanes per cell (latency); bitwise equal to LANE   */
#define GGP_KERNEL_WAVE 3     /* one wave per cell, table-driven outputs (latency);
                                 agrees with LANE/GROUP to ~1e-10, not bitwise        */
#define GGP_KERNEL_PAIR 4     /* one lane per cell, each step split over two waves
                                 (mid-size levels); bitwise equal to LANE             */
/* Launch form (per shard, fixed at creation): when every level takes the wave schedule and the
 * shard has at most as many leaves as the device holds wave blocks, an evaluation is ONE launch
 * (a block per root-to-leaf path, the sum formed in-launch); otherwise one launch per level plus
 * a reduction.  Both give the same bits.  Environment (read at creation, tuning only):
 * GGP_WAVE_PATHS_MAX (paths allowed in one launch; 0 = always level launches),
 * GGP_WAVE_MAX_CELLS / GGP_GROUP_MAX_CELLS / GGP_PAIR_MAX_CELLS (auto's thresholds),
 * GGP_AUTO_SMALL=group, GGP_PAIR_CPW (32: 32 cells per lane-pair workgroup), GGP_PAIR_Q (2 or 4
 * waves per lane-pair cell), GGP_SMOOTHER_LANE=1 (-p levels on the lane schedule only),
 * GGP_COMBINE_EXACT=1 (ggp_predict's combine with the oracle's operations; default: through
 * reciprocal pivots, within ~1e-11 of them, DESIGN.md "Smoother"). */

int ggp_forest_create(const ggp_forest_desc *desc, ggp_forest **out);
void ggp_forest_destroy(ggp_forest *f);

/* +ll of the whole forest (total_likelihood 2-arg form).  params: 11 doubles.
 * nan_cell / nan_row (may be NULL) receive the first NaN (cell index in input order,
 * row within the cell) or -1.  Returns GGP_OK, GGP_ENAN, GGP_EDEV. */
int ggp_total_loglik(ggp_forest *f, const double *params, double *ll, int64_t *nan_cell,
                     int64_t *nan_row);

/* Batched objective (opt-in; SURVEY.md §8(f) 2 -- the Hessian of likelihood.h:211-258 needs 4k^2
 * independent points): params is n_pts*11 doubles; ll[i] receives point i's +ll and status[i]
 * GGP_OK or GGP_ENAN (ll[i] = NaN).  Every point starts from the carried state as it is at the
 * call, and the carried state is left unchanged -- the reference instead chains each call's
 * state into the next (this is the documented difference of the batched mode).  A point's value
 * is bitwise that of ggp_total_loglik with GGP_KERNEL_LANE from the same state.  Returns GGP_OK,
 * GGP_EINVAL, GGP_ENOMEM or GGP_EDEV. */
int ggp_total_loglik_batch(ggp_forest *f, int32_t n_pts, const double *params, double *ll,
                           int32_t *status);

/* Chained objective: n_pts evaluations (params: n_pts*11 doubles) in order, each from the carried
 * state the previous one left -- the results, the NaN location and the carried state afterwards
 * are bitwise those of n_pts successive ggp_total_loglik calls.  ll[i] receives point i's +ll.
 * Stops at the first point whose evaluation fails: returns its code (GGP_ENAN / GGP_ETIMEOUT,
 * ll = NaN, nan_cell / nan_row as ggp_total_loglik reports them) with *n_ok = its index; else
 * GGP_OK with *n_ok = n_pts.  Only a root's state crosses from one evaluation to the next
 * (predictions.h:63-82), so on a path-launch handle (every level on the wave schedule) the points
 * run in one launch per chunk, point i's root waiting for point i-1's and its trees overlapping
 * with the later points'; other handles run the calls one by one (GGP_CHAIN_FUSED=0: always).
 * A chunk holds at most 2^22 rows of chained roots.  A wait of the chained schedule that times
 * out is not the calls' failure: the carried state becomes the last completed point's and the
 * remaining points run one by one (the same values; ggp_chain_fallbacks counts such chains), so
 * GGP_ETIMEOUT comes back only when a one-by-one call stalls too. */
int ggp_total_loglik_chain(ggp_forest *f, int32_t n_pts, const double *params, double *ll,
                           int32_t *n_ok, int64_t *nan_cell, int64_t *nan_row);
/* chained calls of this handle that finished one by one after a stall of the chained schedule */
int ggp_chain_fallbacks(const ggp_forest *f, int64_t *n);

/* Speculative evaluation (the -m optimiser's lookahead): n_pts points in one launch,
 * point i's roots starting from the state point pred[i] left (pred[i] in [-1, i); -1 = the
 * carried state), every other cell from its parent within its point.  ll[i] / status[i] (GGP_OK,
 * GGP_ENAN, GGP_ETIMEOUT) and, if not NULL, nan_cell[i] / nan_row[i] are what a ggp_total_loglik
 * call of point i after the calls of its pred chain would return.  The carried state is left
 * unchanged; ggp_keep_point_state(i) then makes it the state point i left (valid until the next
 * tree, chain or batch call).  Needs a path-launch handle without a communicator (else
 * GGP_EINVAL) and at most one launch's points (the batch workspace; else GGP_EINVAL). */
int ggp_total_loglik_tree(ggp_forest *f, int32_t n_pts, const double *params, const int32_t *pred,
                          double *ll, int32_t *status, int64_t *nan_cell, int64_t *nan_row);
int ggp_keep_point_state(ggp_forest *f, int32_t point);

/* Asynchronous form for drivers that pipeline: enqueue one evaluation on the handle's
 * stream; ggp_loglik_result() waits and returns what ggp_total_loglik would have. */
int ggp_total_loglik_async(ggp_forest *f, const double *params);
int ggp_loglik_result(ggp_forest *f, double *ll, int64_t *nan_cell, int64_t *nan_row);

/* -p smoother.  params: n_seg*11 doubles (one Parameter_set per segment).
 * out_fwd/out_bwd/out_comb: [n_rows*20] each (NULL = not requested).  out_bwd is in
 * normal (un-reversed) coordinates as stored in MOMAdata::mean_backward. */
int ggp_predict(ggp_forest *f, const double *params, int32_t n_seg, double *out_fwd,
                double *out_bwd, double *out_comb);

/* measurement hook (bench.py): HIP-event device time of the last completed ggp_predict on
 * the handle's stream -- the forward + backward level launches, and k_combine.  The copies
 * back to the host are excluded. */
int ggp_predict_profile(ggp_forest *f, float *ms_smooth, float *ms_combine);

/* -j compute: collect_joint_distributions (correlation_tree.h:464-651).  Runs the smoother,
 * then for every start row r in [r_lo, r_hi) (input order) the joints P(z_target, z_r | D)
 * the reference adds to its Joint_vector, in the order it adds them: out_idx[2k] = r,
 * out_idx[2k+1] = target row, out_val[72k..] = mean[8] then cov[64] row-major.  *n_out is the
 * number of joints; they are stored only when *n_out <= cap (else call again with a larger
 * cap or a smaller row range).  A launch costs its longest walk (one lane per start row), so
 * large ranges are cheap: each start is walked once into device slots sized by its bound and
 * packed, while the range's slots fit GGP_JOINT_SLOT_MB (environment, read at creation; default
 * 2048; 0 = count, then emit: two walks); the joints are the same either way. */
int ggp_joints(ggp_forest *f, const double *params, int32_t n_seg, double tol, int64_t r_lo,
               int64_t r_hi, int64_t cap, int64_t *out_idx, double *out_val, int64_t *n_out);

/* ggp_joints with 44 values per joint, what the -j writer prints (sc_joint_distributions,
 * correlation_tree.h; output_upper_triangle, predictions.h:540-551): out_val[44k..] = mean[8],
 * then the covariance's upper triangle row by row (C00, C01, .., C07, C11, .., C77).  The same
 * joints, values and order as ggp_joints; 39% fewer bytes to copy to the host. */
int ggp_joints_packed(ggp_forest *f, const double *params, int32_t n_seg, double tol, int64_t r_lo,
                      int64_t r_hi, int64_t cap, int64_t *out_idx, double *out_val, int64_t *n_out);

/* combined rows [r_lo, r_hi) (input order) of the last ggp_predict -> out[(r - r_lo) * 20]:
 * the -p writer streams a forest far larger than host memory by row ranges
 * (write_predictions_to_file, predictions.h:563-602).  The rows stay in HBM between calls. */
int ggp_predict_rows(ggp_forest *f, int64_t r_lo, int64_t r_hi, double *out);

/* the shards the handle made: *n shards; per shard (k < cap) its device, rows and cells */
int ggp_forest_shards(ggp_forest *f, int32_t *n, int32_t *device, int64_t *rows, int64_t *cells, int32_t cap);

/* test-only device math (tests/test_gpu_device_math.py), one kernel launch on `device`:
 *   ggp_debug_dawson: Faddeeva::Dawson (Faddeeva.cc:467-471) as the kernels evaluate it;
 *                     variant 0 = the lane/group form, 1 = the wave schedule's branch-free form
 *   ggp_debug_tauint: in[6i..6i+5] = (k, t0, t1, a, b, c) -> the k-th tauint of
 *                     mean_cov_model.h:9-67 from the device primitives (k = 0..3) */
int ggp_debug_dawson(int32_t device, int32_t variant, const double *x, int64_t n, double *out);
int ggp_debug_tauint(int32_t device, const double *in, int64_t n, double *out);

/* carried state: zero it (fresh cells), read it back, or restore one read earlier
 * ([n_cells*20], cells in input order) -- a checkpoint of the MOMAdata mean/cov a scan or
 * optimiser run has reached, so a resumed run continues the same chain of values */
int ggp_reset_state(ggp_forest *f);
int ggp_get_state(ggp_forest *f, double *out);
int ggp_set_state(ggp_forest *f, const double *in);

/* measurement hooks (bench.py): HIP-event timings of the launches of the last
 * ggp_total_loglik on the handle's stream.  ms[i], rows[i], kernel[i] for i < *n (cap
 * entries); kernel[i] = GGP_KERNEL_LANE << 8 | 1 or GGP_KERNEL_GROUP << 8 | G (lanes per
 * cell); GGP_KERNEL_LANE << 8 | 2 is one launch over a run of lane-schedule levels (the lane
 * queue, rows = the run's rows).  The first call only switches the events on (*n = 0); a call with cap < 0 switches them
 * off again (*n = 0). */
int ggp_last_launch_profile(ggp_forest *f, float *ms, int64_t *rows, int32_t *kernel, int32_t cap,
                            int32_t *n);
int ggp_forest_info(ggp_forest *f, int64_t *n_levels, int64_t *max_level_cells,
                    int32_t *kernel_used);

/* One process per GPU (north_star "a single RCCL collective per NLopt objective
 * call"): the handle holds this process's whole-tree shard (one device), and after
 * ggp_comm_attach every ggp_total_loglik / ggp_loglik_result returns the total over all ranks.
 * The collective is enqueued by the engine on the shard's stream right behind the evaluation:
 * a one-workgroup kernel forms this rank's partial (ggp_loglik_result's pairwise tree over its
 * blocks, and its first-NaN flag), one RCCL all-gather moves 16 B per rank over xGMI, and a
 * one-thread kernel sums the partials in rank order into mapped host memory (the host spins on
 * it): the same bits as distributed.ShardedObjective's all_gather + combine_partials.  A NaN
 * partial on any rank makes the call return GGP_ENAN on every rank (GGP_ETIMEOUT when the first
 * bad rank's first bad cell stalled); *nan_cell / *nan_row are this rank's own first NaN (-1 when
 * this rank was clean), ggp_comm_nan_rank the lowest bad rank, ggp_comm_local_nan whether this
 * rank's own evaluation was bad (its carried state is then unspecified, as after GGP_ENAN).
 * A wait for the collective is bounded (GGP_COMM_TIMEOUT_S, default 600 s: GGP_ETIMEOUT); after
 * any failure once the shard was enqueued the communicator is aborted (ncclCommAbort) and every
 * later call returns GGP_EDEV: a failed collective evaluation is fatal for the group.
 *   rccl_lib: the RCCL library to use (the one torch already loaded, so the process holds one
 *             RCCL; NULL = "librccl.so.1")
 *   id: 128 bytes (ncclUniqueId) made by ggp_comm_unique_id on rank 0 and given to every rank
 *       (ggp_comm_unique_id with id NULL only checks that the library and its entry points load:
 *       the other ranks' check before they join)
 * The shard's device must be the process's current device for RCCL (one device per handle).
 * Only the objective is collective: ggp_total_loglik_batch, ggp_predict and ggp_joints stay
 * per-rank (each rank's own trees), as distributed.py's ShardedPredictor expects. */
int ggp_comm_unique_id(const char *rccl_lib, unsigned char *id);
int ggp_comm_attach(ggp_forest *f, const char *rccl_lib, int32_t nranks, int32_t rank, const unsigned char *id);
int32_t ggp_comm_nan_rank(const ggp_forest *f);   /* first NaN rank of the last call, -1 none */
/* The shader clock the last path launch (the wave schedule's one-launch evaluation) ran at, as its
 * block 0 measured it over its path: s_memtime cycles per s_memrealtime tick (100 MHz) -- the
 * DVFS clock of a real evaluation, for a benchmark line.  GGP_EINVAL if none ran on this handle. */
int ggp_launch_clock(const ggp_forest *f, double *shader_mhz, double *window_us);
/* The host split of the handle's last objective calls (ggp_total_loglik, or ggp_total_loglik_async +
 * ggp_loglik_result), for a benchmark line: out[6i..6i+5] for the last *n = min(calls, cap, 512)
 * calls, oldest first = (enqueue_us: entry to the launches enqueued, wait_us: enqueued to the
 * completion seen through mapped memory, result_us: the host's sum and return, kernel_us: the path
 * launch's first block start to its publishing block's end on the device's 100 MHz counter (0 without
 * a path launch), shader_mhz: that launch's clock as ggp_launch_clock reports it, call: the call's
 * index on the handle).  wait_us - kernel_us is the launch's dispatch plus the completion's trip to
 * the host.  Two clock reads per call; no device work beyond the path launch's clock counters. */
int ggp_call_trace(const ggp_forest *f, int32_t cap, double *out, int32_t *n);
int32_t ggp_comm_size(const ggp_forest *f);       /* ranks of the attached RCCL communicator as RCCL
                                                     counts them (ncclCommCount); 0 = not attached,
                                                     -1 = the library lacks ncclCommCount */
int32_t ggp_comm_local_nan(const ggp_forest *f);  /* 1: this rank's own last evaluation was bad */

int ggp_device_count(int32_t *n);
const char *ggp_strerror(int code);
const char *ggp_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GGP_H */
