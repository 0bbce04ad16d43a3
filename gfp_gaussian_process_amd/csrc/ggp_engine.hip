// ggp_engine.hip -- MI355X (gfx950) lineage-tree likelihood engine behind include/ggp.h.
//
// Data layout in HBM (one ggp_forest, one device):
//   time/log_length/fp [n_rows] f64, cell-major in input order   (read 24 B per update)
//   row_off [n_cells+1] i64, parent [n_cells] i32, segment [n_rows] i32
//   state   [n_cells][20] f64   carried MOMAdata mean/cov (likelihood)
//   pstate  [n_cells][20] f64   smoother working state (fresh per ggp_predict)
//   level cells [n_cells] i32   cells grouped by generation depth, each level sorted by
//                               row count (longest first) so a wave's lanes finish together
//   cell_ll [n_cells] f64, cell_nan [n_cells] i32, dfs_order [n_cells] i32
//
// Schedule: the recursion likelihood_recr (likelihood.h:110-122) only orders a daughter
// after its parent; every cell of one generation depth is independent.  One launch per
// depth processes all cells of that depth; inside a cell the rows are sequential (each
// prior depends on the previous posterior, mean_cov_model is nonlinear, no parallel
// scan exists).  A final single-workgroup kernel sums the per-cell partials in DFS order
// with a fixed reduction tree (bitwise reproducible) and finds the first NaN.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "ggp.h"
#include "ggp_device.h"
#include "ggp_prop.h"
#include "ggp_outtab.h"
#include "ggp_wave.h"
#include "ggp_predict.h"
#include "ggp_joints.h"

#ifdef GGP_EXACT
#define GGP_VERSION "ggp-mi355x 0.2.0 exact arithmetic (reference gfp_gaussian_process 0.4.2)"
#else
#define GGP_VERSION "ggp-mi355x 0.2.0 (reference gfp_gaussian_process 0.4.2)"
#endif

namespace {

struct DevForest {
    const double *time, *logl, *fp;
    const int64_t *row_off;
    const int32_t *parent, *d1, *d2, *seg;
    const int32_t *dfs_rank;   // cell -> its position in the DFS order (the reduction's order)
    double root_mean0, root_mean1, root_var0, root_var1;
    double leaf_mean0, leaf_var0, leaf_mean1, leaf_var1;
    double fp_auto, two_log_2pi, log2;
    int scaled, binomial;
};

constexpr int kNanNone = 0x7fffffff;
constexpr int kRowStall = 0xffffff;   // a cell never has 2^24 - 1 rows (ggp_forest_create checks)

// agent-coherent (every XCD) loads and stores: the hand-offs between workgroups of one launch
GGP_DEV unsigned add_agent(unsigned *p) { return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
GGP_DEV void zero_agent(unsigned *p) { __hip_atomic_store(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
GGP_DEV double ld_agent(const double *p)
{
    return __longlong_as_double(
        (long long)__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
GGP_DEV void st_agent(double *p, const double v)
{
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
GGP_DEV T ld_agent_i(const T *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <class T>
GGP_DEV void st_agent_i(T *p, const T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// lane-schedule kernels' register budget (tools/lane_wpe_ab.py builds a GGP_LANE_WPE=2 variant)
#ifdef GGP_LANE_WPE
#define GGP_LANE_ATTR __attribute__((amdgpu_waves_per_eu(GGP_LANE_WPE)))
#else
#define GGP_LANE_ATTR
#endif

// Dawson coefficient table copied to LDS once per workgroup (LDS gather ~100 cycles vs an
// L2 round trip per coefficient from constant memory).  Every lane issues all its global loads
// before the first LDS store (one memory latency per launch, not one per 64 coefficients:
// the loop form waited for each load, ~8 us of a level launch's fixed cost).
// (GGP_EXACT: the same array continues with glibc's exp table, ggp_prop.h kPropTabN)
constexpr int kDawsonTab = ggp::kExact ? ggp::kPropTabN : ggp::kDawsonTabN;
template <int N, class SRC>
GGP_DEV void lds_fill(double *dst, const int lane, const SRC &src)
{
    constexpr int R = (N + 63) / 64;
    double v[R];
#pragma unroll
    for (int j = 0; j < R; ++j) v[j] = src(min(lane + 64 * j, N - 1));
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (lane + 64 * j < N) dst[lane + 64 * j] = v[j];
}

GGP_DEV void load_dawson_table(double *s_tab, int lane)
{
    lds_fill<kDawsonTab>(s_tab, lane, [](const int k) { return ggp::prop_tab_entry(k); });
}

// ------------------------------------------------------------------------------------------
// Cell prologue shared by both schedules: init_sc_distribution (predictions.h:63-82).
// Root: mean + diagonal from init_cells_f and the parameters; the off-diagonals keep this
// root's state from the previous evaluation (carried state).  Daughter: a copy of the
// parent's final posterior, to be propagated over dt and mapped through the division.
// ------------------------------------------------------------------------------------------
GGP_DEV void root_init(const DevForest &F, const double *p, double *m, double *C)
{
    m[0] = F.root_mean0;
    m[1] = F.root_mean1;
    C[0] = F.root_var0;
    C[5] = F.root_var1;
    m[2] = p[0];
    m[3] = p[3];
    C[10] = p[2] / (2. * p[1]);
    C[15] = p[5] / (2. * p[4]);
}

GGP_DEV bool cell_prologue(const DevForest &F, const double *p, const double *state, int c,
                           int64_t r0, double *m, double *C, double &dt_div)
{
    const int par = F.parent[c];
    if (par < 0) {
        const double *st = state + (size_t)20 * c;
#pragma unroll
        for (int k = 0; k < 16; ++k) C[k] = st[4 + k];
        root_init(F, p, m, C);
        dt_div = 0.0;
        return false;
    }
    const double *ps = state + (size_t)20 * par;
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = ps[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) C[k] = ps[4 + k];
    dt_div = F.time[r0] - F.time[F.row_off[par + 1] - 1];
    return true;
}

// ------------------------------------------------------------------------------------------
// LANE schedule: one lane per cell.  sc_likelihood (likelihood.h:36-103) for every cell of
// one generation depth.  `cpw` cells per 64-lane wave: < 64 spreads a small level over
// more SIMDs (latency), 64 packs waves (throughput); results do not depend on it.
// ------------------------------------------------------------------------------------------
// one cell of the lane schedule (the cell's lane).  QUEUE (k_loglik_lane_queue): a parent in the
// same launch is read with agent-coherent loads once its done flag is seen, a stalled wait makes
// the cell a stall (no rows run), and a cell with daughters in the launch publishes its final
// state (coherent stores, then its flag); the arithmetic is the same either way
template <bool QUEUE>
GGP_DEV void lane_cell_body(const DevForest &F, const double *p, const int c, double *__restrict__ state,
                            double *__restrict__ cell_ll, int32_t *__restrict__ cell_nan, const double *s_tab,
                            const bool stall = false, const bool publish = false, unsigned *cell_done = nullptr,
                            const unsigned epoch = 0)
{
    const ggp::OU ou = ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    double m[4], C[16];
    const int64_t r0 = F.row_off[c], r1 = F.row_off[c + 1];
    double dt = 0.0;
    bool pending;
    if constexpr (QUEUE) {
        const int par = F.parent[c];
        if (par < 0) {
            pending = cell_prologue(F, p, state, c, r0, m, C, dt);
        } else {   // the parent's final posterior, written by another workgroup of this launch
            const double *ps = state + (size_t)20 * par;
#pragma unroll
            for (int k = 0; k < 4; ++k) m[k] = ld_agent(ps + k);
#pragma unroll
            for (int k = 0; k < 16; ++k) C[k] = ld_agent(ps + 4 + k);
            dt = F.time[r0] - F.time[F.row_off[par + 1] - 1];
            pending = true;
        }
    } else {
        pending = cell_prologue(F, p, state, c, r0, m, C, dt);
    }
    bool divide = pending;
    double cl = 0.0;
    int nan_row = kNanNone;
    double t_cur = F.time[r0];
    int64_t r_end = r1;
    if (QUEUE && stall) {   // the parent never published: no row runs, the cell reports the stall
        cl = __longlong_as_double(0x7ff8000000000000LL);
        nan_row = kRowStall;
        r_end = r0;
    }
    for (int64_t r = r0; r < r_end; ++r) {
        // this row's data and the next row's time, loaded before the propagation they would
        // otherwise wait behind (the same values)
        const double y_l = F.logl[r], y_f = F.fp[r];
        const double t_next = r + 1 < r1 ? F.time[r + 1] : 0.0;
        if (pending) {   // mean_cov_model over dt (likelihood.h:97-101 / predictions.h:28-31)
            ggp::propagate_lane(m, C, dt, ou, s_tab);
            if (divide) {
                ggp::division_map(m, C, p[9], p[10], F.binomial, F.log2);
                divide = false;
            }
        }
        const double x0 = y_l - m[0];
        const double x1 = y_f - m[1];
        ggp_innov v;
        ggp_innovation(m, C, p[7], p[8], F.scaled, F.fp_auto, v);
        cl += ggp_ll_term(x0, x1, v, F.two_log_2pi);
        if (cl != cl) {
            nan_row = (int)(r - r0);
            break;
        }
        ggp_posterior(m, C, x0, x1, v);
        pending = r + 1 < r1;
        if (pending) dt = t_next - t_cur;
        t_cur = t_next;
    }
    double *st = state + (size_t)20 * c;
    if (QUEUE && publish) {
#pragma unroll
        for (int k = 0; k < 4; ++k) st_agent(st + k, m[k]);
#pragma unroll
        for (int k = 0; k < 16; ++k) st_agent(st + 4 + k, C[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) st[k] = m[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) st[4 + k] = C[k];
    }
    cell_ll[F.dfs_rank[c]] = cl;
    cell_nan[F.dfs_rank[c]] = nan_row;
    if (QUEUE && publish) {
        __builtin_amdgcn_s_waitcnt(0);   // the state at the coherence point, then the flag
        __hip_atomic_store(cell_done + c, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

GGP_DEV void loglik_lane_cell(const DevForest &F, const double *p, const int32_t *__restrict__ cells,
                              const int n, const int cpw, double *__restrict__ state,
                              double *__restrict__ cell_ll, int32_t *__restrict__ cell_nan,
                              const double *s_tab, const int lane)
{
    if (lane >= cpw) return;
    const int i = blockIdx.x * cpw + lane;
    if (i >= n) return;
    lane_cell_body<false>(F, p, cells[i], state, cell_ll, cell_nan, s_tab);
}

__global__ __launch_bounds__(64) GGP_LANE_ATTR void k_loglik_level(DevForest F, ggp_params P,
                                                      const int32_t *__restrict__ cells, int n,
                                                      int cpw, double *__restrict__ state,
                                                      double *__restrict__ cell_ll,
                                                      int32_t *__restrict__ cell_nan)
{
    __shared__ double s_tab[kDawsonTab];
    const int lane = threadIdx.x;
    load_dawson_table(s_tab, lane);
    __syncthreads();
    loglik_lane_cell(F, P.p, cells, n, cpw, state, cell_ll, cell_nan, s_tab, lane);
}

// Batched objective (ggp_total_loglik_batch): blockIdx.y = parameter point.  Each point has
// its own parameter row, state slice [n_cells x 20] and per-cell ll / NaN slices; the cell
// body is the lane schedule's, so a point's result is bitwise that of a single lane-schedule
// evaluation from the same starting state.
__global__ __launch_bounds__(64) GGP_LANE_ATTR void k_loglik_level_batch(DevForest F, const double *__restrict__ ptab,
                                                            const int32_t *__restrict__ cells, int n, int cpw,
                                                            int64_t n_cells, double *__restrict__ state,
                                                            double *__restrict__ cell_ll,
                                                            int32_t *__restrict__ cell_nan)
{
    __shared__ double s_tab[kDawsonTab];
    const int lane = threadIdx.x;
    load_dawson_table(s_tab, lane);
    __syncthreads();
    const int64_t pt = blockIdx.y;
    loglik_lane_cell(F, ptab + 11 * pt, cells, n, cpw, state + pt * n_cells * 20, cell_ll + pt * n_cells,
                     cell_nan + pt * n_cells, s_tab, lane);
}

// ------------------------------------------------------------------------------------------
// LANE QUEUE: a run of consecutive lane-schedule levels in one persistent launch.  The levels'
// cells are cut into chunks of up to 64 (one cell per lane, the level order), and one workgroup
// per SIMD takes chunks from a counter until none is left.  A chunk of a later level of the run
// waits, lane by lane, for its cells' parents' done flags; every chunk ahead of it in the queue
// is held by a running workgroup, so the waits end.  Level-by-level launches leave the SIMDs
// idle on the last round of each level: C4 (1e5 roots of 100 rows, then 2e5 daughters of 50)
// takes 2 rounds of roots and 4 of daughters, 400 row-steps, where the queue starts daughters in
// the roots' second round, 350.  The cell body is the lane schedule's (lane_cell_body): results
// are bitwise the level launches'.
// ------------------------------------------------------------------------------------------
struct QChunk {
    int32_t a, n;        // the chunk's cells: level_cells[a .. a + n)
    int32_t wait;        // 1: the cells' parents are in the launch (their flags are waited for)
    int32_t publish;     // 1: the cells' daughters are in the launch (flags published)
};

__global__ __launch_bounds__(64) GGP_LANE_ATTR void k_loglik_lane_queue(
    DevForest F, ggp_params P, const int32_t *__restrict__ cells, const QChunk *__restrict__ chunks, int n_chunks,
    unsigned *qctr, unsigned *cell_done, unsigned epoch, unsigned spin_max, double *__restrict__ state,
    double *__restrict__ cell_ll, int32_t *__restrict__ cell_nan)
{
    __shared__ double s_tab[kDawsonTab];
    const int lane = threadIdx.x;
    load_dawson_table(s_tab, lane);
    __syncthreads();
    for (;;) {   // every workgroup ends when the counter passes n_chunks
        unsigned k = 0;
        if (lane == 0) k = add_agent(qctr);
        k = (unsigned)__builtin_amdgcn_readfirstlane((int)k);
        if (k >= (unsigned)n_chunks) break;
        const QChunk q = chunks[k];
        if (lane < q.n) {
            const int c = cells[q.a + lane];
            bool stall = false;
            if (q.wait) {
                const int par = F.parent[c];
                unsigned spins = 0;
                while (par >= 0 && ld_agent_i(cell_done + par) != epoch) {
                    if (++spins > spin_max) {
                        stall = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            }
            lane_cell_body<true>(F, P.p, c, state, cell_ll, cell_nan, s_tab, stall, q.publish != 0, cell_done, epoch);
        }
    }
}

// ------------------------------------------------------------------------------------------
// LANE-PAIR schedule (k_loglik_pair<Q, CPW>): the lane schedule with every step of a cell split
// over the Q = 2 or 4 waves of a workgroup.  Lane l of every wave holds cell l (CPW cells per
// workgroup); wave w forms the w-th Q-th of the exponentials, of the Dawson values and of the
// integrals, and waves 0 and 1 one output group each (ggp::outputs<1>, <2>); each part goes
// through LDS to the other waves (three workgroup barriers per step), and every wave runs the
// measurement update.  Every value is the lane schedule's expression (the same task bodies,
// index sequences and outputs text), so results are bitwise the lane schedule's; a step issues
// ~1/Q of the lane schedule's task work per wave, for levels too small to fill the SIMDs with
// 64-cell lane waves (C3, C4 shards), where the lane schedule waits on its ~4.1k-instruction step.
// ------------------------------------------------------------------------------------------
namespace pair {
// the output groups of ggp::outputs<PARTS> (bits 1, 2, 4, 8) and the covariance slots each forms;
// wave w of Q forms the groups of kParts[Q / 4][w], the others come through LDS slot kOSlot
constexpr int kOGroups[4][6] = {{1, -1}, {0, 2, 3, 6, 10, -1}, {7, 11, 15, -1}, {5, -1}};
constexpr int kOSlot[16] = {1, 0, 2, 3, -1, 9, 4, 6, -1, -1, 5, 7, -1, -1, -1, 8};
constexpr int kOSlots = 10;
constexpr int kParts[2][4] = {{1 | 2, 4 | 8, 0, 0}, {1, 2, 4, 8}};

template <int OFF, size_t... J>
GGP_DEV void exps(const ggp::Step &S, double *Xc, const double *tab, std::index_sequence<J...> seq, bool &cold)
{
    ggp::lane_exps_flagged<OFF>(S, Xc, tab, seq, cold);   // the lane schedule's computed exponentials (ggp_prop.h), OFF + J
}
template <int OFF, size_t... J>
GGP_DEV void dawsons(const ggp::Step &S, double *Dw, const double *tab, std::index_sequence<J...>)
{
    ((Dw[OFF + J] = ggp_dawson_tab(ggp::zval(S, ggp::kDT[OFF + J].iB, ggp::kDT[OFF + J].it), tab)), ...);
}
template <int OFF, class XA, class DA, class PA, size_t... J>
GGP_DEV void taus(const ggp::Step &S, const XA &X, const DA &Dw, const PA &PW, double *I, std::index_sequence<J...>)
{
    ((I[OFF + J] = ggp::lane_tau<(int)(OFF + J)>(S, X, Dw, PW)), ...);
}

// wave W's part [N W / Q, N (W + 1) / Q) of N tasks: own values to LDS (slot-major, [slot][CPW])
// before the barrier, the other waves' into the register array after it
template <int N, int W, int Q, int CPW>
GGP_DEV void put_part(const double *v, double *L, const int lane)
{
    constexpr int lo = N * W / Q, hi = N * (W + 1) / Q;
#pragma unroll
    for (int j = lo; j < hi; ++j) L[j * CPW + lane] = v[j];
}
template <int N, int W, int Q, int CPW>
GGP_DEV void get_rest(double *v, const double *L, const int lane)
{
    constexpr int lo = N * W / Q, hi = N * (W + 1) / Q;
#pragma unroll
    for (int j = 0; j < lo; ++j) v[j] = L[j * CPW + lane];
#pragma unroll
    for (int j = hi; j < N; ++j) v[j] = L[j * CPW + lane];
}

// one propagation (propagate_lane's order) by wave W of Q; Xl/Dl/Il/Ol: LDS [slot][CPW]
template <int W, int Q, int CPW>
GGP_DEV void propagate(double *m, double *C, const double t, const ggp::OU &P, const double *tab, double *Xl,
                       double *Dl, double *Il, double *Ol, const int lane)
{
    constexpr int X0 = ggp::NXC * W / Q, XN = ggp::NXC * (W + 1) / Q - X0;
    constexpr int D0 = ggp::ND * W / Q, DN = ggp::ND * (W + 1) / Q - D0;
    constexpr int I0 = ggp::NI * W / Q, IN = ggp::NI * (W + 1) / Q - I0;
    ggp::Step S;
    ggp::step_init(S, m, C, t, P);
    double Xc[ggp::NXC], X[ggp::NXE], Dw[ggp::ND];
    bool cold = false;   // GGP_EXACT: an exponential argument outside exp_glibc's main path
    exps<X0>(S, Xc, tab, std::make_index_sequence<XN>{}, cold);
    dawsons<D0>(S, Dw, tab, std::make_index_sequence<DN>{});
    const bool own = lane < CPW;   // lanes past CPW hold no cell and store nothing
    const int ln = own ? lane : 0;
    if (own) {
        put_part<ggp::NXC, W, Q, CPW>(Xc, Xl, lane);
        put_part<ggp::ND, W, Q, CPW>(Dw, Dl, lane);
    }
    if constexpr (ggp::kExact) {
        if (__builtin_expect(own && cold, 0)) {   // an argument of this wave's share outside exp_glibc's
            // main path: the share again through exp_glibc's special paths, one rolled loop (one copy of
            // the code) into the LDS slots, and this wave's registers back from them
            for (int k = X0; k < X0 + XN; ++k)
                Xl[k * CPW + lane] = ggp::exp_glibc(ggp::exp_arg_body(S, ggp::unpack_x(ggp::kXCPacked.w[k])),
                                                    ggp::exp_tab_of(tab));
#pragma unroll
            for (int j = X0; j < X0 + XN; ++j) Xc[j] = Xl[j * CPW + lane];
        }
    }
    __syncthreads();
    get_rest<ggp::NXC, W, Q, CPW>(Xc, Xl, ln);
    get_rest<ggp::ND, W, Q, CPW>(Dw, Dl, ln);
    ggp::lane_expand(Xc, X);   // the slots, X_ONE and the products, in every wave
    ggp::lane_guard_products(S, X, tab);
    double PW[ggp::NPW];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        PW[q] = ggp::pow_task(S, q);
        PW[3 + q] = ggp::frcp(PW[q]);   // rdiv seeds
    }
    double I[ggp::NI];
    taus<I0>(S, X, Dw, PW, I, std::make_index_sequence<IN>{});
    if (own) put_part<ggp::NI, W, Q, CPW>(I, Il, lane);
    __syncthreads();
    get_rest<ggp::NI, W, Q, CPW>(I, Il, ln);
    double Co[16];
    constexpr int PM = kParts[Q / 4][W];
    ggp::outputs<PM>(S, I, X, m, Co);   // the means in every wave, this wave's output groups
    if (own) {
#pragma unroll
        for (int gi = 0; gi < 4; ++gi)
            if ((PM >> gi) & 1)
#pragma unroll
                for (int k = 0; k < 6 && kOGroups[gi][k] >= 0; ++k) Ol[kOSlot[kOGroups[gi][k]] * CPW + lane] = Co[kOGroups[gi][k]];
    }
    __syncthreads();
#pragma unroll
    for (int gi = 0; gi < 4; ++gi)
        if (!((PM >> gi) & 1))
#pragma unroll
            for (int k = 0; k < 6 && kOGroups[gi][k] >= 0; ++k) Co[kOGroups[gi][k]] = Ol[kOSlot[kOGroups[gi][k]] * CPW + ln];
    Co[4] = Co[1]; Co[8] = Co[2]; Co[12] = Co[3]; Co[9] = Co[6]; Co[13] = Co[7]; Co[14] = Co[11];
#pragma unroll
    for (int k = 0; k < 16; ++k) C[k] = Co[k];
}
// wave w's body (w is wave-uniform): one instantiation per wave of the workgroup
template <int W, int Q, int CPW>
GGP_DEV void propagate_from(const int w, double *m, double *C, const double t, const ggp::OU &P, const double *tab,
                            double *Xl, double *Dl, double *Il, double *Ol, const int lane)
{
    if constexpr (W + 1 == Q) {
        propagate<W, Q, CPW>(m, C, t, P, tab, Xl, Dl, Il, Ol, lane);
    } else {
        if (w == W) propagate<W, Q, CPW>(m, C, t, P, tab, Xl, Dl, Il, Ol, lane);
        else propagate_from<W + 1, Q, CPW>(w, m, C, t, P, tab, Xl, Dl, Il, Ol, lane);
    }
}
template <int Q, int CPW>
GGP_DEV void propagate_w(const int w, double *m, double *C, const double t, const ggp::OU &P, const double *tab,
                         double *Xl, double *Dl, double *Il, double *Ol, const int lane)
{
    propagate_from<0, Q, CPW>(w, m, C, t, P, tab, Xl, Dl, Il, Ol, lane);
}
}  // namespace pair

template <int Q, int CPW>
__global__ __launch_bounds__(64 * Q) void k_loglik_pair(DevForest F, ggp_params P, const int32_t *__restrict__ cells, int n,
                                                        double *__restrict__ state, double *__restrict__ cell_ll,
                                                        int32_t *__restrict__ cell_nan)
{
    static_assert(Q == 2 || Q == 4, "two or four waves per workgroup");
    __shared__ double s_tab[kDawsonTab];
    __shared__ double s_x[ggp::NXC * CPW], s_d[ggp::ND * CPW], s_i[ggp::NI * CPW],
        s_o[pair::kOSlots * CPW];
    __shared__ int s_rows[64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w == 0) load_dawson_table(s_tab, lane);
    const int i = blockIdx.x * CPW + lane;
    const bool valid = lane < CPW && i < n;
    const double *p = P.p;
    const ggp::OU ou = ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    int c = 0, nrows = 0;
    int64_t r0 = 0;
    double m[4] = {0, 0, 0, 0}, C[16] = {0};
    double dt = 0.0, t_cur = 0.0;   // t_cur: this row's time, carried from the previous row's load
    bool pending = false, divide = false;
    if (valid) {
        c = cells[i];
        r0 = F.row_off[c];
        nrows = (int)(F.row_off[c + 1] - r0);
        pending = cell_prologue(F, p, state, c, r0, m, C, dt);
        divide = pending;
        if (nrows > 0) t_cur = F.time[r0];
    }
    // lanes without a cell propagate lane 0's state (never stored): finite operands, so they
    // take none of the Dawson's rare branches
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const double v = __shfl(m[q], 0);
        m[q] = valid ? m[q] : v;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const double v = __shfl(C[q], 0);
        C[q] = valid ? C[q] : v;
    }
    {
        const double v = __shfl(dt, 0);
        dt = valid ? dt : v;
    }
    // the steps every wave takes: the longest cell of the workgroup (a barrier count all share)
    if (w == 0) s_rows[lane] = nrows;
    __syncthreads();
    int kmax = 0;
    for (int l = 0; l < CPW; ++l) kmax = max(kmax, s_rows[l]);
    double cl = 0.0;
    int nan_row = kNanNone;
    bool live = valid && nrows > 0;
    for (int k = 0; k < kmax; ++k) {
        const int64_t r = r0 + k;
        double y_l = 0.0, y_f = 0.0, t_next = 0.0;
        if (live) {
            y_l = F.logl[r];
            y_f = F.fp[r];
            if (k + 1 < nrows) t_next = F.time[r + 1];
        }
        // every wave decides alike: the same cells, the same flags
        if (__builtin_amdgcn_ballot_w64(live && pending)) {
            double mn[4], Cn[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) mn[q] = m[q];
#pragma unroll
            for (int q = 0; q < 16; ++q) Cn[q] = C[q];
            pair::propagate_w<Q, CPW>(w, mn, Cn, dt, ou, s_tab, s_x, s_d, s_i, s_o, lane);
            if (live && pending) {
#pragma unroll
                for (int q = 0; q < 4; ++q) m[q] = mn[q];
#pragma unroll
                for (int q = 0; q < 16; ++q) C[q] = Cn[q];
                if (divide) {
                    ggp::division_map(m, C, p[9], p[10], F.binomial, F.log2);
                    divide = false;
                }
            }
        }
        if (live) {   // likelihood.h:53-69, as loglik_lane_cell
            const double x0 = y_l - m[0];
            const double x1 = y_f - m[1];
            ggp_innov v;
            ggp_innovation(m, C, p[7], p[8], F.scaled, F.fp_auto, v);
            cl += ggp_ll_term(x0, x1, v, F.two_log_2pi);
            if (cl != cl) {
                nan_row = k;
                live = false;
            } else {
                ggp_posterior(m, C, x0, x1, v);
                pending = k + 1 < nrows;
                if (pending) dt = t_next - t_cur;   // no load on the step's chain
                t_cur = t_next;
                live = k + 1 < nrows;
            }
        }
    }
    if (valid && w == 0) {
        double *st = state + (size_t)20 * c;
#pragma unroll
        for (int q = 0; q < 4; ++q) st[q] = m[q];
#pragma unroll
        for (int q = 0; q < 16; ++q) st[4 + q] = C[q];
        cell_ll[F.dfs_rank[c]] = cl;
        cell_nan[F.dfs_rank[c]] = nan_row;
    }
}

// every batch point starts from the handle's carried state: dst[pt] = src, for pt < n_pts
__global__ __launch_bounds__(256) void k_replicate(const double *__restrict__ src, int64_t n,
                                                   double *__restrict__ dst, int64_t n_pts)
{
    const int64_t total = n * n_pts;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i % n];
}

// ------------------------------------------------------------------------------------------
// GROUP schedule: G lanes per cell, 64/G cells per single-wave workgroup.  The Kalman update
// and the scalar bookkeeping run redundantly in the G lanes of a cell; the propagation's
// 54 computed exponentials (then the 22 products) + 14 Dawson values + 3 powers and then its
// 45 integrals are spread over the G lanes through LDS (ggp_prop.h tasks), cutting the per-step latency that bounds
// small forests.  Bitwise identical to the lane schedule.
// ------------------------------------------------------------------------------------------
// Optional launch timeline (tools/timeline.hip builds this file with GGP_TIMELINE; the shipped
// library never does): lane 0 of each path block writes the constant 100 MHz clock at the
// phases of its launch, g_tl[block][phase], so the fixed cost of a launch can be attributed.
#ifdef GGP_TIMELINE
__device__ unsigned long long g_tl[8192 * 8];
#define GGP_TL(k)                                                                              \
    do {                                                                                       \
        __builtin_amdgcn_s_waitcnt(0);                                                         \
        if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 8192)                          \
            g_tl[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                     \
    } while (0)
// per-launch event counts (g_cnt): steady steps, steps whose stage B took a rare branch (some
// lane), dt-cache refreshes, row-chunk loads
__device__ unsigned long long g_cnt[4];
#define GGP_TL_CNT_DECL unsigned tl_cnt[4] = {0, 0, 0, 0}
#define GGP_TL_CNT(k, cond) tl_cnt[k] += (cond) ? 1u : 0u
#define GGP_TL_CNT_FLUSH()                                                                     \
    do {                                                                                       \
        if (threadIdx.x == 0)                                                                  \
            for (int k_ = 0; k_ < 4; ++k_) atomicAdd(&g_cnt[k_], (unsigned long long)tl_cnt[k_]); \
    } while (0)
// where the block runs: HW_ID (wave, SIMD, CU, SH, SE) in the low word, XCC_ID in the high word
#define GGP_TL_HWID()                                                                          \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 8192)                          \
            g_tl[blockIdx.x * 8 + 7] = (unsigned long long)__builtin_amdgcn_s_getreg(63492) |  \
                                       ((unsigned long long)__builtin_amdgcn_s_getreg(63508) << 32); \
    } while (0)
// the hand-off to a second daughter: the parent's publish time by cell (g_tlc), and in the
// daughter's block the time its wait saw the flag and its first step began (g_tlx[block][0..1])
__device__ unsigned long long g_tlc[1 << 16];
__device__ unsigned long long g_tlx[8192 * 2];
#define GGP_TL_PUB(c)                                                                          \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.y == 0 && (c) < (1 << 16))                            \
            __hip_atomic_store(&g_tlc[(c)], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, \
                               __HIP_MEMORY_SCOPE_AGENT);                                      \
    } while (0)
#define GGP_TL_SEEN(k)                                                                         \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 8192)                          \
            g_tlx[blockIdx.x * 2 + (k)] = __builtin_amdgcn_s_memrealtime();                    \
    } while (0)
#else
#define GGP_TL(k)
#define GGP_TL_PUB(c)
#define GGP_TL_SEEN(k)
#define GGP_TL_HWID()
#define GGP_TL_CNT_DECL
#define GGP_TL_CNT(k, cond)
#define GGP_TL_CNT_FLUSH()
#endif
// Optional per-stage cycle stamps (tools/stamp_group.hip builds this file with GGP_STAMPS;
// the shipped library never does).
#ifdef GGP_STAMPS
__device__ unsigned long long g_stamp[64];   // [16 * log2(cells per wave) + stage]
#define GGP_STAMP_DECL unsigned long long st_acc[15] = {0}, st_prev = 0, st_now = 0; int st_steps = 0
#define GGP_STAMP(k)                                                                       \
    do {                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_now)::"memory");   \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        if ((k) > 0) st_acc[(k) - 1] += st_now - st_prev;                                  \
        st_prev = st_now;                                                                  \
    } while (0)
#define GGP_STAMP_STEP() ++st_steps
// restart the interval clock without charging a stage (the cell's first step is not a steady one)
#define GGP_STAMP_RESET() asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory")
// phases of a launch (wave schedule): everything issued so far completes, then the stamp
__device__ unsigned long long g_pstamp[2][9];   // [level > 1024 cells][phase], [.][8] = launches
#define GGP_PSTAMP_DECL unsigned long long pst[8] = {0}
#define GGP_PSTAMP(k) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(pst[k])::"memory")
#define GGP_PSTAMP_FLUSH()                                                                 \
    do {                                                                                   \
        if (threadIdx.x == 0) {                                                            \
            const int s_ = gridDim.x <= 1024 ? 0 : 1;                                      \
            for (int k_ = 1; k_ < 8; ++k_) atomicAdd(&g_pstamp[s_][k_], pst[k_] - pst[k_ - 1]); \
            atomicAdd(&g_pstamp[s_][8], 1ull);                                             \
        }                                                                                  \
    } while (0)
#define GGP_STAMP_FLUSH()                                                                  \
    do {                                                                                   \
        if (threadIdx.x == 0) {                                                            \
            const int o_ = 16 * (CPW == 1 ? 0 : CPW == 2 ? 1 : CPW == 4 ? 2 : 3);          \
            for (int k_ = 0; k_ < 15; ++k_) atomicAdd(&g_stamp[o_ + k_], st_acc[k_]);      \
            atomicAdd(&g_stamp[o_ + 15], (unsigned long long)st_steps);                    \
        }                                                                                  \
    } while (0)
#elif defined(GGP_MARKS)   // assembly comments at the stamp points (tools/isa_segments.py)
#define GGP_STAMP_DECL
#define GGP_STAMP(k) asm volatile(";@mark " #k)
#define GGP_STAMP_STEP()
#define GGP_STAMP_RESET()
#define GGP_STAMP_FLUSH()
#define GGP_PSTAMP_DECL
#define GGP_PSTAMP(k) asm volatile(";@pmark " #k)
#define GGP_PSTAMP_FLUSH()
#else
#define GGP_STAMP_DECL
#define GGP_STAMP(k)
#define GGP_STAMP_STEP()
#define GGP_STAMP_RESET()
#define GGP_STAMP_FLUSH()
#define GGP_PSTAMP_DECL
#define GGP_PSTAMP(k)
#define GGP_PSTAMP_FLUSH()
#endif

constexpr int kSlot = ggp::NXE + ggp::ND + ggp::NPW + ggp::NI + ggp::SB_N;   // doubles of LDS per cell


template <int G>
__global__ __launch_bounds__(64) void k_loglik_group(DevForest F, ggp_params P,
                                                     const int32_t *__restrict__ cells, int n,
                                                     double *__restrict__ state,
                                                     double *__restrict__ cell_ll,
                                                     int32_t *__restrict__ cell_nan)
{
    constexpr int CPW = 64 / G;
    constexpr int NXB = (ggp::NXC + G - 1) / G;   // computed exponentials per lane
    constexpr int NPB = ggp::NXPU ? (ggp::NXPU + G - 1) / G : 1;   // product exponentials per lane
    constexpr int NDB = (ggp::ND + G - 1) / G;    // Dawson slots per lane
    constexpr int NCB = (ggp::NI + G - 1) / G;    // integral slots per lane
    __shared__ double lds[CPW * kSlot];
    __shared__ double s_ou[ggp::OU_N];
    __shared__ double s_tab[kDawsonTab];
    const int lane = threadIdx.x;
    load_dawson_table(s_tab, lane);
    const int slot = lane / G, lg = lane % G;
    const int i = blockIdx.x * CPW + slot;
    const bool valid = i < n;
    double *Xl = lds + slot * kSlot;
    double *Dl = Xl + ggp::NXE;
    double *Pl = Dl + ggp::ND;
    double *Il = Pl + ggp::NPW;
    double *Sb = Il + ggp::NI;        // the step block (ggp_prop.h)
    // this lane's task descriptors never change: keep them in registers (no loads in the step
    // loop).  Slots past the end of a list run task 0 and are not stored, so every slot is
    // computed unconditionally and the compiler can overlap their dependency chains.
    uint32_t xd[NXB], xj[NXB], pd[NPB], dd[NDB];
    ggp::ITask cd[NCB];
#pragma unroll
    for (int q = 0; q < NXB; ++q) {
        const int j = lg + q * G;
        xd[q] = ggp::pack_x(ggp::kXC.T[j < ggp::NXC ? j : 0]);
        xj[q] = ggp::kXC.j[j < ggp::NXC ? j : 0];
    }
#pragma unroll
    for (int q = 0; q < NPB; ++q) {
        const int j = lg + q * G;
        const ggp::XProd d = ggp::kXP[j < ggp::NXPU ? j : 0];
        pd[q] = d.j | d.rep << 8 | (uint32_t)d.fac << 16;
    }
#pragma unroll
    for (int q = 0; q < NDB; ++q) {
        const int j = lg + q * G;
        dd[q] = ggp::pack_d(ggp::kDT[j < ggp::ND ? j : 0]);
    }
#pragma unroll
    for (int q = 0; q < NCB; ++q) {
        const int j = lg + q * G;
        cd[q] = ggp::kIT[j < ggp::NI ? j : 0];
    }
    const double *p = P.p;
    if (lane == 0) ggp::store_ou(ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]), s_ou);
    double m[4] = {0, 0, 0, 0}, C[16] = {0};
    int c = 0;
    int64_t r = 0, r1 = 0, r0 = 0;
    double dt = 0.0, t_cur = 0.0;
    bool pending = false, divide = false;
    if (valid) {
        c = cells[i];
        r0 = F.row_off[c];
        r1 = F.row_off[c + 1];
        r = r0;
        pending = cell_prologue(F, p, state, c, r0, m, C, dt);
        divide = pending;
        t_cur = F.time[r0];
    }
    if (lg == 0) Xl[ggp::X_ONE] = 1.0;
    __syncthreads();   // s_tab, s_ou
    double cl = 0.0;
    int nan_row = kNanNone;
    bool live = valid;
    GGP_STAMP_DECL;
    while (__any(live)) {   // wave-uniform loop over steps
        GGP_STAMP(0);
        GGP_STAMP_STEP();
        // row data of this step, loaded now and consumed after the propagation (~10k cycles)
        double y_l = 0.0, y_f = 0.0, t_next = 0.0;
        if (live) {
            y_l = F.logl[r];
            y_f = F.fp[r];
            if (r + 1 < r1) t_next = F.time[r + 1];
        }
        const bool prop = live && pending;
        if (prop && lg == 0) {
            ggp::Step S;
            ggp::step_init(S, m, C, dt, ggp::load_ou(s_ou));
            ggp::store_step(S, Sb);
        }
        __syncthreads();
        GGP_STAMP(1);
        const ggp::StepL S(Sb);
        if (prop) {
            double ev[NXB], dv[NDB];
#pragma unroll
            for (int q = 0; q < NXB; ++q) ev[q] = ggp::exp_body(S, ggp::unpack_x(xd[q]), s_tab);
#pragma unroll
            for (int q = 0; q < NDB; ++q) dv[q] = ggp::dawson_body(S, ggp::unpack_d(dd[q]), s_tab);
            const double pw = ggp::pow_task(S, lg < 3 ? lg : 0);
#pragma unroll
            for (int q = 0; q < NXB; ++q)
                if (lg + q * G < ggp::NXC) Xl[xj[q]] = ev[q];
#pragma unroll
            for (int q = 0; q < NDB; ++q)
                if (lg + q * G < ggp::ND) Dl[lg + q * G] = dv[q];
            if (lg < 3) {
                Pl[lg] = pw;
                Pl[3 + lg] = 1.0 / pw;
            }
        }
        GGP_STAMP(2);
        __syncthreads();
        if (prop) {   // the product exponentials (ggp_prop.h kXP), from the computed ones
#pragma unroll
            for (int q = 0; q < NPB; ++q)
                if (lg + q * G < ggp::NXPU) Xl[pd[q] & 0xff] = Xl[pd[q] >> 8 & 0xff] * Xl[pd[q] >> 16];
        }
        __syncthreads();
        GGP_STAMP(3);
        if (prop) {
            double iv[NCB];
#pragma unroll
            for (int q = 0; q < NCB; ++q) iv[q] = ggp::tau_body(S, cd[q], Xl, Dl, Pl);
#pragma unroll
            for (int q = 0; q < NCB; ++q)
                if (lg + q * G < ggp::NI) Il[lg + q * G] = iv[q];
        }
        GGP_STAMP(4);
        __syncthreads();
        GGP_STAMP(5);
        if (prop) {
            ggp::Step SR;
            ggp::load_step(SR, Sb, s_ou);
            ggp::outputs(SR, Il, Xl, m, C);
            if (divide) {
                ggp::division_map(m, C, p[9], p[10], F.binomial, F.log2);
                divide = false;
            }
        }
        GGP_STAMP(6);
        if (live) {
            const double x0 = y_l - m[0];
            const double x1 = y_f - m[1];
            ggp_innov v;
            ggp_innovation(m, C, p[7], p[8], F.scaled, F.fp_auto, v);
            cl += ggp_ll_term(x0, x1, v, F.two_log_2pi);
            if (cl != cl) {
                nan_row = (int)(r - r0);
                live = false;
            } else {
                ggp_posterior(m, C, x0, x1, v);
                pending = r + 1 < r1;
                if (pending) dt = t_next - t_cur;
                t_cur = t_next;
                ++r;
                live = r < r1;
            }
        }
        GGP_STAMP(7);
        __syncthreads();   // LDS slots are rewritten by the next step
        GGP_STAMP(8);
    }
    GGP_STAMP_FLUSH();
    if (valid && lg == 0) {
        double *st = state + (size_t)20 * c;
#pragma unroll
        for (int k = 0; k < 4; ++k) st[k] = m[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) st[4 + k] = C[k];
        cell_ll[F.dfs_rank[c]] = cl;
        cell_nan[F.dfs_rank[c]] = nan_row;
    }
}


// ------------------------------------------------------------------------------------------
// WAVE schedule: one 64-lane wave per cell (ggp_wave.h).  Every stage of a step is one task per
// lane -- the 46 state-dependent exponentials and 14 Dawson values in one Horner stream, the 45
// integrals, the outputs' trilinear form over 60 state monomials (a DPP butterfly per output
// block) -- and the 20-double state is distributed over lanes 0-19 (lane e owns entry e: the
// innovation runs in every lane, the posterior one entry per lane).  What depends on the
// parameters and dt only (exp(s t), the 18 exp-derived basis values) is formed when dt changes
// and kept in LDS.  The determinant and log of the ll term are off the critical path: x and S go
// to an LDS ring, and every 64 rows (or at the cell's end) 64 lanes take the quadratic forms,
// determinants and logs at once and one lane adds the terms in row order (the reference's
// summation order; the first NaN row is found there).  The outputs are the same polynomial as
// ggp::outputs summed in another order, 22 exponentials are products exp(c + ...) exp(k t), and
// the update uses fused multiply-adds, so results agree with the lane/group schedules to ~1e-10
// relative on the total, not bitwise (DESIGN.md "Parity").
// ------------------------------------------------------------------------------------------
template <int CTRL>
GGP_DEV double dpp_f64(const double v)
{
    const long long b = __double_as_longlong(v);
    // every lane is written (full row/bank masks, in-row patterns): no old value to initialise
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Level launches: block b runs cell cells[b].  Path launches (one launch for a whole forest
// whose levels all take the wave schedule): block b runs the path cells[seq[b] .. seq[b+1]),
// a root or second daughter followed by first daughters down to a leaf; each cell after the
// first inherits its parent's posterior in LDS.  The tables and the lane constants are set up
// once per block.  A path's first cell, if a second daughter, waits for its parent's done flag
// (this evaluation's epoch: relaxed agent-scope polls); a cell with a second daughter publishes
// its state (lanes 0-19, agent-scope stores), waits for the stores (s_waitcnt vmcnt(0)), then
// its flag.  Paths are ordered by the depth of their first cell, so a waiting block's parent
// has a lower block index.  What progress relies on:
//   - the single-call path launch (grid = n_paths <= the blocks the device holds resident, from
//     the occupancy query at creation): every block is resident at once, so every wait ends;
//   - chained and tree launches (k_loglik_wave<true>, grid n_paths x points, blockIdx.y = point,
//     a point's roots waiting for its predecessor point's roots): the grid may exceed residency,
//     and then progress relies on the dispatcher starting a lower linear block index no later
//     than a higher one (a waiting block only ever waits on a lower index), which the hardware
//     does but the programming guide does not promise.  Each chained launch is capped so its
//     chain of roots stays within kChainRowsPerLaunch rows (ggp_total_loglik_chain), well inside
//     one wait's budget.
// A wait that exceeds spin_max polls ends as a stall (GGP_ETIMEOUT), never as a hang or a model
// NaN; ggp_total_loglik_chain then finishes the remaining points call by call from the last
// completed point's state, and the -m lookahead evaluates a stalled node's call normally.
// chain[c] = {parent to wait for or -1, 1 if a second daughter waits for c, the division's dt}.
struct CellLink {
    int32_t x, y;   // a second daughter's parent to wait for (or -1); 1: a second daughter waits for c
    double dt;      // a daughter's division dt, time[its first row] - time[the parent's last row]
                    // (the same subtraction the step would make: bitwise), 0 for a root
};
constexpr unsigned kChainSpinMax = 1u << 24;   // ~20 s of polling (GGP_CHAIN_SPIN_MAX)
// rows of chained roots one chained launch may hold (~1 us per row: a few seconds, against the
// ~20 s a wait may take before it counts as a stall)
constexpr int64_t kChainRowsPerLaunch = int64_t(1) << 22;
constexpr unsigned kChainQuietPerRow = 1100;    // s_memtime units (~0.5 us) of unpolled sleep per parent row

// In-launch reduction of a path launch (replaces k_reduce_blocks there, with the same sums):
// the last path of a reduction block to finish forms the block's tree sums (each in DFS order)
// and its block sum (k_reduce_blocks' 64-wide LDS tree, emulated on the block's <= 8 trees: a
// path launch has at most as many leaves as the device holds wave blocks, so B <= 8), writes
// the block result straight to its mapped host slots and counts the block; the last block
// publishes the call's sequence number.  Counters are agent-scope atomics with few arrivals
// (a block: its paths; done: the blocks); the last arrival resets its counter for the next call.
// The ChainRed travels as a kernel argument (no pointer to chase at the end of the launch), and
// each path's block, its path count and tree bounds are loaded at the launch's start
// (RedPre): the reduction's only round trips are the block count, the cells' results (all
// lanes at once), the host slots and the done count.
// A path launch's block b: what its setup reads before its first row loads, in one place (one
// scalar load) instead of a chain of four dependent loads (path_seq -> path_cells -> row_off ->
// rows; path_blk -> block tables -> tree_dfs)
struct PathDesc {
    int32_t i_lo, i_hi, c0, j;    // the path's cells [i_lo, i_hi) of path_cells, its first cell, its block
    int32_t npaths, nb, t0, pad;  // the block's path count, tree count and first tree
    int64_t r0, r1;               // the first cell's rows
    CellLink l0;                  // the first cell's chain entry
};

struct ChainRed {
    const PathDesc *pdesc;        // per path (nullptr: the tables below / the level launch's cells)
    const int32_t *path_blk;      // local block of each path
    const int32_t *blk_npaths;    // paths per local block
    const int64_t *tree_dfs;      // DFS start of each local tree, then the end
    const int32_t *blk_t0, *blk_nt, *gdfs;
    unsigned *cnt_blk, *done;
    int64_t *out_seq;
    double *host_sum;
    long long *host_nan;
    int n_lblocks;                // 0: no in-launch reduction
    unsigned long long *clk;      // mapped: block 0's shader-clock and 100 MHz ticks over its path, its
                                  // start (100 MHz counter), the publishing block's end (ggp_call_trace)
};
constexpr long long kChainNoNan = 0x7fffffffffffffffLL;


// what the reduction of path b needs, loaded at the launch's start and parked in LDS (red[0..63]:
// lane k <= nb the DFS start of the block's tree k, k = nb its end; red[64..66]: the block j, its
// path count, nb), so no register holds it through the steps
struct RedPre {
    int j, npaths, nb;
    int64_t tb;
};
GGP_DEV RedPre red_load(const ChainRed &R, const int b, const int lane)
{
    RedPre q{0, 0, 0, 0};
    if (R.n_lblocks <= 0) return q;
    int t0;
    if (R.pdesc) {
        const PathDesc &pd = R.pdesc[b];
        q.j = pd.j;
        q.npaths = pd.npaths;
        q.nb = pd.nb;
        t0 = pd.t0;
    } else {
        q.j = R.path_blk[b];
        q.npaths = R.blk_npaths[q.j];
        q.nb = R.blk_nt[q.j];
        t0 = R.blk_t0[q.j];
    }
    q.tb = lane <= q.nb ? R.tree_dfs[t0 + lane] : 0;
    return q;
}
GGP_DEV void red_park(const RedPre &q, double *red, const int lane)
{
    red[lane] = __longlong_as_double((long long)q.tb);
    if (lane == 0) {
        red[64] = (double)q.j;
        red[65] = (double)q.npaths;
        red[66] = (double)q.nb;
    }
}
GGP_DEV RedPre red_unpark(const double *red, const int lane)
{
    RedPre q;
    q.tb = (int64_t)__double_as_longlong(red[lane]);
    q.j = __builtin_amdgcn_readfirstlane((int)red[64]);
    q.npaths = __builtin_amdgcn_readfirstlane((int)red[65]);
    q.nb = __builtin_amdgcn_readfirstlane((int)red[66]);
    return q;
}

// every lane of the path's wave calls it after the path's last cell results are stored; scr:
// 192 doubles of the wave's LDS that nothing reads any more
GGP_DEV void chain_reduce(const ChainRed &R, const RedPre &q, const int64_t seq, const int lane, const double *cell_ll,
                          const int32_t *cell_nan, double *scr)
{
    __builtin_amdgcn_s_waitcnt(0);   // this path's cell results are at the coherence point
    int last = 0;
    if (lane == 0) last = add_agent(R.cnt_blk + q.j) + 1 == (unsigned)q.npaths;
    if (__builtin_amdgcn_readfirstlane(last) == 0) return;
    if (lane == 0) zero_agent(R.cnt_blk + q.j);
    // the block's cells [c_lo, c_hi) in DFS order, 64 at a time: every lane loads one cell's
    // result, lane 0 adds them tree by tree in DFS order (k_reduce_blocks' per-thread loop)
    const int nb = q.nb;
    double *s_ll = scr, *s_end = scr + 128;
    int32_t *s_nan = reinterpret_cast<int32_t *>(scr + 64);
    s_end[lane] = __longlong_as_double((long long)q.tb);
    const int64_t c_lo = (int64_t)__shfl((long long)q.tb, 0, 64);
    const int64_t c_hi = (int64_t)__shfl((long long)q.tb, nb, 64);
    double sv[8];
    long long sn[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sv[k] = 0.0;
        sn[k] = kChainNoNan;
    }
    int k = 0;
    int64_t k_end = 0;
    for (int64_t base = c_lo; base < c_hi; base += 64) {
        const int64_t i = base + lane;
        double x = 0.0;
        int nr = kNanNone;
        if (i < c_hi) {
            x = ld_agent(cell_ll + i);
            nr = ld_agent_i(cell_nan + i);
        }
        s_ll[lane] = x;
        s_nan[lane] = nr;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            const int64_t top = base + 64 < c_hi ? base + 64 : c_hi;
            if (base == c_lo) k_end = (int64_t)__double_as_longlong(s_end[1]);
            for (int64_t c = base; c < top; ++c) {
                while (c >= k_end && k + 1 < nb) {
                    ++k;
                    k_end = (int64_t)__double_as_longlong(s_end[k + 1]);
                }
                const double v = s_ll[c - base];
                const int r = s_nan[c - base];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (u == k) {
                        sv[u] += v;
                        if (r != kNanNone && sn[u] == kChainNoNan) sn[u] = ((long long)R.gdfs[c] << 24) | (long long)r;
                    }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (lane != 0) return;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1)   // k_reduce_blocks' tree over 64 slots; slots >= 8 hold 0
#pragma unroll
        for (int u = 0; u < 8 && u < w; ++u) {
            sv[u] = sv[u] + (u + w < 8 ? sv[(u + w) & 7] : 0.0);
            sn[u] = min(sn[u], u + w < 8 ? sn[(u + w) & 7] : kChainNoNan);
        }
    // the block result to its mapped host slots (system-coherent stores), complete before the count
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(R.host_sum + q.j), (unsigned long long)__double_as_longlong(sv[0]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(R.host_nan + q.j, sn[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_waitcnt(0);
    if (add_agent(R.done) + 1 != (unsigned)R.n_lblocks) return;
    zero_agent(R.done);
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    // every block's slots reached host memory before its count: each block's system-scope stores to
    // the fine-grained (uncached) host slots are acknowledged by the fabric before its s_waitcnt(0)
    // lets the count go out, so they are host-visible when the last block sees the full count.
    // The sequence number goes last with a system-scope release (the memory model's
    // ordering, not only the hardware's; one per launch -- A/B in DESIGN.md §6)
#ifdef GGP_SEQ_RELAXED
    __hip_atomic_store(R.out_seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
    __hip_atomic_store(R.out_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    // the launch's end on the 100 MHz counter (ggp_call_trace), AFTER the sequence number: nothing
    // waits for it (the host reads it when it next enters the handle, long after it landed)
    if (R.clk) __hip_atomic_store(R.clk + 3, t_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------------------------------
// k_loglik_wave: the wave schedule.  Path launch: seq != nullptr, block b runs the path
// cells[seq[b] .. seq[b+1]) and the sum is formed in-launch (red); level launch: one cell per
// block.  A second daughter whose parent does not finish within spin_max polls ends as a stall
// (NaN total, row kRowStall: GGP_ETIMEOUT on the host).
// ------------------------------------------------------------------------------------------

// k_loglik_wave's workgroups are one wave: the LDS executes a wave's DS instructions in issue
// order, so a write is seen by every later read of the same wave without waiting for it (no
// lgkmcnt(0) drain, which __syncthreads' workgroup fence would emit); this keeps the compiler from
// moving LDS accesses across the point and costs no instruction.
GGP_DEV void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <bool CHAIN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_loglik_wave(
    DevForest F, ggp_params P, const int32_t *__restrict__ cells, int n, double *__restrict__ state,
    double *__restrict__ cell_ll, int32_t *__restrict__ cell_nan, const CellLink *__restrict__ chain, unsigned *cell_done,
    const unsigned epoch, const int32_t *__restrict__ seq, const ChainRed red, const int64_t call_seq,
    const unsigned spin_max, const double *__restrict__ ptab, const double *__restrict__ carry,
    const int32_t *__restrict__ pt_pred)
{
    namespace W = ggp::wave;
    [[maybe_unused]] const int CPW = gridDim.x <= 1024 ? 8 : 4;   // GGP_STAMPS builds only
    __shared__ __attribute__((aligned(16))) double lds[W::kLds];
    const int lane = threadIdx.x;
    // the launch's shader clock (ggp_launch_clock): block 0 reads the shader-clock counter and the
    // constant 100 MHz counter at its start and after its path (two scalar reads each)
    const unsigned long long clk_c0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
    GGP_PSTAMP_DECL;
    GGP_PSTAMP(0);
    GGP_TL(0);
    GGP_TL_HWID();
    GGP_TL_CNT_DECL;
    // every global load of the launch's setup is issued before the first wait: the reduction's
    // block tables, the Dawson/exp table, this lane's row of the lane constants and the first
    // cell's first 64 rows; make_ou runs while they are in flight
    const RedPre rq0 = red_load(red, blockIdx.x, lane);
    constexpr int kTabN2 = W::kTabRows * W::kTabRow / 2, kTabR = (kTabN2 + 63) / 64;   // 16-byte pieces
    double2 tab_v[kTabR];
    const double2 *tab_img = reinterpret_cast<const double2 *>(W::kTabImg.v);
#pragma unroll
    for (int j = 0; j < kTabR; ++j) tab_v[j] = tab_img[min(lane + 64 * j, kTabN2 - 1)];
    const PathDesc *pd = red.pdesc ? red.pdesc + blockIdx.x : nullptr;
    const int i_lo = pd ? pd->i_lo : seq ? seq[blockIdx.x] : (int)blockIdx.x;
    const int i_hi = pd ? pd->i_hi : seq ? seq[blockIdx.x + 1] : i_lo + 1;
    double pre_l = 0.0, pre_f = 0.0, pre_t = 0.0, pre_t64 = 0.0;   // the first cell's chunk [r0, r0 + 64)
    {
        const int c = pd ? pd->c0 : cells[i_lo];
        const int64_t r0 = pd ? pd->r0 : F.row_off[c], r1 = pd ? pd->r1 : F.row_off[c + 1], rr = r0 + lane;
        if (rr < r1) {
            pre_l = F.logl[rr];
            pre_f = F.fp[rr];
            pre_t = F.time[rr];
        }
        if (lane == 0 && r0 + 64 < r1) pre_t64 = F.time[r0 + 64];
    }
    const double *p = P.p;
    // chained evaluations (ggp_total_loglik_chain / _tree): blockIdx.y = point; the point's
    // parameter row and its state / ll / NaN / done slices of n cells each.  A point's roots start
    // from the state point pred left (pt_pred[pt], or pt - 1; -1: the handle's carried state)
    const int pt = CHAIN ? (int)blockIdx.y : 0;
    const int pred = CHAIN ? (pt_pred ? pt_pred[pt] : pt - 1) : -1;
    if constexpr (CHAIN) {
        p = ptab + 11 * pt;
        state += (size_t)20 * n * pt;
        cell_ll += (size_t)n * pt;
        cell_nan += (size_t)n * pt;
        cell_done += (size_t)n * pt;
    }
    const W::LaneC LC = W::unpack_lane(W::kLanePTab.l[lane]);   // this lane's row of the compile-time table (packed)
    W::Lane L;
    {
        const ggp::OU ou = ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
        const double kap = W::lane_kappa(lane, ou);
#pragma unroll
        for (int j = 0; j < kTabR; ++j)
            if (lane + 64 * j < kTabN2) reinterpret_cast<double2 *>(lds + W::L_TAB)[lane + 64 * j] = tab_v[j];
        if (red.n_lblocks > 0) red_park(rq0, lds + W::L_RED, lane);
        lds[W::L_ROWL + lane] = pre_l;   // the first cell's chunk (its loop iteration loads no rows)
        lds[W::L_ROWF + lane] = pre_f;
        lds[W::L_ROWT + lane] = pre_t;
        if (lane == 0) lds[W::L_ROWT + 64] = pre_t64;
        GGP_PSTAMP(1);
        GGP_TL(1);
        lds[W::L_MONO + lane] = kap;   // the 33 kappas, one per lane (MONO is free here)
        wave_sync();
        L = W::lane_from(lane, LC, ou, lds + W::L_MONO);
        wave_sync();
    }
    const double var_x = p[7], var_g = p[8], var_dx = p[9], var_dg = p[10], b = p[6];
    const double g_sc = F.scaled ? var_g : 0.0, g_0 = F.scaled ? 0.0 : var_g;   // W::uinnov's D11
    if (lane == 0) {
        lds[W::L_X + ggp::X_ONE] = 1.0;
        lds[W::L_BV + ggp::BV_ONE] = 1.0;
        lds[W::L_V + ggp::V_ONE] = 1.0;
        lds[W::L_ONE1] = 1.0;
        lds[W::L_ZERO] = 0.0;
    }
    GGP_PSTAMP(2);
    GGP_TL(2);
    // exp(s t) and the exp-derived basis depend on the parameters and dt only; dt compared by its
    // bits (a NaN pattern no time difference produces: nothing cached yet)
    unsigned long long dt_cached = 0x7ff4dead0000beefULL;
    // the dt cache's keys start as that pattern too; way dt_victim is replaced next
    if (lane < W::kDtWays) lds[W::L_DTK + lane] = __longlong_as_double((long long)dt_cached);
    int dt_victim = 0;
    const int dt_my_slot = W::dt_slot(lane < W::kDtVals ? lane : 0);
    GGP_STAMP_DECL;
    // the cell's first state into POST (lanes' entries) and V (stage D's variables), from registers
    // holding the same values in every lane (once per cell)
    auto scatter = [&](const double *m, const double *C) {
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v = lane == k ? m[k] : v;
#pragma unroll
        for (int k = 0; k < 16; ++k) v = lane == 4 + k ? C[k] : v;
        lds[L.u_post] = v;
        lds[L.u_v] = v - L.u_vshift;
    };
    // one propagation of the state in POST / V over dt: the raw outputs in OUT (after a barrier)
    auto propagate = [&](const double dt) {
        GGP_STAMP(0);
        const long long db = __double_as_longlong(dt);
        const unsigned long long dbits = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(db >> 32)) << 32) |
                                         (unsigned)__builtin_amdgcn_readfirstlane((int)(db & 0xffffffff));
        GGP_TL_CNT(2, dbits != dt_cached);
        if (dbits != dt_cached) {   // lane constants and kernel arguments only: no OU values live in the loop
            // a cached way of this dt (lane w compares key w): its values to the working slots;
            // else computed, then saved into way dt_victim (bitwise the same values either way)
            const unsigned long long key = (unsigned long long)__double_as_longlong(lds[W::L_DTK + (lane & (W::kDtWays - 1))]);
            const unsigned long long hit = __ballot(lane < W::kDtWays && key == dbits);
            if (hit != 0ull) {
                const int way = __builtin_ctzll(hit);
                if (lane < W::kDtVals) lds[dt_my_slot] = lds[W::L_DTC + W::kDtVals * way + lane];
                if (lane == 0) lds[W::L_V + ggp::V_T] = dt;
                wave_sync();
            } else {
                if (lane < 7) lds[lane < 6 ? W::L_X + ggp::XS_bt + lane : W::L_XPGQ] = exp(L.c_sv * dt);
                wave_sync();
                if (lane < ggp::kNDerived)
                    lds[W::L_BV + ggp::BV_R_EBT + lane] = ggp::derived_generic(ggp::kDerived[lane], lds + W::L_X, p[1], dt);
                if (lane == 0) lds[W::L_V + ggp::V_T] = dt;
                wave_sync();
                if (lane < W::kDtVals) lds[W::L_DTC + W::kDtVals * dt_victim + lane] = lds[dt_my_slot];
                if (lane == 0) lds[W::L_DTK + dt_victim] = __longlong_as_double((long long)dbits);
                dt_victim = (dt_victim + 1) & (W::kDtWays - 1);
                __builtin_amdgcn_s_waitcnt(0x0F70);   // (the derived values' table loads: none outlives the miss)
            }
            dt_cached = dbits;
        }
        const double *po = lds + W::L_POST;
        const W::WStep S = W::wstep2(po[0], po[2], po[4], po[6], po[14], dt, b);
        lds[L.mo_dst] = W::mono(L, lds);   // stage D's monomials of this state
        GGP_STAMP(1);
        {   // stage B: one exponential or Dawson value per lane
            const W::BOut o = W::stageB(S, L, lds);
            double v = o.v;
            GGP_TL_CNT(1, __builtin_amdgcn_readfirstlane(__ballot(o.rare) != 0 ? 1 : 0));
            if (o.rare) v = W::stageB_rare(L.b_isD, o.arg, o.z, o.v);   // skipped (execz) when no lane needs it
            lds[L.b_dst] = v;
        }
        GGP_STAMP(2);
        wave_sync();
        GGP_STAMP(3);
        lds[L.i_dst] = W::stageC(S, L, lds);   // stage C: one integral per lane
        GGP_STAMP(4);
        wave_sync();
        GGP_STAMP(5);
        double acc = W::stageD(L, lds);   // stage D: the lane's output terms
        GGP_STAMP(6);
        {   // block sums: DPP butterfly (ggp::out_partner)
            const int bs = L.d_bs;
            double w;
            w = dpp_f64<0xB1>(acc);  acc = bs > 1 ? acc + w : acc;
            w = dpp_f64<0x4E>(acc);  acc = bs > 2 ? acc + w : acc;
            w = dpp_f64<0x141>(acc); acc = bs > 4 ? acc + w : acc;
            w = dpp_f64<0x140>(acc); acc = bs > 8 ? acc + w : acc;
        }
        lds[L.d_out] = acc;
        GGP_STAMP(7);
        wave_sync();
    };
    bool next_pre = false;   // the previous cell's last flush loaded this cell's first chunk
    // the cell, its chain entry and rows, loaded while the previous cell ran (the path's first
    // cell: from its descriptor), so a cell starts without a chain of dependent loads
    int c_cur = pd ? pd->c0 : cells[i_lo];
    CellLink ch_cur = pd ? pd->l0 : chain[c_cur];
    int64_t r0_cur = pd ? pd->r0 : F.row_off[c_cur], r1_cur = pd ? pd->r1 : F.row_off[c_cur + 1];
    for (int i = i_lo; i < i_hi; ++i) {
        const int c = c_cur;
        const CellLink ch = ch_cur;
        bool chain_broken = false;
        // the path's next cell: its first chunk is loaded during this cell's last flush
        const int c_nx = i + 1 < i_hi ? cells[i + 1] : -1;
        const int64_t r0n = c_nx >= 0 ? F.row_off[c_nx] : 0, r1n = c_nx >= 0 ? F.row_off[c_nx + 1] : 0;
        const CellLink ch_nx = c_nx >= 0 ? chain[c_nx] : CellLink{-1, 0, 0.0};
        // the cell to wait for: a second daughter's parent; in a chain also a root's own state at
        // the end of the previous point (its carried state)
        int wc = ch.x;
        const unsigned *wdone = cell_done;
        bool carried_prev = false, publish = ch.y != 0;
        if constexpr (CHAIN) {
            const bool root = F.parent[c] < 0;
            carried_prev = root && pred >= 0;
            publish = publish || (root && (pt_pred != nullptr || pt + 1 < (int)gridDim.y));
            if (carried_prev) {
                wc = c;
                wdone = cell_done + (ptrdiff_t)n * (pred - pt);
            }
        }
        if (wc >= 0 && __hip_atomic_load(wdone + wc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
            // the cell runs in this launch and is not done: sleep through ~0.5 us per row of it
            // without polling, then poll (relaxed agent-scope loads); spin_max polls at most
            if (spin_max > 0) {
                const unsigned long long t_start = __builtin_amdgcn_s_memtime();
                const unsigned long long quiet = (unsigned long long)(F.row_off[wc + 1] - F.row_off[wc]) * kChainQuietPerRow;
                while (__builtin_amdgcn_s_memtime() - t_start < quiet) __builtin_amdgcn_s_sleep(127);
            }
            unsigned spins = 0;
            while (__hip_atomic_load(wdone + wc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
                if (++spins > spin_max) {
                    chain_broken = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2)   /* short: the poll's own load is most of an iteration */;
            }
        }
        // a root whose predecessor point's root stalled stalls too (its state would be that
        // root's unfinished one): the tree's dependent points report GGP_ETIMEOUT, not a value
        if (CHAIN && carried_prev && !chain_broken &&
            ld_agent_i(cell_nan + (wdone - cell_done) + F.dfs_rank[c]) == kRowStall)
            chain_broken = true;
        if (i == i_lo && wc >= 0) GGP_TL_SEEN(0);
        const int64_t r0 = r0_cur, r1 = r1_cur;
        c_cur = c_nx;   // the next iteration's cell
        ch_cur = ch_nx;
        r0_cur = r0n;
        r1_cur = r1n;
        double dt = 0.0;
        bool pending;
        if (i > i_lo) {   // the first daughter of the previous cell: its posterior is in POST / V
            pending = true;
            dt = ch.dt;
        } else if (ch.x >= 0) {   // a second daughter of a cell in another path: lane e takes entry e
            if (lane < 20) {
                const double v = ld_agent(state + (size_t)20 * ch.x + lane);
                lds[L.u_post] = v;
                lds[L.u_v] = v - L.u_vshift;
            }
            pending = true;
            dt = ch.dt;
        } else {
            double m[4], C[16];
            if (CHAIN && carried_prev) {   // a root: the previous point's final state of it (coherent loads)
                const double *st = state + (ptrdiff_t)20 * n * (pred - pt) + (size_t)20 * c;
#pragma unroll
                for (int k = 0; k < 16; ++k) C[k] = ld_agent(st + 4 + k);
                root_init(F, p, m, C);
                pending = false;
            } else {
                pending = cell_prologue(F, p, CHAIN && F.parent[c] < 0 ? carry : state, c, r0, m, C, dt);
            }
            scatter(m, C);
        }
        const bool divide = pending;
        GGP_PSTAMP(3);
        if (i == i_lo) GGP_TL(3);
        if (i == i_lo && ch.x >= 0) GGP_TL_SEEN(1);
        // the rows of the chunk [base, base + 64) go to LDS once (one coalesced load per lane)
        auto load_chunk = [&](const int64_t base) {
            const int64_t rr = base + lane;
            double a = 0.0, bb = 0.0, t = 0.0;
            if (rr < r1) {
                a = F.logl[rr];
                bb = F.fp[rr];
                t = F.time[rr];
            }
            lds[W::L_ROWL + lane] = a;
            lds[W::L_ROWF + lane] = bb;
            lds[W::L_ROWT + lane] = t;
            if (lane == 0) lds[W::L_ROWT + 64] = base + 64 < r1 ? F.time[base + 64] : 0.0;
        };
        // the first cell's chunk is in LDS since the launch's start, a later one's since its
        // predecessor's last flush (unless that stopped at a NaN)
        if (i != i_lo && !next_pre) load_chunk(r0);
        next_pre = false;
        wave_sync();
        // the row time from LDS (no global load the step loop's waits would have to cover)
        double t_cur = lds[W::L_ROWT];
        double cl = 0.0;
        int nan_row = kNanNone;
        int slot = 0;                    // row - chunk base
        const int nrows = (int)(r1 - r0);
        int left = nrows;                // rows from the chunk's first on (updated at each flush)
        int slot_end = min(64, nrows);   // the chunk's rows: the step that fills them flushes
        bool live = !chain_broken;
        if (chain_broken) {
            cl = __longlong_as_double(0x7ff8000000000000LL);
            nan_row = kRowStall;
        }
        // after the step whose row ends a chunk (slot == slot_end: 64 rows, or the cell's last): the
        // ll ring is flushed, then the next chunk loaded (left, live: after this chunk).  false =
        // stop (a NaN term; nan_row set)
        auto flush = [&]() -> bool {
            left -= slot;
            live = left > 0;
            {
                const int done = nrows - left;
                const int64_t base = done - slot;
                // the next chunk (this cell's, or the path's next cell's first) is loaded while the
                // flush runs, and goes to LDS after the flush has read this chunk's rows
                const bool nx = live || c_nx >= 0;
                const int64_t nb0 = live ? r0 + done : r0n, ne = live ? r1 : r1n;
                double na = 0.0, nf = 0.0, nt = 0.0, nt64 = 0.0;
                if (nx) {
                    const int64_t rr = nb0 + lane;
                    if (rr < ne) {
                        na = F.logl[rr];
                        nf = F.fp[rr];
                        nt = F.time[rr];
                    }
                    if (lane == 0 && nb0 + 64 < ne) nt64 = F.time[nb0 + 64];
                }
                wave_sync();
                if (lane < slot) {
                    const double s00 = lds[W::L_RS0 + lane], s01 = lds[W::L_RS1 + lane], s11 = lds[W::L_RS2 + lane];
                    // the ring holds the prior means: -x = m - y formed here, 64 rows at once (the
                    // quadratic form is even in x)
                    lds[W::L_RT + lane] = W::ll_quad(lds[W::L_RX0 + lane] - lds[W::L_ROWL + lane],
                                                     lds[W::L_RX1 + lane] - lds[W::L_ROWF + lane], s00, s01, s11) -
                                           0.5 * log(ggp_det_pplu(s00, s01, s01, s11)) - F.two_log_2pi;
                }
                wave_sync();
                bool ok = true;
                if (lane == 0) {
                    // the terms in row order (the reference's running sum), unrolled for a full chunk;
                    // the scan for the first NaN row only when the chunk's sum is NaN
                    double acc = cl;
                    if (slot == 64) {
#pragma unroll
                        for (int k = 0; k < 64; ++k) acc += lds[W::L_RT + k];
                    } else {
                        for (int k = 0; k < slot; ++k) acc += lds[W::L_RT + k];
                    }
                    if (acc != acc) {
                        acc = cl;
                        for (int k = 0; k < slot; ++k) {
                            acc += lds[W::L_RT + k];
                            if (acc != acc) {
                                nan_row = (int)(base + k);
                                ok = false;
                                break;
                            }
                        }
                    }
                    cl = acc;
                }
                // no global load outlives the flush, on either exit (s_waitcnt vmcnt(0)): the step
                // loop then needs no vmcnt waits for the registers its loads wrote
                __builtin_amdgcn_s_waitcnt(0x0F70);
                if (__builtin_amdgcn_readfirstlane(ok ? 1 : 0) == 0) return false;
                slot = 0;
                slot_end = min(64, left);
                if (nx) {
                    wave_sync();   // every lane has read this chunk's rows (lane 0's sum: the ll terms only)
                    lds[W::L_ROWL + lane] = na;
                    lds[W::L_ROWF + lane] = nf;
                    lds[W::L_ROWT + lane] = nt;
                    if (lane == 0) lds[W::L_ROWT + 64] = nt64;
                }
                next_pre = !live && c_nx >= 0;
                GGP_TL_CNT(3, nx);
            }
            return true;
        };
        GGP_PSTAMP(4);
        if (live) {   // the cell's first step: uniform registers (no propagation / division map)
            const double y_l = lds[W::L_ROWL], y_f = lds[W::L_ROWF];
            const double t_next = left > 1 ? lds[W::L_ROWT + 1] : 0.0;
            double m[4], C[16];
            if (pending) {
                propagate(dt);
                double o[ggp::kOutN];
#pragma unroll
                for (int k = 0; k < ggp::kOutN; ++k) o[k] = lds[W::L_OUT + k];
#pragma unroll
                for (int k = 0; k < ggp::kOutN; ++k)   // out_finish: the covariances' sum - nm_i nm_j
                    if (ggp::kOutNm[k][0] >= 0) o[k] = __builtin_fma(-o[ggp::kOutNm[k][0]], o[ggp::kOutNm[k][1]], o[k]);
                ggp::out_store(o, m, C);
                if (divide) ggp::division_map(m, C, var_dx, var_dg, F.binomial, F.log2);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) m[k] = lds[W::L_POST + k];
#pragma unroll
                for (int k = 0; k < 16; ++k) C[k] = lds[W::L_POST + 4 + k];
            }
            const double x0 = y_l - m[0], x1 = y_f - m[1];
            const W::WInnov v = W::innovation(m, C, var_x, var_g, F.scaled, F.fp_auto);
            if (lane == 0) {   // the ll term's inputs: the prior means (the flush forms m - y) and S
                lds[W::L_RX0 + slot] = m[0];
                lds[W::L_RX1 + slot] = m[1];
                lds[W::L_RS0 + slot] = v.S00;
                lds[W::L_RS1 + slot] = v.S01;
                lds[W::L_RS2 + slot] = v.S11;
            }
            W::posterior(m, C, x0, x1, v, true);
            scatter(m, C);
            pending = left > 1;
            if (pending) dt = t_next - t_cur;
            t_cur = t_next;
            GGP_STAMP_RESET();
            ++slot;
            if (slot == slot_end && !flush()) live = false;
            wave_sync();   // the LDS slots are rewritten by the next step
        }
        GGP_PSTAMP(5);
        __builtin_amdgcn_s_waitcnt(0x0F70);   // (vmcnt(0): see the flush)
        // steady steps, the state distributed over lanes 0-19: the chunk's rows [slot, slot_end) in
        // a counted loop (one exit), then the flush; the row times from LDS in one read (ROWT[64]:
        // the next chunk's first time; the next time is unused on the cell's last row)
        // the row's slot as a byte offset in a vector register (sv = 8 slot): the slot-indexed LDS
        // accesses of a step take it as their address, with the region in the offset field
        auto at = [&](const int sv, const int region) -> double & {
            return *reinterpret_cast<double *>(reinterpret_cast<char *>(lds + region) + sv);
        };
        while (live) {
            int sv;
            asm volatile("v_mov_b32 %0, %1" : "=v"(sv) : "s"(slot << 3));
            do {
                wave_sync();   // the previous step's (or the flush's) LDS slots are complete
                GGP_STAMP_STEP();
                GGP_TL_CNT(0, true);
                const double t_now = at(sv, W::L_ROWT), t_next = at(sv + 8, W::L_ROWT);
                propagate(dt);
                {
                    // every lane forms the innovation from the raw outputs (the values lanes 1, 4, 5, 9,
                    // 20, 24 finish: fma(-o0, o1, o5) = C01, fma(-o1, o1, o8) = C11), its loads issued
                    // with the finish's before any store
                    const double *o = lds + W::L_OUT;
                    const double o0 = o[0], o1 = o[1], o4 = o[4], o5 = o[5], o8 = o[8];
                    const double fv = W::finish_sv(L, lds, sv);   // the prior's entries, -x0, -x1
                    lds[L.f_dst] = fv;
                    const W::UInnov v = W::uinnov(o1, o4, __builtin_fma(-o0, o1, o5), __builtin_fma(-o1, o1, o8), var_x,
                                                  g_sc, g_0, F.fp_auto);
                    {   // the ll term's inputs: the prior means (the flush forms m - y) and S, the same
                        // values from every lane to one address (no exec mask around the stores)
                        at(sv, W::L_RX0) = o0;
                        at(sv, W::L_RX1) = o1;
                        at(sv, W::L_RS0) = v.S00;
                        at(sv, W::L_RS1) = v.S01;
                        at(sv, W::L_RS2) = v.S11;
                    }
                    GGP_STAMP(8);
                    wave_sync();
                    const W::UOps q = W::upost_load(L, lds);
                    W::sched_fence();   // the operand reads issued before the update's arithmetic
                    const double up = W::upost(q, fv, v);
                    lds[L.u_post] = up;
                    lds[L.u_v] = up - L.u_vshift;
                }
                GGP_STAMP(9);
                dt = t_next - t_now;
                GGP_STAMP(10);
                sv += 8;
            } while (++slot != slot_end);
            wave_sync();
            const bool stop = !flush() || !live;
            GGP_STAMP(10);
            wave_sync();
            if (stop) break;
        }
        GGP_PSTAMP(6);
        GGP_TL(4);
        wave_sync();
        // the cell's results; its state from lanes 0-19 (one coalesced store), agent-coherent with
        // the flag after it when a second daughter waits for it
        if (lane == 0) {
            st_agent(cell_ll + F.dfs_rank[c], cl);   // coherent: a path launch sums them in-launch
            st_agent_i(cell_nan + F.dfs_rank[c], nan_row);
        }
        if (lane < 20) {
            const double v = lds[W::L_POST + lane];
            if (publish)
                st_agent(state + (size_t)20 * c + lane, v);
            else if (i + 1 != i_hi)   // (the path's last cell: stored after the reduction's count)
                state[(size_t)20 * c + lane] = v;
        }
        if (publish) {
            __builtin_amdgcn_s_waitcnt(0);   // every lane's stores at the coherence point, then the flag
            GGP_TL_PUB(c);
            if (lane == 0) __hip_atomic_store(cell_done + c, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        GGP_PSTAMP(7);
        GGP_TL(5);
        wave_sync();   // the LDS rows and ring are the next cell's
    }
    GGP_STAMP_FLUSH();
    GGP_PSTAMP_FLUSH();
    if (red.clk && blockIdx.x == 0 && blockIdx.y == 0 && lane == 0) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_store(red.clk, c1 - clk_c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(red.clk + 1, r1 - clk_r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(red.clk + 2, clk_r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // the path's last cell's state: nothing in this launch reads it unless it was published above
    // (then this stores the same values again), so its store is issued after the reduction's count
    // and its completion is no part of the wait in front of that count
    const int c_last = cells[i_hi - 1];
    const double v_last = lane < 20 ? lds[W::L_POST + lane] : 0.0;
    if (red.n_lblocks > 0) chain_reduce(red, red_unpark(lds + W::L_RED, lane), call_seq, lane, cell_ll, cell_nan, lds + W::L_RX0);
    if (lane < 20) state[(size_t)20 * c_last + lane] = v_last;
    GGP_TL(6);
    GGP_TL_CNT_FLUSH();
}


// ------------------------------------------------------------------------------------------
// -p smoother kernels (lane schedule).  Parameters per row come from the segment table.
// ------------------------------------------------------------------------------------------
GGP_DEV const double *seg_params(const DevForest &F, const double *ptab, int n_seg, int64_t r)
{
    int s = F.seg ? F.seg[r] : 0;
    if (s < 0 || s >= n_seg) s = 0;
    return ptab + 11 * s;
}

// a row's parameter row from its raw segment index, clamped as seg_params clamps it
GGP_DEV const double *seg_row(const double *ptab, int n_seg, int s)
{
    if (s < 0 || s >= n_seg) s = 0;
    return ptab + 11 * s;
}

GGP_DEV void store20(double *dst, const double *m, const double *C)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = m[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) dst[4 + k] = C[k];
}

// The lane smoother's row loop is pipelined one row ahead: row r - 1's (backward) or r + 1's
// (forward) data, segment, time and forward row are loaded at the end of row r, before row r's
// stores.  vmcnt counts loads and stores in issue order, so a wait for a load issued after a store
// drains the store too: loaded first, the next row's operands are waited for without it, and they
// arrive behind this row's propagation.  SL: the parameter rows staged in LDS (n_seg <= kSegLds:
// the CLI's -b segments), so the per-row parameter reads are LDS reads, outside vmcnt altogether.
constexpr int kSegLds = 32;

template <bool SL>
GGP_DEV const double *stage_params(double *s_par, const double *ptab, const int n_seg, const int lane)
{
    if constexpr (SL) {
        for (int k = lane; k < 11 * n_seg; k += 64) s_par[k] = ptab[k];
        return s_par;
    } else {
        return ptab;
    }
}

// prediction_forward / sc_prediction_forward (predictions.h:93-173)
template <bool SL>
__global__ __launch_bounds__(64) GGP_LANE_ATTR void k_fwd_level(DevForest F, const double *__restrict__ ptab, int n_seg,
                                                  const int32_t *__restrict__ cells, int n, int cpw,
                                                  double *__restrict__ pstate, double *__restrict__ out)
{
    __shared__ double s_tab[kDawsonTab];
    __shared__ double s_par[SL ? 11 * kSegLds : 1];
    const int lane = threadIdx.x;
    load_dawson_table(s_tab, lane);
    const double *PT = stage_params<SL>(s_par, ptab, n_seg, lane);
    __syncthreads();
    if (lane >= cpw) return;
    const int i = blockIdx.x * cpw + lane;
    if (i >= n) return;
    const int c = cells[i];
    const int64_t r0 = F.row_off[c], r1 = F.row_off[c + 1];
    const int par = F.parent[c];
    // root: segment of its first row; daughter: the parent's last segment (:103-108)
    const double *pi = seg_params(F, PT, n_seg, par < 0 ? r0 : F.row_off[par + 1] - 1);
    double m[4], C[16], dt = 0.0;
    bool pending = cell_prologue(F, pi, pstate, c, r0, m, C, dt);
    bool divide = pending;
    const double *pprop = pi;
    // the OU constants (six divisions and a pow) are formed again only when the segment changes
    const double *ou_src = nullptr;
    ggp::OU ou{};
    double t_cur = F.time[r0];
    // row r's operands, loaded during row r - 1 (the look-ahead index is clamped to the cell's last
    // row instead of a branch: the last row's look-ahead reads a valid row and nothing uses it)
    const int64_t r_last = r1 - 1;
    double y_l_n = F.logl[r0], y_f_n = F.fp[r0], t_nx_n = F.time[min(r0 + 1, r_last)];
    int seg_n = F.seg ? F.seg[r0] : 0;
    // the prologue's loads complete here, so the loop's waits are the look-ahead's alone
    __builtin_amdgcn_s_waitcnt(0);
    for (int64_t r = r0; r < r1; ++r) {
        const double y_l = y_l_n, y_f = y_f_n, t_next = t_nx_n;
        const double *p = seg_row(PT, n_seg, seg_n);
        const double var_x = p[7], var_g = p[8];
        if (pending) {
            if (pprop != ou_src) {
                ou = ggp::make_ou(pprop[0], pprop[1], pprop[2], pprop[3], pprop[4], pprop[5], pprop[6]);
                ou_src = pprop;
            }
            ggp::propagate_lane(m, C, dt, ou, s_tab);
            if (divide) {
                ggp::division_map(m, C, pi[9], pi[10], F.binomial, F.log2);
                divide = false;
            }
        }
        const double x0 = y_l - m[0];
        const double x1 = y_f - m[1];
        ggp_innov v;
        ggp_innovation(m, C, var_x, var_g, F.scaled, F.fp_auto, v);
        ggp_posterior(m, C, x0, x1, v);
        {   // row r + 1's operands, ahead of row r's store
            const int64_t rn = min(r + 1, r_last);
            y_l_n = F.logl[rn];
            y_f_n = F.fp[rn];
            t_nx_n = F.time[min(r + 2, r_last)];
            if (F.seg) seg_n = F.seg[rn];
        }
        __builtin_amdgcn_sched_barrier(0);   // the loads above issue before the store below
        store20(out + (size_t)20 * r, m, C);
        pending = r + 1 < r1;
        if (pending) dt = t_next - t_cur;
        t_cur = t_next;
        pprop = p;   // the step t -> t+1 uses row t's parameters (:143-146)
    }
    store20(pstate + (size_t)20 * c, m, C);
}

// prediction_backward / sc_prediction_backward (predictions.h:368-444), levels bottom-up.
// COMB: combine_predictions (predictions.h:466-499, k_combine<true>'s combine_info) fused in: each
// row's backward prior is combined with its forward row as soon as it is formed, into comb; the
// backward rows themselves are stored only when out is given.  The same operations per row as
// k_combine<true>, so the combined rows are bitwise the separate kernel's.
template <bool COMB, bool SL>
__global__ __launch_bounds__(64) GGP_LANE_ATTR void k_bwd_level(DevForest F, const double *__restrict__ ptab, int n_seg,
                                                  const int32_t *__restrict__ cells, int n, int cpw,
                                                  double *__restrict__ pstate, double *__restrict__ out,
                                                  const int32_t *__restrict__ prior_seg,
                                                  const double *__restrict__ fwd, double *__restrict__ comb)
{
    __shared__ double s_tab[kDawsonTab];
    __shared__ double s_par[SL ? 11 * kSegLds : 1];
    const int lane = threadIdx.x;
    load_dawson_table(s_tab, lane);
    const double *PT = stage_params<SL>(s_par, ptab, n_seg, lane);
    __syncthreads();
    if (lane >= cpw) return;
    const int i = blockIdx.x * cpw + lane;
    if (i >= n) return;
    const int c = cells[i];
    const int64_t r0 = F.row_off[c], r1 = F.row_off[c + 1];
    const double *pi = seg_params(F, PT, n_seg, r1 - 1);          // :376-378
    const int d1 = F.d1[c], d2 = F.d2[c];
    double m[4], C[16];
    // the propagation before row r's update (one call site: the division's and the rows' steps)
    bool pend = false;
    double dtp = 0.0;
    const double *pq = pi;   // its parameters (the reversed model)
    if (d1 < 0 && d2 < 0) {
        // init_sc_distribution_r leaf branch (:317-332): on top of the forward final state
        const double *st = pstate + (size_t)20 * c;
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = st[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) C[k] = st[4 + k];
        m[0] = F.leaf_mean0;
        m[1] = F.leaf_mean1;
        C[0] = F.leaf_var0;
        C[5] = F.leaf_var1;
        m[2] = -pi[0];
        m[3] = -pi[3];
        C[10] = pi[2] / (2. * pi[1]);
        C[15] = pi[5] / (2. * pi[4]);
    } else {
        // mean_cov_after_division_r (:201-275); a cell with only daughter2 does not occur
        // (build_cell_genealogy fills daughter1 first)
        const double *s1 = pstate + (size_t)20 * d1;
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = s1[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) C[k] = s1[4 + k];
        ggp::division_map_r(m, C, pi[9], pi[10], F.binomial, F.log2);
        if (d2 >= 0) {
            double m2[4], C2[16];
            const double *s2 = pstate + (size_t)20 * d2;
#pragma unroll
            for (int k = 0; k < 4; ++k) m2[k] = s2[k];
#pragma unroll
            for (int k = 0; k < 16; ++k) C2[k] = s2[4 + k];
            ggp::division_map_r(m2, C2, pi[9], pi[10], F.binomial, F.log2);
            ggp::mult_gauss(m, C, m2, C2);
        }
        dtp = F.time[F.row_off[d1]] - F.time[r1 - 1];
        pend = true;
    }
    const double *ou_src = nullptr;   // as k_fwd_level: the OU constants per segment change only
    ggp::OU ou{};
    // row r's operands, loaded during row r + 1 (k_fwd_level's pipeline, downwards; indices clamped
    // to the cell's first row)
    double y_l_n, y_f_n, t_r_n, t_prev_n, fw_n[20];
    int seg_r_n, seg_p_n, sp_n = 0;
    auto load_row = [&](const int64_t rr) {
        const int64_t rp = max(rr - 1, r0);
        y_l_n = F.logl[rr];
        y_f_n = F.fp[rr];
        t_r_n = F.time[rr];
        t_prev_n = F.time[rp];
        seg_p_n = F.seg ? F.seg[rp] : 0;   // row rr - 1's: the propagation after row rr
        if constexpr (COMB) {
            sp_n = prior_seg[rr];
            const double *fr = fwd + (size_t)20 * rr;
#pragma unroll
            for (int k = 0; k < 20; ++k) fw_n[k] = fr[k];
        }
    };
    seg_r_n = F.seg ? F.seg[r1 - 1] : 0;
    load_row(r1 - 1);
    __builtin_amdgcn_s_waitcnt(0);   // the prologue's loads complete here (k_fwd_level)
    for (int64_t r = r1 - 1; r >= r0; --r) {
        const double y_l = y_l_n, y_f = y_f_n, t_r = t_r_n, t_prev = t_prev_n;
        const int seg_p = seg_p_n;
        const double *p = seg_row(PT, n_seg, seg_r_n);
        const double var_x = p[7], var_g = p[8];
        if (pend) {
            if (pq != ou_src) {
                ou = ggp::make_ou(-pq[0], pq[1], pq[2], -pq[3], pq[4], pq[5], -pq[6]);
                ou_src = pq;
            }
            ggp::propagate_lane(m, C, dtp, ou, s_tab);
        }
        double rm[4], rC[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) rm[k] = m[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) rC[k] = C[k];
        ggp::reverse_state(rm, rC);
        double mf[4], Cf[16];
        int sp = 0;
        if constexpr (COMB) {   // k_combine<true> on this row
#pragma unroll
            for (int k = 0; k < 4; ++k) mf[k] = fw_n[k];
#pragma unroll
            for (int k = 0; k < 16; ++k) Cf[k] = fw_n[4 + k];
            sp = sp_n;
            if (sp < 0 || sp >= n_seg) sp = 0;
            ggp::combine_info(mf, Cf, rm, rC, PT + 11 * sp);
        }
        const double x0 = y_l - m[0];
        const double x1 = y_f - m[1];
        ggp_innov v;
        ggp_innovation(m, C, var_x, var_g, F.scaled, F.fp_auto, v);
        ggp_posterior(m, C, x0, x1, v);
        seg_r_n = seg_p;
        load_row(max(r - 1, r0));   // row r - 1's operands, ahead of row r's stores
        __builtin_amdgcn_sched_barrier(0);
        if (!COMB || out) store20(out + (size_t)20 * r, rm, rC);  // the prior, before the update
        if constexpr (COMB) store20(comb + (size_t)20 * r, mf, Cf);
        pend = r > r0;
        if (pend) {
            pq = seg_row(PT, n_seg, seg_p);   // row r - 1's parameters (seg_params(r - 1))
            dtp = t_r - t_prev;
        }
    }
    store20(pstate + (size_t)20 * c, m, C);
}

// ------------------------------------------------------------------------------------------
// The smoother's levels on the lane-pair split (k_fwd_pair / k_bwd_pair<Q, CPW>): k_fwd_level /
// k_bwd_level with each propagation split over the Q waves of a workgroup (pair::propagate, the
// lane schedule's expressions: bitwise the lane smoother).  The row loop is workgroup-uniform
// (the longest cell of the workgroup; a cell past its rows computes on its frozen state and
// stores nothing); wave 0 stores the rows.  For levels up to pair_max_cells (the example's deep
// trees, per-GPU shards of C3/C4-sized forests), where the lane smoother waits on its step.
// ------------------------------------------------------------------------------------------
namespace pair {
// the workgroup's step count (its longest cell) and lane 0's operands for lanes without a cell
template <int CPW>
GGP_DEV int wg_rows(int *s_rows, const int w, const int lane, const int nrows)
{
    if (w == 0) s_rows[lane] = nrows;
    __syncthreads();
    int kmax = 0;
    for (int l = 0; l < CPW; ++l) kmax = max(kmax, s_rows[l]);
    return kmax;
}
GGP_DEV void adopt_lane0(const bool valid, double *m, double *C, double &dt)
{
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const double v = __shfl(m[q], 0);
        m[q] = valid ? m[q] : v;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const double v = __shfl(C[q], 0);
        C[q] = valid ? C[q] : v;
    }
    const double v = __shfl(dt, 0);
    dt = valid ? dt : v;
}
}  // namespace pair

#define GGP_PAIR_LDS(CPW)                                                                         \
    __shared__ double s_tab[kDawsonTab];                                                          \
    __shared__ double s_x[ggp::NXC * (CPW)], s_d[ggp::ND * (CPW)], s_i[ggp::NI * (CPW)],          \
        s_o[pair::kOSlots * (CPW)];                                                               \
    __shared__ int s_rows[64]

// prediction_forward (predictions.h:93-173) on the split: k_fwd_level's row loop
template <int Q, int CPW>
__global__ __launch_bounds__(64 * Q) void k_fwd_pair(DevForest F, const double *__restrict__ ptab, int n_seg,
                                                     const int32_t *__restrict__ cells, int n, double *__restrict__ pstate,
                                                     double *__restrict__ out)
{
    GGP_PAIR_LDS(CPW);
    __shared__ double s_par[11 * kSegLds];   // the parameter rows (n_seg <= kSegLds: the launch checks)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w == 0) load_dawson_table(s_tab, lane);
    if (w == 1 % Q) stage_params<true>(s_par, ptab, n_seg, lane);
    __syncthreads();
    const double *PT = s_par;
    const int i = blockIdx.x * CPW + lane;
    const bool valid = lane < CPW && i < n;
    int c = 0, nrows = 0;
    int64_t r0 = 0;
    const double *pi = PT, *pprop = PT;
    double m[4] = {0, 0, 0, 0}, C[16] = {0}, dt = 0.0;
    bool pending = false, divide = false;
    if (valid) {
        c = cells[i];
        r0 = F.row_off[c];
        nrows = (int)(F.row_off[c + 1] - r0);
        const int par = F.parent[c];
        pi = seg_params(F, PT, n_seg, par < 0 ? r0 : F.row_off[par + 1] - 1);   // :103-108
        pending = cell_prologue(F, pi, pstate, c, r0, m, C, dt);
        divide = pending;
        pprop = pi;
    }
    pair::adopt_lane0(valid, m, C, dt);
    const int kmax = pair::wg_rows<CPW>(s_rows, w, lane, nrows);
    bool live = valid && nrows > 0;
    const double *ou_src = nullptr;   // the OU constants per segment change only (k_fwd_level)
    ggp::OU ou{};
    // row r's operands (its data, time, the next row's time, its raw segment index) are loaded
    // during row r - 1, after its propagation and before its store (k_fwd_level's pipeline:
    // unconditional loads, indices clamped to the cell's rows; a lane without a cell reads row 0)
    const int64_t r_last = r0 + max(nrows, 1) - 1;
    double y_l_n = F.logl[r0], y_f_n = F.fp[r0], t_r_n = F.time[r0], t_nx_n = F.time[min(r0 + 1, r_last)];
    int seg_n = F.seg ? F.seg[r0] : 0;
    __builtin_amdgcn_s_waitcnt(0);   // the prologue's loads complete here (k_fwd_level)
    for (int k = 0; k < kmax; ++k) {
        const int64_t r = r0 + k;
        const double y_l = y_l_n, y_f = y_f_n, t_r = t_r_n, t_nx = t_nx_n;
        const int seg_r = seg_n;
        if (__builtin_amdgcn_ballot_w64(live && pending)) {
            double mn[4], Cn[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) mn[q] = m[q];
#pragma unroll
            for (int q = 0; q < 16; ++q) Cn[q] = C[q];
            if (pprop != ou_src) {
                ou = ggp::make_ou(pprop[0], pprop[1], pprop[2], pprop[3], pprop[4], pprop[5], pprop[6]);
                ou_src = pprop;
            }
            pair::propagate_w<Q, CPW>(w, mn, Cn, dt, ou, s_tab, s_x, s_d, s_i, s_o, lane);
            if (live && pending) {
#pragma unroll
                for (int q = 0; q < 4; ++q) m[q] = mn[q];
#pragma unroll
                for (int q = 0; q < 16; ++q) C[q] = Cn[q];
                if (divide) {
                    ggp::division_map(m, C, pi[9], pi[10], F.binomial, F.log2);
                    divide = false;
                }
            }
        }
        {   // row r + 1's operands, ahead of row r's store
            const int64_t rn = min(r + 1, r_last);
            y_l_n = F.logl[rn];
            y_f_n = F.fp[rn];
            t_r_n = F.time[rn];
            t_nx_n = F.time[min(r + 2, r_last)];
            if (F.seg) seg_n = F.seg[rn];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (live) {
            const double *p = seg_row(PT, n_seg, seg_r);
            const double x0 = y_l - m[0];
            const double x1 = y_f - m[1];
            ggp_innov v;
            ggp_innovation(m, C, p[7], p[8], F.scaled, F.fp_auto, v);
            ggp_posterior(m, C, x0, x1, v);
            if (w == 0) store20(out + (size_t)20 * r, m, C);
            pending = k + 1 < nrows;
            if (pending) dt = t_nx - t_r;
            pprop = p;   // the step t -> t+1 uses row t's parameters (:143-146)
            live = k + 1 < nrows;
        }
    }
    if (valid && w == 0) store20(pstate + (size_t)20 * c, m, C);
}

// prediction_backward (predictions.h:368-444) on the split: k_bwd_level's row loop, bottom-up
template <int Q, int CPW>
__global__ __launch_bounds__(64 * Q) void k_bwd_pair(DevForest F, const double *__restrict__ ptab, int n_seg,
                                                     const int32_t *__restrict__ cells, int n, double *__restrict__ pstate,
                                                     double *__restrict__ out)
{
    GGP_PAIR_LDS(CPW);
    __shared__ double s_par[11 * kSegLds];   // the parameter rows (n_seg <= kSegLds: the launch checks)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w == 0) load_dawson_table(s_tab, lane);
    if (w == 1 % Q) stage_params<true>(s_par, ptab, n_seg, lane);
    __syncthreads();
    const double *PT = s_par;
    const int i = blockIdx.x * CPW + lane;
    const bool valid = lane < CPW && i < n;
    int c = 0, nrows = 0, d1 = -1;
    int64_t r0 = 0, r1 = 0;
    const double *pi = PT;
    double m[4] = {0, 0, 0, 0}, C[16] = {0}, dt = 0.0;
    bool internal = false;
    if (valid) {
        c = cells[i];
        r0 = F.row_off[c];
        r1 = F.row_off[c + 1];
        nrows = (int)(r1 - r0);
        pi = seg_params(F, PT, n_seg, r1 - 1);   // :376-378
        d1 = F.d1[c];
        const int d2 = F.d2[c];
        if (d1 < 0 && d2 < 0) {   // init_sc_distribution_r leaf branch (:317-332)
            const double *st = pstate + (size_t)20 * c;
#pragma unroll
            for (int k = 0; k < 4; ++k) m[k] = st[k];
#pragma unroll
            for (int k = 0; k < 16; ++k) C[k] = st[4 + k];
            m[0] = F.leaf_mean0;
            m[1] = F.leaf_mean1;
            C[0] = F.leaf_var0;
            C[5] = F.leaf_var1;
            m[2] = -pi[0];
            m[3] = -pi[3];
            C[10] = pi[2] / (2. * pi[1]);
            C[15] = pi[5] / (2. * pi[4]);
        } else {   // mean_cov_after_division_r (:201-275), then the propagation below
            const double *s1 = pstate + (size_t)20 * d1;
#pragma unroll
            for (int k = 0; k < 4; ++k) m[k] = s1[k];
#pragma unroll
            for (int k = 0; k < 16; ++k) C[k] = s1[4 + k];
            ggp::division_map_r(m, C, pi[9], pi[10], F.binomial, F.log2);
            if (d2 >= 0) {
                double m2[4], C2[16];
                const double *s2 = pstate + (size_t)20 * d2;
#pragma unroll
                for (int k = 0; k < 4; ++k) m2[k] = s2[k];
#pragma unroll
                for (int k = 0; k < 16; ++k) C2[k] = s2[4 + k];
                ggp::division_map_r(m2, C2, pi[9], pi[10], F.binomial, F.log2);
                ggp::mult_gauss(m, C, m2, C2);
            }
            dt = F.time[F.row_off[d1]] - F.time[r1 - 1];
            internal = true;
        }
    }
    pair::adopt_lane0(valid, m, C, dt);
    const int kmax = pair::wg_rows<CPW>(s_rows, w, lane, nrows);
    const double *pq = pi;   // the next propagation's parameters (the reversed model)
    const double *ou_src = nullptr;   // the OU constants per segment change only (k_fwd_level)
    ggp::OU ou{};
    auto prop = [&](const bool act, const double t) {
        double mn[4], Cn[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) mn[q] = m[q];
#pragma unroll
        for (int q = 0; q < 16; ++q) Cn[q] = C[q];
        if (pq != ou_src) {
            ou = ggp::make_ou(-pq[0], pq[1], pq[2], -pq[3], pq[4], pq[5], -pq[6]);
            ou_src = pq;
        }
        pair::propagate_w<Q, CPW>(w, mn, Cn, t, ou, s_tab, s_x, s_d, s_i, s_o, lane);
        if (act) {
#pragma unroll
            for (int q = 0; q < 4; ++q) m[q] = mn[q];
#pragma unroll
            for (int q = 0; q < 16; ++q) C[q] = Cn[q];
        }
    };
    bool live = valid && nrows > 0;
    bool pend = internal;   // the propagation before this row's update (one call site)
    // row r's operands (its data and time, the previous row's time and raw segment index) are
    // loaded during row r + 1, after its propagation and before its store (k_fwd_pair, downwards;
    // indices clamped to the cell's rows, a lane without a cell reads row 0)
    const int64_t r_first = r0, r_top = r1 > r0 ? r1 - 1 : r0;
    auto seg_at = [&](const int64_t rr) { return F.seg ? F.seg[rr] : 0; };
    double y_l_n = F.logl[r_top], y_f_n = F.fp[r_top], t_r_n = F.time[r_top], t_p_n = F.time[max(r_top - 1, r_first)];
    int seg_r_n = seg_at(r_top), seg_p_n = seg_at(max(r_top - 1, r_first));
    __builtin_amdgcn_s_waitcnt(0);   // the prologue's loads complete here (k_fwd_level)
    for (int k = 0; k < kmax; ++k) {
        const int64_t r = r1 - 1 - k;
        const double y_l = y_l_n, y_f = y_f_n, t_r = t_r_n, t_p = t_p_n;
        const int seg_r = seg_r_n, seg_p = seg_p_n;
        if (__builtin_amdgcn_ballot_w64(pend)) prop(pend, dt);
        {   // row r - 1's operands, ahead of row r's store
            const int64_t rn = max(r - 1, r_first), rp = max(r - 2, r_first);
            y_l_n = F.logl[rn];
            y_f_n = F.fp[rn];
            t_r_n = F.time[rn];
            t_p_n = F.time[rp];
            seg_r_n = seg_p;
            seg_p_n = seg_at(rp);
        }
        __builtin_amdgcn_sched_barrier(0);
        bool more = false;
        if (live) {
            double rm[4], rC[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) rm[q] = m[q];
#pragma unroll
            for (int q = 0; q < 16; ++q) rC[q] = C[q];
            ggp::reverse_state(rm, rC);
            if (w == 0) store20(out + (size_t)20 * r, rm, rC);   // the prior, before the update
            const double *p = seg_row(PT, n_seg, seg_r);
            const double x0 = y_l - m[0];
            const double x1 = y_f - m[1];
            ggp_innov v;
            ggp_innovation(m, C, p[7], p[8], F.scaled, F.fp_auto, v);
            ggp_posterior(m, C, x0, x1, v);
            more = r > r0;
            if (more) {
                pq = seg_row(PT, n_seg, seg_p);   // seg_params(r - 1)
                dt = t_r - t_p;
            }
        }
        pend = more;
        live = more;
    }
    if (valid && w == 0) store20(pstate + (size_t)20 * c, m, C);
}

// combine_predictions (predictions.h:466-499): one lane per row.  FAST (the default): the
// inverses through reciprocal pivots, the product's mean reassociated (ggp_predict.h);
// GGP_COMBINE_EXACT=1: the oracle's operations
template <bool FAST>
__global__ __launch_bounds__(256) void k_combine(const double *__restrict__ ptab, int n_seg,
                                                 const int32_t *__restrict__ prior_seg, int64_t n_rows,
                                                 const double *__restrict__ fwd, const double *__restrict__ bwd,
                                                 double *__restrict__ out)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    double m[4], C[16], mb[4], Cb[16];
    const double *f = fwd + (size_t)20 * r, *b = bwd + (size_t)20 * r;
#pragma unroll
    for (int k = 0; k < 4; ++k) { m[k] = f[k]; mb[k] = b[k]; }
#pragma unroll
    for (int k = 0; k < 16; ++k) { C[k] = f[4 + k]; Cb[k] = b[4 + k]; }
    int s = prior_seg[r];
    if (s < 0 || s >= n_seg) s = 0;
    if constexpr (FAST) {
        ggp::combine_info(m, C, mb, Cb, ptab + 11 * s);
    } else {   // the oracle's operations (GGP_COMBINE_EXACT=1): multiply_gaussian, then divide_by_prior
        ggp::mult_gauss<false>(m, C, mb, Cb);
        ggp::divide_prior<false>(m, C, ptab + 11 * s);
    }
    store20(out + (size_t)20 * r, m, C);
}

// ------------------------------------------------------------------------------------------
// -j kernels (ggp_joints.h).  Per-row tables: back [20] = the backward factor over the prior,
// cond [36] = a, F, A of the step conditional, start [72] = the start joint.
// ------------------------------------------------------------------------------------------
constexpr int kJBack = 20, kJCond = 36, kJStart = 72;

GGP_DEV void load_g4(const double *src, ggp::G4 &g)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) g.m[k] = src[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) g.C[k] = src[4 + k];
}

GGP_DEV void store_a4(double *dst, const ggp::A4 &g)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = g.a[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        dst[4 + k] = g.F[k];
        dst[20 + k] = g.A[k];
    }
}

GGP_DEV ggp::A4 load_a4(const double *src)
{
    ggp::A4 g;
#pragma unroll
    for (int k = 0; k < 4; ++k) g.a[k] = src[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        g.F[k] = src[4 + k];
        g.A[k] = src[20 + k];
    }
    return g;
}

GGP_DEV void store_g8(double *dst, const ggp::G8 &g)
{
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k] = g.m[k];
#pragma unroll
    for (int k = 0; k < 64; ++k) dst[8 + k] = g.C[k];
}

GGP_DEV void load_g8(const double *src, ggp::G8 &g)
{
#pragma unroll
    for (int k = 0; k < 8; ++k) g.m[k] = src[k];
#pragma unroll
    for (int k = 0; k < 64; ++k) g.C[k] = src[8 + k];
}

__global__ __launch_bounds__(64) void k_joint_rows(DevForest F, const double *__restrict__ ptab, int n_seg,
                                                   const int32_t *__restrict__ row_cell, int64_t n_rows,
                                                   const double *__restrict__ fwd, const double *__restrict__ bwd,
                                                   double *__restrict__ back, double *__restrict__ cond,
                                                   double *__restrict__ start)
{
    __shared__ double s_tab[kDawsonTab];
    const int lane = threadIdx.x;
    load_dawson_table(s_tab, lane);
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * 64 + lane;
    if (r >= n_rows) return;
    const int c = row_cell[r];
    const int64_t r1 = F.row_off[c + 1];
    const double *p = seg_params(F, ptab, n_seg, r);
    const ggp::G4 bk = ggp::backward_over_prior(bwd + (size_t)20 * r, p);
    store20(back + (size_t)kJBack * r, bk.m, bk.C);
    const double *ft = fwd + (size_t)20 * r;
    const ggp::OU ou = ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    double m2[4], C2[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) m2[k] = ft[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) C2[k] = ft[4 + k];
    ggp::G8 j;
    ggp::A4 cd;
    if (r + 1 < r1) {
        // consecutive_joint / consecutive_conditional (correlation_tree.h:285-356)
        double K[16], Kt[16];
        ggp::propagate_lane(m2, C2, F.time[r + 1] - F.time[r], ou, s_tab, K);
        ggp::jt<4, 4>(K, Kt);
        ggp::join8(m2, ft, C2, K, Kt, ft + 4, j);
        ggp::G8 jc;
        ggp::join8(ft, m2, ft + 4, Kt, K, C2, jc);
        ggp::G4 mg;
        ggp::A4 sc;
        ggp::separate(jc, mg, sc);
        cd = ggp::a_transform(sc);
    } else if (F.d1[c] >= 0) {
        // consecutive_{joint,conditional}_cell_division (correlation_tree.h:158-283)
        const double dtd = F.time[F.row_off[F.d1[c]]] - F.time[r];
        if (F.binomial) {
            double mb[4], Cb[16], cross[16], crossT[16];
            ggp::propagate_lane(m2, C2, dtd, ou, s_tab);
            ggp::division_binomial_j(p, m2, C2, ft, mb, Cb, cross);
            ggp::jt<4, 4>(cross, crossT);
            ggp::join8(mb, ft, Cb, cross, crossT, ft + 4, j);
            ggp::G8 jc;
            ggp::join8(ft, mb, ft + 4, crossT, cross, Cb, jc);
            ggp::G4 mg;
            ggp::A4 sc;
            ggp::separate(jc, mg, sc);
            cd = ggp::a_transform(sc);
        } else {
            ggp::G4 mg;
            load_g4(ft, mg);
            const ggp::A4 dv = ggp::division_affine(p);
            j = ggp::flip_xy(ggp::to_joint(mg, dv));
            cd = ggp::a_transform(dv);
        }
    } else {
        return;   // a leaf's last row starts no walk and is never stepped from
    }
    store_g8(start + (size_t)kJStart * r, j);
    store_a4(cond + (size_t)kJCond * r, cd);
}

// One lane per start row.  emit == nullptr: count the joints into counts[i]; else write them
// from out_off[i] on (start, target, mean[8], cov[64]).  stack: depth x (cell, joint) per lane.
__global__ __launch_bounds__(64) void k_joint_walk(DevForest F, const double *__restrict__ ptab, int n_seg,
                                                   const int32_t *__restrict__ row_cell,
                                                   const double *__restrict__ bstate,
                                                   const double *__restrict__ back, const double *__restrict__ cond,
                                                   const double *__restrict__ start, double tol, int64_t r_lo,
                                                   int64_t n_starts, int depth, double *__restrict__ stack_j,
                                                   int32_t *__restrict__ stack_c, int64_t *__restrict__ counts,
                                                   const int64_t *__restrict__ out_off, int64_t *__restrict__ out_idx,
                                                   double *__restrict__ out_val)
{
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= n_starts) return;
    const int64_t r = r_lo + i;
    int cur = row_cell[r];
    const int64_t rows0 = F.row_off[cur + 1] - F.row_off[cur];
    int64_t cn = r - F.row_off[cur];
    bool at_div = false;
    int64_t cnt = 0;
    // this start's slots [out_off[i], out_off[i + 1]): exact counts (two-pass) or the walk's bound
    // (single pass); a joint past the end is counted, not stored (the host then redoes the range)
    int64_t out = out_off ? out_off[i] : 0;
    const int64_t out_end = out_off ? out_off[i + 1] : 0;
    if (cn == rows0 - 1) {
        if (F.d1[cur] < 0) {
            counts[i] = 0;
            return;
        }
        at_div = true;
    }
    ggp::G8 J;
    load_g8(start + (size_t)kJStart * r, J);
    double *sj = stack_j + (size_t)i * depth * kJStart;
    int32_t *sc = stack_c + (size_t)i * depth;
    int sp = 0;
    for (;;) {
        bool stop = false;
        if (!at_div) {
            // calc_joint_distributions (correlation_tree.h:464-524)
            const int64_t rr0 = F.row_off[cur], rows = F.row_off[cur + 1] - rr0;
            const double mean1 = bstate[(size_t)20 * cur + 1];   // cell.mean(1) after -p
            const bool has_d1 = F.d1[cur] >= 0;
            for (int64_t m = 1; cn + m < rows; ++m) {
                const int64_t rr = rr0 + cn + m;
                const double *p = seg_params(F, ptab, n_seg, rr);
                const double D[4] = {p[7], 0.0, 0.0, F.scaled ? p[8] * (mean1 + F.fp_auto) : p[8]};
                ggp::include_measurement(J, D, F.logl[rr], F.fp[rr]);
                ggp::G4 mg, bk;
                ggp::A4 sep;
                ggp::separate(J, mg, sep);
                load_g4(back + (size_t)kJBack * rr, bk);
                const ggp::G8 comb = ggp::to_joint(ggp::g_multiply(mg, bk), sep);
                if (ggp::cross_small(comb, tol)) {
                    stop = true;
                    break;
                }
                if (out < out_end) {
                    out_idx[2 * out] = r;
                    out_idx[2 * out + 1] = rr;
                    store_g8(out_val + (size_t)kJStart * out, comb);
                    ++out;
                }
                ++cnt;
                if (cn + m < rows - 1 || has_d1) J = ggp::next_joint(J, load_a4(cond + (size_t)kJCond * rr));
            }
        }
        if (!stop && F.d1[cur] >= 0) {   // joint_distributions_recr: daughter1, then daughter2
            if (F.d2[cur] >= 0 && sp < depth) {
                sc[sp] = F.d2[cur];
                store_g8(sj + (size_t)kJStart * sp, J);
                ++sp;
            }
            cur = F.d1[cur];
            cn = -1;
            at_div = false;
            continue;
        }
        if (sp == 0) break;
        --sp;
        cur = sc[sp];
        load_g8(sj + (size_t)kJStart * sp, J);
        cn = -1;
        at_div = false;
    }
    counts[i] = cnt;
}

// the packed joint record (ggp_joints_packed): the 8 means, then the covariance's upper triangle
// row by row (output_upper_triangle, predictions.h:540-551) -- the 44 values the CLI prints
constexpr int kJPacked = 44;
struct JUpper {
    unsigned char off[kJPacked];   // record value -> offset in the 72-value record
};
constexpr JUpper make_jupper()
{
    JUpper u{};
    for (int k = 0; k < 8; ++k) u.off[k] = (unsigned char)k;
    int q = 8;
    for (int m = 0; m < 8; ++m)
        for (int k = m; k < 8; ++k) u.off[q++] = (unsigned char)(8 + 8 * m + k);
    return u;
}
GGP_DEV constexpr JUpper kJUpper = make_jupper();

// -j: start i's joints from its slots [boff[i], ...) of the 72-value records to the output at
// coff[i] in W-value records (72: as they are; 44: packed), one workgroup per start
template <int W>
__global__ __launch_bounds__(256) void k_joint_pack(int64_t n_starts, const int64_t *__restrict__ boff,
                                                    const int64_t *__restrict__ coff, const int64_t *__restrict__ counts,
                                                    const int64_t *__restrict__ src_idx, const double *__restrict__ src_val,
                                                    int64_t *__restrict__ dst_idx, double *__restrict__ dst_val)
{
    const int64_t i = blockIdx.x;
    if (i >= n_starts) return;
    const int64_t n = counts[i], b = boff[i], c = coff[i];
    for (int64_t k = threadIdx.x; k < 2 * n; k += blockDim.x) dst_idx[2 * c + k] = src_idx[2 * b + k];
    for (int64_t k = threadIdx.x; k < (int64_t)W * n; k += blockDim.x) {
        const int64_t q = k / W;
        const int e = (int)(k - q * W);
        dst_val[(size_t)W * c + k] = src_val[(size_t)kJStart * (b + q) + (W == kJStart ? e : kJUpper.off[e])];
    }
}


// ------------------------------------------------------------------------------------------
// Deterministic total whose bits do not depend on how the forest is sharded over devices:
//   tree sum  : a tree's cell partials in DFS pre-order, added one after another (within a
//               tree: the reference's own accumulation order, likelihood.h:110-122, at cell
//               granularity)
//   block sum : B consecutive trees of the global root order (B from the tree count only),
//               one workgroup, a fixed LDS tree
//   total     : the block sums in global block order, a fixed pairwise tree (host, top_sum)
// A block always lives whole on one shard, so N shards give the same bits as one.  The first
// NaN is the min over (global DFS rank << 24 | row): the reference's order (likelihood.h:71-93).
// ------------------------------------------------------------------------------------------
constexpr int kRedMax = 1024;
constexpr long long kNoNan = 0x7fffffffffffffffLL;

__global__ __launch_bounds__(kRedMax) void k_reduce_blocks(int64_t n_cells, const double *__restrict__ cell_ll,
                                                            const int32_t *__restrict__ cell_nan,
                                                            const int64_t *__restrict__ tree_dfs,
                                                            const int32_t *__restrict__ blk_t0,
                                                            const int32_t *__restrict__ blk_nt,
                                                            const int32_t *__restrict__ gdfs, int n_lblocks,
                                                            double *__restrict__ out_sum, int64_t *__restrict__ out_nan,
                                                            unsigned *__restrict__ done, int64_t *__restrict__ out_seq,
                                                            int64_t seq, double *__restrict__ host_sum,
                                                            int64_t *__restrict__ host_nan)
{
    __shared__ double s_sum[kRedMax];
    __shared__ long long s_nan[kRedMax];
    const int tid = threadIdx.x, nt = blockDim.x, j = blockIdx.x;
    const int64_t pt = blockIdx.y;             // batch point (a single evaluation: 0)
    cell_ll += pt * n_cells;
    cell_nan += pt * n_cells;
    double v = 0.0;
    long long code = kNoNan;
    if (tid < blk_nt[j]) {
        const int64_t t = blk_t0[j] + tid;
        for (int64_t i = tree_dfs[t]; i < tree_dfs[t + 1]; ++i) {
            v += cell_ll[i];
            const int nr = cell_nan[i];
            if (nr != kNanNone && code == kNoNan) code = ((long long)gdfs[i] << 24) | (long long)nr;
        }
    }
    s_sum[tid] = v;
    s_nan[tid] = code;
    __syncthreads();
    for (int w = nt / 2; w > 0; w >>= 1) {
        if (tid < w) {
            s_sum[tid] = s_sum[tid] + s_sum[tid + w];
            s_nan[tid] = min(s_nan[tid], s_nan[tid + w]);
        }
        __syncthreads();
    }
    __shared__ bool s_last;
    if (tid == 0) {
        out_sum[pt * n_lblocks + j] = s_sum[0];
        out_nan[pt * n_lblocks + j] = s_nan[0];
        s_last = false;
        if (out_seq) {
            // device-scope fence, then count: the last workgroup to finish sees every block
            __threadfence();
            const unsigned prev = atomicAdd(done, 1u);
            s_last = prev + 1 == gridDim.x * gridDim.y;
        }
    }
    if (!out_seq) return;
    __syncthreads();
    if (!s_last) return;
    // the last workgroup copies the block results to the mapped host slots in one burst, then
    // publishes the call's sequence number (the host polls it, ggp_loglik_result)
    __threadfence();
    for (int k = tid; k < n_lblocks; k += nt) {
        host_sum[k] = __hip_atomic_load(out_sum + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        host_nan[k] = __hip_atomic_load(out_nan + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tid == 0) {
        *done = 0u;                            // ready for the next call (stream ordered)
        __threadfence_system();
        __hip_atomic_store(out_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ------------------------------------------------------------------------------------------
// Multi-process evaluation (ggp_comm_attach): this rank's partial, the RCCL all-gather, the
// rank-order sum -- all on the shard's stream behind the evaluation.
// k_rank_partial: ggp_loglik_result's total on the device: the block results (mapped host
// memory, written by the reduction of this evaluation) zero-padded to np2 and summed by the same
// fixed pairwise tree (v[i] = v[2i] + v[2i+1], level by level: top_sum's bits), and the flag of
// a NaN partial (a first-NaN code, or a NaN sum: ggp_loglik_result's GGP_ENAN cases).
// part = {sum, flag as a double}: the 16 B this rank sends.
// ------------------------------------------------------------------------------------------
constexpr int kPartMax = 4096;   // blocks a rank may hold (4096 x 1024 trees)

__global__ __launch_bounds__(256) void k_rank_partial(const double *__restrict__ blk, const int64_t *__restrict__ code, int nb,
                                                      int np2, double *__restrict__ part)
{
    __shared__ double v[kPartMax];
    __shared__ long long cm[256];
    const int t = threadIdx.x;
    long long c = kNoNan;
    for (int i = t; i < np2; i += 256) {
        double x = 0.0;
        if (i < nb) {   // fine-grained host memory: system-scope loads
            x = __longlong_as_double(
                (long long)__hip_atomic_load(reinterpret_cast<const unsigned long long *>(blk + i), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM));
            c = min(c, (long long)__hip_atomic_load(code + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        }
        v[i] = x;
    }
    cm[t] = c;
    __syncthreads();
    constexpr int R = kPartMax / 512;   // pairs per thread at the widest level
    for (int n = np2; n > 1; n >>= 1) {
        double x[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int i = t + 256 * j;
            x[j] = i < n / 2 ? v[2 * i] + v[2 * i + 1] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int i = t + 256 * j;
            if (i < n / 2) v[i] = x[j];
        }
        __syncthreads();
    }
    if (t == 0) {
        long long mc = kNoNan;
        for (int k = 0; k < 256; ++k) mc = min(mc, cm[k]);
        const double s = v[0];
        part[0] = s;
        // 2: this rank's first bad cell stalled (GGP_ETIMEOUT on every rank), 1: a NaN
        part[1] = (mc != kNoNan && (mc & 0xffffff) == kRowStall) ? 2.0 : (mc != kNoNan || s != s) ? 1.0 : 0.0;
    }
}

// distributed.combine_partials on the gathered {sum, flag} of every rank: the first rank with a
// flag decides (NaN), else 0.0 + p_0 + p_1 + ... in rank order; the result and that rank to the
// mapped host slots, then the call's sequence number (system-scope release; the host spins on it)
__global__ void k_rank_sum(const double *__restrict__ g, int nranks, double *out_sum, int64_t *out_rank, int64_t *out_seq,
                           int64_t seq)
{
    if (threadIdx.x != 0) return;
    double s = 0.0;
    long long nr = -1;
    for (int r = 0; r < nranks; ++r) {
        // the first bad rank, + 2^32 when its first bad cell stalled
        if (nr < 0 && g[2 * r + 1] != 0.0) nr = r + (g[2 * r + 1] == 2.0 ? (1LL << 32) : 0);
        s = s + g[2 * r];
    }
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(out_sum),
                       (unsigned long long)__double_as_longlong(nr >= 0 ? __longlong_as_double(0x7ff8000000000000LL) : s),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out_rank, (int64_t)nr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(out_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------------------------------
// Test-only device entry points (tests/test_gpu_device_math.py): the device Dawson in both
// forms the kernels use, and the four tauint integrals of mean_cov_model.h:9-67 built from
// the same device primitives (rdiv, ocml exp, table Dawson, a^k sqrt(a)) in tau_body's
// expression order, at arbitrary (t0, t1, a, b, c).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_debug_dawson(const double *__restrict__ x, int64_t n, int variant,
                                                     double *__restrict__ out)
{
    namespace W = ggp::wave;
    __shared__ double s_tab[kDawsonTab];
    __shared__ __attribute__((aligned(16))) double s_w[W::kTabRows * W::kTabRow];
    load_dawson_table(s_tab, threadIdx.x);
    lds_fill<W::kTabRows * W::kTabRow>(s_w, threadIdx.x, [](const int k) { return W::tab_entry(k); });
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const double v = i < n ? x[i] : 0.0;
    double r;
    if (variant == 0) {
        r = ggp_dawson_tab(v, s_tab);
    } else {
        // the wave schedule's stage B on a Dawson lane (ggp_wave.h stageB): z = rdiv(B + 2a 0, 1, 1)
        // = B = fma(0, 1, v) + 0 = v exactly, then the lane's reduction, table row, Horner, sign
        // and, where needed, the rare branches -- the same instructions the kernel runs
        W::WStep S{};
        S.t = 0.0; S.a = 1.0; S.two_a = 2.0; S.four_a = 4.0; S.four_aa = 4.0; S.two_sa = 1.0; S.m2sa = -1.0;
        S.r_two_sa = 1.0; S.r_two_sa0 = 1.0; S.r_four_a = 0.25; S.bbl = v; S.Cxl = 0.0; S.bx = 0.0; S.Cxx = 0.0;
        W::Lane L{};
        L.b_tau = 0.0; L.b_km = 1.0; L.b_gqks = 0.0; L.b_m1 = 1.0; L.b_m2 = 0.5; L.b_kc = 0.0;
        L.b_mult = GGP_SPI2; L.b_sgn = (int)0x80000000u; L.b_isE = 0; L.b_isA = 0; L.b_isD = 1; L.b_exmask = 0;
        const W::BOut o = W::stageB(S, L, s_w);
        r = o.rare ? W::stageB_rare(true, o.arg, o.z, o.v) : o.v;
    }
    if (i < n) out[i] = r;
}

GGP_DEV double debug_tauint(const int k, const double t0, const double t1, const double a, const double b,
                            const double c, const double *tab)
{
    // the tauint formulas with the integral bounds as given (mean_cov_model.h:9-67); z, the
    // exponentials and the powers formed as the propagator forms them (ggp_prop.h)
    const double sa = sqrt(a);
    const double two_sa = 2. * sa, m2sa = -2. * sa, two_a = 2. * a, four_a = 4. * a, four_aa = 4 * (a * a);
    const double r_two_sa = ggp::frcp(two_sa), r_four_a = ggp::frcp(four_a);
    const double z0 = ggp::rdiv(b + two_a * t0, two_sa, r_two_sa), z1 = ggp::rdiv(b + two_a * t1, two_sa, r_two_sa);
    const double D0 = ggp_dawson_tab(z0, tab), D1 = ggp_dawson_tab(z1, tab);
    const double n_ = ggp::rdiv(-(b * b), four_a, r_four_a);
    if (k == 0) {
        const double Z0 = exp(a * (t0 * t0) + b * t0 + c), Z1 = exp(a * (t1 * t1) + b * t1 + c);
        return ggp::rdiv(2. * (-Z0 * D0 + Z1 * D1), two_sa, r_two_sa);
    }
    const double E0 = exp(n_ + c + z0 * z0), E1 = exp(n_ + c + z1 * z1);
    const double ec = exp(c), ea0 = exp(t0 * (b + a * t0)), ea1 = exp(t1 * (b + a * t1));
    const double pw = k == 1 ? 4. * (a * sa) : k == 2 ? 8. * ((a * a) * sa) : 16. * (((a * a) * a) * sa);
    const double rpw = ggp::frcp(pw);
    const double B = b;
    double x;
    if (k == 1)
        x = (m2sa * ec * (ea0 - ea1) + B * 2. * (E0 * D0 - E1 * D1));
    else if (k == 2)
        x = (two_sa * ec * (ea0 * (B - two_a * t0) - ea1 * (B - two_a * t1)) +
             (E0 * (two_a - B * B) * 2. * D0 + E1 * (-two_a + B * B) * 2. * D1));
    else
        x = (m2sa * ec *
             ((B * B) * (ea0 - ea1) - two_a * ea0 * (2. + B * t0) + two_a * ea1 * (2 + B * t1) +
              four_aa * (ea0 * (t0 * t0) - ea1 * (t1 * t1)))) +
            E0 * B * (-6. * a + B * B) * 2. * D0 - E1 * B * (-6 * a + B * B) * 2. * D1;
    return ggp::rdiv(x, pw, rpw);
}

__global__ __launch_bounds__(64) void k_debug_tauint(const double *__restrict__ in, int64_t n,
                                                     double *__restrict__ out)
{
    __shared__ double s_tab[kDawsonTab];
    load_dawson_table(s_tab, threadIdx.x);
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const double *q = in + 6 * i;   // k, t0, t1, a, b, c
    out[i] = debug_tauint((int)q[0], q[1], q[2], q[3], q[4], q[5], s_tab);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
thread_local std::string g_last_err;

// Every exported entry point that touches a device restores the caller's current HIP device on
// return: the engine switches devices per shard (hipSetDevice), and a caller (torch, another
// library) must find its own current device unchanged after any ggp_* call.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard()
    {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard()
    {
        int now = -1;   // hipSetDevice only when a shard switched it (the common one-device case: never)
        if (dev >= 0 && (hipGetDevice(&now) != hipSuccess || now != dev)) (void)hipSetDevice(dev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            g_last_err = std::string(#expr) + ": " + hipGetErrorString(_e);                 \
            return GGP_EDEV;                                                                \
        }                                                                                   \
    } while (0)

template <typename T>
int dev_upload(T **dst, const T *src, size_t n)
{
    *dst = nullptr;
    if (n == 0) return GGP_OK;
    if (hipMalloc((void **)dst, n * sizeof(T)) != hipSuccess) {
        g_last_err = "hipMalloc failed";
        return GGP_ENOMEM;
    }
    if (src) HIPCHK(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return GGP_OK;
}

// trees per reduction block: a function of the tree count only (the sum's shape must not depend
// on the sharding); at most 1024 (one workgroup), about 256-512 blocks for large forests
int64_t block_trees_for(int64_t n_trees)
{
    int64_t B = 1;
    while (B < kRedMax && B * 256 < n_trees) B *= 2;
    return B;
}

// fixed pairwise tree over the block sums in global order (zero padded to a power of two)
double top_sum(std::vector<double> v)
{
    size_t n = 1;
    while (n < v.size()) n *= 2;
    v.resize(n, 0.0);
    for (; n > 1; n /= 2)
        for (size_t i = 0; i < n / 2; ++i) v[i] = v[2 * i] + v[2 * i + 1];
    return v.empty() ? 0.0 : v[0];
}

// top_sum in place on a buffer already zero-padded to a power of two (n_pow2 entries): the same
// tree, no allocation (the objective's result path, once per call)
double top_sum_inplace(double *v, size_t n_pow2)
{
    for (size_t n = n_pow2; n > 1; n /= 2)
        for (size_t i = 0; i < n / 2; ++i) v[i] = v[2 * i] + v[2 * i + 1];
    return n_pow2 ? v[0] : 0.0;
}

}  // namespace

// One device (HIP ordinal) used by the handle: its stream, and the -p workspace its shards
// share (forward + backward rows, sized to the largest shard on the device; shards on one
// device are smoothed one after another on its stream).
struct DeviceCtx {
    int id = 0;
    hipStream_t stream = nullptr;
    int n_cu = 256;
    double *sm_fwd = nullptr, *sm_bwd = nullptr;
    int64_t sm_rows = 0;
};

// One shard: whole trees (whole reduction blocks) of the forest, cells in input order, on one
// device.  Everything below works on the shard's local numbering.
struct Shard {
    DeviceCtx *dev = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t n_cells = 0, n_rows = 0;
    int n_cu = 256;
    int kernel_pref = GGP_KERNEL_AUTO;
    // auto's schedule for small levels; the GGP_EXACT engine has no wave schedule (its table-driven
    // outputs sum in another order than the reference expressions): the group schedule there
    int auto_small = ggp::kExact ? GGP_KERNEL_GROUP : GGP_KERNEL_WAVE;
    int64_t wave_max_cells = 5120;    // auto: wave schedule for levels up to this size
    int64_t group_max_cells = 8192;   // auto with GGP_AUTO_SMALL=group: group schedule above that
    int64_t pair_max_cells = 32768;   // auto: lane-pair schedule above that, up to this size
    int tune_lane_cpw = 0, tune_group_cpw = 0;   // GGP_LANE_CPW / GGP_GROUP_CPW (tuning only)
    int tune_pair_cpw = 64;                      // GGP_PAIR_CPW: cells per lane-pair workgroup (32, 64)
    bool combine_exact = ggp::kExact;            // GGP_COMBINE_EXACT=1: k_combine with the oracle's operations
    bool combine_fused = true;                   // GGP_COMBINE_FUSED=0: k_combine after the backward pass always
    int tune_pair_q = 0;                         // GGP_PAIR_Q: waves per cell (2, 4; 0 = by level size)
    bool smoother_lane = false;                  // GGP_SMOOTHER_LANE=1: the lane smoother on every level
    int kernel_used = GGP_KERNEL_LANE;
    int32_t last_code = 0;
    DevForest F{};
    // device buffers
    double *d_time = nullptr, *d_logl = nullptr, *d_fp = nullptr;
    int64_t *d_row_off = nullptr;
    int32_t *d_parent = nullptr, *d_d1 = nullptr, *d_d2 = nullptr, *d_seg = nullptr;
    int32_t *d_level_cells = nullptr, *d_dfs_rank = nullptr;
    int32_t *d_prior_seg = nullptr;   // -p: segment of the stationary prior per row
    int32_t *d_row_cell = nullptr;    // -j: cell of every row
    double *d_state = nullptr, *d_cell_ll = nullptr;
    int32_t *d_cell_nan = nullptr;
    // chained wave launches (k_loglik_wave): per cell {parent to wait for, has a waiting daughter},
    // done flags holding the epoch of the evaluation that finished the cell
    CellLink *d_chain = nullptr;
    unsigned *d_cell_done = nullptr;
    unsigned epoch = 0;
    int wave_resident = 2048;          // k_loglik_wave blocks the device holds at once
    unsigned spin_max = kChainSpinMax; // GGP_CHAIN_SPIN_MAX: polls of a waiting second daughter
    int32_t *d_path_cells = nullptr, *d_path_seq = nullptr;   // path launch: cells, [n_paths + 1] starts
    int64_t n_paths = 0;               // 0: level launches
    // path launch's in-launch reduction (ChainRed): path -> block, paths per block, the blocks'
    // arrival counters
    int32_t *d_path_blk = nullptr, *d_blk_npaths = nullptr;
    unsigned *d_cnt_blk = nullptr;
    ChainRed red{};                    // the path launch's in-launch reduction (a kernel argument)
    std::vector<int32_t> level_kind;   // GGP_KERNEL_* each level runs
    // lane queue (k_loglik_lane_queue): runs of >= 2 consecutive lane-schedule levels, each one
    // persistent launch over its chunks; the launch's chunk counter (zeroed before it)
    struct QRun {
        int la, lb;                    // levels la .. lb - 1
        int64_t off, n, rows;          // chunks d_qchunks[off .. off + n), the run's rows
    };
    std::vector<QRun> qruns;
    std::vector<int32_t> qrun_at;      // level -> its run (-1: none / not the run's first level)
    QChunk *d_qchunks = nullptr;
    unsigned *d_qctr = nullptr;
    bool lane_queue = true;            // GGP_LANE_QUEUE=0: level-by-level lane launches
    int queue_resident = 1024;         // k_loglik_lane_queue workgroups the device holds at once
    // reduction (k_reduce_blocks): local trees in DFS order, the shard's blocks, global DFS ranks
    int64_t n_trees = 0, n_lblocks = 0;
    int red_threads = 64;
    int64_t *d_tree_dfs = nullptr;
    int32_t *d_blk_t0 = nullptr, *d_blk_nt = nullptr, *d_gdfs = nullptr;
    unsigned *d_done = nullptr;
    double *d_blk_sum = nullptr;       // this evaluation's block results (device), before the
    int64_t *d_blk_nan = nullptr;      // last workgroup copies them to the mapped host slots
    std::vector<int64_t> blk_global;   // local block -> global block
    // the result: pinned, mapped host memory k_reduce_blocks writes directly (no copy back):
    // block sums [n_lblocks], first-NaN codes [n_lblocks], then the call's sequence number
    // (the host spins on it instead of waiting for the kernel-completion signal, with
    // hipStreamQuery as the way out if the stream fails; GGP_SPIN=0: synchronise)
    void *h_res = nullptr;
    double *h_sum = nullptr, *m_sum = nullptr;
    int64_t *h_nan = nullptr, *m_nan = nullptr;
    volatile int64_t *h_seq = nullptr;
    int64_t *m_seq = nullptr;
    volatile unsigned long long *h_clk = nullptr;   // path launches: block 0's clock counters
    PathDesc *d_pdesc = nullptr;                    // path launches: per path (PathDesc)
    unsigned long long clk_snap[4] = {0, 0, 0, 0}; // h_clk as the last completed launch left it
    unsigned long long *m_clk = nullptr;
    // the largest |dt| of any propagation of the shard (in-cell steps and divisions): with the
    // parameters it bounds |k dt| for the wave schedule's product factors exp(-gl dt), exp(-gq dt),
    // exp(-b dt), exp(gq dt) (wave_products_risky)
    double max_dt = 0.0;
    bool used_path = false;                         // the last launch_levels took the path launch
    int64_t seq = 0;
    bool seq_pending = false;
    bool spin = true;
    // numbering
    std::vector<int32_t> cell_g;       // local cell -> global cell (ascending); empty = identity
    std::vector<int64_t> row_off;      // local row_offset (host copy)
    // schedule
    std::vector<int64_t> level_start;  // [n_levels+1] into level_cells
    // profiling
    bool profile = false;
    std::vector<hipEvent_t> ev;
    std::vector<int64_t> ev_rows;
    std::vector<int32_t> ev_kernel;   // per profiled launch: kind << 8 | lanes per cell
    std::vector<int64_t> ev_rows_launch;
    int n_prof = 0;
    // -p: per-cell working state, the combined rows (kept in HBM until the next ggp_predict so
    // ggp_predict_rows can stream them), the parameter table; device-time events
    double *d_sm_ptab = nullptr, *d_sm_pstate = nullptr, *d_sm_comb = nullptr;
    int32_t sm_ptab_cap = 0;
    hipEvent_t ev_pred[3] = {nullptr, nullptr, nullptr};   // start, after fwd+bwd, after combine
    bool pred_timed = false;
    // batched-objective workspace (ggp_total_loglik_batch), grown on demand
    double *d_b_ptab = nullptr, *d_b_state = nullptr, *d_b_ll = nullptr, *d_b_sum = nullptr;
    int32_t *d_b_nan = nullptr;
    int64_t *d_b_code = nullptr;
    unsigned *d_b_done = nullptr;   // ggp_total_loglik_chain / _tree: per point, the cells' done flags
    int32_t *d_b_pred = nullptr;    // ggp_total_loglik_tree: each point's predecessor
    int64_t b_cap = 0;   // points the workspace holds
    // -j: the smoother and the per-row joint tables, kept for the parameters they were made with
    // (the CLI asks for many start-row ranges with the same parameters)
    double *d_j_ptab = nullptr, *d_j_pstate = nullptr, *d_j_fwd = nullptr, *d_j_bwd = nullptr;
    double *d_j_back = nullptr, *d_j_cond = nullptr, *d_j_start = nullptr;
    std::vector<double> j_params;      // the table the joint tables hold (empty: none)
    // -j per-call buffers, grow-only (no hipMalloc / synchronising hipFree per start-row range):
    // the walks' stacks and counts, sized by start rows x depth, and the emitted joints
    void *d_jw_stack = nullptr, *d_jw_small = nullptr, *d_jw_out = nullptr, *d_jw_bnd = nullptr;
    size_t jw_stack_bytes = 0, jw_small_bytes = 0, jw_out_bytes = 0, jw_bnd_bytes = 0;
    // rows below every cell (all its descendants'): with the rows after a start row in its own cell,
    // the most joints that start's walk can emit (the single-pass emit's slots)
    std::vector<int64_t> j_below;
    size_t joint_slot_bytes = (size_t)2 << 30;   // GGP_JOINT_SLOT_MB: the single pass's slot budget (0: two passes)
};

// RCCL entry points, resolved at run time from the library the caller names (the one torch
// loaded, so the process holds a single RCCL): rccl.h signatures, the unique id by value
struct ggp_rccl_id {
    char internal[128];
};
struct RcclApi {
    void *lib = nullptr;
    int (*get_unique_id)(ggp_rccl_id *) = nullptr;
    int (*comm_init_rank)(void **, int, ggp_rccl_id, int) = nullptr;
    int (*all_gather)(const void *, void *, size_t, int, void *, hipStream_t) = nullptr;
    int (*comm_destroy)(void *) = nullptr;
    int (*comm_abort)(void *) = nullptr;   // ncclCommAbort (optional)
    int (*comm_count)(const void *, int *) = nullptr;   // ncclCommCount (optional)
    const char *(*error_string)(int) = nullptr;
};
constexpr int kRcclUint8 = 1;   // ncclUint8 (rccl.h ncclDataType_t)

// one rank of a group of one-GPU processes (ggp_comm_attach)
struct Comm {
    RcclApi api;
    void *nc = nullptr;                // ncclComm_t
    int nranks = 1, rank = 0;
    double *d_part = nullptr;          // this rank's {sum, flag}
    double *d_gath = nullptr;          // every rank's, in rank order
    void *h_res = nullptr;             // mapped: the total, the first NaN rank, the sequence number
    volatile double *h_sum = nullptr;
    volatile int64_t *h_rank = nullptr, *h_seq = nullptr;
    double *m_sum = nullptr;
    int64_t *m_rank = nullptr, *m_seq = nullptr;
    int64_t seq = 0;
    int32_t last_nan_rank = -1;
    int32_t local_nan = 0;             // this rank's own evaluation had a NaN (or stalled) last call
    bool failed = false;               // a failed collective evaluation: the communicator was aborted
};

// A failed evaluation after the collective may have been entered on other ranks (an enqueue error,
// a timeout) is fatal for the group: the communicator is aborted (ncclCommAbort, so no peer waits
// forever on it) and every later call on the handle returns GGP_EDEV.
static void comm_fail(Comm *c)
{
    if (c->failed) return;
    c->failed = true;
    if (c->nc) {
        if (c->api.comm_abort) c->api.comm_abort(c->nc);
        c->nc = nullptr;
    }
}

// one objective call's host split (ggp_call_trace)
struct CallRec {
    double enqueue_us, wait_us, result_us, kernel_us, shader_mhz, call;
};
constexpr int kCallRing = 512;

struct ggp_forest {
    int64_t n_cells = 0, n_rows = 0, n_trees = 0, blk_trees = 1, n_blocks = 0;
    std::chrono::steady_clock::time_point tr_t0, tr_t1, tr_t2;   // the pending call's entry, enqueue end, wait end
    bool tr_pending = false;
    int64_t tr_open = -1;              // ring entry whose kernel end stamp is still to be read
    int64_t tr_n = 0;                  // calls recorded
    CallRec tr_ring[kCallRing];
    std::vector<DeviceCtx *> devs;
    std::vector<Shard *> shards;
    std::vector<int32_t> dfs_order;    // global DFS position -> global cell
    std::vector<double> res_blocks;    // the result path's block sums, padded to a power of two
    std::vector<int64_t> row_off;      // global row_offset
    Comm *comm = nullptr;              // multi-process mode (ggp_comm_attach)
    int32_t tree_pts = 0;              // points of the last ggp_total_loglik_tree (ggp_keep_point_state)
    int64_t max_root_rows = 1;         // rows of the longest root cell (the chained launch's cap)
    int64_t chain_fallbacks = 0;       // chained calls finished call by call after a stall
};

namespace {

// Lane schedule: a wave's cost per step does not depend on how many of its lanes hold a
// cell (FP64 issue is per wave-instruction, and the clock falls with the number of busy
// SIMDs), so cells are packed 64 per wave at every level size (tools/lane_scan.py: 1k-30k
// trees, cpw 64 fastest everywhere).
int lane_cpw(const Shard *f) { return f->tune_lane_cpw > 0 ? f->tune_lane_cpw : 64; }

// the schedule of a level of n cells: the handle's choice, or auto (measured,
// profiles/r08_schedule_scan.txt): up to 5 cells per SIMD the wave schedule (GGP_AUTO_SMALL=group:
// the bitwise-lane-equal one), up to 8 per SIMD the group schedule with 1-8 cells per wave,
// above that the lane schedule
int level_kind(const Shard *f, int64_t n)
{
    if (f->kernel_pref != GGP_KERNEL_AUTO) return f->kernel_pref;
    if (n <= f->wave_max_cells) return f->auto_small;
    if (f->auto_small == GGP_KERNEL_GROUP && n <= f->group_max_cells) return GGP_KERNEL_GROUP;
    return n <= f->pair_max_cells ? GGP_KERNEL_PAIR : GGP_KERNEL_LANE;
}

// The wave schedule forms 22 exponentials as products exp(c_rep + ...) exp(+-k dt).  Beyond
// |k dt| ~ 700 a factor under- or overflows while the direct exponential may not (the lane
// schedules guard this per step: ggp_prop.h lane_guard_products; the wave, one cell per wave, has
// no room for a second form).  So an evaluation whose parameters reach |k| max_dt > 200 anywhere
// on the shard runs its wave levels on the lane-pair (or lane) schedule -- the same values to the
// bar -- and its chains call by call: a dt of days at the example's rates, where the reference's
// own integrals overflow soon after (tests/test_gpu_parity.py long-dt test)
constexpr double kWaveProductSafe = 200.0;
bool wave_products_risky(const Shard *f, const double *p)
{
    const double k = std::max(std::fabs(p[1]), std::max(std::fabs(p[4]), std::fabs(p[6])));
    return !(k * f->max_dt <= kWaveProductSafe);
}

int launch_levels(Shard *f, const ggp_params &P)
{
    const int n_levels = (int)f->level_start.size() - 1;
    f->n_prof = 0;
    ++f->epoch;
    auto prof_begin = [&]() -> hipError_t {
        if (f->profile && 2 * (f->n_prof + 1) <= (int)f->ev.size()) return hipEventRecord(f->ev[2 * f->n_prof], f->stream);
        return hipSuccess;
    };
    auto prof_end = [&](int64_t rows) -> hipError_t {
        if (f->profile && 2 * (f->n_prof + 1) <= (int)f->ev.size()) {
            const hipError_t e = hipEventRecord(f->ev[2 * f->n_prof + 1], f->stream);
            f->ev_kernel[f->n_prof] = f->last_code;
            f->ev_rows_launch[f->n_prof] = rows;
            f->n_prof++;
            return e;
        }
        return hipSuccess;
    };
    const bool risky = wave_products_risky(f, P.p);
    f->used_path = f->n_paths > 0 && !risky;
    if (f->used_path) {   // every level on the wave schedule: one launch, one block per path
        HIPCHK(prof_begin());
        hipLaunchKernelGGL(k_loglik_wave<false>, dim3((unsigned)f->n_paths), dim3(64), 0, f->stream, f->F, P,
                           f->d_path_cells, (int)f->n_cells, f->d_state, f->d_cell_ll, f->d_cell_nan, f->d_chain,
                           f->d_cell_done, f->epoch, f->d_path_seq, f->red, f->seq, f->spin_max,
                           (const double *)nullptr, (const double *)nullptr, (const int32_t *)nullptr);
        HIPCHK(hipGetLastError());
        f->kernel_used = GGP_KERNEL_WAVE;
        f->last_code = GGP_KERNEL_WAVE << 8 | 64;
        HIPCHK(prof_end(f->n_rows));
        return GGP_OK;
    }
    for (int L = 0; L < n_levels; ++L) {
        const int64_t a = f->level_start[L], b = f->level_start[L + 1];
        const int n = (int)(b - a);
        if (n <= 0) continue;
        HIPCHK(prof_begin());
        if (f->lane_queue && f->qrun_at[L] >= 0) {   // levels la .. lb - 1 in one persistent launch
            const Shard::QRun &R = f->qruns[(size_t)f->qrun_at[L]];
            HIPCHK(hipMemsetAsync(f->d_qctr, 0, sizeof(unsigned), f->stream));
            const int grid = (int)std::min<int64_t>(R.n, f->queue_resident);
            hipLaunchKernelGGL(k_loglik_lane_queue, dim3(grid), dim3(64), 0, f->stream, f->F, P, f->d_level_cells,
                               f->d_qchunks + R.off, (int)R.n, f->d_qctr, f->d_cell_done, f->epoch, f->spin_max,
                               f->d_state, f->d_cell_ll, f->d_cell_nan);
            HIPCHK(hipGetLastError());
            f->kernel_used = GGP_KERNEL_LANE;
            f->last_code = GGP_KERNEL_LANE << 8 | 2;
            HIPCHK(prof_end(R.rows));
            L = R.lb - 1;
            continue;
        }
        const int64_t n_simd = (int64_t)f->n_cu * 4;
        int kind = f->level_kind[L];
        if (kind == GGP_KERNEL_WAVE && risky) kind = n <= f->pair_max_cells ? GGP_KERNEL_PAIR : GGP_KERNEL_LANE;
        if (kind == GGP_KERNEL_WAVE) {
            hipLaunchKernelGGL(k_loglik_wave<false>, dim3(n), dim3(64), 0, f->stream, f->F, P, f->d_level_cells + a, n,
                               f->d_state, f->d_cell_ll, f->d_cell_nan, f->d_chain, f->d_cell_done, f->epoch,
                               (const int32_t *)nullptr, ChainRed{}, (int64_t)0, f->spin_max,
                               (const double *)nullptr, (const double *)nullptr, (const int32_t *)nullptr);
            f->kernel_used = GGP_KERNEL_WAVE;
            f->last_code = GGP_KERNEL_WAVE << 8 | 64;
        } else if (kind == GGP_KERNEL_PAIR) {
            // four waves per cell while one 64-cell workgroup per CU holds the level, else two
            const int q = f->tune_pair_q > 0 ? f->tune_pair_q : (n <= (int64_t)f->n_cu * 64 ? 4 : 2);
            const int cpw = f->tune_pair_cpw;
            const int blocks = (n + cpw - 1) / cpw;
            if (q == 4 && cpw == 64)
                hipLaunchKernelGGL((k_loglik_pair<4, 64>), dim3(blocks), dim3(256), 0, f->stream, f->F, P, f->d_level_cells + a,
                                   n, f->d_state, f->d_cell_ll, f->d_cell_nan);
            else if (q == 4)
                hipLaunchKernelGGL((k_loglik_pair<4, 32>), dim3(blocks), dim3(256), 0, f->stream, f->F, P, f->d_level_cells + a,
                                   n, f->d_state, f->d_cell_ll, f->d_cell_nan);
            else if (cpw == 32)
                hipLaunchKernelGGL((k_loglik_pair<2, 32>), dim3(blocks), dim3(128), 0, f->stream, f->F, P, f->d_level_cells + a,
                                   n, f->d_state, f->d_cell_ll, f->d_cell_nan);
            else
                hipLaunchKernelGGL((k_loglik_pair<2, 64>), dim3(blocks), dim3(128), 0, f->stream, f->F, P, f->d_level_cells + a,
                                   n, f->d_state, f->d_cell_ll, f->d_cell_nan);
            f->kernel_used = GGP_KERNEL_PAIR;
            f->last_code = GGP_KERNEL_PAIR << 8 | q;
        } else if (kind == GGP_KERNEL_GROUP) {
            // one cell per wave while that fits one wave per SIMD, else two (G = 32); the
            // auto threshold keeps bigger levels on the lane schedule (tools/lane_scan.py)
            int cpw = 1;
            while (cpw < 8 && (n + cpw - 1) / cpw > n_simd) cpw *= 2;
            if (f->tune_group_cpw > 0) cpw = f->tune_group_cpw;
            const int blocks = (n + cpw - 1) / cpw;
            switch (cpw) {
            case 1: hipLaunchKernelGGL(k_loglik_group<64>, dim3(blocks), dim3(64), 0, f->stream, f->F, P,
                                       f->d_level_cells + a, n, f->d_state, f->d_cell_ll, f->d_cell_nan); break;
            case 2: hipLaunchKernelGGL(k_loglik_group<32>, dim3(blocks), dim3(64), 0, f->stream, f->F, P,
                                       f->d_level_cells + a, n, f->d_state, f->d_cell_ll, f->d_cell_nan); break;
            case 4: hipLaunchKernelGGL(k_loglik_group<16>, dim3(blocks), dim3(64), 0, f->stream, f->F, P,
                                       f->d_level_cells + a, n, f->d_state, f->d_cell_ll, f->d_cell_nan); break;
            default: hipLaunchKernelGGL(k_loglik_group<8>, dim3(blocks), dim3(64), 0, f->stream, f->F, P,
                                        f->d_level_cells + a, n, f->d_state, f->d_cell_ll, f->d_cell_nan); break;
            }
            f->kernel_used = GGP_KERNEL_GROUP;
            f->last_code = GGP_KERNEL_GROUP << 8 | (64 / cpw);
        } else {
            const int cpw = lane_cpw(f);
            const int blocks = (n + cpw - 1) / cpw;
            hipLaunchKernelGGL(k_loglik_level, dim3(blocks), dim3(64), 0, f->stream, f->F, P,
                               f->d_level_cells + a, n, cpw, f->d_state, f->d_cell_ll, f->d_cell_nan);
            f->kernel_used = GGP_KERNEL_LANE;
            f->last_code = GGP_KERNEL_LANE << 8 | 1;
        }
        HIPCHK(hipGetLastError());
        HIPCHK(prof_end(f->ev_rows[L]));
    }
    return GGP_OK;
}

// a chained / tree launch's ChainRed: no in-launch reduction, only the per-path setup descriptors
ChainRed chain_red_setup(const Shard *s)
{
    ChainRed R{};
    R.pdesc = s->d_pdesc;
    return R;
}

// one evaluation on a shard: the levels, then the block sums straight into mapped host memory
int shard_launch(Shard *s, const ggp_params &P)
{
    if (s->n_cells == 0) return GGP_OK;
    HIPCHK(hipSetDevice(s->device));
    ++s->seq;
    const int rc = launch_levels(s, P);
    if (rc != GGP_OK) return rc;
    if (s->used_path) {   // the path launch reduced in-launch
        s->seq_pending = true;
        return GGP_OK;
    }
    hipLaunchKernelGGL(k_reduce_blocks, dim3((unsigned)s->n_lblocks, 1), dim3(s->red_threads), 0, s->stream,
                       s->n_cells, s->d_cell_ll, s->d_cell_nan, s->d_tree_dfs, s->d_blk_t0, s->d_blk_nt, s->d_gdfs,
                       (int)s->n_lblocks, s->d_blk_sum, s->d_blk_nan, s->d_done, s->m_seq, s->seq, s->m_sum, s->m_nan);
    s->seq_pending = true;
    HIPCHK(hipGetLastError());
    return GGP_OK;
}

int shard_wait(Shard *s)
{
    if (s->n_cells == 0) return GGP_OK;
    bool seen = false;
    if (s->spin && s->seq_pending) {
        for (uint32_t it = 1;; ++it) {
            if (*s->h_seq == s->seq) { seen = true; break; }
            if ((it & 1023) == 0 && hipStreamQuery(s->stream) != hipErrorNotReady) break;
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        if (seen && s->used_path && s->h_clk)   // the launch's counters, complete before its sequence number
            for (int k = 0; k < 4; ++k) s->clk_snap[k] = s->h_clk[k];
    }
    s->seq_pending = false;
    if (!seen || s->profile) {
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    return GGP_OK;
}

// whether every level of the smoother takes the lane kernels (no lane-pair level): the backward
// pass can then form the combined rows itself (k_bwd_level<true>)
bool smoother_all_lane(const Shard *f)
{
    if (f->smoother_lane) return true;
    for (size_t L = 0; L + 1 < f->level_start.size(); ++L) {
        const int64_t n = f->level_start[L + 1] - f->level_start[L];
        if (n > 0 && n <= f->pair_max_cells) return false;
    }
    return true;
}

// forward then backward pass of the smoother (predictions.h:93-444) into device buffers; pstate
// is left holding every cell's backward final state (MOMAdata::mean/cov after -p).  d_comb (only
// when smoother_all_lane): the backward pass also forms the combined rows there, and d_bwd may
// then be null (the backward rows not stored)
hipError_t run_smoother(Shard *f, const double *d_ptab, int n_seg, double *d_pstate, double *d_fwd, double *d_bwd,
                        double *d_comb = nullptr)
{
    const int n_levels = (int)f->level_start.size() - 1;
    // a level up to pair_max_cells takes the lane-pair split (four waves per cell while one
    // 64-cell workgroup per CU holds it, else two; bitwise the lane smoother), larger ones the
    // lane smoother (GGP_SMOOTHER_LANE=1: every level)
    auto launch = [&](const bool fwd, const int64_t a, const int n) {
        if (!f->smoother_lane && n <= f->pair_max_cells && n_seg <= kSegLds) {   // (the pair kernels stage <= kSegLds rows)
            const int q = n <= (int64_t)f->n_cu * 64 ? 4 : 2;
            const dim3 grid((n + 63) / 64);
            if (fwd && q == 4)
                hipLaunchKernelGGL((k_fwd_pair<4, 64>), grid, dim3(256), 0, f->stream, f->F, d_ptab, n_seg, f->d_level_cells + a, n,
                                   d_pstate, d_fwd);
            else if (fwd)
                hipLaunchKernelGGL((k_fwd_pair<2, 64>), grid, dim3(128), 0, f->stream, f->F, d_ptab, n_seg, f->d_level_cells + a, n,
                                   d_pstate, d_fwd);
            else if (q == 4)
                hipLaunchKernelGGL((k_bwd_pair<4, 64>), grid, dim3(256), 0, f->stream, f->F, d_ptab, n_seg, f->d_level_cells + a, n,
                                   d_pstate, d_bwd);
            else
                hipLaunchKernelGGL((k_bwd_pair<2, 64>), grid, dim3(128), 0, f->stream, f->F, d_ptab, n_seg, f->d_level_cells + a, n,
                                   d_pstate, d_bwd);
            return;
        }
        const int cpw = lane_cpw(f);
        const dim3 grid((n + cpw - 1) / cpw);
        const bool sl = n_seg <= kSegLds;   // the parameter rows in LDS
        if (fwd && sl)
            hipLaunchKernelGGL(k_fwd_level<true>, grid, dim3(64), 0, f->stream, f->F, d_ptab, n_seg, f->d_level_cells + a, n,
                               cpw, d_pstate, d_fwd);
        else if (fwd)
            hipLaunchKernelGGL(k_fwd_level<false>, grid, dim3(64), 0, f->stream, f->F, d_ptab, n_seg, f->d_level_cells + a, n,
                               cpw, d_pstate, d_fwd);
        else if (d_comb && sl)
            hipLaunchKernelGGL((k_bwd_level<true, true>), grid, dim3(64), 0, f->stream, f->F, d_ptab, n_seg,
                               f->d_level_cells + a, n, cpw, d_pstate, d_bwd, f->d_prior_seg, (const double *)d_fwd, d_comb);
        else if (d_comb)
            hipLaunchKernelGGL((k_bwd_level<true, false>), grid, dim3(64), 0, f->stream, f->F, d_ptab, n_seg,
                               f->d_level_cells + a, n, cpw, d_pstate, d_bwd, f->d_prior_seg, (const double *)d_fwd, d_comb);
        else if (sl)
            hipLaunchKernelGGL((k_bwd_level<false, true>), grid, dim3(64), 0, f->stream, f->F, d_ptab, n_seg,
                               f->d_level_cells + a, n, cpw, d_pstate, d_bwd, (const int32_t *)nullptr,
                               (const double *)nullptr, (double *)nullptr);
        else
            hipLaunchKernelGGL((k_bwd_level<false, false>), grid, dim3(64), 0, f->stream, f->F, d_ptab, n_seg,
                               f->d_level_cells + a, n, cpw, d_pstate, d_bwd, (const int32_t *)nullptr,
                               (const double *)nullptr, (double *)nullptr);
    };
    hipError_t e = hipMemsetAsync(d_pstate, 0, (size_t)f->n_cells * 20 * sizeof(double), f->stream);
    for (int L = 0; L < n_levels && e == hipSuccess; ++L) {        // forward: roots first
        const int64_t a = f->level_start[L];
        const int n = (int)(f->level_start[L + 1] - a);
        if (n <= 0) continue;
        launch(true, a, n);
        e = hipGetLastError();
    }
    for (int L = n_levels - 1; L >= 0 && e == hipSuccess; --L) {   // backward: leaves first
        const int64_t a = f->level_start[L];
        const int n = (int)(f->level_start[L + 1] - a);
        if (n <= 0) continue;
        launch(false, a, n);
        e = hipGetLastError();
    }
    return e;
}

void shard_free_joints(Shard *f)
{
    for (double **p : {&f->d_j_ptab, &f->d_j_pstate, &f->d_j_fwd, &f->d_j_bwd, &f->d_j_back, &f->d_j_cond,
                       &f->d_j_start}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    for (void **p : {&f->d_jw_stack, &f->d_jw_small, &f->d_jw_out, &f->d_jw_bnd}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    f->jw_stack_bytes = f->jw_small_bytes = f->jw_out_bytes = f->jw_bnd_bytes = 0;
    f->j_params.clear();
}

// a grow-only device buffer of at least `bytes` (the stream is idle when this is called)
void *jw_reserve(void **buf, size_t *have, size_t bytes)
{
    bytes = std::max<size_t>(bytes, 256);
    if (*buf && *have >= bytes) return *buf;
    const size_t want = std::max(bytes, *have + *have / 2);
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    if (hipMalloc(buf, want) != hipSuccess) {
        *buf = nullptr;
        return nullptr;
    }
    *have = want;
    return *buf;
}

void batch_free(Shard *f)
{
    for (void *p : {(void *)f->d_b_ptab, (void *)f->d_b_state, (void *)f->d_b_ll, (void *)f->d_b_sum,
                    (void *)f->d_b_nan, (void *)f->d_b_code, (void *)f->d_b_done, (void *)f->d_b_pred})
        if (p) (void)hipFree(p);
    f->d_b_ptab = f->d_b_state = f->d_b_ll = f->d_b_sum = nullptr;
    f->d_b_nan = nullptr;
    f->d_b_code = nullptr;
    f->d_b_done = nullptr;
    f->d_b_pred = nullptr;
    f->b_cap = 0;
}

void shard_destroy(Shard *f)
{
    if (!f) return;
    (void)hipSetDevice(f->device);
    if (f->stream) (void)hipStreamSynchronize(f->stream);
    for (void *p : {(void *)f->d_time, (void *)f->d_logl, (void *)f->d_fp, (void *)f->d_row_off,
                    (void *)f->d_parent, (void *)f->d_d1, (void *)f->d_d2, (void *)f->d_seg,
                    (void *)f->d_level_cells, (void *)f->d_dfs_rank, (void *)f->d_prior_seg, (void *)f->d_row_cell,
                    (void *)f->d_state, (void *)f->d_cell_ll, (void *)f->d_cell_nan, (void *)f->d_tree_dfs,
                    (void *)f->d_blk_t0, (void *)f->d_blk_nt, (void *)f->d_gdfs, (void *)f->d_done,
                    (void *)f->d_blk_sum, (void *)f->d_blk_nan, (void *)f->d_chain, (void *)f->d_cell_done,
                    (void *)f->d_path_cells, (void *)f->d_path_seq, (void *)f->d_path_blk,
                    (void *)f->d_blk_npaths, (void *)f->d_cnt_blk, (void *)f->d_pdesc,
                    (void *)f->d_qchunks, (void *)f->d_qctr,
                    (void *)f->d_sm_ptab, (void *)f->d_sm_pstate, (void *)f->d_sm_comb})
        if (p) (void)hipFree(p);
    batch_free(f);
    shard_free_joints(f);
    for (auto &e : f->ev_pred)
        if (e) (void)hipEventDestroy(e);
    if (f->h_res) (void)hipHostFree(f->h_res);
    for (auto &e : f->ev) (void)hipEventDestroy(e);
    delete f;
}

// validated topology of a descriptor: generation depth per cell, the DFS pre-order (roots in
// input order, daughter1 before daughter2: likelihood_recr) and where each tree starts in it
int check_topology(const ggp_forest_desc *d, std::vector<int32_t> &depth, std::vector<int32_t> &dfs,
                   std::vector<int64_t> &tree_start)
{
    const int64_t nc = d->n_cells, nr = d->n_rows;
    if (nc < 0 || nr < 0 || (nc > 0 && (!d->row_offset || !d->parent || !d->daughter1 || !d->daughter2)) ||
        (nr > 0 && (!d->time || !d->log_length || !d->fp))) {
        g_last_err = "incomplete forest descriptor";
        return GGP_EINVAL;
    }
    if (nc >= (int64_t)1 << 31 || nr >= (int64_t)1 << 40) { g_last_err = "forest too large"; return GGP_EINVAL; }
    // bad indices would fault on the device: validate on the host
    if (nc > 0 && (d->row_offset[0] != 0 || d->row_offset[nc] != nr)) {
        g_last_err = "row_offset must start at 0 and end at n_rows";
        return GGP_EINVAL;
    }
    for (int64_t c = 0; c < nc; ++c) {
        if (d->row_offset[c + 1] <= d->row_offset[c]) { g_last_err = "every cell needs >= 1 row"; return GGP_EINVAL; }
        if (d->row_offset[c + 1] - d->row_offset[c] >= (int64_t)1 << 24) { g_last_err = "a cell has >= 2^24 rows"; return GGP_EINVAL; }
        for (int32_t v : {d->parent[c], d->daughter1[c], d->daughter2[c]})
            if (v < -1 || v >= nc || v == c) { g_last_err = "genealogy index out of range"; return GGP_EINVAL; }
    }
    depth.assign(nc, -1);
    dfs.clear();
    dfs.reserve(nc);
    tree_start.clear();
    std::vector<int32_t> stack;
    for (int64_t r = 0; r < nc; ++r) {
        if (d->parent[r] != -1) continue;
        tree_start.push_back((int64_t)dfs.size());
        depth[r] = 0;
        stack.push_back((int32_t)r);
        while (!stack.empty()) {
            int32_t c = stack.back();
            stack.pop_back();
            dfs.push_back(c);
            for (int32_t ch : {d->daughter2[c], d->daughter1[c]}) {
                if (ch < 0) continue;
                if (depth[ch] != -1) { g_last_err = "genealogy is not a forest"; return GGP_EINVAL; }
                depth[ch] = depth[c] + 1;
                stack.push_back(ch);
            }
        }
    }
    tree_start.push_back((int64_t)dfs.size());
    for (int64_t c = 0; c < nc; ++c)
        if (depth[c] < 0) { g_last_err = "cell not reachable from a root (cycle)"; return GGP_EINVAL; }
    // a daughter's parent pointer must be the cell that lists it (single-parent forest)
    for (int64_t c = 0; c < nc; ++c)
        for (int32_t ch : {d->daughter1[c], d->daughter2[c]})
            if (ch >= 0 && d->parent[ch] != c) {
                g_last_err = "daughter/parent pointers disagree";
                return GGP_EINVAL;
            }
    return GGP_OK;
}

// A shard from a (sub-)forest descriptor `d` in its own numbering.  gdfs_of_cell: the global
// DFS rank of every local cell; blk_ntrees: the shard's reduction blocks in order (trees each,
// consecutive local trees), blk_global: their global indices; B: trees per block.
int shard_create(const ggp_forest_desc *d, DeviceCtx *dev, const std::vector<int32_t> &gdfs_of_cell,
                 const std::vector<int32_t> &blk_ntrees, const std::vector<int64_t> &blk_global, int64_t B,
                 Shard **out)
{
    *out = nullptr;
    const int64_t nc = d->n_cells, nr = d->n_rows;
    std::vector<int32_t> depth, dfs;
    std::vector<int64_t> tree_start;
    int rc = check_topology(d, depth, dfs, tree_start);
    if (rc != GGP_OK) return rc;
    auto *f = new Shard();
    f->dev = dev;
    f->device = dev->id;
    f->stream = dev->stream;
    f->n_cells = nc;
    f->n_rows = nr;
    f->kernel_pref = d->kernel;
    f->n_cu = dev->n_cu;
    f->wave_max_cells = (int64_t)f->n_cu * 4 * 5;   // r08 scan: wave ahead of group up to ~5 cells/SIMD
    f->group_max_cells = (int64_t)f->n_cu * 4 * 8;   // 8 cells per wave, one wave per SIMD
    f->pair_max_cells = (int64_t)f->n_cu * 64 * 2;   // r13 scan: two rounds of 64-cell pair workgroups
    if (const char *e = getenv("GGP_WAVE_MAX_CELLS")) f->wave_max_cells = atoll(e);
    if (const char *e = getenv("GGP_CHAIN_SPIN_MAX")) f->spin_max = (unsigned)strtoul(e, nullptr, 10);
    if (const char *e = getenv("GGP_SPIN")) f->spin = atoi(e) != 0;
    if (const char *e = getenv("GGP_LANE_CPW")) f->tune_lane_cpw = std::max(0, std::min(64, atoi(e)));
    if (const char *e = getenv("GGP_GROUP_CPW")) {
        const int v = atoi(e);
        f->tune_group_cpw = (v == 1 || v == 2 || v == 4 || v == 8) ? v : 0;
    }
    if (const char *e = getenv("GGP_GROUP_MAX_CELLS")) f->group_max_cells = atoll(e);
    if (const char *e = getenv("GGP_PAIR_CPW")) f->tune_pair_cpw = atoi(e) == 32 ? 32 : 64;
    if (const char *e = getenv("GGP_PAIR_MAX_CELLS")) f->pair_max_cells = atoll(e);
    if (const char *e = getenv("GGP_COMBINE_EXACT")) f->combine_exact = atoi(e) != 0;
    if (const char *e = getenv("GGP_COMBINE_FUSED")) f->combine_fused = atoi(e) != 0;
    if (const char *e = getenv("GGP_JOINT_SLOT_MB")) f->joint_slot_bytes = (size_t)std::max(0, atoi(e)) << 20;
    if (const char *e = getenv("GGP_PAIR_Q")) f->tune_pair_q = atoi(e) == 4 ? 4 : atoi(e) == 2 ? 2 : 0;
    if (const char *e = getenv("GGP_SMOOTHER_LANE")) f->smoother_lane = atoi(e) != 0;
    if (const char *e = getenv("GGP_LANE_QUEUE")) f->lane_queue = atoi(e) != 0;
    if (const char *e = getenv("GGP_AUTO_SMALL"); e && !ggp::kExact)
        f->auto_small = std::string(e) == "group" ? GGP_KERNEL_GROUP : GGP_KERNEL_WAVE;
    f->row_off.assign(d->row_offset, d->row_offset + nc + 1);
    if (nc == 0) f->row_off.assign(1, 0);
    for (int64_t c = 0; c < nc; ++c) {
        const int64_t a = d->row_offset[c], b = d->row_offset[c + 1];
        for (int64_t r = a + 1; r < b; ++r) f->max_dt = std::max(f->max_dt, std::fabs(d->time[r] - d->time[r - 1]));
        if (d->parent[c] >= 0 && b > a)
            f->max_dt = std::max(f->max_dt, std::fabs(d->time[a] - d->time[d->row_offset[d->parent[c] + 1] - 1]));
    }
    if (hipSetDevice(f->device) != hipSuccess) {
        g_last_err = "hipSetDevice failed";
        delete f;
        return GGP_EDEV;
    }
    auto check = [&](int r) { if (r != GGP_OK && rc == GGP_OK) rc = r; };
    // ---- level schedule: cells by generation depth, each level longest first ----
    int32_t max_depth = 0;
    for (int64_t c = 0; c < nc; ++c) max_depth = std::max(max_depth, depth[c]);
    std::vector<int32_t> level_cells(nc);
    std::iota(level_cells.begin(), level_cells.end(), 0);
    std::stable_sort(level_cells.begin(), level_cells.end(), [&](int32_t a, int32_t b) {
        if (depth[a] != depth[b]) return depth[a] < depth[b];
        return (d->row_offset[a + 1] - d->row_offset[a]) > (d->row_offset[b + 1] - d->row_offset[b]);
    });
    f->level_start.assign(nc > 0 ? max_depth + 2 : 1, 0);
    for (int64_t c = 0; c < nc; ++c) f->level_start[depth[c] + 1]++;
    for (size_t L = 1; L < f->level_start.size(); ++L) f->level_start[L] += f->level_start[L - 1];
    // rows below each cell, deepest cells first (a daughter is one generation below its parent)
    f->j_below.assign(nc, 0);
    for (int64_t k = nc - 1; k >= 0; --k) {
        const int32_t c = level_cells[k], par = d->parent[c];
        if (par >= 0) f->j_below[par] += (d->row_offset[c + 1] - d->row_offset[c]) + f->j_below[c];
    }
    // ---- uploads ----
    check(dev_upload(&f->d_time, d->time, nr));
    check(dev_upload(&f->d_logl, d->log_length, nr));
    check(dev_upload(&f->d_fp, d->fp, nr));
    check(dev_upload(&f->d_row_off, d->row_offset, nc + 1));
    check(dev_upload(&f->d_parent, d->parent, nc));
    check(dev_upload(&f->d_d1, d->daughter1, nc));
    check(dev_upload(&f->d_d2, d->daughter2, nc));
    if (d->segment) check(dev_upload(&f->d_seg, d->segment, nr));
    check(dev_upload(&f->d_level_cells, level_cells.data(), nc));
    {
        std::vector<int32_t> rank(nc), gd(nc);
        for (int64_t k = 0; k < nc; ++k) {
            rank[dfs[k]] = (int32_t)k;
            gd[k] = gdfs_of_cell[dfs[k]];
        }
        check(dev_upload(&f->d_dfs_rank, rank.data(), nc));
        check(dev_upload(&f->d_gdfs, gd.data(), nc));
    }
    {
        // combine_predictions' prior (predictions.h:475-490): a cell's first row divides by the
        // parameters that initialised it (its own for a root, the parent's last row otherwise)
        std::vector<int32_t> prior(nr, 0);
        if (d->segment) {
            for (int64_t c = 0; c < nc; ++c) {
                const int64_t r0 = d->row_offset[c];
                for (int64_t r = r0; r < d->row_offset[c + 1]; ++r) prior[r] = d->segment[r];
                if (d->parent[c] >= 0) prior[r0] = d->segment[d->row_offset[d->parent[c] + 1] - 1];
            }
        }
        check(dev_upload(&f->d_prior_seg, prior.data(), nr));
        std::vector<int32_t> row_cell(nr);
        for (int64_t c = 0; c < nc; ++c)
            for (int64_t r = d->row_offset[c]; r < d->row_offset[c + 1]; ++r) row_cell[r] = (int32_t)c;
        check(dev_upload(&f->d_row_cell, row_cell.data(), nr));
    }
    check(dev_upload<double>(&f->d_state, nullptr, (size_t)nc * 20));
    check(dev_upload<double>(&f->d_cell_ll, nullptr, nc));
    check(dev_upload<int32_t>(&f->d_cell_nan, nullptr, nc));
    if (rc == GGP_OK && nc > 0 && hipMemset(f->d_state, 0, (size_t)nc * 20 * sizeof(double)) != hipSuccess) rc = GGP_EDEV;
    // ---- reduction blocks ----
    f->n_trees = (int64_t)tree_start.size() - 1;
    f->n_lblocks = (int64_t)blk_ntrees.size();
    f->blk_global = blk_global;
    f->red_threads = (int)std::max<int64_t>(64, B);
    {
        std::vector<int32_t> t0(f->n_lblocks);
        int64_t t = 0;
        for (int64_t j = 0; j < f->n_lblocks; ++j) {
            t0[j] = (int32_t)t;
            t += blk_ntrees[j];
        }
        if (t != f->n_trees && rc == GGP_OK) {
            g_last_err = "shard blocks do not cover its trees";
            rc = GGP_EINVAL;
        }
        check(dev_upload(&f->d_tree_dfs, tree_start.data(), tree_start.size()));
        check(dev_upload(&f->d_blk_t0, t0.data(), t0.size()));
        check(dev_upload(&f->d_blk_nt, blk_ntrees.data(), blk_ntrees.size()));
        check(dev_upload<unsigned>(&f->d_done, nullptr, 1));
        check(dev_upload<double>(&f->d_blk_sum, nullptr, (size_t)std::max<int64_t>(1, f->n_lblocks)));
        check(dev_upload<int64_t>(&f->d_blk_nan, nullptr, (size_t)std::max<int64_t>(1, f->n_lblocks)));
        if (rc == GGP_OK && f->d_done && hipMemset(f->d_done, 0, sizeof(unsigned)) != hipSuccess) rc = GGP_EDEV;
    }
    if (rc == GGP_OK) {   // the result slots: pinned host memory the reduction writes over the bus
        const size_t slots = 2 * (size_t)f->n_lblocks + 1 + 4;   // + the launch clock's four counters
        void *h = nullptr, *m = nullptr;
        if (hipHostMalloc(&h, slots * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            rc = GGP_ENOMEM;
        } else {
            f->h_res = h;
            f->h_sum = (double *)h;
            f->h_nan = (int64_t *)((char *)h + f->n_lblocks * sizeof(double));
            f->h_seq = (volatile int64_t *)((char *)h + 2 * f->n_lblocks * sizeof(double));
            *f->h_seq = 0;
            if (hipHostGetDevicePointer(&m, h, 0) != hipSuccess) rc = GGP_EDEV;
            f->m_sum = (double *)m;
            f->m_nan = (int64_t *)((char *)m + f->n_lblocks * sizeof(double));
            f->m_seq = (int64_t *)((char *)m + 2 * f->n_lblocks * sizeof(double));
            f->h_clk = (volatile unsigned long long *)((char *)h + (2 * f->n_lblocks + 1) * sizeof(double));
            f->m_clk = (unsigned long long *)((char *)m + (2 * f->n_lblocks + 1) * sizeof(double));
            f->h_clk[0] = f->h_clk[1] = f->h_clk[2] = f->h_clk[3] = 0;
        }
    }
    if (rc != GGP_OK) {
        shard_destroy(f);
        return rc;
    }
    DevForest &F = f->F;
    F.time = f->d_time; F.logl = f->d_logl; F.fp = f->d_fp;
    F.row_off = f->d_row_off; F.parent = f->d_parent; F.d1 = f->d_d1; F.d2 = f->d_d2; F.seg = f->d_seg;
    F.dfs_rank = f->d_dfs_rank;
    F.root_mean0 = d->root_mean_xg[0]; F.root_mean1 = d->root_mean_xg[1];
    F.root_var0 = d->root_var_xg[0]; F.root_var1 = d->root_var_xg[1];
    F.leaf_mean0 = d->leaf_mean_xg[0]; F.leaf_mean1 = d->leaf_mean_xg[1];
    F.leaf_var0 = d->leaf_var_xg[0]; F.leaf_var1 = d->leaf_var_xg[1];
    F.fp_auto = d->fp_auto;
    F.two_log_2pi = 2 * std::log(2 * M_PI);
    F.log2 = std::log(2.);
    F.scaled = d->noise_scaled ? 1 : 0;
    F.binomial = d->division_binomial ? 1 : 0;
    // schedule per level; when every level takes the wave schedule and the forest has at most as
    // many leaves as the device holds wave blocks, one path launch (k_loglik_wave): paths
    // (a root or second daughter, then first daughters to a leaf) ordered by the depth of
    // their first cell, and the chain table of the second daughters' waits
    {
        const int n_levels = (int)f->level_start.size() - 1;
        f->level_kind.assign(std::max(0, n_levels), GGP_KERNEL_LANE);
        bool all_wave = n_levels > 0;
        for (int L = 0; L < n_levels; ++L) {
            f->level_kind[L] = level_kind(f, f->level_start[L + 1] - f->level_start[L]);
            all_wave = all_wave && f->level_kind[L] == GGP_KERNEL_WAVE;
        }
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_loglik_wave<false>, 64, 0) == hipSuccess && per_cu > 0)
            f->wave_resident = per_cu * f->n_cu;
        if (const char *e = getenv("GGP_WAVE_PATHS_MAX")) f->wave_resident = atoi(e);
        std::vector<CellLink> ch(nc, CellLink{-1, 0, 0.0});
        for (int64_t c = 0; c < nc; ++c)   // the division dt of every daughter (the step's own subtraction)
            if (d->parent[c] >= 0) ch[c].dt = d->time[d->row_offset[c]] - d->time[d->row_offset[d->parent[c] + 1] - 1];
        std::vector<int32_t> heads, pcells, pseq;
        auto next_of = [&](int32_t c) { return d->daughter1[c] >= 0 ? d->daughter1[c] : d->daughter2[c]; };
        if (all_wave) {
            for (int64_t c = 0; c < nc; ++c) {
                const int32_t pa = d->parent[c];
                if (pa < 0 || next_of(pa) != c) heads.push_back((int32_t)c);
            }
            std::stable_sort(heads.begin(), heads.end(), [&](int32_t a2, int32_t b2) { return depth[a2] < depth[b2]; });
        }
        // the in-launch reduction emulates k_reduce_blocks' 64-wide tree on <= 8 trees per block
        bool small_blocks = f->red_threads == 64;
        for (int32_t v : blk_ntrees) small_blocks = small_blocks && v <= 8;
        if (all_wave && small_blocks && (int64_t)heads.size() <= f->wave_resident) {
            pseq.push_back(0);
            for (int32_t h : heads) {
                for (int32_t c = h; c >= 0 && (int64_t)pcells.size() <= nc; c = next_of(c)) pcells.push_back(c);
                pseq.push_back((int32_t)pcells.size());
                const int32_t pa = d->parent[h];
                if (pa >= 0) {
                    ch[h].x = pa;
                    ch[pa].y = 1;
                }
            }
            if ((int64_t)pcells.size() != nc && rc == GGP_OK) {
                g_last_err = "path decomposition does not cover the forest";
                rc = GGP_EINVAL;
            }
            f->n_paths = (int64_t)heads.size();
            check(dev_upload(&f->d_path_cells, pcells.data(), pcells.size()));
            check(dev_upload(&f->d_path_seq, pseq.data(), pseq.size()));
            // reduction tables: the block of each path (by its first cell's DFS position and
            // that tree's block), paths per block
            std::vector<int32_t> rank(nc);
            for (int64_t k = 0; k < nc; ++k) rank[dfs[k]] = (int32_t)k;
            const int64_t ntr = (int64_t)tree_start.size() - 1;
            std::vector<int32_t> tblk(std::max<int64_t>(1, ntr), 0);
            for (int64_t j = 0, t = 0; j < (int64_t)blk_ntrees.size(); ++j)
                for (int32_t u = 0; u < blk_ntrees[j]; ++u, ++t) tblk[t] = (int32_t)j;
            std::vector<int32_t> pblk(heads.size()), bnp(std::max<size_t>(1, blk_ntrees.size()), 0);
            for (size_t q = 0; q < heads.size(); ++q) {
                const int64_t k = rank[heads[q]];
                const int32_t t = (int32_t)(std::upper_bound(tree_start.begin(), tree_start.end(), k) - tree_start.begin() - 1);
                pblk[q] = tblk[t];
                bnp[tblk[t]]++;
            }
            check(dev_upload(&f->d_path_blk, pblk.data(), pblk.size()));
            check(dev_upload(&f->d_blk_npaths, bnp.data(), bnp.size()));
            {
                std::vector<int32_t> bt0(blk_ntrees.size() + 1, 0);   // each block's first tree (blk_t0)
                for (size_t jj = 0; jj < blk_ntrees.size(); ++jj) bt0[jj + 1] = bt0[jj] + blk_ntrees[jj];
                std::vector<PathDesc> pdv(heads.size());
                for (size_t q = 0; q < heads.size(); ++q) {
                    PathDesc &P = pdv[q];
                    P.i_lo = pseq[q];
                    P.i_hi = pseq[q + 1];
                    P.c0 = pcells[(size_t)pseq[q]];
                    P.j = pblk[q];
                    P.npaths = bnp[(size_t)pblk[q]];
                    P.nb = blk_ntrees[(size_t)pblk[q]];
                    P.t0 = bt0[(size_t)pblk[q]];
                    P.pad = 0;
                    P.r0 = d->row_offset[P.c0];
                    P.r1 = d->row_offset[P.c0 + 1];
                    P.l0 = ch[(size_t)P.c0];
                }
                check(dev_upload(&f->d_pdesc, pdv.data(), pdv.size()));
            }
            check(dev_upload<unsigned>(&f->d_cnt_blk, nullptr, bnp.size()));
            if (rc == GGP_OK && hipMemset(f->d_cnt_blk, 0, bnp.size() * sizeof(unsigned)) != hipSuccess) rc = GGP_EDEV;
            if (rc == GGP_OK) {
                ChainRed R{};
                R.pdesc = f->d_pdesc;
                R.path_blk = f->d_path_blk;
                R.blk_npaths = f->d_blk_npaths;
                R.tree_dfs = f->d_tree_dfs;
                R.blk_t0 = f->d_blk_t0;
                R.blk_nt = f->d_blk_nt;
                R.gdfs = f->d_gdfs;
                R.cnt_blk = f->d_cnt_blk;
                R.done = f->d_done;
                R.out_seq = f->m_seq;
                R.host_sum = f->m_sum;
                R.host_nan = (long long *)f->m_nan;
                R.n_lblocks = (int)f->n_lblocks;
                R.clk = f->m_clk;
                f->red = R;
            }
        }
        check(dev_upload(&f->d_chain, ch.data(), nc));
        check(dev_upload<unsigned>(&f->d_cell_done, nullptr, nc));
        if (rc == GGP_OK && nc > 0 && hipMemset(f->d_cell_done, 0, (size_t)nc * sizeof(unsigned)) != hipSuccess) rc = GGP_EDEV;
        // lane queue runs: >= 2 consecutive levels the lane schedule takes, their cells in chunks of
        // lane_cpw in level order; a chunk waits when its level is not the run's first and
        // publishes when its level is not the run's last
        f->qrun_at.assign(std::max(0, n_levels), -1);
        if (f->lane_queue && f->n_paths == 0) {
            std::vector<QChunk> qc;
            const int cpw = lane_cpw(f);
            for (int L = 0; L < n_levels;) {
                int lb = L;
                while (lb < n_levels && f->level_kind[lb] == GGP_KERNEL_LANE) ++lb;
                if (lb - L >= 2) {
                    Shard::QRun R{L, lb, (int64_t)qc.size(), 0, 0};
                    for (int l = L; l < lb; ++l) {
                        const int64_t a = f->level_start[l], b = f->level_start[l + 1];
                        for (int64_t x = a; x < b; x += cpw)
                            qc.push_back(QChunk{(int32_t)x, (int32_t)std::min<int64_t>(cpw, b - x), l > L ? 1 : 0,
                                                l + 1 < lb ? 1 : 0});
                    }
                    R.n = (int64_t)qc.size() - R.off;
                    f->qrun_at[L] = (int32_t)f->qruns.size();
                    f->qruns.push_back(R);
                }
                L = std::max(lb, L + 1);
            }
            if (!qc.empty()) {
                check(dev_upload(&f->d_qchunks, qc.data(), qc.size()));
                check(dev_upload<unsigned>(&f->d_qctr, nullptr, 1));
                int per_cu = 0;
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_loglik_lane_queue, 64, 0) == hipSuccess && per_cu > 0)
                    f->queue_resident = per_cu * f->n_cu;
            }
        }
        if (rc != GGP_OK) {
            shard_destroy(f);
            return rc;
        }
    }
    // per-level rows for the roofline bookkeeping
    f->ev_rows.assign(f->level_start.size() - 1, 0);
    for (size_t L = 0; L + 1 < f->level_start.size(); ++L)
        for (int64_t i = f->level_start[L]; i < f->level_start[L + 1]; ++i) {
            int32_t c = level_cells[i];
            f->ev_rows[L] += d->row_offset[c + 1] - d->row_offset[c];
        }
    for (auto &R : f->qruns)
        for (int L = R.la; L < R.lb; ++L) R.rows += f->ev_rows[L];
    *out = f;
    return GGP_OK;
}

// ---- numbering helpers -------------------------------------------------------------------
int64_t g_cell(const Shard *s, int64_t lc) { return s->cell_g.empty() ? lc : s->cell_g[lc]; }

// the shard's local rows whose global rows fall in [r_lo, r_hi) (a contiguous local range:
// the shard keeps its cells in input order)
void local_rows(const ggp_forest *f, const Shard *s, int64_t r_lo, int64_t r_hi, int64_t &l_lo, int64_t &l_hi)
{
    l_lo = l_hi = 0;
    if (r_hi <= r_lo || s->n_cells == 0) return;
    if (s->cell_g.empty()) {
        l_lo = r_lo;
        l_hi = r_hi;
        return;
    }
    const auto &G = f->row_off;
    const int64_t gc_lo = (int64_t)(std::upper_bound(G.begin(), G.end(), r_lo) - G.begin()) - 1;
    const int64_t gc_hi = (int64_t)(std::upper_bound(G.begin(), G.end(), r_hi - 1) - G.begin()) - 1;
    const int64_t lc0 = std::lower_bound(s->cell_g.begin(), s->cell_g.end(), (int32_t)gc_lo) - s->cell_g.begin();
    const int64_t lc1 = std::upper_bound(s->cell_g.begin(), s->cell_g.end(), (int32_t)gc_hi) - s->cell_g.begin();
    if (lc0 >= lc1) return;
    const int64_t gc0 = s->cell_g[lc0], gcl = s->cell_g[lc1 - 1];
    l_lo = s->row_off[lc0] + std::max<int64_t>(0, r_lo - G[gc0]);
    l_hi = s->row_off[lc1 - 1] + std::min(G[gcl + 1], r_hi) - G[gcl];
}

int64_t g_row(const ggp_forest *f, const Shard *s, int64_t lr)
{
    if (s->cell_g.empty()) return lr;
    const int64_t lc = (int64_t)(std::upper_bound(s->row_off.begin(), s->row_off.end(), lr) - s->row_off.begin()) - 1;
    return f->row_off[s->cell_g[lc]] + (lr - s->row_off[lc]);
}

// local rows [l_lo, l_hi) of a [rows x w] host array -> their global rows of out (row base r_base)
void scatter_rows(const ggp_forest *f, const Shard *s, const double *src, int64_t l_lo, int64_t l_hi, int w,
                  double *out, int64_t r_base)
{
    if (l_hi <= l_lo) return;
    int64_t lc = (int64_t)(std::upper_bound(s->row_off.begin(), s->row_off.end(), l_lo) - s->row_off.begin()) - 1;
    for (int64_t lr = l_lo; lr < l_hi;) {
        const int64_t end = std::min(l_hi, s->row_off[lc + 1]);
        const int64_t gr = f->row_off[g_cell(s, lc)] + (lr - s->row_off[lc]);
        std::memcpy(out + (gr - r_base) * w, src + (lr - l_lo) * w, (size_t)(end - lr) * w * sizeof(double));
        lr = end;
        ++lc;
    }
}

// -j on one shard (local start rows [r_lo, r_hi)): collect_joint_distributions (correlation_tree.h
// :464-651).  The smoother and the per-row tables are kept for the parameters they were made with.
int shard_joints(Shard *f, const double *params, int32_t n_seg, double tol, int64_t r_lo, int64_t r_hi, int64_t cap,
                 int64_t *out_idx, double *out_val, int64_t *n_out, int width)
{
    const int64_t nc = f->n_cells, nr = f->n_rows;
    *n_out = 0;
    if (nc == 0 || r_hi <= r_lo) return GGP_OK;
    HIPCHK(hipSetDevice(f->device));
    HIPCHK(hipStreamSynchronize(f->stream));
    const std::vector<double> key(params, params + (size_t)n_seg * 11);
    if (!f->d_j_back) {
        int rc = GGP_OK;
        auto check = [&](int r) { if (r != GGP_OK && rc == GGP_OK) rc = r; };
        check(dev_upload<double>(&f->d_j_pstate, nullptr, (size_t)nc * 20));
        check(dev_upload<double>(&f->d_j_fwd, nullptr, (size_t)nr * 20));
        check(dev_upload<double>(&f->d_j_bwd, nullptr, (size_t)nr * 20));
        check(dev_upload<double>(&f->d_j_back, nullptr, (size_t)nr * kJBack));
        check(dev_upload<double>(&f->d_j_cond, nullptr, (size_t)nr * kJCond));
        check(dev_upload<double>(&f->d_j_start, nullptr, (size_t)nr * kJStart));
        if (rc != GGP_OK) {
            shard_free_joints(f);
            g_last_err = "ggp_joints: device allocation failed";
            return rc;
        }
    }
    hipError_t e = hipSuccess;
    if (key != f->j_params) {   // smoother + per-row tables for these parameters
        f->j_params.clear();
        if (f->d_j_ptab) (void)hipFree(f->d_j_ptab);
        f->d_j_ptab = nullptr;
        const int rc = dev_upload(&f->d_j_ptab, params, (size_t)n_seg * 11);
        if (rc != GGP_OK) return rc;
        e = run_smoother(f, f->d_j_ptab, n_seg, f->d_j_pstate, f->d_j_fwd, f->d_j_bwd);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_joint_rows, dim3((unsigned)((nr + 63) / 64)), dim3(64), 0, f->stream, f->F,
                               f->d_j_ptab, n_seg, f->d_row_cell, nr, f->d_j_fwd, f->d_j_bwd, f->d_j_back,
                               f->d_j_cond, f->d_j_start);
            e = hipGetLastError();
        }
        if (e == hipSuccess) f->j_params = key;
    }
    auto cleanup = [&]() { (void)hipStreamSynchronize(f->stream); };
    if (e == hipSuccess) e = hipStreamSynchronize(f->stream);   // the grow-only buffers are idle
    const int64_t ns = r_hi - r_lo;
    const int depth = (int)f->level_start.size();   // generations below any start, plus one
    const size_t b_stack_j = (size_t)ns * depth * kJStart * sizeof(double);
    const size_t b_stack_c = ((size_t)ns * depth * sizeof(int32_t) + 255) & ~(size_t)255;
    auto *stack = (char *)jw_reserve(&f->d_jw_stack, &f->jw_stack_bytes, b_stack_j + b_stack_c);
    // counts [ns], slot offsets [ns + 1], packed offsets [ns + 1]
    auto *small = (int64_t *)jw_reserve(&f->d_jw_small, &f->jw_small_bytes, (size_t)(3 * ns + 2) * sizeof(int64_t));
    if (!stack || !small) { cleanup(); g_last_err = "ggp_joints: device allocation failed"; return GGP_ENOMEM; }
    auto *d_stack_c = (int32_t *)stack;
    auto *d_stack_j = (double *)(stack + b_stack_c);
    int64_t *d_counts = small, *d_off = small + ns, *d_coff = small + 2 * ns + 1;
    const unsigned wblocks = (unsigned)((ns + 63) / 64);
    constexpr size_t kJointBytes = 2 * sizeof(int64_t) + kJStart * sizeof(double);
    auto walk = [&](const int64_t *offs, int64_t *o_idx, double *o_val) {
        hipLaunchKernelGGL(k_joint_walk, dim3(wblocks), dim3(64), 0, f->stream, f->F, f->d_j_ptab, n_seg,
                           f->d_row_cell, f->d_j_pstate, f->d_j_back, f->d_j_cond, f->d_j_start, tol, r_lo, ns, depth,
                           d_stack_j, d_stack_c, d_counts, offs, o_idx, o_val);
        return hipGetLastError();
    };
    // the output buffer for `total` joints: (start, target) pairs, then width values each
    auto out_buf = [&](int64_t total, int64_t *&d_idx, double *&d_val) {
        const size_t b_idx = (size_t)total * 2 * sizeof(int64_t);
        auto *out = (char *)jw_reserve(&f->d_jw_out, &f->jw_out_bytes,
                                       b_idx + (size_t)total * width * sizeof(double));
        d_idx = (int64_t *)out;
        d_val = out ? (double *)(out + b_idx) : nullptr;
        return out != nullptr;
    };
    // start i's joints from slots [from[i], ...) of 72-value records to [to[i], ...) in width-value records
    auto pack = [&](const int64_t *from, const int64_t *to, const int64_t *s_idx, const double *s_val, int64_t *o_idx,
                    double *o_val) {
        if (width == kJStart)
            hipLaunchKernelGGL(k_joint_pack<kJStart>, dim3((unsigned)ns), dim3(256), 0, f->stream, ns, from, to,
                               (const int64_t *)d_counts, s_idx, s_val, o_idx, o_val);
        else
            hipLaunchKernelGGL(k_joint_pack<kJPacked>, dim3((unsigned)ns), dim3(256), 0, f->stream, ns, from, to,
                               (const int64_t *)d_counts, s_idx, s_val, o_idx, o_val);
        return hipGetLastError();
    };
    std::vector<int64_t> counts(ns), off(ns + 1);
    // single pass: every start walks once into slots sized by its bound (the rows after it in its
    // cell plus every row below the cell), then the joints are packed on the device; when the
    // caller takes joints and the slots fit joint_slot_bytes, 2 GiB (else, or if a walk outgrew
    // its slots, the two passes: count, then emit at the exact offsets)
    bool single = e == hipSuccess && cap > 0 && out_idx && out_val;
    std::vector<int64_t> boff;
    if (single) {
        boff.resize(ns + 1);
        int64_t c = (int64_t)(std::upper_bound(f->row_off.begin(), f->row_off.end(), r_lo) - f->row_off.begin()) - 1;
        int64_t acc = 0;
        for (int64_t k = 0; k < ns; ++k) {
            const int64_t r = r_lo + k;
            while (f->row_off[c + 1] <= r) ++c;
            boff[k] = acc;
            acc += (f->row_off[c + 1] - 1 - r) + f->j_below[c];
        }
        boff[ns] = acc;
        single = (size_t)acc * kJointBytes <= f->joint_slot_bytes;
    }
    char *bnd = nullptr;
    if (single) {
        bnd = (char *)jw_reserve(&f->d_jw_bnd, &f->jw_bnd_bytes, (size_t)boff[ns] * kJointBytes);
        single = bnd != nullptr;
    }
    if (single) {
        auto *b_idx = (int64_t *)bnd;
        auto *b_val = (double *)(bnd + (size_t)boff[ns] * 2 * sizeof(int64_t));
        e = hipMemcpyAsync(d_off, boff.data(), (ns + 1) * sizeof(int64_t), hipMemcpyHostToDevice, f->stream);
        if (e == hipSuccess) e = walk(d_off, b_idx, b_val);
        if (e == hipSuccess) e = hipMemcpyAsync(counts.data(), d_counts, ns * sizeof(int64_t), hipMemcpyDeviceToHost, f->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(f->stream);
        int64_t total = 0;
        for (int64_t k = 0; k < ns && e == hipSuccess; ++k) {
            if (counts[k] > boff[k + 1] - boff[k]) {   // not expected: the two passes redo the range
                single = false;
                break;
            }
            off[k] = total;
            total += counts[k];
        }
        off[ns] = total;
        if (e == hipSuccess && single) {
            *n_out = total;
            if (total > 0 && total <= cap) {
                int64_t *d_idx = nullptr;
                double *d_val = nullptr;
                if (!out_buf(total, d_idx, d_val)) {
                    cleanup();
                    g_last_err = "ggp_joints: device allocation failed";
                    return GGP_ENOMEM;
                }
                e = hipMemcpyAsync(d_coff, off.data(), (ns + 1) * sizeof(int64_t), hipMemcpyHostToDevice, f->stream);
                if (e == hipSuccess) e = pack(d_off, d_coff, b_idx, b_val, d_idx, d_val);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(out_idx, d_idx, (size_t)total * 2 * sizeof(int64_t), hipMemcpyDeviceToHost, f->stream);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(out_val, d_val, (size_t)total * width * sizeof(double), hipMemcpyDeviceToHost, f->stream);
                if (e == hipSuccess) e = hipStreamSynchronize(f->stream);
            }
        }
    }
    if (e == hipSuccess && !single) {
        e = walk(nullptr, nullptr, nullptr);   // pass 1: count
        if (e == hipSuccess) e = hipMemcpyAsync(counts.data(), d_counts, ns * sizeof(int64_t), hipMemcpyDeviceToHost, f->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(f->stream);
        int64_t total = 0;
        for (int64_t k = 0; k < ns; ++k) {
            off[k] = total;
            total += counts[k];
        }
        off[ns] = total;
        *n_out = total;
        if (e == hipSuccess && total > 0 && total <= cap && out_idx && out_val) {   // pass 2: emit
            int64_t *d_idx = nullptr;
            double *d_val = nullptr;
            if (!out_buf(total, d_idx, d_val)) {
                cleanup();
                g_last_err = "ggp_joints: device allocation failed";
                return GGP_ENOMEM;
            }
            e = hipMemcpyAsync(d_off, off.data(), (ns + 1) * sizeof(int64_t), hipMemcpyHostToDevice, f->stream);
            if (e == hipSuccess && width == kJStart) {
                e = walk(d_off, d_idx, d_val);
            } else if (e == hipSuccess) {   // packed: emit 72-value records, then pack them
                auto *raw = (char *)jw_reserve(&f->d_jw_bnd, &f->jw_bnd_bytes, (size_t)total * kJointBytes);
                if (!raw) {
                    cleanup();
                    g_last_err = "ggp_joints: device allocation failed";
                    return GGP_ENOMEM;
                }
                auto *r_idx = (int64_t *)raw;
                auto *r_val = (double *)(raw + (size_t)total * 2 * sizeof(int64_t));
                e = walk(d_off, r_idx, r_val);
                if (e == hipSuccess) e = pack(d_off, d_off, r_idx, r_val, d_idx, d_val);
            }
            if (e == hipSuccess)
                e = hipMemcpyAsync(out_idx, d_idx, (size_t)total * 2 * sizeof(int64_t), hipMemcpyDeviceToHost, f->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(out_val, d_val, (size_t)total * width * sizeof(double), hipMemcpyDeviceToHost, f->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(f->stream);
        }
    }
    cleanup();
    if (e != hipSuccess) {
        f->j_params.clear();
        g_last_err = std::string("ggp_joints: ") + hipGetErrorString(e);
        return GGP_EDEV;
    }
    return GGP_OK;
}

// sub-forest descriptor of the cells `cells` (global indices, ascending; whole trees)
struct SubDesc {
    ggp_forest_desc d{};
    std::vector<int64_t> row_offset;
    std::vector<int32_t> parent, d1, d2, segment;
    std::vector<double> time, logl, fp;
};

void make_subdesc(const ggp_forest_desc *g, const std::vector<int32_t> &cells, SubDesc &s)
{
    const int64_t n = (int64_t)cells.size();
    std::unordered_map<int32_t, int32_t> remap;
    remap.reserve((size_t)n * 2);
    for (int64_t k = 0; k < n; ++k) remap[cells[k]] = (int32_t)k;
    auto rm = [&](int32_t v) { return v < 0 ? -1 : remap.at(v); };
    s.row_offset.assign(n + 1, 0);
    for (int64_t k = 0; k < n; ++k)
        s.row_offset[k + 1] = s.row_offset[k] + (g->row_offset[cells[k] + 1] - g->row_offset[cells[k]]);
    const int64_t nr = s.row_offset[n];
    s.parent.resize(n);
    s.d1.resize(n);
    s.d2.resize(n);
    for (int64_t k = 0; k < n; ++k) {
        s.parent[k] = rm(g->parent[cells[k]]);
        s.d1[k] = rm(g->daughter1[cells[k]]);
        s.d2[k] = rm(g->daughter2[cells[k]]);
    }
    s.time.resize(nr);
    s.logl.resize(nr);
    s.fp.resize(nr);
    if (g->segment) s.segment.resize(nr);
    for (int64_t k = 0; k < n; ++k) {
        const int64_t a = g->row_offset[cells[k]], b = g->row_offset[cells[k] + 1], o = s.row_offset[k];
        std::memcpy(&s.time[o], g->time + a, (size_t)(b - a) * sizeof(double));
        std::memcpy(&s.logl[o], g->log_length + a, (size_t)(b - a) * sizeof(double));
        std::memcpy(&s.fp[o], g->fp + a, (size_t)(b - a) * sizeof(double));
        if (g->segment) std::memcpy(&s.segment[o], g->segment + a, (size_t)(b - a) * sizeof(int32_t));
    }
    s.d = *g;
    s.d.n_cells = n;
    s.d.n_rows = nr;
    s.d.row_offset = s.row_offset.data();
    s.d.parent = s.parent.data();
    s.d.daughter1 = s.d1.data();
    s.d.daughter2 = s.d2.data();
    s.d.segment = g->segment ? s.segment.data() : nullptr;
    s.d.time = s.time.data();
    s.d.log_length = s.logl.data();
    s.d.fp = s.fp.data();
}

}  // namespace

extern "C" {

const char *ggp_strerror(int code)
{
    switch (code) {
    case GGP_OK: return "ok";
    case GGP_EINVAL: return g_last_err.empty() ? "invalid argument" : g_last_err.c_str();
    case GGP_ENAN: return "Likelihood is Nan";
    case GGP_EDEV: return g_last_err.empty() ? "HIP device error" : g_last_err.c_str();
    case GGP_ENOMEM: return "device allocation failed";
    case GGP_ETIMEOUT: return g_last_err.empty() ? "evaluation stalled (timeout)" : g_last_err.c_str();
    default: return "unknown error";
    }
}

const char *ggp_version(void) { return GGP_VERSION; }

static int rccl_load(const char *path, RcclApi &a)
{
    const char *lib = path && *path ? path : "librccl.so.1";
    a.lib = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!a.lib) {
        g_last_err = std::string("cannot load ") + lib + ": " + dlerror();
        return GGP_EDEV;
    }
    a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(a.lib, "ncclGetUniqueId"));
    a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(dlsym(a.lib, "ncclCommInitRank"));
    a.all_gather = reinterpret_cast<decltype(a.all_gather)>(dlsym(a.lib, "ncclAllGather"));
    a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(a.lib, "ncclCommDestroy"));
    a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(a.lib, "ncclGetErrorString"));
    a.comm_abort = reinterpret_cast<decltype(a.comm_abort)>(dlsym(a.lib, "ncclCommAbort"));
    a.comm_count = reinterpret_cast<decltype(a.comm_count)>(dlsym(a.lib, "ncclCommCount"));
    if (!a.get_unique_id || !a.comm_init_rank || !a.all_gather || !a.comm_destroy) {
        g_last_err = std::string(lib) + " lacks the RCCL entry points";
        return GGP_EDEV;
    }
    return GGP_OK;
}

int ggp_comm_unique_id(const char *rccl_lib, unsigned char *id)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    RcclApi a;
    int rc = rccl_load(rccl_lib, a);
    if (rc != GGP_OK || !id) return rc;   // id NULL: only check that the library can be used
    ggp_rccl_id u;
    const int e = a.get_unique_id(&u);
    if (e != 0) {
        g_last_err = std::string("ncclGetUniqueId: ") + (a.error_string ? a.error_string(e) : "error");
        return GGP_EDEV;
    }
    std::memcpy(id, u.internal, sizeof u.internal);
    return GGP_OK;
}

int ggp_comm_attach(ggp_forest *f, const char *rccl_lib, int32_t nranks, int32_t rank, const unsigned char *id)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !id || nranks < 1 || rank < 0 || rank >= nranks) return GGP_EINVAL;
    if (f->comm) {
        g_last_err = "ggp_comm_attach: the handle is already attached";
        return GGP_EINVAL;
    }
    if (f->shards.size() != 1 || f->shards[0]->n_lblocks > kPartMax) {
        g_last_err = "ggp_comm_attach: the handle must hold one shard (one device per process) of at most 4096 blocks";
        return GGP_EINVAL;
    }
    Shard *s = f->shards[0];
    Comm *c = new Comm;
    c->nranks = nranks;
    c->rank = rank;
    int rc = rccl_load(rccl_lib, c->api);
    auto fail = [&](int code) {
        if (c->d_part) (void)hipFree(c->d_part);
        if (c->d_gath) (void)hipFree(c->d_gath);
        if (c->h_res) (void)hipHostFree(c->h_res);
        if (c->nc) c->api.comm_destroy(c->nc);
        delete c;
        return code;
    };
    if (rc != GGP_OK) return fail(rc);
    if (hipSetDevice(s->device) != hipSuccess || hipMalloc(&c->d_part, 2 * sizeof(double)) != hipSuccess ||
        hipMalloc(&c->d_gath, 2 * sizeof(double) * (size_t)nranks) != hipSuccess) {
        g_last_err = "ggp_comm_attach: device buffers";
        return fail(GGP_ENOMEM);
    }
    void *m = nullptr;
    if (hipHostMalloc(&c->h_res, 3 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(&m, c->h_res, 0) != hipSuccess) {
        g_last_err = "ggp_comm_attach: mapped result slots";
        return fail(GGP_ENOMEM);
    }
    c->h_sum = (volatile double *)c->h_res;
    c->h_rank = (volatile int64_t *)((char *)c->h_res + sizeof(double));
    c->h_seq = (volatile int64_t *)((char *)c->h_res + 2 * sizeof(double));
    *c->h_seq = 0;
    c->m_sum = (double *)m;
    c->m_rank = (int64_t *)((char *)m + sizeof(double));
    c->m_seq = (int64_t *)((char *)m + 2 * sizeof(double));
    ggp_rccl_id u;
    std::memcpy(u.internal, id, sizeof u.internal);
    const int e = c->api.comm_init_rank(&c->nc, nranks, u, rank);   // every rank of the group joins
    if (e != 0) {
        g_last_err = std::string("ncclCommInitRank: ") + (c->api.error_string ? c->api.error_string(e) : "error");
        c->nc = nullptr;
        return fail(GGP_EDEV);
    }
    f->comm = c;
    return GGP_OK;
}

int ggp_launch_clock(const ggp_forest *f, double *shader_mhz, double *window_us)
{
    if (!f || f->shards.empty() || !f->shards[0]->h_clk) return GGP_EINVAL;
    const Shard *s = f->shards[0];
    // the last COMPLETED launch's counters (snapshotted when its sequence number was seen), never a
    // launch still in flight
    const unsigned long long c = s->clk_snap[0], r = s->clk_snap[1];
    if (r == 0) return GGP_EINVAL;   // no path launch has completed on this handle
    if (shader_mhz) *shader_mhz = (double)c / (double)r * 100.0;   // s_memrealtime: 100 MHz
    if (window_us) *window_us = (double)r / 100.0;
    return GGP_OK;
}

int32_t ggp_comm_size(const ggp_forest *f)
{
    if (!f || !f->comm || !f->comm->nc) return 0;
    int n = 0;
    if (f->comm->api.comm_count && f->comm->api.comm_count(f->comm->nc, &n) == 0) return n;
    return -1;
}

int32_t ggp_comm_nan_rank(const ggp_forest *f)
{
    return f && f->comm ? f->comm->last_nan_rank : -1;
}

int32_t ggp_comm_local_nan(const ggp_forest *f)
{
    return f && f->comm ? f->comm->local_nan : 0;
}

int ggp_device_count(int32_t *n)
{
    int c = 0;
    HIPCHK(hipGetDeviceCount(&c));
    *n = c;
    return GGP_OK;
}

void ggp_forest_destroy(ggp_forest *f)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f) return;
    if (Comm *c = f->comm) {
        if (!f->shards.empty()) {
            (void)hipSetDevice(f->shards[0]->device);
            (void)hipStreamSynchronize(f->shards[0]->stream);
        }
        if (c->nc && c->api.comm_destroy) c->api.comm_destroy(c->nc);
        if (c->d_part) (void)hipFree(c->d_part);
        if (c->d_gath) (void)hipFree(c->d_gath);
        if (c->h_res) (void)hipHostFree(c->h_res);
        delete c;   // the RCCL library stays loaded (the process's other users hold it too)
    }
    for (Shard *s : f->shards) shard_destroy(s);
    for (DeviceCtx *d : f->devs) {
        (void)hipSetDevice(d->id);
        if (d->stream) (void)hipStreamSynchronize(d->stream);
        if (d->sm_fwd) (void)hipFree(d->sm_fwd);
        if (d->sm_bwd) (void)hipFree(d->sm_bwd);
        if (d->stream) (void)hipStreamDestroy(d->stream);
        delete d;
    }
    delete f;
}

int ggp_forest_create(const ggp_forest_desc *d, ggp_forest **out)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!d || !out) { g_last_err = "null argument"; return GGP_EINVAL; }
    *out = nullptr;
    if (d->kernel < GGP_KERNEL_AUTO || d->kernel > GGP_KERNEL_PAIR) {
        g_last_err = "ggp_forest_create: unknown kernel policy";
        return GGP_EINVAL;
    }
    if (ggp::kExact && d->kernel == GGP_KERNEL_WAVE) {
        g_last_err = "ggp_forest_create: the exact-arithmetic engine (libggp_exact.so) has no wave schedule";
        return GGP_EINVAL;
    }
    std::vector<int32_t> depth, dfs;
    std::vector<int64_t> tree_start;
    int rc = check_topology(d, depth, dfs, tree_start);
    if (rc != GGP_OK) return rc;
    // ---- devices ----
    int n_vis = 0;
    if (hipGetDeviceCount(&n_vis) != hipSuccess || n_vis <= 0) {
        g_last_err = "no HIP device";
        return GGP_EDEV;
    }
    // n_devices: > 0 the list (or 0..n-1), 0 device 0 (a zero-filled descriptor), GGP_ALL_DEVICES
    // every visible device
    if (d->n_devices < 0 && d->n_devices != GGP_ALL_DEVICES) { g_last_err = "n_devices < 0 and not GGP_ALL_DEVICES"; return GGP_EINVAL; }
    std::vector<int32_t> devlist;
    const int nd = d->n_devices > 0 ? d->n_devices : d->n_devices == 0 ? 1 : n_vis;
    for (int k = 0; k < nd; ++k) {
        const int32_t id = (d->n_devices > 0 && d->devices) ? d->devices[k] : k;
        if (id < 0 || id >= n_vis) { g_last_err = "device ordinal out of range"; return GGP_EINVAL; }
        devlist.push_back(id);
    }
    auto *f = new ggp_forest();
    const int64_t nc = d->n_cells, nr = d->n_rows;
    f->n_cells = nc;
    f->n_rows = nr;
    f->n_trees = (int64_t)tree_start.size() - 1;
    for (int64_t c = 0; c < nc; ++c)
        if (d->parent[c] < 0) f->max_root_rows = std::max<int64_t>(f->max_root_rows, d->row_offset[c + 1] - d->row_offset[c]);
    f->dfs_order = dfs;
    f->row_off.assign(d->row_offset ? d->row_offset : nullptr, d->row_offset ? d->row_offset + nc + 1 : nullptr);
    if (nc == 0) f->row_off.assign(1, 0);
    f->blk_trees = block_trees_for(f->n_trees);
    f->n_blocks = (f->n_trees + f->blk_trees - 1) / f->blk_trees;
    // ---- shards: whole reduction blocks, LPT over the blocks' row counts ----
    int64_t n_shards = (int64_t)devlist.size();
    if (d->max_shard_rows > 0) n_shards = std::max<int64_t>(n_shards, (nr + d->max_shard_rows - 1) / d->max_shard_rows);
    n_shards = std::max<int64_t>(1, std::min<int64_t>(n_shards, std::max<int64_t>(1, f->n_blocks)));
    std::vector<int32_t> tree_of_cell(nc, 0);
    std::vector<int64_t> blk_rows(f->n_blocks, 0);
    for (int64_t t = 0; t < f->n_trees; ++t)
        for (int64_t k = tree_start[t]; k < tree_start[t + 1]; ++k) {
            const int32_t c = dfs[k];
            tree_of_cell[c] = (int32_t)t;
            blk_rows[t / f->blk_trees] += d->row_offset[c + 1] - d->row_offset[c];
        }
    std::vector<int32_t> blk_shard(f->n_blocks, 0);
    {
        std::vector<int64_t> order(f->n_blocks);
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return blk_rows[a] > blk_rows[b]; });
        // LPT; with a row cap, more shards until every shard fits it (a block is never split)
        for (;;) {
            std::vector<int64_t> load(n_shards, 0);
            for (int64_t b : order) {
                const int64_t s = std::min_element(load.begin(), load.end()) - load.begin();
                blk_shard[b] = (int32_t)s;
                load[s] += blk_rows[b];
            }
            const int64_t mx = load.empty() ? 0 : *std::max_element(load.begin(), load.end());
            if (d->max_shard_rows <= 0 || mx <= d->max_shard_rows || n_shards >= f->n_blocks) break;
            ++n_shards;
        }
    }
    // ---- device contexts (one per distinct ordinal) ----
    std::vector<DeviceCtx *> shard_dev(n_shards, nullptr);
    for (int64_t s = 0; s < n_shards && rc == GGP_OK; ++s) {
        const int id = devlist[s % devlist.size()];
        DeviceCtx *ctx = nullptr;
        for (DeviceCtx *c : f->devs)
            if (c->id == id) ctx = c;
        if (!ctx) {
            ctx = new DeviceCtx();
            ctx->id = id;
            f->devs.push_back(ctx);
            if (hipSetDevice(id) != hipSuccess ||
                hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
                g_last_err = "hipSetDevice / hipStreamCreate failed";
                rc = GGP_EDEV;
                break;
            }
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, id) == hipSuccess) ctx->n_cu = prop.multiProcessorCount;
        }
        shard_dev[s] = ctx;
    }
    std::vector<int32_t> gdfs_rank(nc);
    for (int64_t k = 0; k < nc; ++k) gdfs_rank[dfs[k]] = (int32_t)k;
    for (int64_t s = 0; s < n_shards && rc == GGP_OK; ++s) {
        std::vector<int32_t> ntrees;
        std::vector<int64_t> bglob;
        for (int64_t b = 0; b < f->n_blocks; ++b)
            if (blk_shard[b] == s) {
                bglob.push_back(b);
                ntrees.push_back((int32_t)(std::min(f->n_trees, (b + 1) * f->blk_trees) - b * f->blk_trees));
            }
        Shard *sh = nullptr;
        if (n_shards == 1) {
            rc = shard_create(d, shard_dev[s], gdfs_rank, ntrees, bglob, f->blk_trees, &sh);
        } else {
            std::vector<int32_t> cells;
            for (int64_t c = 0; c < nc; ++c)
                if (blk_shard[tree_of_cell[c] / f->blk_trees] == s) cells.push_back((int32_t)c);
            SubDesc sd;
            make_subdesc(d, cells, sd);
            std::vector<int32_t> gd(cells.size());
            for (size_t k = 0; k < cells.size(); ++k) gd[k] = gdfs_rank[cells[k]];
            rc = shard_create(&sd.d, shard_dev[s], gd, ntrees, bglob, f->blk_trees, &sh);
            if (sh) sh->cell_g = std::move(cells);
        }
        if (sh) f->shards.push_back(sh);
    }
    if (rc != GGP_OK) {
        ggp_forest_destroy(f);
        return rc;
    }
    *out = f;
    return GGP_OK;
}

int ggp_forest_shards(ggp_forest *f, int32_t *n, int32_t *device, int64_t *rows, int64_t *cells, int32_t cap)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !n) return GGP_EINVAL;
    *n = (int32_t)f->shards.size();
    for (int32_t k = 0; k < *n && k < cap; ++k) {
        if (device) device[k] = f->shards[k]->device;
        if (rows) rows[k] = f->shards[k]->n_rows;
        if (cells) cells[k] = f->shards[k]->n_cells;
    }
    return GGP_OK;
}

int ggp_reset_state(ggp_forest *f)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f) return GGP_EINVAL;
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipMemsetAsync(s->d_state, 0, (size_t)s->n_cells * 20 * sizeof(double), s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    return GGP_OK;
}

int ggp_get_state(ggp_forest *f, double *out)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !out) return GGP_EINVAL;
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipStreamSynchronize(s->stream));
        if (s->cell_g.empty()) {
            HIPCHK(hipMemcpy(out, s->d_state, (size_t)s->n_cells * 20 * sizeof(double), hipMemcpyDeviceToHost));
            continue;
        }
        std::vector<double> tmp((size_t)s->n_cells * 20);
        HIPCHK(hipMemcpy(tmp.data(), s->d_state, tmp.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int64_t c = 0; c < s->n_cells; ++c)
            std::memcpy(out + (size_t)20 * s->cell_g[c], &tmp[(size_t)20 * c], 20 * sizeof(double));
    }
    return GGP_OK;
}

int ggp_set_state(ggp_forest *f, const double *in)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !in) return GGP_EINVAL;
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipStreamSynchronize(s->stream));
        if (s->cell_g.empty()) {
            HIPCHK(hipMemcpy(s->d_state, in, (size_t)s->n_cells * 20 * sizeof(double), hipMemcpyHostToDevice));
            continue;
        }
        std::vector<double> tmp((size_t)s->n_cells * 20);
        for (int64_t c = 0; c < s->n_cells; ++c)
            std::memcpy(&tmp[(size_t)20 * c], in + (size_t)20 * s->cell_g[c], 20 * sizeof(double));
        HIPCHK(hipMemcpy(s->d_state, tmp.data(), tmp.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    return GGP_OK;
}

// the last path launch's device time into its ring entry: its first block's start (written before
// the sequence number) and its publishing block's end (written just after it; a stamp older than
// the start is one that has not landed: the entry keeps kernel_us = 0)
static void trace_finalize(ggp_forest *f)
{
    if (f->tr_open < 0 || f->shards.empty()) return;
    const Shard *s0 = f->shards[0];
    CallRec &r = f->tr_ring[f->tr_open];
    f->tr_open = -1;
    if (!s0->h_clk) return;
    const unsigned long long t0 = s0->clk_snap[2], t1 = s0->h_clk[3];
    if (t1 > t0) r.kernel_us = (double)(t1 - t0) / 100.0;   // s_memrealtime: 100 MHz
}

int ggp_total_loglik_async(ggp_forest *f, const double *params)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !params) return GGP_EINVAL;
    if (f->comm && f->comm->failed) {
        g_last_err = "the handle's communicator was aborted after a failed collective evaluation; re-create the group";
        return GGP_EDEV;
    }
    f->tr_t0 = std::chrono::steady_clock::now();
    trace_finalize(f);   // before the next launch can overwrite the stamps
    ggp_params P;
    std::memcpy(P.p, params, sizeof P.p);
    for (Shard *s : f->shards) {   // every device enqueued before any is waited for
        const int rc = shard_launch(s, P);
        if (rc != GGP_OK) {
            if (f->comm) comm_fail(f->comm);   // the peers would wait for this rank's all-gather
            return rc;
        }
    }
    if (Comm *c = f->comm) {   // behind the evaluation: partial, all-gather, rank-order sum
        Shard *s = f->shards[0];
        int np2 = 1;
        while (np2 < s->n_lblocks) np2 *= 2;
        hipLaunchKernelGGL(k_rank_partial, dim3(1), dim3(256), 0, s->stream, s->m_sum, s->m_nan, (int)s->n_lblocks, np2,
                           c->d_part);
        if (hipGetLastError() != hipSuccess) {
            g_last_err = "k_rank_partial launch failed";
            comm_fail(c);
            return GGP_EDEV;
        }
        const int e = c->api.all_gather(c->d_part, c->d_gath, 2 * sizeof(double), kRcclUint8, c->nc, s->stream);
        if (e != 0) {
            g_last_err = std::string("RCCL all-gather: ") + (c->api.error_string ? c->api.error_string(e) : "error");
            comm_fail(c);
            return GGP_EDEV;
        }
        ++c->seq;
        hipLaunchKernelGGL(k_rank_sum, dim3(1), dim3(64), 0, s->stream, c->d_gath, c->nranks, c->m_sum, c->m_rank, c->m_seq,
                           c->seq);
        if (hipGetLastError() != hipSuccess) {
            g_last_err = "k_rank_sum launch failed";
            comm_fail(c);
            return GGP_EDEV;
        }
    }
    f->tr_t1 = std::chrono::steady_clock::now();
    f->tr_pending = true;
    return GGP_OK;
}

// multi-process result: spin on the sequence number k_rank_sum releases (hipStreamQuery as the
// way out when the stream fails; a wall-clock bound, GGP_COMM_TIMEOUT_S (default 600 s), when a
// peer never reaches the collective: GGP_ETIMEOUT and the communicator is aborted).  This rank's
// own first NaN (or stall) is always read from its block results: nan_cell / nan_row hold it
// (-1 if this rank was clean) and ggp_comm_local_nan reports it, whatever the lowest bad rank is.
static int comm_result(ggp_forest *f, double *ll, int64_t *nan_cell, int64_t *nan_row)
{
    Comm *c = f->comm;
    Shard *s = f->shards[0];
    if (c->failed) {
        g_last_err = "the handle's communicator was aborted after a failed collective evaluation; re-create the group";
        return GGP_EDEV;
    }
    static const double limit_s = [] {
        const char *e = getenv("GGP_COMM_TIMEOUT_S");
        return e ? atof(e) : 600.0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false, timed_out = false;
    for (uint32_t it = 1;; ++it) {
        if (*c->h_seq == c->seq) { seen = true; break; }
        if ((it & 1023) == 0) {
            if (hipStreamQuery(s->stream) != hipErrorNotReady) break;
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) {
                timed_out = true;
                break;
            }
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    s->seq_pending = false;
    f->tr_t2 = std::chrono::steady_clock::now();
    if (seen && s->used_path && s->h_clk)   // the path launch completed before k_rank_sum (stream order)
        for (int k = 0; k < 4; ++k) s->clk_snap[k] = s->h_clk[k];
    if (timed_out) {
        g_last_err = "multi-process evaluation did not complete within GGP_COMM_TIMEOUT_S (a peer rank never reached the collective); communicator aborted";
        comm_fail(c);
        return GGP_ETIMEOUT;
    }
    if (!seen || s->profile) {
        HIPCHK(hipSetDevice(s->device));
        const hipError_t e = hipStreamSynchronize(s->stream);
        if (e != hipSuccess || *c->h_seq != c->seq) {
            g_last_err = "multi-process evaluation did not complete";
            comm_fail(c);
            return GGP_EDEV;
        }
    }
    const double v = *c->h_sum;
    const int64_t code_rank = *c->h_rank;
    const bool stall = code_rank >= 0 && (code_rank >> 32) != 0;
    c->last_nan_rank = code_rank < 0 ? -1 : (int32_t)(code_rank & 0xffffffff);
    if (ll) *ll = v;
    if (nan_cell) *nan_cell = -1;
    if (nan_row) *nan_row = -1;
    // this rank's own first bad cell, as ggp_loglik_result finds it
    long long code = kNoNan;
    bool own_nan_sum = false;
    for (int64_t j = 0; j < s->n_lblocks; ++j) {
        code = std::min<long long>(code, s->h_nan[j]);
        own_nan_sum = own_nan_sum || std::isnan(s->h_sum[j]);
    }
    c->local_nan = (code != kNoNan || own_nan_sum) ? 1 : 0;
    if (code != kNoNan) {
        if (nan_cell) *nan_cell = f->dfs_order[code >> 24];
        if (nan_row) *nan_row = (code & 0xffffff) == kRowStall ? -1 : (code & 0xffffff);
    }
    if (c->last_nan_rank < 0) return GGP_OK;
    if (stall) {
        g_last_err = "evaluation stalled on rank " + std::to_string(c->last_nan_rank) +
                     ": a daughter cell's wait for its parent timed out (a scheduling stall, not a NaN)";
        return GGP_ETIMEOUT;
    }
    return GGP_ENAN;
}

static int loglik_result(ggp_forest *f, double *ll, int64_t *nan_cell, int64_t *nan_row)
{
    if (f->comm) return comm_result(f, ll, nan_cell, nan_row);
    long long code = kNoNan;
    for (Shard *s : f->shards) {
        const int rc = shard_wait(s);
        if (rc != GGP_OK) return rc;
    }
    f->tr_t2 = std::chrono::steady_clock::now();
    size_t np2 = 1;
    while (np2 < (size_t)f->n_blocks) np2 *= 2;
    if (f->res_blocks.size() != np2) f->res_blocks.assign(np2, 0.0);
    double *blocks = f->res_blocks.data();
    std::fill(blocks + f->n_blocks, blocks + np2, 0.0);   // the pad (the tree overwrites the low slots)
    for (Shard *s : f->shards) {
        const int64_t *gj = s->blk_global.data();
        for (int64_t j = 0; j < s->n_lblocks; ++j) {
            blocks[(size_t)gj[j]] = s->h_sum[j];
            code = std::min<long long>(code, s->h_nan[j]);
        }
    }
    const double v = f->n_blocks ? top_sum_inplace(blocks, np2) : 0.0;
    if (ll) *ll = v;
    if (nan_cell) *nan_cell = -1;
    if (nan_row) *nan_row = -1;
    if (code != kNoNan) {
        const int64_t rank = code >> 24, row = code & 0xffffff;
        if (nan_cell) *nan_cell = f->dfs_order[rank];
        if (nan_row) *nan_row = row == kRowStall ? -1 : row;
        if (ll) *ll = std::nan("");
        if (row == kRowStall) {   // the first bad cell in reference order waited for its parent too long
            g_last_err = "evaluation stalled: a daughter cell's wait for its parent timed out (a scheduling stall, not a NaN)";
            return GGP_ETIMEOUT;
        }
        return GGP_ENAN;
    }
    if (std::isnan(v)) return GGP_ENAN;   // NaN from +inf + -inf across cells (see include/ggp.h)
    return GGP_OK;
}

int ggp_loglik_result(ggp_forest *f, double *ll, int64_t *nan_cell, int64_t *nan_row)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f) return GGP_EINVAL;
    f->tr_t2 = {};
    const int rc = loglik_result(f, ll, nan_cell, nan_row);
    if (f->tr_pending) {   // the call's host split (ggp_call_trace)
        f->tr_pending = false;
        const auto t3 = std::chrono::steady_clock::now();
        const auto t2 = f->tr_t2 == std::chrono::steady_clock::time_point{} ? t3 : f->tr_t2;
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        CallRec &r = f->tr_ring[f->tr_n % kCallRing];
        r.enqueue_us = us(f->tr_t0, f->tr_t1);
        r.wait_us = us(f->tr_t1, t2);
        r.result_us = us(t2, t3);
        r.kernel_us = r.shader_mhz = 0.0;
        const Shard *s0 = f->shards.empty() ? nullptr : f->shards[0];
        if (s0 && s0->used_path && s0->clk_snap[1] > 0)
            r.shader_mhz = (double)s0->clk_snap[0] / (double)s0->clk_snap[1] * 100.0;
        // the kernel's end stamp lands just after the sequence number: read when the handle is next
        // entered (trace_finalize)
        f->tr_open = s0 && s0->used_path ? (int64_t)(f->tr_n % kCallRing) : -1;
        r.call = (double)f->tr_n;
        ++f->tr_n;
    }
    return rc;
}

int ggp_call_trace(const ggp_forest *f, int32_t cap, double *out, int32_t *n)
{
    if (!f || cap < 0 || (cap > 0 && !out)) return GGP_EINVAL;
    trace_finalize(const_cast<ggp_forest *>(f));
    const int64_t have = std::min<int64_t>(f->tr_n, kCallRing);
    const int32_t k = (int32_t)std::min<int64_t>(have, cap);
    for (int32_t i = 0; i < k; ++i) {   // the last k calls, oldest first
        const CallRec &r = f->tr_ring[(f->tr_n - k + i) % kCallRing];
        const double v[6] = {r.enqueue_us, r.wait_us, r.result_us, r.kernel_us, r.shader_mhz, r.call};
        std::memcpy(out + 6 * (size_t)i, v, sizeof v);
    }
    if (n) *n = k;
    return GGP_OK;
}

int ggp_total_loglik(ggp_forest *f, const double *params, double *ll, int64_t *nan_cell, int64_t *nan_row)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    int rc = ggp_total_loglik_async(f, params);
    if (rc != GGP_OK) return rc;
    return ggp_loglik_result(f, ll, nan_cell, nan_row);
}

// Batched objective: n_pts parameter points, each evaluated from the handle's carried state as
// it is at the call (the carried state itself is left unchanged).  Points run in chunks that
// keep the per-point state slices under kBatchBytes per shard; every level of a chunk is one
// launch of the lane schedule with blockIdx.y = point, then the block sums of every point.
static constexpr int64_t kBatchBytes = int64_t(4) << 30;

// the per-point workspace of a batch or chain call, for up to min(n_pts, what keeps a shard's
// slices under kBatchBytes) points; returns that chunk (<= 0: an error code, negated)
static int64_t batch_reserve(ggp_forest *f, int32_t n_pts)
{
    int64_t chunk = std::min<int64_t>((int64_t)n_pts, 65535);
    if (const char *e = std::getenv("GGP_BATCH_CHUNK"))   // tests: chunk boundaries
        if (std::atoll(e) > 0) chunk = std::min<int64_t>(chunk, std::atoll(e));
    for (Shard *s : f->shards)
        if (s->n_cells) chunk = std::min<int64_t>(chunk, std::max<int64_t>(1, kBatchBytes / (s->n_cells * (20 * 8 + 8 + 4 + 4))));
    for (Shard *s : f->shards) {
        if (!s->n_cells || chunk <= s->b_cap) continue;
        if (hipSetDevice(s->device) != hipSuccess || hipStreamSynchronize(s->stream) != hipSuccess) {
            g_last_err = "HIP error before the batch workspace";
            return -GGP_EDEV;
        }
        batch_free(s);
        int rc = GGP_OK;
        auto check = [&](int r) { if (r != GGP_OK && rc == GGP_OK) rc = r; };
        const int64_t nc = s->n_cells;
        check(dev_upload<double>(&s->d_b_ptab, nullptr, (size_t)chunk * 11));
        check(dev_upload<double>(&s->d_b_state, nullptr, (size_t)chunk * nc * 20));
        check(dev_upload<double>(&s->d_b_ll, nullptr, (size_t)chunk * nc));
        check(dev_upload<int32_t>(&s->d_b_nan, nullptr, (size_t)chunk * nc));
        check(dev_upload<double>(&s->d_b_sum, nullptr, (size_t)chunk * s->n_lblocks));
        check(dev_upload<int64_t>(&s->d_b_code, nullptr, (size_t)chunk * s->n_lblocks));
        check(dev_upload<unsigned>(&s->d_b_done, nullptr, (size_t)chunk * nc));
        check(dev_upload<int32_t>(&s->d_b_pred, nullptr, (size_t)chunk));
        if (rc == GGP_OK && hipMemset(s->d_b_done, 0, (size_t)chunk * nc * sizeof(unsigned)) != hipSuccess) rc = GGP_EDEV;
        if (rc != GGP_OK) { batch_free(s); return -rc; }
        s->b_cap = chunk;
    }
    return chunk;
}

int ggp_total_loglik_batch(ggp_forest *f, int32_t n_pts, const double *params, double *ll, int32_t *status)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || n_pts < 0 || (n_pts > 0 && (!params || !ll || !status))) {
        g_last_err = "ggp_total_loglik_batch: bad arguments";
        return GGP_EINVAL;
    }
    if (n_pts == 0) return GGP_OK;
    if (f->n_cells == 0) {
        for (int32_t i = 0; i < n_pts; ++i) { ll[i] = 0.0; status[i] = GGP_OK; }
        return GGP_OK;
    }
    f->tree_pts = 0;
    const int64_t chunk = batch_reserve(f, n_pts);
    if (chunk <= 0) return (int)-chunk;
    const size_t ns = f->shards.size();
    std::vector<std::vector<double>> sums(ns);
    std::vector<std::vector<int64_t>> codes(ns);
    for (int64_t p0 = 0; p0 < n_pts; p0 += chunk) {
        const int64_t np = std::min<int64_t>(chunk, n_pts - p0);
        for (size_t k = 0; k < ns; ++k) {   // enqueue every shard
            Shard *s = f->shards[k];
            if (!s->n_cells) continue;
            const int64_t nc = s->n_cells;
            HIPCHK(hipSetDevice(s->device));
            HIPCHK(hipMemcpyAsync(s->d_b_ptab, params + 11 * p0, (size_t)np * 11 * sizeof(double),
                                  hipMemcpyHostToDevice, s->stream));
            const int64_t total = nc * 20 * np;
            const int rblocks = (int)std::min<int64_t>((total + 255) / 256, 65536);
            hipLaunchKernelGGL(k_replicate, dim3(rblocks), dim3(256), 0, s->stream, s->d_state, nc * 20, s->d_b_state, np);
            HIPCHK(hipGetLastError());
            const int n_levels = (int)s->level_start.size() - 1;
            const int cpw = lane_cpw(s);
            for (int L = 0; L < n_levels; ++L) {
                const int64_t a = s->level_start[L];
                const int n = (int)(s->level_start[L + 1] - a);
                if (n <= 0) continue;
                hipLaunchKernelGGL(k_loglik_level_batch, dim3((n + cpw - 1) / cpw, (unsigned)np), dim3(64), 0,
                                   s->stream, s->F, s->d_b_ptab, s->d_level_cells + a, n, cpw, nc, s->d_b_state,
                                   s->d_b_ll, s->d_b_nan);
                HIPCHK(hipGetLastError());
            }
            hipLaunchKernelGGL(k_reduce_blocks, dim3((unsigned)s->n_lblocks, (unsigned)np), dim3(s->red_threads), 0,
                               s->stream, nc, s->d_b_ll, s->d_b_nan, s->d_tree_dfs, s->d_blk_t0, s->d_blk_nt,
                               s->d_gdfs, (int)s->n_lblocks, s->d_b_sum, s->d_b_code, (unsigned *)nullptr,
                               (int64_t *)nullptr, (int64_t)0, (double *)nullptr, (int64_t *)nullptr);
            HIPCHK(hipGetLastError());
            sums[k].resize((size_t)np * s->n_lblocks);
            codes[k].resize((size_t)np * s->n_lblocks);
            HIPCHK(hipMemcpyAsync(sums[k].data(), s->d_b_sum, sums[k].size() * sizeof(double), hipMemcpyDeviceToHost,
                                  s->stream));
            HIPCHK(hipMemcpyAsync(codes[k].data(), s->d_b_code, codes[k].size() * sizeof(int64_t),
                                  hipMemcpyDeviceToHost, s->stream));
        }
        for (Shard *s : f->shards) {
            if (!s->n_cells) continue;
            HIPCHK(hipSetDevice(s->device));
            HIPCHK(hipStreamSynchronize(s->stream));
        }
        for (int64_t i = 0; i < np; ++i) {
            std::vector<double> blocks((size_t)f->n_blocks, 0.0);
            bool bad = false;
            for (size_t k = 0; k < ns; ++k) {
                const Shard *s = f->shards[k];
                for (int64_t j = 0; j < s->n_lblocks; ++j) {
                    blocks[(size_t)s->blk_global[j]] = sums[k][(size_t)(i * s->n_lblocks + j)];
                    bad = bad || codes[k][(size_t)(i * s->n_lblocks + j)] != kNoNan;
                }
            }
            const double v = top_sum(std::move(blocks));
            bad = bad || std::isnan(v);
            status[p0 + i] = bad ? GGP_ENAN : GGP_OK;
            ll[p0 + i] = bad ? std::nan("") : v;
        }
    }
    return GGP_OK;
}

// Chained objective: n_pts evaluations in order, each from the carried state the previous one
// left -- bitwise n_pts ggp_total_loglik calls (the reference's own sequences: num_hessian_ll's
// 4k^2 calls, likelihood.h:211-258; the -s scan, main.cpp:80-114).  Only a root's state crosses
// from one evaluation to the next (init_sc_distribution keeps its off-diagonals,
// predictions.h:63-82), so on path-launch shards one k_loglik_wave<true> launch runs a chunk of
// points (blockIdx.y = point): a root of point i waits for the same root of point i - 1, every
// other cell only for its parent within its point, and the points' trees overlap on the device.
// Per point: k_reduce_blocks' sums (bitwise the in-launch reduction) and the host's top_sum.
// Other handles (level launches, a communicator) run the calls one by one.
// chained points on the path-launch shards: np points of params, point i's roots from the state
// point pred[i] left (pred NULL: i - 1; -1: the carried state); per shard its block sums and
// first-NaN codes per point, on the host once the shards are synchronised
static bool chain_fusable(const ggp_forest *f, int64_t np = 0, const double *params = nullptr)
{
    bool fused = f->comm == nullptr;
    if (const char *e = std::getenv("GGP_CHAIN_FUSED")) fused = fused && std::atoi(e) != 0;
    for (const Shard *s : f->shards) {
        if (s->n_cells && s->n_paths == 0) fused = false;
        for (int64_t i = 0; fused && s->n_cells && i < np; ++i)
            if (wave_products_risky(s, params + 11 * i)) fused = false;   // launch_levels' other schedules
    }
    return fused;
}

static int run_points(ggp_forest *f, int64_t np, const double *params, const int32_t *pred,
                      std::vector<std::vector<double>> &sums, std::vector<std::vector<int64_t>> &codes)
{
    const size_t ns = f->shards.size();
    sums.assign(ns, {});
    codes.assign(ns, {});
    ggp_params P0{};
    for (size_t k = 0; k < ns; ++k) {   // enqueue every shard
        Shard *s = f->shards[k];
        if (!s->n_cells) continue;
        const int64_t nc = s->n_cells;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipMemcpyAsync(s->d_b_ptab, params, (size_t)np * 11 * sizeof(double), hipMemcpyHostToDevice, s->stream));
        if (pred)
            HIPCHK(hipMemcpyAsync(s->d_b_pred, pred, (size_t)np * sizeof(int32_t), hipMemcpyHostToDevice, s->stream));
        ++s->epoch;
        hipLaunchKernelGGL(k_loglik_wave<true>, dim3((unsigned)s->n_paths, (unsigned)np), dim3(64), 0, s->stream, s->F, P0,
                           s->d_path_cells, (int)nc, s->d_b_state, s->d_b_ll, s->d_b_nan, s->d_chain, s->d_b_done, s->epoch,
                           s->d_path_seq, chain_red_setup(s), (int64_t)0, s->spin_max, (const double *)s->d_b_ptab,
                           (const double *)s->d_state, pred ? (const int32_t *)s->d_b_pred : (const int32_t *)nullptr);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_reduce_blocks, dim3((unsigned)s->n_lblocks, (unsigned)np), dim3(s->red_threads), 0,
                           s->stream, nc, s->d_b_ll, s->d_b_nan, s->d_tree_dfs, s->d_blk_t0, s->d_blk_nt,
                           s->d_gdfs, (int)s->n_lblocks, s->d_b_sum, s->d_b_code, (unsigned *)nullptr,
                           (int64_t *)nullptr, (int64_t)0, (double *)nullptr, (int64_t *)nullptr);
        HIPCHK(hipGetLastError());
        sums[k].resize((size_t)np * s->n_lblocks);
        codes[k].resize((size_t)np * s->n_lblocks);
        HIPCHK(hipMemcpyAsync(sums[k].data(), s->d_b_sum, sums[k].size() * sizeof(double), hipMemcpyDeviceToHost,
                              s->stream));
        HIPCHK(hipMemcpyAsync(codes[k].data(), s->d_b_code, codes[k].size() * sizeof(int64_t), hipMemcpyDeviceToHost,
                              s->stream));
    }
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    return GGP_OK;
}

// point i's result as ggp_loglik_result forms it: the code, the value, the NaN location
static int point_result(const ggp_forest *f, const std::vector<std::vector<double>> &sums,
                        const std::vector<std::vector<int64_t>> &codes, int64_t i, double *ll, int64_t *nan_cell,
                        int64_t *nan_row)
{
    std::vector<double> blocks((size_t)f->n_blocks, 0.0);
    long long code = kNoNan;
    for (size_t k = 0; k < f->shards.size(); ++k) {
        const Shard *s = f->shards[k];
        for (int64_t j = 0; j < s->n_lblocks; ++j) {
            blocks[(size_t)s->blk_global[j]] = sums[k][(size_t)(i * s->n_lblocks + j)];
            code = std::min<long long>(code, codes[k][(size_t)(i * s->n_lblocks + j)]);
        }
    }
    const double v = top_sum(std::move(blocks));
    if (nan_cell) *nan_cell = -1;
    if (nan_row) *nan_row = -1;
    *ll = v;
    if (code != kNoNan) {
        const int64_t rank = code >> 24, row = code & 0xffffff;
        if (nan_cell) *nan_cell = f->dfs_order[rank];
        if (nan_row) *nan_row = row == kRowStall ? -1 : row;
        *ll = std::nan("");
        return row == kRowStall ? GGP_ETIMEOUT : GGP_ENAN;
    }
    return std::isnan(v) ? GGP_ENAN : GGP_OK;   // NaN from +inf + -inf across cells
}

static const char *kStallMsg =
    "evaluation stalled: a cell's wait for the cell it depends on timed out (a scheduling stall, not a NaN)";

// the carried state becomes the state point `point` of the last run_points left (every cell, as
// its sequential call leaves it); the copies are enqueued on each shard's stream
static int adopt_point_state(ggp_forest *f, int64_t point)
{
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        const int64_t nc = s->n_cells;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipMemcpyAsync(s->d_state, s->d_b_state + (size_t)point * nc * 20, (size_t)nc * 20 * sizeof(double),
                              hipMemcpyDeviceToDevice, s->stream));
    }
    return GGP_OK;
}

int ggp_total_loglik_chain(ggp_forest *f, int32_t n_pts, const double *params, double *ll, int32_t *n_ok,
                           int64_t *nan_cell, int64_t *nan_row)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || n_pts < 0 || !n_ok || (n_pts > 0 && (!params || !ll))) {
        g_last_err = "ggp_total_loglik_chain: bad arguments";
        return GGP_EINVAL;
    }
    *n_ok = 0;
    if (nan_cell) *nan_cell = -1;
    if (nan_row) *nan_row = -1;
    f->tree_pts = 0;
    if (!chain_fusable(f, n_pts, params) || f->n_cells == 0) {
        for (int32_t i = 0; i < n_pts; ++i) {
            const int rc = ggp_total_loglik(f, params + (size_t)11 * i, ll + i, nan_cell, nan_row);
            if (rc != GGP_OK) return rc;
            *n_ok = i + 1;
        }
        return GGP_OK;
    }
    if (n_pts == 0) return GGP_OK;
    int64_t chunk = batch_reserve(f, n_pts);
    if (chunk <= 0) return (int)-chunk;
    // a launch's chain of roots (point i's roots wait for point i - 1's) stays within
    // kChainRowsPerLaunch rows, so no wait in it comes near the stall budget
    int64_t rows_cap = kChainRowsPerLaunch;
    if (const char *e = std::getenv("GGP_CHAIN_ROWS_PER_LAUNCH"))   // tests: the cap's chunk boundaries
        if (std::atoll(e) > 0) rows_cap = std::atoll(e);
    chunk = std::min<int64_t>(chunk, std::max<int64_t>(1, rows_cap / f->max_root_rows));
    std::vector<std::vector<double>> sums;
    std::vector<std::vector<int64_t>> codes;
    for (int64_t p0 = 0; p0 < n_pts; p0 += chunk) {
        const int64_t np = std::min<int64_t>(chunk, n_pts - p0);
        int rc = run_points(f, np, params + 11 * p0, nullptr, sums, codes);
        if (rc != GGP_OK) return rc;
        int64_t i = 0;
        int r = GGP_OK;
        for (; i < np; ++i) {
            r = point_result(f, sums, codes, i, ll + p0 + i, nan_cell, nan_row);
            if (r != GGP_OK) break;
            *n_ok = (int32_t)(p0 + i + 1);
        }
        if (r == GGP_OK || r == GGP_ENAN) {   // after a NaN the carried state is unspecified (as one by one)
            if ((rc = adopt_point_state(f, r == GGP_OK ? np - 1 : i)) != GGP_OK) return rc;
            if (r != GGP_OK) return r;
            continue;
        }
        // a stall (GGP_ETIMEOUT) is the chained schedule's, not the calls': the carried state
        // becomes the last completed point's (or stays the one before this launch), and the
        // remaining points run one by one -- the same calls, so the same values
        if (i > 0 && (rc = adopt_point_state(f, i - 1)) != GGP_OK) return rc;
        ++f->chain_fallbacks;
        for (int64_t q = p0 + i; q < n_pts; ++q) {
            const int rq = ggp_total_loglik(f, params + (size_t)11 * q, ll + q, nan_cell, nan_row);
            if (rq == GGP_ETIMEOUT) g_last_err = kStallMsg;
            if (rq != GGP_OK) return rq;
            *n_ok = (int32_t)(q + 1);
        }
        return GGP_OK;
    }
    return GGP_OK;
}

int ggp_chain_fallbacks(const ggp_forest *f, int64_t *n)
{
    if (!f || !n) {
        g_last_err = "ggp_chain_fallbacks: bad arguments";
        return GGP_EINVAL;
    }
    *n = f->chain_fallbacks;
    return GGP_OK;
}

// Speculative evaluation (the -m optimiser's next calls): points whose roots start from the state
// another point of the call left, all in one launch; the carried state is left unchanged until
// ggp_keep_point_state picks the point whose state the caller's sequence of calls would have left.
int ggp_total_loglik_tree(ggp_forest *f, int32_t n_pts, const double *params, const int32_t *pred, double *ll,
                          int32_t *status, int64_t *nan_cell, int64_t *nan_row)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || n_pts < 0 || (n_pts > 0 && (!params || !pred || !ll || !status))) {
        g_last_err = "ggp_total_loglik_tree: bad arguments";
        return GGP_EINVAL;
    }
    for (int32_t i = 0; i < n_pts; ++i)
        if (pred[i] < -1 || pred[i] >= i) {
            g_last_err = "ggp_total_loglik_tree: pred[i] must lie in [-1, i)";
            return GGP_EINVAL;
        }
    f->tree_pts = 0;
    if (!chain_fusable(f, n_pts, params)) {
        g_last_err = "ggp_total_loglik_tree: the handle has no path launch (or is attached to a communicator, or "
                     "the points' rates x dt leave the wave schedule's product range)";
        return GGP_EINVAL;
    }
    if (n_pts == 0) return GGP_OK;
    if (f->n_cells == 0) {
        for (int32_t i = 0; i < n_pts; ++i) {
            ll[i] = 0.0;
            status[i] = GGP_OK;
            if (nan_cell) nan_cell[i] = -1;
            if (nan_row) nan_row[i] = -1;
        }
        f->tree_pts = n_pts;
        return GGP_OK;
    }
    const int64_t chunk = batch_reserve(f, n_pts);
    if (chunk <= 0) return (int)-chunk;
    if (chunk < n_pts) {
        g_last_err = "ggp_total_loglik_tree: more points than one launch holds";
        return GGP_EINVAL;
    }
    std::vector<std::vector<double>> sums;
    std::vector<std::vector<int64_t>> codes;
    const int rc = run_points(f, n_pts, params, pred, sums, codes);
    if (rc != GGP_OK) return rc;
    for (int32_t i = 0; i < n_pts; ++i)
        status[i] = point_result(f, sums, codes, i, ll + i, nan_cell ? nan_cell + i : nullptr, nan_row ? nan_row + i : nullptr);
    f->tree_pts = n_pts;
    return GGP_OK;
}

int ggp_keep_point_state(ggp_forest *f, int32_t point)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || point < 0 || point >= f->tree_pts) {
        g_last_err = "ggp_keep_point_state: no such point of the last ggp_total_loglik_tree call";
        return GGP_EINVAL;
    }
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        const int64_t nc = s->n_cells;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipMemcpyAsync(s->d_state, s->d_b_state + (size_t)point * nc * 20, (size_t)nc * 20 * sizeof(double),
                              hipMemcpyDeviceToDevice, s->stream));
    }
    return GGP_OK;
}

int ggp_last_launch_profile(ggp_forest *ff, float *ms, int64_t *rows, int32_t *kernel, int32_t cap, int32_t *n)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!ff || !n || ff->shards.empty()) return GGP_EINVAL;
    Shard *f = ff->shards[0];   // the first shard's launches
    if (cap < 0) {   // switch the events off again (the spin wait returns)
        *n = 0;
        if (!f->profile) return GGP_OK;
        HIPCHK(hipSetDevice(f->device));
        HIPCHK(hipStreamSynchronize(f->stream));
        for (auto &e : f->ev) (void)hipEventDestroy(e);
        f->ev.clear();
        f->n_prof = 0;
        f->profile = false;
        return GGP_OK;
    }
    if (!f->profile) {
        // enable for subsequent calls: one event pair per level
        HIPCHK(hipSetDevice(f->device));
        const size_t levels = f->level_start.size() - 1;
        f->ev.resize(2 * levels);
        for (auto &e : f->ev) HIPCHK(hipEventCreate(&e));
        f->ev_kernel.assign(levels, 0);
        f->ev_rows_launch.assign(levels, 0);
        f->profile = true;
        *n = 0;
        return GGP_OK;
    }
    HIPCHK(hipSetDevice(f->device));
    HIPCHK(hipStreamSynchronize(f->stream));
    int k = 0;
    for (int L = 0; L < f->n_prof && k < cap; ++L, ++k) {
        float t = 0;
        HIPCHK(hipEventElapsedTime(&t, f->ev[2 * L], f->ev[2 * L + 1]));
        if (ms) ms[k] = t;
        if (rows) rows[k] = f->ev_rows_launch[L];
        if (kernel) kernel[k] = f->ev_kernel[L];
    }
    *n = k;
    return GGP_OK;
}

int ggp_forest_info(ggp_forest *f, int64_t *n_levels, int64_t *max_level_cells, int32_t *kernel_used)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f) return GGP_EINVAL;
    int64_t mx = 0, nl = 0;
    for (const Shard *s : f->shards) {
        for (size_t L = 0; L + 1 < s->level_start.size(); ++L)
            mx = std::max(mx, s->level_start[L + 1] - s->level_start[L]);
        nl = std::max(nl, (int64_t)s->level_start.size() - 1);
    }
    if (n_levels) *n_levels = nl;
    if (max_level_cells) *max_level_cells = mx;
    if (kernel_used) *kernel_used = f->shards.empty() ? GGP_KERNEL_LANE : f->shards[0]->kernel_used;
    return GGP_OK;
}

int ggp_predict_profile(ggp_forest *f, float *ms_smooth, float *ms_combine)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f) return GGP_EINVAL;
    // per device: its shards run one after another; report the slowest device
    float best_a = 0, best_b = 0;
    bool any = false;
    for (const DeviceCtx *dv : f->devs) {
        float a = 0, b = 0;
        for (Shard *s : f->shards) {
            if (s->dev != dv || !s->n_cells) continue;
            if (!s->pred_timed) { g_last_err = "ggp_predict_profile: no completed ggp_predict"; return GGP_EINVAL; }
            HIPCHK(hipSetDevice(s->device));
            float x = 0, y = 0;
            HIPCHK(hipEventElapsedTime(&x, s->ev_pred[0], s->ev_pred[1]));
            HIPCHK(hipEventElapsedTime(&y, s->ev_pred[1], s->ev_pred[2]));
            a += x;
            b += y;
            any = true;
        }
        if (a + b > best_a + best_b) { best_a = a; best_b = b; }
    }
    if (!any) { g_last_err = "ggp_predict_profile: no completed ggp_predict"; return GGP_EINVAL; }
    if (ms_smooth) *ms_smooth = best_a;
    if (ms_combine) *ms_combine = best_b;
    return GGP_OK;
}

// -p: per device, its shards one after another through the device's forward/backward workspace;
// each shard's combined rows stay in HBM (ggp_predict_rows streams them)
int ggp_predict(ggp_forest *f, const double *params, int32_t n_seg, double *out_fwd, double *out_bwd,
                double *out_comb)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !params || n_seg < 1) { g_last_err = "ggp_predict: null params or n_seg < 1"; return GGP_EINVAL; }
    if (f->n_cells == 0) return GGP_OK;
    // ---- workspaces ----
    for (DeviceCtx *dv : f->devs) {
        int64_t need = 0;
        for (const Shard *s : f->shards)
            if (s->dev == dv) need = std::max(need, s->n_rows);
        if (need <= dv->sm_rows) continue;
        HIPCHK(hipSetDevice(dv->id));
        HIPCHK(hipStreamSynchronize(dv->stream));
        for (double **p : {&dv->sm_fwd, &dv->sm_bwd}) {
            if (*p) (void)hipFree(*p);
            *p = nullptr;
        }
        dv->sm_rows = 0;
        int rc = GGP_OK;
        auto check = [&](int r) { if (r != GGP_OK && rc == GGP_OK) rc = r; };
        check(dev_upload<double>(&dv->sm_fwd, nullptr, (size_t)need * 20));
        check(dev_upload<double>(&dv->sm_bwd, nullptr, (size_t)need * 20));
        if (rc != GGP_OK) {
            for (double **p : {&dv->sm_fwd, &dv->sm_bwd}) {
                if (*p) (void)hipFree(*p);
                *p = nullptr;
            }
            return rc;
        }
        dv->sm_rows = need;
    }
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        HIPCHK(hipSetDevice(s->device));
        if (!s->d_sm_pstate) {
            int rc = GGP_OK;
            auto check = [&](int r) { if (r != GGP_OK && rc == GGP_OK) rc = r; };
            check(dev_upload<double>(&s->d_sm_pstate, nullptr, (size_t)s->n_cells * 20));
            check(dev_upload<double>(&s->d_sm_comb, nullptr, (size_t)s->n_rows * 20));
            for (auto &ev : s->ev_pred)
                if (rc == GGP_OK && hipEventCreate(&ev) != hipSuccess) rc = GGP_EDEV;
            if (rc != GGP_OK) return rc;
        }
        if (n_seg > s->sm_ptab_cap) {
            HIPCHK(hipStreamSynchronize(s->stream));
            if (s->d_sm_ptab) (void)hipFree(s->d_sm_ptab);
            s->d_sm_ptab = nullptr;
            s->sm_ptab_cap = 0;
            const int rc = dev_upload<double>(&s->d_sm_ptab, nullptr, (size_t)n_seg * 11);
            if (rc != GGP_OK) return rc;
            s->sm_ptab_cap = n_seg;
        }
        s->pred_timed = false;
    }
    // ---- smoother + combine, shard by shard on each device (devices run concurrently) ----
    const bool direct = f->shards.size() == 1 && f->shards[0]->cell_g.empty();
    std::vector<double> stage;
    hipError_t e = hipSuccess;
    for (Shard *s : f->shards) {
        if (!s->n_cells || e != hipSuccess) continue;
        DeviceCtx *dv = s->dev;
        e = hipSetDevice(s->device);
        if (e == hipSuccess)
            e = hipMemcpyAsync(s->d_sm_ptab, params, (size_t)n_seg * 11 * sizeof(double), hipMemcpyHostToDevice,
                               s->stream);
        if (e == hipSuccess) e = hipEventRecord(s->ev_pred[0], s->stream);
        // the combine fused into the backward pass where every level runs the lane smoother (C5-sized
        // levels; the same rows bitwise), else k_combine after it
        const bool fuse = s->combine_fused && !s->combine_exact && smoother_all_lane(s);
        if (e == hipSuccess)
            e = run_smoother(s, s->d_sm_ptab, n_seg, s->d_sm_pstate, dv->sm_fwd, fuse && !out_bwd ? nullptr : dv->sm_bwd,
                             fuse ? s->d_sm_comb : nullptr);
        if (e == hipSuccess) e = hipEventRecord(s->ev_pred[1], s->stream);
        if (e == hipSuccess && !fuse) {
            const int64_t blocks = (s->n_rows + 255) / 256;
            auto *kc = s->combine_exact ? k_combine<false> : k_combine<true>;
            hipLaunchKernelGGL(kc, dim3((unsigned)blocks), dim3(256), 0, s->stream, s->d_sm_ptab, n_seg,
                               s->d_prior_seg, s->n_rows, dv->sm_fwd, dv->sm_bwd, s->d_sm_comb);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(s->ev_pred[2], s->stream);
        // forward / backward rows leave the shared workspace before the device's next shard
        const size_t bytes = (size_t)s->n_rows * 20 * sizeof(double);
        for (int which = 0; which < 2 && e == hipSuccess; ++which) {
            double *dst = which == 0 ? out_fwd : out_bwd;
            const double *src = which == 0 ? dv->sm_fwd : dv->sm_bwd;
            if (!dst) continue;
            if (direct) {
                e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s->stream);
            } else {
                stage.resize((size_t)s->n_rows * 20);
                e = hipMemcpyAsync(stage.data(), src, bytes, hipMemcpyDeviceToHost, s->stream);
                if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
                if (e == hipSuccess) scatter_rows(f, s, stage.data(), 0, s->n_rows, 20, dst, 0);
            }
        }
    }
    for (Shard *s : f->shards) {
        if (!s->n_cells || e != hipSuccess) continue;
        e = hipSetDevice(s->device);
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
        if (e == hipSuccess) s->pred_timed = true;
    }
    if (e != hipSuccess) {
        g_last_err = std::string("ggp_predict: ") + hipGetErrorString(e);
        return GGP_EDEV;
    }
    if (out_comb) return ggp_predict_rows(f, 0, f->n_rows, out_comb);
    return GGP_OK;
}

// combined rows [r_lo, r_hi) of the last ggp_predict (input order) -> out[(r - r_lo) * 20]
int ggp_predict_rows(ggp_forest *f, int64_t r_lo, int64_t r_hi, double *out)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !out || r_lo < 0 || r_hi > f->n_rows || r_hi < r_lo) {
        g_last_err = "ggp_predict_rows: bad arguments";
        return GGP_EINVAL;
    }
    std::vector<double> stage;
    for (Shard *s : f->shards) {
        if (!s->n_cells) continue;
        if (!s->pred_timed || !s->d_sm_comb) { g_last_err = "ggp_predict_rows: no completed ggp_predict"; return GGP_EINVAL; }
        int64_t l_lo, l_hi;
        local_rows(f, s, r_lo, r_hi, l_lo, l_hi);
        if (l_hi <= l_lo) continue;
        HIPCHK(hipSetDevice(s->device));
        const size_t bytes = (size_t)(l_hi - l_lo) * 20 * sizeof(double);
        if (s->cell_g.empty()) {
            HIPCHK(hipMemcpy(out + (l_lo - r_lo) * 20, s->d_sm_comb + l_lo * 20, bytes, hipMemcpyDeviceToHost));
            continue;
        }
        stage.resize((size_t)(l_hi - l_lo) * 20);
        HIPCHK(hipMemcpy(stage.data(), s->d_sm_comb + l_lo * 20, bytes, hipMemcpyDeviceToHost));
        scatter_rows(f, s, stage.data(), l_lo, l_hi, 20, out, r_lo);
    }
    return GGP_OK;
}

static int joints_impl(ggp_forest *f, const double *params, int32_t n_seg, double tol, int64_t r_lo, int64_t r_hi,
                       int64_t cap, int64_t *out_idx, double *out_val, int64_t *n_out, int width)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!f || !params || n_seg < 1 || !n_out) { g_last_err = "ggp_joints: bad arguments"; return GGP_EINVAL; }
    if (r_lo < 0) r_lo = 0;
    if (r_hi > f->n_rows) r_hi = f->n_rows;
    *n_out = 0;
    if (f->n_cells == 0 || r_hi <= r_lo) return GGP_OK;
    if (f->shards.size() == 1 && f->shards[0]->cell_g.empty())
        return shard_joints(f->shards[0], params, n_seg, tol, r_lo, r_hi, cap, out_idx, out_val, n_out, width);
    // several shards: every start row belongs to one; count first, then each shard's joints in
    // global numbering, merged by start row (each start's joints keep their add order)
    const size_t ns = f->shards.size();
    std::vector<int64_t> lo(ns), hi(ns), cnt(ns, 0);
    int64_t total = 0;
    for (size_t k = 0; k < ns; ++k) {
        local_rows(f, f->shards[k], r_lo, r_hi, lo[k], hi[k]);
        const int rc = shard_joints(f->shards[k], params, n_seg, tol, lo[k], hi[k], 0, nullptr, nullptr, &cnt[k], width);
        if (rc != GGP_OK) return rc;
        total += cnt[k];
    }
    *n_out = total;
    if (total == 0 || total > cap || !out_idx || !out_val) return GGP_OK;
    std::vector<int64_t> idx;
    std::vector<double> val;
    std::vector<std::pair<int64_t, int64_t>> order;   // (global start, position in idx/val)
    order.reserve((size_t)total);
    idx.reserve((size_t)total * 2);
    val.reserve((size_t)total * width);
    for (size_t k = 0; k < ns; ++k) {
        if (!cnt[k]) continue;
        std::vector<int64_t> li((size_t)cnt[k] * 2);
        std::vector<double> lv((size_t)cnt[k] * width);
        int64_t got = 0;
        const int rc = shard_joints(f->shards[k], params, n_seg, tol, lo[k], hi[k], cnt[k], li.data(), lv.data(), &got, width);
        if (rc != GGP_OK) return rc;
        for (int64_t q = 0; q < got; ++q) {
            const int64_t gs = g_row(f, f->shards[k], li[2 * q]), gt = g_row(f, f->shards[k], li[2 * q + 1]);
            order.emplace_back(gs, (int64_t)idx.size() / 2);
            idx.push_back(gs);
            idx.push_back(gt);
        }
        val.insert(val.end(), lv.begin(), lv.begin() + got * width);
    }
    std::stable_sort(order.begin(), order.end(),
                     [](const std::pair<int64_t, int64_t> &a, const std::pair<int64_t, int64_t> &b) { return a.first < b.first; });
    for (size_t q = 0; q < order.size(); ++q) {
        const int64_t p = order[q].second;
        out_idx[2 * q] = idx[2 * p];
        out_idx[2 * q + 1] = idx[2 * p + 1];
        std::memcpy(out_val + q * width, &val[(size_t)p * width], width * sizeof(double));
    }
    return GGP_OK;
}

int ggp_joints(ggp_forest *f, const double *params, int32_t n_seg, double tol, int64_t r_lo, int64_t r_hi,
               int64_t cap, int64_t *out_idx, double *out_val, int64_t *n_out)
{
    return joints_impl(f, params, n_seg, tol, r_lo, r_hi, cap, out_idx, out_val, n_out, kJStart);
}

int ggp_joints_packed(ggp_forest *f, const double *params, int32_t n_seg, double tol, int64_t r_lo, int64_t r_hi,
                      int64_t cap, int64_t *out_idx, double *out_val, int64_t *n_out)
{
    return joints_impl(f, params, n_seg, tol, r_lo, r_hi, cap, out_idx, out_val, n_out, kJPacked);
}

// ---- test-only device math (tests/test_gpu_device_math.py) --------------------------------
int ggp_debug_dawson(int32_t device, int32_t variant, const double *x, int64_t n, double *out)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!x || !out || n < 0 || variant < 0 || variant > 1) { g_last_err = "ggp_debug_dawson: bad arguments"; return GGP_EINVAL; }
    if (n == 0) return GGP_OK;
    HIPCHK(hipSetDevice(device));
    double *dx = nullptr, *dy = nullptr;
    int rc = dev_upload(&dx, x, (size_t)n);
    if (rc == GGP_OK) rc = dev_upload<double>(&dy, nullptr, (size_t)n);
    if (rc == GGP_OK) {
        hipLaunchKernelGGL(k_debug_dawson, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, dx, n, variant, dy);
        if (hipGetLastError() != hipSuccess || hipMemcpy(out, dy, (size_t)n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
            g_last_err = "ggp_debug_dawson: launch failed";
            rc = GGP_EDEV;
        }
    }
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    return rc;
}

int ggp_debug_tauint(int32_t device, const double *in, int64_t n, double *out)
{
    DeviceGuard device_guard_;   // the caller's current device is restored on return
    if (!in || !out || n < 0) { g_last_err = "ggp_debug_tauint: bad arguments"; return GGP_EINVAL; }
    for (int64_t i = 0; i < n; ++i)
        if (in[6 * i] < 0 || in[6 * i] > 3 || in[6 * i] != (double)(int)in[6 * i]) {
            g_last_err = "ggp_debug_tauint: k must be 0..3";
            return GGP_EINVAL;
        }
    if (n == 0) return GGP_OK;
    HIPCHK(hipSetDevice(device));
    double *di = nullptr, *dy = nullptr;
    int rc = dev_upload(&di, in, (size_t)n * 6);
    if (rc == GGP_OK) rc = dev_upload<double>(&dy, nullptr, (size_t)n);
    if (rc == GGP_OK) {
        hipLaunchKernelGGL(k_debug_tauint, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, di, n, dy);
        if (hipGetLastError() != hipSuccess || hipMemcpy(out, dy, (size_t)n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
            g_last_err = "ggp_debug_tauint: launch failed";
            rc = GGP_EDEV;
        }
    }
    if (di) (void)hipFree(di);
    if (dy) (void)hipFree(dy);
    return rc;
}

}  // extern "C"
