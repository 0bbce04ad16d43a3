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

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "ggp.h"
#include "ggp_device.h"

#define GGP_VERSION "ggp-mi355x 0.1.0 (reference gfp_gaussian_process 0.4.2)"

namespace {

struct DevForest {
    const double *time, *logl, *fp;
    const int64_t *row_off;
    const int32_t *parent, *d1, *d2, *seg;
    double root_mean0, root_mean1, root_var0, root_var1;
    double leaf_mean0, leaf_var0, leaf_mean1, leaf_var1;
    double fp_auto, two_log_2pi, log2;
    int scaled, binomial;
};

constexpr int kNanNone = 0x7fffffff;

// ------------------------------------------------------------------------------------------
// likelihood, one lane per cell.  sc_likelihood (likelihood.h:36-103) for every cell of
// one generation depth.  `cpw` cells per 64-lane wave: < 64 spreads a small level over
// more SIMDs (latency), 64 packs waves (throughput); results do not depend on it.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_loglik_level(DevForest F, ggp_params P,
                                                      const int32_t *__restrict__ cells, int n,
                                                      int cpw, double *__restrict__ state,
                                                      double *__restrict__ cell_ll,
                                                      int32_t *__restrict__ cell_nan)
{
    const int lane = threadIdx.x;
    if (lane >= cpw) return;
    const int i = blockIdx.x * cpw + lane;
    if (i >= n) return;
    const int c = cells[i];
    const double *p = P.p;
    double m[4], C[16];
    double *st = state + (size_t)20 * c;
    const int64_t r0 = F.row_off[c], r1 = F.row_off[c + 1];
    const int par = F.parent[c];
    if (par < 0) {
        // init_sc_distribution root branch (predictions.h:63-78): the off-diagonals keep
        // this root's state from the previous evaluation (carried state)
#pragma unroll
        for (int k = 0; k < 16; ++k) C[k] = st[4 + k];
        m[0] = F.root_mean0;
        m[1] = F.root_mean1;
        C[0] = F.root_var0;
        C[5] = F.root_var1;
        m[2] = p[0];
        m[3] = p[3];
        C[10] = p[2] / (2. * p[1]);
        C[15] = p[5] / (2. * p[4]);
    } else {
        const double *ps = state + (size_t)20 * par;
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = ps[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) C[k] = ps[4 + k];
        const double dt = F.time[r0] - F.time[F.row_off[par + 1] - 1];
        ggp_after_division(m, C, dt, P, F.binomial, F.log2);
    }
    double cl = 0.0;
    int nan_row = kNanNone;
    double tn = F.time[r0], xn = F.logl[r0], gn = F.fp[r0];
    for (int64_t r = r0; r < r1; ++r) {
        const double tc = tn, x = xn, g = gn;
        if (r + 1 < r1) {   // prefetch the next row while this one computes
            tn = F.time[r + 1];
            xn = F.logl[r + 1];
            gn = F.fp[r + 1];
        }
        const double x0 = x - m[0];
        const double x1 = g - m[1];
        ggp_innov v;
        ggp_innovation(m, C, p[7], p[8], F.scaled, F.fp_auto, v);
        const double term = ggp_ll_term(x0, x1, v, F.two_log_2pi);
        cl += term;
        if (cl != cl) {
            nan_row = (int)(r - r0);
            break;
        }
        ggp_posterior(m, C, x0, x1, v);
        if (r + 1 < r1) ggp_propagate(m, C, tn - tc, p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) st[k] = m[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) st[4 + k] = C[k];
    cell_ll[c] = cl;
    cell_nan[c] = nan_row;
}

// ------------------------------------------------------------------------------------------
// Deterministic total: sum cell_ll in DFS pre-order (the reference's accumulation order at
// cell granularity) with a fixed-shape tree; first NaN = min over (dfs rank, row).
// ------------------------------------------------------------------------------------------
constexpr int kRedThreads = 1024;

__global__ __launch_bounds__(kRedThreads) void k_reduce(const int32_t *__restrict__ dfs_order, int64_t n,
                                                         const double *__restrict__ cell_ll,
                                                         const int32_t *__restrict__ cell_nan,
                                                         double *__restrict__ out_ll,
                                                         int64_t *__restrict__ out_nan)
{
    __shared__ double s_sum[kRedThreads];
    __shared__ long long s_nan[kRedThreads];
    const int tid = threadIdx.x;
    const int64_t lo = n * tid / kRedThreads, hi = n * (tid + 1) / kRedThreads;
    double acc = 0.0;
    long long first = 0x7fffffffffffffffLL;
    for (int64_t i = lo; i < hi; ++i) {
        const int c = dfs_order[i];
        acc += cell_ll[c];
        const int nr = cell_nan[c];
        if (nr != kNanNone && first == 0x7fffffffffffffffLL) first = (i << 24) | (long long)nr;
    }
    s_sum[tid] = acc;
    s_nan[tid] = first;
    __syncthreads();
    for (int w = kRedThreads / 2; w > 0; w >>= 1) {
        if (tid < w) {
            s_sum[tid] = s_sum[tid] + s_sum[tid + w];
            s_nan[tid] = min(s_nan[tid], s_nan[tid + w]);
        }
        __syncthreads();
    }
    if (tid == 0) {
        out_ll[0] = s_sum[0];
        out_nan[0] = s_nan[0];
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
thread_local std::string g_last_err;

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

}  // namespace

struct ggp_forest {
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t n_cells = 0, n_rows = 0;
    int n_cu = 256;
    int kernel_pref = GGP_KERNEL_AUTO;
    int kernel_used = GGP_KERNEL_LANE;
    DevForest F{};
    // device buffers
    double *d_time = nullptr, *d_logl = nullptr, *d_fp = nullptr;
    int64_t *d_row_off = nullptr;
    int32_t *d_parent = nullptr, *d_d1 = nullptr, *d_d2 = nullptr, *d_seg = nullptr;
    int32_t *d_level_cells = nullptr, *d_dfs_order = nullptr;
    double *d_state = nullptr, *d_cell_ll = nullptr;
    int32_t *d_cell_nan = nullptr;
    double *d_out_ll = nullptr;
    int64_t *d_out_nan = nullptr;
    // pinned host result
    double *h_out_ll = nullptr;
    int64_t *h_out_nan = nullptr;
    // schedule
    std::vector<int64_t> level_start;       // [n_levels+1] into level_cells
    std::vector<int32_t> h_dfs_order;
    // profiling
    bool profile = false;
    std::vector<hipEvent_t> ev;
    std::vector<int64_t> ev_rows;
    int n_prof = 0;
};

static int launch_levels(ggp_forest *f, const ggp_params &P)
{
    const int n_levels = (int)f->level_start.size() - 1;
    f->n_prof = 0;
    for (int L = 0; L < n_levels; ++L) {
        const int64_t a = f->level_start[L], b = f->level_start[L + 1];
        const int n = (int)(b - a);
        if (n <= 0) continue;
        // spread small levels: aim for >= 4 waves per CU before packing lanes
        const int64_t target_waves = (int64_t)f->n_cu * 8;
        int cpw = (int)std::min<int64_t>(64, std::max<int64_t>(1, (n + target_waves - 1) / target_waves));
        const int blocks = (n + cpw - 1) / cpw;
        if (f->profile && 2 * (f->n_prof + 1) <= (int)f->ev.size()) {
            HIPCHK(hipEventRecord(f->ev[2 * f->n_prof], f->stream));
        }
        hipLaunchKernelGGL(k_loglik_level, dim3(blocks), dim3(64), 0, f->stream, f->F, P,
                           f->d_level_cells + a, n, cpw, f->d_state, f->d_cell_ll, f->d_cell_nan);
        HIPCHK(hipGetLastError());
        if (f->profile && 2 * (f->n_prof + 1) <= (int)f->ev.size()) {
            HIPCHK(hipEventRecord(f->ev[2 * f->n_prof + 1], f->stream));
            int64_t rows = 0;
            // rows of this level (host copy of offsets kept implicitly via ev_rows)
            rows = f->ev_rows.empty() ? 0 : f->ev_rows[L];
            (void)rows;
            f->n_prof++;
        }
    }
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kRedThreads), 0, f->stream, f->d_dfs_order,
                       f->n_cells, f->d_cell_ll, f->d_cell_nan, f->d_out_ll, f->d_out_nan);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(f->h_out_ll, f->d_out_ll, sizeof(double), hipMemcpyDeviceToHost, f->stream));
    HIPCHK(hipMemcpyAsync(f->h_out_nan, f->d_out_nan, sizeof(int64_t), hipMemcpyDeviceToHost, f->stream));
    return GGP_OK;
}

extern "C" {

const char *ggp_strerror(int code)
{
    switch (code) {
    case GGP_OK: return "ok";
    case GGP_EINVAL: return g_last_err.empty() ? "invalid argument" : g_last_err.c_str();
    case GGP_ENAN: return "Likelihood is Nan";
    case GGP_EDEV: return g_last_err.empty() ? "HIP device error" : g_last_err.c_str();
    case GGP_ENOMEM: return "device allocation failed";
    default: return "unknown error";
    }
}

const char *ggp_version(void) { return GGP_VERSION; }

int ggp_device_count(int32_t *n)
{
    int c = 0;
    HIPCHK(hipGetDeviceCount(&c));
    *n = c;
    return GGP_OK;
}

void ggp_forest_destroy(ggp_forest *f)
{
    if (!f) return;
    (void)hipSetDevice(f->device);
    if (f->stream) (void)hipStreamSynchronize(f->stream);
    for (void *p : {(void *)f->d_time, (void *)f->d_logl, (void *)f->d_fp, (void *)f->d_row_off,
                    (void *)f->d_parent, (void *)f->d_d1, (void *)f->d_d2, (void *)f->d_seg,
                    (void *)f->d_level_cells, (void *)f->d_dfs_order, (void *)f->d_state,
                    (void *)f->d_cell_ll, (void *)f->d_cell_nan, (void *)f->d_out_ll,
                    (void *)f->d_out_nan})
        if (p) (void)hipFree(p);
    if (f->h_out_ll) (void)hipHostFree(f->h_out_ll);
    if (f->h_out_nan) (void)hipHostFree(f->h_out_nan);
    for (auto &e : f->ev) (void)hipEventDestroy(e);
    if (f->stream) (void)hipStreamDestroy(f->stream);
    delete f;
}

int ggp_forest_create(const ggp_forest_desc *d, ggp_forest **out)
{
    if (!d || !out) { g_last_err = "null argument"; return GGP_EINVAL; }
    *out = nullptr;
    const int64_t nc = d->n_cells, nr = d->n_rows;
    if (nc < 0 || nr < 0 || (nc > 0 && (!d->row_offset || !d->parent || !d->daughter1 || !d->daughter2)) ||
        (nr > 0 && (!d->time || !d->log_length || !d->fp))) {
        g_last_err = "incomplete forest descriptor";
        return GGP_EINVAL;
    }
    if (nc >= (int64_t)1 << 31 || nr >= (int64_t)1 << 40) { g_last_err = "forest too large"; return GGP_EINVAL; }
    // ---- validate topology on the host (bad indices would fault on the device) ----
    if (nc > 0 && (d->row_offset[0] != 0 || d->row_offset[nc] != nr)) {
        g_last_err = "row_offset must start at 0 and end at n_rows";
        return GGP_EINVAL;
    }
    for (int64_t c = 0; c < nc; ++c) {
        if (d->row_offset[c + 1] <= d->row_offset[c]) { g_last_err = "every cell needs >= 1 row"; return GGP_EINVAL; }
        for (int32_t v : {d->parent[c], d->daughter1[c], d->daughter2[c]})
            if (v < -1 || v >= nc || v == c) { g_last_err = "genealogy index out of range"; return GGP_EINVAL; }
    }
    // ---- generation depth (iterative, parents may follow children in input order) ----
    std::vector<int32_t> depth(nc, -1);
    std::vector<int32_t> dfs;
    dfs.reserve(nc);
    {
        std::vector<int32_t> stack;
        for (int64_t r = 0; r < nc; ++r) {
            if (d->parent[r] != -1) continue;
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
        for (int64_t c = 0; c < nc; ++c)
            if (depth[c] < 0) { g_last_err = "cell not reachable from a root (cycle)"; return GGP_EINVAL; }
        // a daughter's parent pointer must be the cell that lists it (single-parent forest)
        for (int64_t c = 0; c < nc; ++c)
            for (int32_t ch : {d->daughter1[c], d->daughter2[c]})
                if (ch >= 0 && d->parent[ch] != c) {
                    g_last_err = "daughter/parent pointers disagree";
                    return GGP_EINVAL;
                }
    }
    auto *f = new ggp_forest();
    f->device = d->device;
    f->n_cells = nc;
    f->n_rows = nr;
    f->kernel_pref = d->kernel;
    if (hipSetDevice(d->device) != hipSuccess) {
        g_last_err = "hipSetDevice failed";
        delete f;
        return GGP_EDEV;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d->device) == hipSuccess) f->n_cu = prop.multiProcessorCount;
    int rc = GGP_OK;
    auto check = [&](int r) { if (r != GGP_OK && rc == GGP_OK) rc = r; };
    check(hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking) == hipSuccess ? GGP_OK : GGP_EDEV);
    // ---- level schedule ----
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
    f->h_dfs_order = dfs;
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
    check(dev_upload(&f->d_dfs_order, dfs.data(), nc));
    check(dev_upload<double>(&f->d_state, nullptr, (size_t)nc * 20));
    check(dev_upload<double>(&f->d_cell_ll, nullptr, nc));
    check(dev_upload<int32_t>(&f->d_cell_nan, nullptr, nc));
    check(dev_upload<double>(&f->d_out_ll, nullptr, 1));
    check(dev_upload<int64_t>(&f->d_out_nan, nullptr, 1));
    if (rc == GGP_OK && nc > 0 && hipMemset(f->d_state, 0, (size_t)nc * 20 * sizeof(double)) != hipSuccess) rc = GGP_EDEV;
    if (rc == GGP_OK && hipHostMalloc((void **)&f->h_out_ll, sizeof(double)) != hipSuccess) rc = GGP_ENOMEM;
    if (rc == GGP_OK && hipHostMalloc((void **)&f->h_out_nan, sizeof(int64_t)) != hipSuccess) rc = GGP_ENOMEM;
    if (rc != GGP_OK) {
        ggp_forest_destroy(f);
        return rc;
    }
    DevForest &F = f->F;
    F.time = f->d_time; F.logl = f->d_logl; F.fp = f->d_fp;
    F.row_off = f->d_row_off; F.parent = f->d_parent; F.d1 = f->d_d1; F.d2 = f->d_d2; F.seg = f->d_seg;
    F.root_mean0 = d->root_mean_xg[0]; F.root_mean1 = d->root_mean_xg[1];
    F.root_var0 = d->root_var_xg[0]; F.root_var1 = d->root_var_xg[1];
    F.leaf_mean0 = d->leaf_mean_xg[0]; F.leaf_mean1 = d->leaf_mean_xg[1];
    F.leaf_var0 = d->leaf_var_xg[0]; F.leaf_var1 = d->leaf_var_xg[1];
    F.fp_auto = d->fp_auto;
    F.two_log_2pi = 2 * std::log(2 * M_PI);
    F.log2 = std::log(2.);
    F.scaled = d->noise_scaled ? 1 : 0;
    F.binomial = d->division_binomial ? 1 : 0;
    // per-level rows for the roofline bookkeeping
    f->ev_rows.assign(f->level_start.size() - 1, 0);
    for (size_t L = 0; L + 1 < f->level_start.size(); ++L)
        for (int64_t i = f->level_start[L]; i < f->level_start[L + 1]; ++i) {
            int32_t c = level_cells[i];
            f->ev_rows[L] += d->row_offset[c + 1] - d->row_offset[c];
        }
    *out = f;
    return GGP_OK;
}

int ggp_reset_state(ggp_forest *f)
{
    if (!f) return GGP_EINVAL;
    HIPCHK(hipSetDevice(f->device));
    if (f->n_cells) HIPCHK(hipMemsetAsync(f->d_state, 0, (size_t)f->n_cells * 20 * sizeof(double), f->stream));
    HIPCHK(hipStreamSynchronize(f->stream));
    return GGP_OK;
}

int ggp_get_state(ggp_forest *f, double *out)
{
    if (!f || !out) return GGP_EINVAL;
    HIPCHK(hipSetDevice(f->device));
    HIPCHK(hipStreamSynchronize(f->stream));
    if (f->n_cells) HIPCHK(hipMemcpy(out, f->d_state, (size_t)f->n_cells * 20 * sizeof(double), hipMemcpyDeviceToHost));
    return GGP_OK;
}

int ggp_total_loglik_async(ggp_forest *f, const double *params)
{
    if (!f || !params) return GGP_EINVAL;
    HIPCHK(hipSetDevice(f->device));
    ggp_params P;
    std::memcpy(P.p, params, sizeof P.p);
    if (f->n_cells == 0) {
        *f->h_out_ll = 0.0;
        *f->h_out_nan = 0x7fffffffffffffffLL;
        return GGP_OK;
    }
    return launch_levels(f, P);
}

int ggp_loglik_result(ggp_forest *f, double *ll, int64_t *nan_cell, int64_t *nan_row)
{
    if (!f) return GGP_EINVAL;
    HIPCHK(hipStreamSynchronize(f->stream));
    const double v = *f->h_out_ll;
    const int64_t code = *f->h_out_nan;
    if (ll) *ll = v;
    if (nan_cell) *nan_cell = -1;
    if (nan_row) *nan_row = -1;
    if (code != 0x7fffffffffffffffLL) {
        const int64_t rank = code >> 24, row = code & 0xffffff;
        if (nan_cell) *nan_cell = f->h_dfs_order[rank];
        if (nan_row) *nan_row = row;
        if (ll) *ll = std::nan("");
        return GGP_ENAN;
    }
    if (std::isnan(v)) {   // NaN from +inf + -inf across cells (see include/ggp.h)
        if (ll) *ll = v;
        return GGP_ENAN;
    }
    return GGP_OK;
}

int ggp_total_loglik(ggp_forest *f, const double *params, double *ll, int64_t *nan_cell, int64_t *nan_row)
{
    int rc = ggp_total_loglik_async(f, params);
    if (rc != GGP_OK) return rc;
    return ggp_loglik_result(f, ll, nan_cell, nan_row);
}

int ggp_last_launch_profile(ggp_forest *f, float *ms, int64_t *rows, int32_t cap, int32_t *n)
{
    if (!f || !n) return GGP_EINVAL;
    if (!f->profile) {
        // enable for subsequent calls: one event pair per level
        const size_t need = 2 * (f->level_start.size() - 1);
        f->ev.resize(need);
        for (auto &e : f->ev) HIPCHK(hipEventCreate(&e));
        f->profile = true;
        *n = 0;
        return GGP_OK;
    }
    HIPCHK(hipStreamSynchronize(f->stream));
    int k = 0;
    for (int L = 0; L < f->n_prof && k < cap; ++L, ++k) {
        float t = 0;
        HIPCHK(hipEventElapsedTime(&t, f->ev[2 * L], f->ev[2 * L + 1]));
        if (ms) ms[k] = t;
        if (rows) rows[k] = f->ev_rows[L];
    }
    *n = k;
    return GGP_OK;
}

int ggp_forest_info(ggp_forest *f, int64_t *n_levels, int64_t *max_level_cells, int32_t *kernel_used)
{
    if (!f) return GGP_EINVAL;
    int64_t mx = 0;
    for (size_t L = 0; L + 1 < f->level_start.size(); ++L)
        mx = std::max(mx, f->level_start[L + 1] - f->level_start[L]);
    if (n_levels) *n_levels = (int64_t)f->level_start.size() - 1;
    if (max_level_cells) *max_level_cells = mx;
    if (kernel_used) *kernel_used = f->kernel_used;
    return GGP_OK;
}

int ggp_predict(ggp_forest *f, const double *params, int32_t n_seg, double *out_fwd, double *out_bwd,
                double *out_comb)
{
    (void)f; (void)params; (void)n_seg; (void)out_fwd; (void)out_bwd; (void)out_comb;
    g_last_err = "ggp_predict: not built in this version";
    return GGP_EINVAL;
}

}  // extern "C"
