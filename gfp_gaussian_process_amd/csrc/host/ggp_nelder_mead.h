// ggp_nelder_mead.h -- the -m optimiser: a restatement of NLopt 2.7.1's LN_NELDERMEAD.
//
// The reference drives NLopt (README.md:58-61 pins 2.7.1; src/minimizer_nlopt.h:112-215 sets
// lower/upper bounds, the initial step, ftol_abs and LN_NELDERMEAD).  NLopt is neither in
// /root/reference nor in this image, so this is a restatement of its published algorithm
// (nldrmd.c, Nelder-Mead with Richardson-Kuester bound pinning, plus optimize.c's handling
// of lb == ub dimensions) and the parity of the trajectory against NLopt is unpinned
// (DESIGN.md).  What is restated:
//
//   * dimensions with lb == ub are eliminated before the simplex is built (NLopt's
//     "elimdim" wrapping for LN_NELDERMEAD) and re-inserted for every evaluation;
//   * initial simplex x + step_i e_i, with the step turned back inside the bounds the way
//     nldrmd does it; a vertex that coincides with x fails (NLOPT_FAILURE);
//   * reflection alpha = 1, expansion 2, contraction 1/2 (inside when the reflected point is
//     no better than the worst), shrink 1/2 towards the best vertex, every new point pinned
//     to [lb, ub]; a step whose new point coincides with the centroid or the old point ends
//     the run with NLOPT_XTOL_REACHED;
//   * vertices ordered by (f, vertex index) -- nldrmd's red-black tree breaks ties by
//     address, i.e. by index;
//   * ftol_abs stop |f_high - f_low| < ftol_abs checked once per iteration;
//   * the best point seen (f <= minf) is returned.
#pragma once
#include <cmath>
#include <algorithm>
#include <cstring>
#include <functional>
#include <vector>

namespace ggp_nm {

enum Result {   // nlopt_result values
    FAILURE = -1, INVALID_ARGS = -2, FORCED_STOP = -5,
    SUCCESS = 1, FTOL_REACHED = 3, XTOL_REACHED = 4, MAXEVAL_REACHED = 5
};

// f(x, &value) -> false to force a stop (the reference's objective throws on a NaN)
using Objective = std::function<bool(const double *x, double *value)>;

inline bool close_pt(double a, double b) { return std::fabs(a - b) <= 1e-13 * (std::fabs(a) + std::fabs(b)); }

// xnew = c + scale (c - xold), pinned to the bounds; false if xnew coincides with c or xold
inline bool reflectpt(int n, double *xnew, const double *c, double scale, const double *xold, const double *lb,
                      const double *ub)
{
    bool equalc = true, equalold = true;
    for (int i = 0; i < n; ++i) {
        double v = c[i] + scale * (c[i] - xold[i]);
        if (v < lb[i]) v = lb[i];
        if (v > ub[i]) v = ub[i];
        equalc = equalc && close_pt(v, c[i]);
        equalold = equalold && close_pt(v, xold[i]);
        xnew[i] = v;
    }
    return !(equalc || equalold);
}

struct Stats {
    long nevals = 0;
    long iterations = 0, expansions = 0, accepts = 0, contractions = 0, shrinks = 0;   // diagnostics
};

// nldrmd_minimize_ on the reduced problem (all lb < ub) as a resumable machine: pending() is the
// point whose objective value the run needs next, feed(f) gives it and advances to the next call
// (or to the end).  The machine is a value (copyable), so a driver can run copies ahead on values
// it does not know yet (speculation) without touching the real run.
class Machine {
public:
    Machine(int n, const double *lb, const double *ub, const double *x, double minf, const double *xstep,
            double ftol_abs, long maxeval, long nevals)
        : n_(n), w_(n + 1), lb_(lb, lb + n), ub_(ub, ub + n), xstep_(xstep, xstep + n), x_(x, x + n),
          pts_((size_t)(n + 1) * (n + 1)), c_(n), xcur_(n), minf_(minf), ftol_(ftol_abs), maxeval_(maxeval)
    {
        st_.nevals = nevals;
        std::memcpy(&pts_[1], x, sizeof(double) * n);
        pts_[0] = minf;
        start_vertex(0);
    }
    bool done() const { return ph_ == DONE; }
    Result result() const { return res_; }
    const double *pending() const
    {
        switch (ph_) {
        case VERTEX: return &pts_[(size_t)(vi_ + 1) * w_ + 1];
        case SHRINK: return &pts_[(size_t)vi_ * w_ + 1];
        case EXPANDED: return &pts_[(size_t)hi_ * w_ + 1];
        default: return xcur_.data();
        }
    }
    const double *best_x() const { return x_.data(); }
    double minf() const { return minf_; }
    const Stats &stats() const { return st_; }
    // the objective values the next transition compares the fed value with, directly or later
    // through the vertex order (every vertex's, the reflected point's)
    std::vector<double> thresholds() const
    {
        std::vector<double> t;
        for (int i = 0; i <= n_; ++i) t.push_back(pts_[(size_t)i * w_]);
        if (ph_ == EXPANDED || ph_ == CONTRACTED) t.push_back(fr_);
        t.push_back(minf_);
        return t;
    }

    void feed(double f)
    {
        switch (ph_) {
        case VERTEX:
            pts_[(size_t)(vi_ + 1) * w_] = f;
            if (!book(pending(), f)) return;
            if (++vi_ < n_)
                start_vertex(vi_);
            else
                start_iteration();
            return;
        case REFLECTED:
            fr_ = f;
            if (!book(xcur_.data(), f)) return;
            if (fr_ < fl_) {   // expand
                ++st_.expansions;
                double *xh = &pts_[(size_t)hi_ * w_ + 1];
                if (!reflectpt(n_, xh, c_.data(), kGamma, xh, lb_.data(), ub_.data())) return finish(XTOL_REACHED);
                ph_ = EXPANDED;
            } else if (fr_ < pts_[(size_t)pred_ * w_]) {   // accept
                ++st_.accepts;
                std::memcpy(&pts_[(size_t)hi_ * w_ + 1], xcur_.data(), sizeof(double) * n_);
                pts_[(size_t)hi_ * w_] = fr_;
                start_iteration();
            } else {   // contract (inside when the reflected point is no better than the worst)
                ++st_.contractions;
                if (!reflectpt(n_, xcur_.data(), c_.data(), fh_ <= fr_ ? -kBeta : kBeta, &pts_[(size_t)hi_ * w_ + 1],
                               lb_.data(), ub_.data()))
                    return finish(XTOL_REACHED);
                ph_ = CONTRACTED;
            }
            return;
        case EXPANDED: {
            double *xh = &pts_[(size_t)hi_ * w_ + 1];
            if (!book(xh, f)) return;
            double fh = f;
            if (fh >= fr_) {
                fh = fr_;
                std::memcpy(xh, xcur_.data(), sizeof(double) * n_);
            }
            pts_[(size_t)hi_ * w_] = fh;
            start_iteration();
            return;
        }
        case CONTRACTED:
            if (!book(xcur_.data(), f)) return;
            if (f < fr_ && f < fh_) {
                std::memcpy(&pts_[(size_t)hi_ * w_ + 1], xcur_.data(), sizeof(double) * n_);
                pts_[(size_t)hi_ * w_] = f;
                start_iteration();
            } else {   // shrink towards the best vertex, then restart (re-sort)
                ++st_.shrinks;
                start_shrink(0);
            }
            return;
        case SHRINK:
            pts_[(size_t)vi_ * w_] = f;
            if (!book(pending(), f)) return;
            start_shrink(vi_ + 1);
            return;
        default:
            return;
        }
    }

private:
    static constexpr double kAlpha = 1, kBeta = 0.5, kGamma = 2, kDelta = 0.5;
    enum Phase { VERTEX, REFLECTED, EXPANDED, CONTRACTED, SHRINK, DONE };
    int n_, w_;
    std::vector<double> lb_, ub_, xstep_, x_, pts_, c_, xcur_;   // pts_ rows: f, x[0..n-1]
    double minf_, ftol_;
    long maxeval_;
    Stats st_;
    Phase ph_ = VERTEX;
    Result res_ = SUCCESS;
    int vi_ = 0, lo_ = 0, hi_ = 0, pred_ = 0;
    double fl_ = 0, fh_ = 0, fr_ = 0;

    void finish(Result r)
    {
        res_ = r;
        ph_ = DONE;
    }
    // an objective value came in (nldrmd's CHECK_EVAL): count, keep the best point, stop at maxeval
    bool book(const double *xc, double f)
    {
        ++st_.nevals;
        if (f <= minf_) {
            minf_ = f;
            std::memcpy(x_.data(), xc, sizeof(double) * n_);
        }
        if (maxeval_ > 0 && st_.nevals >= maxeval_) {
            finish(MAXEVAL_REACHED);
            return false;
        }
        return true;
    }
    // vertex i + 1 of the initial simplex: x (as it is then -- a vertex that improves on minf moves
    // it) with coordinate i stepped, turned back inside the bounds the way nldrmd does it
    void start_vertex(int i)
    {
        double *v = &pts_[(size_t)(i + 1) * w_ + 1];
        const double *x = x_.data();
        std::memcpy(v, x, sizeof(double) * n_);
        v[i] += xstep_[i];
        if (v[i] > ub_[i]) {
            if (ub_[i] - x[i] > std::fabs(xstep_[i]) * 0.1)
                v[i] = ub_[i];
            else
                v[i] = x[i] - std::fabs(xstep_[i]);
        }
        if (v[i] < lb_[i]) {
            if (x[i] - lb_[i] > std::fabs(xstep_[i]) * 0.1) {
                v[i] = lb_[i];
            } else {
                v[i] = x[i] + std::fabs(xstep_[i]);
                if (v[i] > ub_[i]) v[i] = 0.5 * ((ub_[i] - x[i] > x[i] - lb_[i] ? ub_[i] : lb_[i]) + x[i]);
            }
        }
        if (close_pt(v[i], x[i])) return finish(FAILURE);
        vi_ = i;
        ph_ = VERTEX;
    }
    // ordering of vertices: (f, index), the red-black tree's comparator
    bool less(int a, int b) const
    {
        const double fa = pts_[(size_t)a * w_], fb = pts_[(size_t)b * w_];
        if (fa < fb) return true;
        if (fa > fb) return false;
        return a < b;
    }
    void start_iteration()
    {
        lo_ = 0;
        hi_ = 0;   // low, high and the vertex just below high
        for (int i = 1; i <= n_; ++i) {
            if (less(i, lo_)) lo_ = i;
            if (less(hi_, i)) hi_ = i;
        }
        pred_ = -1;
        for (int i = 0; i <= n_; ++i)
            if (i != hi_ && (pred_ < 0 || less(pred_, i))) pred_ = i;
        fl_ = pts_[(size_t)lo_ * w_];
        fh_ = pts_[(size_t)hi_ * w_];
        // nlopt_stop_ftol(stop, fl, fh) with ftol_rel = 0
        if (!std::isinf(fh_) && std::fabs(fl_ - fh_) < ftol_) return finish(FTOL_REACHED);
        std::fill(c_.begin(), c_.end(), 0.0);
        for (int i = 0; i <= n_; ++i)
            if (i != hi_)
                for (int j = 0; j < n_; ++j) c_[j] += pts_[(size_t)i * w_ + 1 + j];
        const double ninv = 1.0 / n_;
        for (int j = 0; j < n_; ++j) c_[j] *= ninv;
        // (nldrmd's x-tolerance test never fires with xtol_rel = xtol_abs = 0)
        if (!reflectpt(n_, xcur_.data(), c_.data(), kAlpha, &pts_[(size_t)hi_ * w_ + 1], lb_.data(), ub_.data()))
            return finish(XTOL_REACHED);
        ++st_.iterations;
        ph_ = REFLECTED;
    }
    // the shrink's calls: every vertex but the best, moved halfway to it, from vertex i on
    void start_shrink(int i)
    {
        const double *xl = &pts_[(size_t)lo_ * w_ + 1];
        for (; i <= n_; ++i) {
            if (i == lo_) continue;
            double *pt = &pts_[(size_t)i * w_ + 1];
            if (!reflectpt(n_, pt, xl, -kDelta, pt, lb_.data(), ub_.data())) return finish(XTOL_REACHED);
            vi_ = i;
            ph_ = SHRINK;
            return;
        }
        start_iteration();
    }
};

// Speculation (optional).  An objective whose calls carry state (each call starts from the state
// the previous one left) can evaluate the run's next calls ahead: a tree of points, each to be
// evaluated from the state its parent leaves, covering the calls the run can make next whatever
// the values turn out to be -- machine copies fed one value from every interval between the
// objective values the next transitions compare with, up to `depth` calls ahead and `max_nodes`
// points.  need(x): the objective cannot serve the call x from what it evaluated ahead; tree():
// evaluate these points ahead (x: the points, pred: each one's parent, -1 = the next call).
// The sequence of calls, and so the trajectory, is unchanged.
struct Lookahead {
    std::function<bool(const double *x)> need;
    std::function<void(const std::vector<std::vector<double>> &x, const std::vector<int> &pred)> tree;
    int depth = 2, max_nodes = 40;   // measured on the example: profiles/r30_example_mp_lookahead_sweep*.json
};

inline void speculate(const Machine &m, int n, const Lookahead &look, std::vector<std::vector<double>> &pts,
                      std::vector<int> &pred)
{
    pts.clear();
    pred.clear();
    if (m.done()) return;
    struct Item {
        Machine m;
        int node;
    };
    std::vector<Item> level{{m, 0}};
    pts.emplace_back(m.pending(), m.pending() + n);
    pred.push_back(-1);
    for (int d = 1; d <= look.depth && !level.empty(); ++d) {
        std::vector<Item> next;
        std::vector<std::vector<double>> npts;
        std::vector<int> npred;
        for (const Item &it : level) {
            std::vector<double> t = it.m.thresholds();
            std::vector<double> v;
            for (double x : t)
                if (std::isfinite(x)) v.push_back(x);
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
            std::vector<double> reps;
            if (v.empty()) {
                reps.push_back(0.0);
            } else {
                reps.push_back(v.front() - 1.0 - std::fabs(v.front()));
                for (size_t k = 0; k + 1 < v.size(); ++k) reps.push_back(v[k] + 0.5 * (v[k + 1] - v[k]));
                reps.push_back(v.back() + 1.0 + std::fabs(v.back()));
            }
            for (double r : reps) {
                Machine c = it.m;
                c.feed(r);
                if (c.done()) continue;
                const double *p = c.pending();
                int node = -1;   // the same point under the same parent: one node
                for (size_t k = 0; k < npts.size() && node < 0; ++k)
                    if (npred[k] == it.node && std::memcmp(npts[k].data(), p, sizeof(double) * n) == 0)
                        node = (int)(pts.size() + k);
                if (node < 0) {
                    node = (int)(pts.size() + npts.size());
                    npts.emplace_back(p, p + n);
                    npred.push_back(it.node);
                }
                next.push_back({c, node});
            }
        }
        if (pts.size() + npts.size() > (size_t)look.max_nodes) break;
        for (size_t k = 0; k < npts.size(); ++k) {
            pts.push_back(npts[k]);
            pred.push_back(npred[k]);
        }
        level.swap(next);
    }
}

// the run: calls the objective for each pending point, speculating when the objective cannot
// serve the next call from what it evaluated ahead
inline Result nldrmd(int n, const Objective &f, const double *lb, const double *ub, double *x, double *minf,
                     const double *xstep, double ftol_abs, long maxeval, Stats &st, const Lookahead *look = nullptr)
{
    Machine m(n, lb, ub, x, *minf, xstep, ftol_abs, maxeval, st.nevals);
    std::vector<std::vector<double>> sp;
    std::vector<int> spred;
    Result r = SUCCESS;
    while (!m.done()) {
        if (look && look->need && look->tree && look->need(m.pending())) {
            speculate(m, n, *look, sp, spred);
            look->tree(sp, spred);
        }
        double v;
        if (!f(m.pending(), &v)) {
            r = FORCED_STOP;
            break;
        }
        m.feed(v);
    }
    if (m.done()) r = m.result();
    st = m.stats();
    std::memcpy(x, m.best_x(), sizeof(double) * n);
    *minf = m.minf();
    return r;
}

// nlopt_optimize for LN_NELDERMEAD: bound check, elimdim, first evaluation, nldrmd
inline Result minimize(int n, const Objective &f, const double *lb, const double *ub, double *x, const double *dx,
                       double ftol_abs, long maxeval, double *minf, Stats &st, const Lookahead *look = nullptr)
{
    for (int i = 0; i < n; ++i)
        if (lb[i] > ub[i] || x[i] < lb[i] || x[i] > ub[i]) return INVALID_ARGS;
    std::vector<int> free_dims;
    for (int i = 0; i < n; ++i)
        if (lb[i] != ub[i]) free_dims.push_back(i);
    const int nd = (int)free_dims.size();
    std::vector<double> full(x, x + n);
    std::vector<double> xr(nd), lbr(nd), ubr(nd), dxr(nd);
    for (int j = 0; j < nd; ++j) {
        const int i = free_dims[j];
        xr[j] = x[i];
        lbr[j] = lb[i];
        ubr[j] = ub[i];
        dxr[j] = dx[i];
    }
    for (int i = 0; i < n; ++i)
        if (lb[i] == ub[i]) full[i] = lb[i];
    std::vector<double> buf(full);
    const Objective fr = [&](const double *xd, double *v) {
        for (int j = 0; j < nd; ++j) buf[free_dims[j]] = xd[j];
        return f(buf.data(), v);
    };
    // the lookahead in full coordinates (the eliminated dimensions re-inserted)
    Lookahead lr;
    if (look) {
        lr.depth = look->depth;
        lr.max_nodes = look->max_nodes;
        lr.need = [&](const double *xd) {
            std::vector<double> v(full);
            for (int j = 0; j < nd; ++j) v[free_dims[j]] = xd[j];
            return look->need(v.data());
        };
        lr.tree = [&](const std::vector<std::vector<double>> &xs, const std::vector<int> &pred) {
            std::vector<std::vector<double>> fx(xs.size(), full);
            for (size_t k = 0; k < xs.size(); ++k)
                for (int j = 0; j < nd; ++j) fx[k][free_dims[j]] = xs[k][j];
            look->tree(fx, pred);
        };
    }
    // nldrmd_minimize: the starting point is evaluated first
    if (!fr(xr.data(), minf)) return FORCED_STOP;
    ++st.nevals;
    Result ret = SUCCESS;
    if (maxeval > 0 && st.nevals >= maxeval) {
        ret = MAXEVAL_REACHED;
    } else if (nd > 0) {
        ret = nldrmd(nd, fr, lbr.data(), ubr.data(), xr.data(), minf, dxr.data(), ftol_abs, maxeval, st,
                     look ? &lr : nullptr);
    }
    for (int j = 0; j < nd; ++j) full[free_dims[j]] = xr[j];
    std::memcpy(x, full.data(), sizeof(double) * n);
    return ret;
}

}  // namespace ggp_nm
