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

// Optional lookahead, called before each reflected point's call with that point and the points
// one of which the next call of the iteration may be -- expansion, outside contraction, inside
// contraction (NULL where that step would end the run instead).  An objective whose calls carry
// state can evaluate them ahead, each from the state the reflected point leaves; the sequence of
// calls, and so the trajectory, is unchanged.
using Lookahead = std::function<void(const double *first, const double *const *next, int n_next)>;

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
};

// nldrmd_minimize_ on the reduced problem (all lb < ub)
inline Result nldrmd(int n, const Objective &f, const double *lb, const double *ub, double *x, double *minf,
                     const double *xstep, double ftol_abs, long maxeval, Stats &st, const Lookahead *look = nullptr)
{
    const double alpha = 1, beta = 0.5, gamm = 2, delta = 0.5;
    const int w = n + 1;                                // row: f, x[0..n-1]
    std::vector<double> pts((size_t)(n + 1) * w), c(n), xcur(n);
    Result ret = SUCCESS;

    auto eval = [&](const double *xc, double *fc) -> Result {
        if (!f(xc, fc)) return FORCED_STOP;
        ++st.nevals;
        if (*fc <= *minf) {
            *minf = *fc;
            std::memcpy(x, xc, sizeof(double) * n);
        }
        if (maxeval > 0 && st.nevals >= maxeval) return MAXEVAL_REACHED;
        return SUCCESS;
    };
    // ordering of vertices: (f, index), the red-black tree's comparator
    auto less = [&](int a, int b) {
        const double fa = pts[(size_t)a * w], fb = pts[(size_t)b * w];
        if (fa < fb) return true;
        if (fa > fb) return false;
        return a < b;
    };

    std::memcpy(&pts[1], x, sizeof(double) * n);
    pts[0] = *minf;
    for (int i = 0; i < n; ++i) {
        double *pt = &pts[(size_t)(i + 1) * w];
        std::memcpy(pt + 1, x, sizeof(double) * n);
        pt[1 + i] += xstep[i];
        if (pt[1 + i] > ub[i]) {
            if (ub[i] - x[i] > std::fabs(xstep[i]) * 0.1)
                pt[1 + i] = ub[i];
            else
                pt[1 + i] = x[i] - std::fabs(xstep[i]);
        }
        if (pt[1 + i] < lb[i]) {
            if (x[i] - lb[i] > std::fabs(xstep[i]) * 0.1) {
                pt[1 + i] = lb[i];
            } else {
                pt[1 + i] = x[i] + std::fabs(xstep[i]);
                if (pt[1 + i] > ub[i]) pt[1 + i] = 0.5 * ((ub[i] - x[i] > x[i] - lb[i] ? ub[i] : lb[i]) + x[i]);
            }
        }
        if (close_pt(pt[1 + i], x[i])) return FAILURE;
        if ((ret = eval(pt + 1, &pt[0])) != SUCCESS) return ret;
    }

    for (;;) {
        // low, high and the vertex just below high
        int lo = 0, hi = 0;
        for (int i = 1; i <= n; ++i) {
            if (less(i, lo)) lo = i;
            if (less(hi, i)) hi = i;
        }
        int pred = -1;
        for (int i = 0; i <= n; ++i)
            if (i != hi && (pred < 0 || less(pred, i))) pred = i;
        const double fl = pts[(size_t)lo * w];
        double fh = pts[(size_t)hi * w];
        const double *xl = &pts[(size_t)lo * w + 1];
        double *xh = &pts[(size_t)hi * w + 1];

        // nlopt_stop_ftol(stop, fl, fh) with ftol_rel = 0
        if (!std::isinf(fh) && std::fabs(fl - fh) < ftol_abs) return FTOL_REACHED;

        std::fill(c.begin(), c.end(), 0.0);
        for (int i = 0; i <= n; ++i) {
            const double *xi = &pts[(size_t)i * w + 1];
            if (xi != xh)
                for (int j = 0; j < n; ++j) c[j] += xi[j];
        }
        const double ninv = 1.0 / n;
        for (int j = 0; j < n; ++j) c[j] *= ninv;
        // (nldrmd's x-tolerance test never fires with xtol_rel = xtol_abs = 0)

        if (!reflectpt(n, xcur.data(), c.data(), alpha, xh, lb, ub)) return XTOL_REACHED;
        if (look && *look) {   // the points the branches below would call next (same expressions)
            std::vector<double> xe(n), xo(n), xi(n);
            const bool ve = reflectpt(n, xe.data(), c.data(), gamm, xh, lb, ub);
            const bool vo = reflectpt(n, xo.data(), c.data(), beta, xh, lb, ub);
            const bool vi = reflectpt(n, xi.data(), c.data(), -beta, xh, lb, ub);
            const double *next[3] = {ve ? xe.data() : nullptr, vo ? xo.data() : nullptr, vi ? xi.data() : nullptr};
            (*look)(xcur.data(), next, 3);
        }
        double fr;
        if ((ret = eval(xcur.data(), &fr)) != SUCCESS) return ret;

        if (fr < fl) {   // expand
            if (!reflectpt(n, xh, c.data(), gamm, xh, lb, ub)) return XTOL_REACHED;
            if ((ret = eval(xh, &fh)) != SUCCESS) return ret;
            if (fh >= fr) {
                fh = fr;
                std::memcpy(xh, xcur.data(), sizeof(double) * n);
            }
        } else if (fr < pts[(size_t)pred * w]) {   // accept
            std::memcpy(xh, xcur.data(), sizeof(double) * n);
            fh = fr;
        } else {   // contract
            double fc;
            if (!reflectpt(n, xcur.data(), c.data(), fh <= fr ? -beta : beta, xh, lb, ub)) return XTOL_REACHED;
            if ((ret = eval(xcur.data(), &fc)) != SUCCESS) return ret;
            if (fc < fr && fc < fh) {
                std::memcpy(xh, xcur.data(), sizeof(double) * n);
                fh = fc;
            } else {   // shrink towards the best vertex, then restart (re-sort)
                for (int i = 0; i <= n; ++i) {
                    double *pt = &pts[(size_t)i * w];
                    if (pt + 1 != xl) {
                        if (!reflectpt(n, pt + 1, xl, -delta, pt + 1, lb, ub)) return XTOL_REACHED;
                        if ((ret = eval(pt + 1, &pt[0])) != SUCCESS) return ret;
                    }
                }
                continue;
            }
        }
        pts[(size_t)hi * w] = fh;
    }
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
    std::vector<std::vector<double>> lbuf(4, full);
    const Lookahead lr = [&](const double *first, const double *const *next, int n_next) {
        const double *fl[3] = {nullptr, nullptr, nullptr};
        for (int k = 0; k <= n_next && k < 4; ++k) {
            const double *src = k == 0 ? first : next[k - 1];
            if (!src) continue;
            for (int j = 0; j < nd; ++j) lbuf[k][free_dims[j]] = src[j];
            if (k > 0) fl[k - 1] = lbuf[k].data();
        }
        (*look)(lbuf[0].data(), fl, n_next < 3 ? n_next : 3);
    };
    // nldrmd_minimize: the starting point is evaluated first
    if (!fr(xr.data(), minf)) return FORCED_STOP;
    ++st.nevals;
    Result ret = SUCCESS;
    if (maxeval > 0 && st.nevals >= maxeval) {
        ret = MAXEVAL_REACHED;
    } else if (nd > 0) {
        ret = nldrmd(nd, fr, lbr.data(), ubr.data(), xr.data(), minf, dxr.data(), ftol_abs, maxeval, st,
                     look && *look ? &lr : nullptr);
    }
    for (int j = 0; j < nd; ++j) full[free_dims[j]] = xr[j];
    std::memcpy(x, full.data(), sizeof(double) * n);
    return ret;
}

}  // namespace ggp_nm
