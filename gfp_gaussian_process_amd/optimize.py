"""The -m / -s layer over an objective: the reference's minimizer_nlopt.h and the error bars
of likelihood.h, with the numerics in libggp_host.so (include/ggp_host.h):

  nldrmd_minimize        NLopt 2.7.1 LN_NELDERMEAD (restated, csrc/host/ggp_nelder_mead.h)
  minimize_wrapper       minimize_wrapper / minimize_wrapper_log_params  minimizer_nlopt.h:10-215
  num_hessian            num_hessian_ll                                    likelihood.h:211-258
  num_hessian_batched    the same points in one ggp_total_loglik_batch call (opt-in, unchained)
  inverse_pplu           Eigen MatrixXd::inverse (partial-pivot LU)
  ll_error_bars          ll_error_bars                                     likelihood.h:260-268
  bound_1dscan           run_bound_1dscan                                  main.cpp:80-114

The objective is any callable params(11) -> +log-likelihood that raises LikelihoodIsNan on a
NaN -- in the product a gfp_gaussian_process_amd.Forest (GPU); in CPU tests the oracle.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

from . import _native as N
from .forest import Forest, ParameterSet

# nlopt_result
FAILURE, INVALID_ARGS, FORCED_STOP = -1, -2, -5
SUCCESS, FTOL_REACHED, XTOL_REACHED, MAXEVAL_REACHED = 1, 3, 4, 5


class _Stop(Exception):
    pass


def _callback(f, n, errors: list):
    def cb(xp, vp, _data):
        if errors:   # a lookahead callback failed: stop the run there (re-raised by the caller)
            return 1
        try:
            vp[0] = float(f(np.ctypeslib.as_array(xp, shape=(n,)).copy()))
            return 0
        except BaseException as e:   # re-raised by the caller after the C side unwinds
            errors.append(e)
            return 1
    return N.OBJECTIVE_FN(cb)


def nldrmd_minimize(f, x0, lb, ub, dx, ftol_abs: float, maxeval: int = 0, ahead=None):
    """minimise f over the box [lb, ub] (lb == ub: a fixed dimension); returns
    (x_best, f_best, result_code, n_evaluations).  An exception raised by f stops the run
    and propagates (the reference's NaN path).  ahead: an _Ahead (the lookahead of a stateful
    objective, ggp_nldrmd_minimize_ahead) -- the same calls and result."""
    x = np.ascontiguousarray(x0, np.float64).copy()
    n = x.size
    lb, ub, dx = (np.ascontiguousarray(v, np.float64) for v in (lb, ub, dx))
    errors: list = []
    cb = _callback(f, n, errors)
    minf = ctypes.c_double()
    nev = ctypes.c_int64()
    dp = lambda a: a.ctypes.data_as(N.c_double_p)  # noqa: E731
    if ahead is None:
        rc = N.host().ggp_nldrmd_minimize(n, cb, None, dp(lb), dp(ub), dp(x), dp(dx), ftol_abs, maxeval,
                                          ctypes.byref(minf), ctypes.byref(nev))
    else:
        need, tree = ahead.callbacks(n, errors)
        rc = N.host().ggp_nldrmd_minimize_ahead(n, cb, need, tree, None, dp(lb), dp(ub), dp(x), dp(dx), ftol_abs,
                                                maxeval, ctypes.byref(minf), ctypes.byref(nev), 0, 0)
    if errors:
        raise errors[0]
    return x, minf.value, rc, nev.value


class _Ahead:
    """The optimiser's lookahead for a Forest objective (include/ggp_host.h
    ggp_nldrmd_minimize_ahead): the run's possible next calls evaluated in one
    ggp_total_loglik_tree launch, each from the state its parent call leaves; call() serves the
    real calls from them while they match (bitwise parameters, from the node last served), else
    evaluates as usual.  to_params: the optimiser's point -> the objective's parameters."""

    def __init__(self, forest, to_params):
        self.f, self.to_params = forest, to_params
        self.active, self.off, self.cur = False, False, -1
        self.keys, self.pred, self.res = [], [], None

    def node(self, p) -> int:
        if not self.active:
            return -1
        key = np.ascontiguousarray(p, np.float64).tobytes()
        for k, (kk, pk) in enumerate(zip(self.keys, self.pred)):
            if pk == self.cur and kk == key:
                return k
        return -1

    def callbacks(self, n, errors):
        def need(xp, _data):
            try:
                return int(self.node(self.to_params(np.ctypeslib.as_array(xp, shape=(n,)).copy())) < 0)
            except BaseException as e:
                errors.append(e)
                return 1

        def tree(xp, predp, n_pts, _data):
            try:
                self.active = False
                if self.off:
                    return
                xs = np.ctypeslib.as_array(xp, shape=(n_pts, n))
                pts = np.stack([self.to_params(xs[k].copy()) for k in range(n_pts)])
                pred = np.ctypeslib.as_array(predp, shape=(n_pts,)).copy()
                r = self.f.total_likelihood_tree(pts, pred)
                if r is None:   # no path launch on this handle: call by call
                    self.off = True
                    return
                self.keys = [np.ascontiguousarray(p).tobytes() for p in pts]
                self.pred, self.res, self.cur, self.active = list(pred), r, -1, True
            except BaseException as e:
                errors.append(e)
                self.off = True
        self._cbs = (N.AHEAD_NEED_FN(need), N.AHEAD_TREE_FN(tree))   # kept alive for the run
        return self._cbs

    def call(self, params) -> float:
        k = self.node(params)
        # a node whose speculative launch stalled (GGP_ETIMEOUT: the lookahead's schedule, not the
        # call) is not served: the call runs as usual from the carried state, the last node served
        if k >= 0 and int(self.res[1][k]) == N.GGP_ETIMEOUT:
            k = -1
        if k < 0:
            self.active = False
            return self.f.total_likelihood(params)
        self.cur = k
        self.f.keep_point_state(k)
        ll, st, nc, nr = (a[k] for a in self.res)
        if st == N.GGP_ENAN:
            raise self.f._nan(int(nc), int(nr))
        self.f._stalled(int(st))
        self.f._check(int(st))
        return float(ll)


def minimize_wrapper(objective, params: ParameterSet, tolerance: float = 1e-10, search_space: str = "log",
                     start=None, maxeval: int = 0):
    """maximise objective(params) over the non-fixed parameters (minimizer_nlopt.h:10-215);
    returns (final parameter vector, maximal log-likelihood, nlopt result).  maxeval > 0 stops
    after that many evaluations (MAXEVAL_REACHED; the reference sets none)"""
    log = search_space == "log"
    init = np.asarray(params.init, np.float64)
    start = init if start is None else np.asarray(start, np.float64)
    lb, ub, dx, x = (np.zeros(11) for _ in range(4))
    ln = (lambda v: float(np.log(np.float64(v)))) if log else float   # log(0) = -inf, as in C
    with np.errstate(divide="ignore"):
        for i, kind in enumerate(params.kind):
            x[i] = ln(start[i])
            if kind == "fixed":
                dx[i] = 1.0
                lb[i] = ub[i] = ln(init[i])
            else:
                dx[i] = math.log(1.0 + params.step[i] / init[i]) if log else params.step[i]
                lb[i] = ln(params.lower[i])
                ub[i] = ln(params.upper[i])
    to_params = (lambda v: np.exp(v)) if log else (lambda v: v)
    forest = _chain_forest(objective)
    ahead = None
    if forest is not None and os.environ.get("GGP_NM_LOOKAHEAD", "1") != "0":
        ahead = _Ahead(forest, to_params)   # a Forest: the lookahead (the same calls)
        objective = ahead.call
    f = lambda v: -objective(to_params(v))  # noqa: E731
    xb, minf, rc, _ = nldrmd_minimize(f, x, lb, ub, dx, tolerance, maxeval, ahead)
    if rc == INVALID_ARGS:
        raise ValueError("nlopt invalid argument")
    if rc == FAILURE:
        raise RuntimeError("nlopt failure")
    return (np.exp(xb) if log else xb), -minf, rc


def _chain_forest(objective):
    """the Forest behind an objective that is a Forest or its bound total_likelihood (whose
    known call sequences can run as one ggp_total_loglik_chain call), else None.  Only the
    Forest's own total_likelihood qualifies: a subclass that overrides it (a prior, a logging
    wrapper) is called one call at a time, so every call goes through the override."""
    if isinstance(objective, Forest):
        return objective if type(objective).total_likelihood is Forest.total_likelihood else None
    owner = getattr(objective, "__self__", None)
    if isinstance(owner, Forest) and getattr(objective, "__func__", None) is Forest.total_likelihood:
        return owner
    return None


def num_hessian(objective, x, idx, epsilon: float) -> np.ndarray:
    """num_hessian_ll (likelihood.h:211-258): H[i, j] = (l++ - l+- - l-+ + l--) / (4 h_i h_j) over
    its 4 k^2 calls in its order, each from the carried state the previous left.  A Forest
    objective runs them as one chained call (bitwise the call-by-call form, ggp_num_hessian)."""
    forest = _chain_forest(objective)
    if forest is not None:
        pts, h = hessian_points(x, idx, epsilon)
        q = forest.total_likelihood_chain(pts).reshape(len(h), len(h), 4)
        out = np.zeros((len(h), len(h)))
        for i in range(len(h)):
            for j in range(len(h)):
                out[i, j] = (q[i, j, 0] - q[i, j, 1] - q[i, j, 2] + q[i, j, 3]) / (4 * h[i] * h[j])
        return out
    x = np.ascontiguousarray(x, np.float64)
    idx32 = np.ascontiguousarray(idx, np.int32)
    k = idx32.size
    out = np.zeros((k, k))
    errors: list = []
    cb = _callback(objective, x.size, errors)
    rc = N.host().ggp_num_hessian(x.size, cb, None, x.ctypes.data_as(N.c_double_p),
                                  idx32.ctypes.data_as(N.c_int32_p), k, epsilon,
                                  out.ctypes.data_as(N.c_double_p))
    if errors:
        raise errors[0]
    if rc != N.GGP_OK:
        raise RuntimeError("ggp_num_hessian failed")
    return out


def hessian_points(x, idx, epsilon: float):
    """the 4 k^2 parameter points num_hessian_ll visits (likelihood.h:211-258), in its order
    (i, j, then ++, +-, -+, --), with its steps h = max(x epsilon, 1e-12); returns (points
    [4 k^2, n], h [k])"""
    x = np.asarray(x, np.float64)
    idx = [int(i) for i in idx]
    h = np.array([max(x[i] * epsilon, 1e-12) for i in idx])
    pts = []
    for a, ii in enumerate(idx):
        for b, jj in enumerate(idx):
            for s1, s2 in ((1, 1), (1, -1), (-1, 1), (-1, -1)):
                xx = x.copy()
                xx[ii] = xx[ii] + h[a] if s1 > 0 else xx[ii] - h[a]
                xx[jj] = xx[jj] + h[b] if s2 > 0 else xx[jj] - h[b]
                pts.append(xx)
    return np.array(pts), h


def num_hessian_batched(forest, x, idx, epsilon: float) -> np.ndarray:
    """opt-in batched num_hessian_ll: the 4 k^2 points in ONE ggp_total_loglik_batch call, each
    from the carried state as it is now (the reference chains the state from call to call, so
    its values differ by that carried state).  Same steps and the same
    (l++ - l+- - l-+ + l--) / (4 h1 h2) expression as num_hessian."""
    from .forest import LikelihoodIsNan
    pts, h = hessian_points(x, idx, epsilon)
    ll, nan = forest.total_likelihood_batch(pts)
    if nan.any():
        raise LikelihoodIsNan(-1, -1)
    k = len(h)
    q = ll.reshape(k, k, 4)
    out = np.zeros((k, k))
    for i in range(k):
        for j in range(k):
            out[i, j] = (q[i, j, 0] - q[i, j, 1] - q[i, j, 2] + q[i, j, 3]) / (4 * h[i] * h[j])
    return out


def inverse_pplu(a) -> np.ndarray:
    a = np.ascontiguousarray(a, np.float64)
    out = np.zeros_like(a)
    N.host().ggp_inverse_pplu(a.shape[0], a.ctypes.data_as(N.c_double_p), out.ctypes.data_as(N.c_double_p))
    return out


def ll_error_bars(objective, x_final, params: ParameterSet, epsilon: float, batched: bool = False) -> np.ndarray:
    """squared error bars -diag(H^-1) of the non-fixed parameters (likelihood.h:260-268);
    batched=True evaluates the Hessian's points in one batch (objective: a Forest)"""
    if batched:
        h = num_hessian_batched(objective, x_final, params.non_fixed(), epsilon)
    else:
        h = num_hessian(objective, x_final, params.non_fixed(), epsilon)
    return -np.diag(inverse_pplu(h))


def arange(start: float, stop: float, step: float) -> list:
    """utils.h arange: accumulate value += step (not start + i*step)"""
    out, v = [], start
    while v < stop:
        out.append(v)
        v += step
    return out


def bound_1dscan(objective, params: ParameterSet, final=None) -> dict:
    """run_bound_1dscan (main.cpp:80-114): for every bound parameter, evaluate the objective
    along arange(lower, upper, step) with the others at their final (else init) values.
    Returns {name: [(value, log_likelihood), ...]} in evaluation order."""
    base = np.asarray(params.init if final is None else final, np.float64)
    forest = _chain_forest(objective)   # a Forest: each parameter's calls as one chained call
    out = {}
    for i in params.bound():
        pv = base.copy()
        vals = arange(params.lower[i], params.upper[i], params.step[i])
        if forest is not None:
            pts = np.repeat(pv[None, :], len(vals), axis=0)
            pts[:, i] = vals
            out[params.names[i]] = list(zip(vals, forest.total_likelihood_chain(pts).tolist()))
            continue
        rows = []
        for v in vals:
            pv[i] = v
            rows.append((v, objective(pv.copy())))
        out[params.names[i]] = rows
    return out
