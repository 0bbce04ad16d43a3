"""ctypes front-end of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by
the product package.  See ggp_oracle.h for what is restated from where and the pinning
status ("parity unpinned" for the Eigen-dependent part: the reference cannot be built
here without Eigen 3.3.7).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
LIB_SENS = os.path.join(HERE, "liboracle_sens.so")
REF_FADDEEVA = os.path.join(HERE, "_ref", "libfaddeeva_ref.so")


class OraForest(ctypes.Structure):
    _fields_ = [("n_cells", ctypes.c_int64), ("n_rows", ctypes.c_int64),
                ("row_off", ctypes.c_void_p), ("parent", ctypes.c_void_p), ("d1", ctypes.c_void_p),
                ("d2", ctypes.c_void_p), ("time", ctypes.c_void_p), ("log_length", ctypes.c_void_p),
                ("fp", ctypes.c_void_p), ("segment", ctypes.c_void_p),
                ("root_mean_xg", ctypes.c_double * 2), ("root_var_xg", ctypes.c_double * 2),
                ("leaf_mean_xg", ctypes.c_double * 2), ("leaf_var_xg", ctypes.c_double * 2),
                ("noise_scaled", ctypes.c_int), ("div_binomial", ctypes.c_int), ("fp_auto", ctypes.c_double)]


_lib = None
_libs = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(sens: bool = False):
    """the oracle library; sens=True: the build with the exp-ulp conditioning probe"""
    global _lib
    if sens:
        if "sens" not in _libs:
            if not os.path.exists(LIB_SENS):
                build()
            _libs["sens"] = _bind(ctypes.CDLL(LIB_SENS))
            _libs["sens"].ora_set_exp_ulp_noise.argtypes = [ctypes.c_uint64]
            _libs["sens"].ora_set_exp_ulp_noise.restype = None
        return _libs["sens"]
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = _bind(ctypes.CDLL(LIB))
    return _lib


def _bind(L):
    dp = ctypes.POINTER(ctypes.c_double)
    L.ora_dawson.restype = ctypes.c_double
    L.ora_dawson.argtypes = [ctypes.c_double]
    L.ora_tauint.restype = ctypes.c_double
    L.ora_tauint.argtypes = [ctypes.c_int] + [ctypes.c_double] * 5
    L.ora_mean_cov_model.restype = None
    L.ora_mean_cov_model.argtypes = [dp, dp, ctypes.c_double, dp]
    L.ora_cross_cov_model.restype = None
    L.ora_cross_cov_model.argtypes = [dp, dp, ctypes.c_double, dp, dp]
    L.ora_total_loglik.restype = ctypes.c_double
    L.ora_total_loglik.argtypes = [ctypes.POINTER(OraForest), dp, dp,
                                   ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), dp]
    L.ora_predict.restype = ctypes.c_int
    L.ora_predict.argtypes = [ctypes.POINTER(OraForest), dp, ctypes.c_int, dp, dp, dp, dp]
    L.ora_joints.restype = ctypes.c_int64
    L.ora_joints.argtypes = [ctypes.POINTER(OraForest), dp, ctypes.c_int, dp, dp, dp, ctypes.c_double,
                             ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                             ctypes.POINTER(ctypes.c_int64), dp]
    return L


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def make_forest(a: dict) -> OraForest:
    """a: the arrays dict of gfp_gaussian_process_amd.HostForest (.a)"""
    f = OraForest()
    keep = {k: np.ascontiguousarray(a[k]) for k in
            ("row_offset", "parent", "daughter1", "daughter2", "time", "log_length", "fp", "segment")}
    f._keep = keep
    f.n_cells = len(keep["parent"])
    f.n_rows = len(keep["time"])
    f.row_off = keep["row_offset"].ctypes.data
    f.parent = keep["parent"].ctypes.data
    f.d1 = keep["daughter1"].ctypes.data
    f.d2 = keep["daughter2"].ctypes.data
    f.time = keep["time"].ctypes.data
    f.log_length = keep["log_length"].ctypes.data
    f.fp = keep["fp"].ctypes.data
    f.segment = keep["segment"].ctypes.data if len(keep["segment"]) else None
    f.root_mean_xg[:] = list(a["root_mean_xg"])
    f.root_var_xg[:] = list(a["root_var_xg"])
    f.leaf_mean_xg[:] = list(a["leaf_mean_xg"])
    f.leaf_var_xg[:] = list(a["leaf_var_xg"])
    f.noise_scaled = int(a["noise_scaled"])
    f.div_binomial = int(a["division_binomial"])
    f.fp_auto = float(a["fp_auto"])
    return f


class OracleForest:
    """CPU oracle over the same arrays, with its own carried state."""

    def __init__(self, arrays: dict, exp_ulp_noise: int = 0, ref_dawson: bool = False):
        """exp_ulp_noise != 0: run on the conditioning-probe build with exp() moved +-1 ulp at
        random (seeded) -- tells a test which outputs rounding alone can move.
        ref_dawson: every Dawson value from the reference's own Faddeeva::Dawson (Faddeeva.cc,
        compiled in place into oracle/_ref; build container only) instead of the restatement's
        table -- the likelihood then runs the reference's own Dawson arithmetic"""
        self.f = make_forest(arrays)
        self._noise = int(exp_ulp_noise)
        self._ref_dawson = bool(ref_dawson)
        if self._ref_dawson and faddeeva_ref() is None:
            raise FileNotFoundError(f"{REF_FADDEEVA} is missing: `make -C oracle ref` (needs /root/reference)")
        self.state = np.zeros((self.f.n_cells, 20))
        self.cell_ll = np.zeros(self.f.n_cells)

    def _L(self):
        if not self._noise and not self._ref_dawson:
            return lib()
        L = lib(sens=True)
        L.ora_set_exp_ulp_noise(self._noise)    # re-seeded per call: deterministic (0: exact exp)
        hook = ctypes.c_void_p.in_dll(L, "ora_dawson_hook")
        hook.value = ctypes.cast(faddeeva_ref(), ctypes.c_void_p).value if self._ref_dawson else None
        return L

    def total_likelihood(self, params):
        p = np.ascontiguousarray(params, np.float64)
        nc, nr = ctypes.c_int64(), ctypes.c_int64()
        v = self._L().ora_total_loglik(ctypes.byref(self.f), _dp(p), _dp(self.state), ctypes.byref(nc),
                                   ctypes.byref(nr), _dp(self.cell_ll))
        return v, nc.value, nr.value

    def reset_state(self):
        self.state[:] = 0.0

    def predict(self, params_per_segment):
        p = np.ascontiguousarray(np.atleast_2d(params_per_segment), np.float64)
        st = np.zeros((self.f.n_cells, 20))
        out = [np.zeros((self.f.n_rows, 20)) for _ in range(3)]
        self._L().ora_predict(ctypes.byref(self.f), _dp(p), p.shape[0], _dp(st), *(_dp(o) for o in out))
        self.after_predict = st          # MOMAdata::mean/cov after -p (the backward final states)
        return tuple(out)

    def joints(self, params_per_segment, tol=1e-10, r_lo=0, r_hi=None, cap=1 << 20):
        """-j for start rows [r_lo, r_hi): (idx [k, 2] = (start, target), val [k, 72])"""
        p = np.ascontiguousarray(np.atleast_2d(params_per_segment), np.float64)
        key = p.tobytes()
        if getattr(self, "_joint_smooth_key", None) != key:   # the smoother once per parameters
            fwd, bwd, _ = self.predict(p)
            self._joint_smooth = (fwd, bwd, self.after_predict.copy())
            self._joint_smooth_key = key
        fwd, bwd, after = self._joint_smooth
        r_hi = self.f.n_rows if r_hi is None else r_hi
        idx = np.zeros((cap, 2), np.int64)
        val = np.zeros((cap, 72))
        n = self._L().ora_joints(ctypes.byref(self.f), _dp(p), p.shape[0], _dp(fwd), _dp(bwd), _dp(after),
                             tol, r_lo, r_hi, cap, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), _dp(val))
        if n > cap:
            raise ValueError(f"{n} joints > cap {cap}")
        return idx[:n], val[:n]


def dawson(x: float) -> float:
    return lib().ora_dawson(float(x))


def tauint(k: int, a: float, b: float, c: float, t1: float, t0: float = 0.0) -> float:
    return lib().ora_tauint(k, a, b, c, t1, t0)


def mean_cov_model(mean, cov, t: float, p7):
    m = np.ascontiguousarray(mean, np.float64).copy()
    C = np.ascontiguousarray(cov, np.float64).reshape(16).copy()
    p = np.ascontiguousarray(p7, np.float64)
    lib().ora_mean_cov_model(_dp(m), _dp(C), float(t), _dp(p))
    return m, C.reshape(4, 4)


_faddeeva = None


def faddeeva_ref():
    """Faddeeva::Dawson(double) of the reference's own Faddeeva.cc, compiled in place into
    oracle/_ref by `make -C oracle ref` (only where /root/reference exists)."""
    global _faddeeva
    if _faddeeva is None:
        if not os.path.exists(REF_FADDEEVA):
            return None
        L = ctypes.CDLL(REF_FADDEEVA)
        fn = L._ZN8Faddeeva6DawsonEd
        fn.restype = ctypes.c_double
        fn.argtypes = [ctypes.c_double]
        _faddeeva = fn
    return _faddeeva
