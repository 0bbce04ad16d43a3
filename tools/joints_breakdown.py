"""Where the -j leg's time goes (diagnostic): 20 C5-shaped trees x 500 tp, every start row.
  wrapper   Forest.joints per 2,048-row range (fresh output arrays per call, as bench.py)
  reuse     ggp_joints per range into one preallocated, already-touched pair of host arrays
  whole     ggp_joints over all start rows in one call (preallocated)
  count     ggp_joints over all start rows with cap 0 (the counting walk only)
Prints one JSON line of seconds."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gfp_gaussian_process_amd as g  # noqa: E402
from gfp_gaussian_process_amd import _native as N  # noqa: E402

P = np.ascontiguousarray(np.atleast_2d([2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04,
                                        3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]), np.float64)
hf = g.HostForest.synthetic(20, 500, seed=20261015, first_tree=2 * 10 ** 6)
f = g.Forest(hf)
nr = hf.n_rows
f.joints(P, 1e-10, 0, 256, cap=1 << 20)   # warm-up: smoother tables cached
L, h = f._lib, f._h
cap = 1 << 21
idx = np.ones((cap, 2), np.int64)
val = np.ones((cap, 72))
n = ctypes.c_int64()


def call(lo, hi, c):
    rc = L.ggp_joints(h, P.ctypes.data_as(N.c_double_p), 1, 1e-10, lo, hi, c, idx.ctypes.data_as(N.c_int64_p),
                      val.ctypes.data_as(N.c_double_p), ctypes.byref(n))
    assert rc == 0, rc
    return n.value


out = {"rows": nr}
for rep in range(2):
    t0 = time.perf_counter()
    tot = 0
    for lo in range(0, nr, 2048):
        tot += len(f.joints(P, 1e-10, lo, min(nr, lo + 2048), cap=cap)[0])
    out["wrapper"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tot2 = sum(call(lo, min(nr, lo + 2048), cap) for lo in range(0, nr, 2048))
    out["reuse"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tot3 = call(0, nr, cap)
    out["whole"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    tot4 = call(0, nr, 0)
    out["count"] = time.perf_counter() - t0
out["joints"] = [tot, tot2, tot3, tot4]
out["bytes_d2h"] = tot3 * (72 * 8 + 16)
print(json.dumps(out), flush=True)
