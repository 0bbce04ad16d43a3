"""Diagnostic: Forest.total_likelihood (ctypes) on a one-tree forest -- the Python floor of one
evaluation call -- beside tools/launch_latency's C++ numbers.  Median of 2000 calls."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (bench.py's process: torch's HIP runtime)
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
f = g.Forest(g.HostForest.synthetic(1, 4))
for _ in range(50):
    f.total_likelihood(P)
t = []
for _ in range(2000):
    a = time.perf_counter()
    f.total_likelihood(P)
    t.append(time.perf_counter() - a)
t.sort()
print(f"Forest.total_likelihood, 1 tree x 4 rows (python, torch runtime) {1e6 * t[len(t) // 2]:7.2f} us")
