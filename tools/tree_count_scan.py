"""C2-shaped forests at several tree counts and rows per tree, wave path launch: ms per
evaluation (median of 40 after 5 warm-ups) and us per critical-path step (3P/4 rows).
Separates the per-step latency (few trees: one wave per SIMD throughout) from the issue
contention of two active waves per SIMD (>= ~1024 trees of 200 rows: root and daughter paths
of different trees share a SIMD in the last P/4 rows).

  python3 tools/tree_count_scan.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def t_eval(trees, rows, reps=40):
    hf = g.HostForest.synthetic(trees, rows)
    f = g.Forest(hf, kernel="auto")
    for _ in range(5):
        f.total_likelihood(P)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f.total_likelihood(P)
        ts.append(time.perf_counter() - t0)
    f.close()
    return float(np.median(ts)) * 1e3


shapes = [(t, 200) for t in (64, 256, 512, 768, 960, 1000, 1024, 1100, 1300, 1600, 2000)]
shapes += [(1000, r) for r in (8, 40, 100, 400)] + [(500, r) for r in (8, 40, 100, 200, 400)]
for trees, rows in shapes:
    ms = t_eval(trees, rows)
    crit = 3 * rows // 4
    print(f"trees={trees:5d} rows/tree={rows:4d} ms={ms:8.4f} us/crit-step={1e3 * ms / crit:7.3f} "
          f"updates/s={trees * rows / ms * 1e3:9.3e}", flush=True)
