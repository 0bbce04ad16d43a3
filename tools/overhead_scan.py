"""Per-launch overhead of the wave schedule (diagnostic): level times of C2-shaped forests with
1000 trees and growing rows per tree; a linear fit of level time against steps per cell gives
the per-step cost and the fixed cost of a level launch (prologue, table load, launch gap)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
trees = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
kern = sys.argv[2] if len(sys.argv) > 2 else "wave"
pts = []
for rows in (8, 20, 40, 100, 200, 400):
    f = g.Forest(g.HostForest.synthetic(trees, rows), kernel=kern)
    for _ in range(3):
        f.total_likelihood(P)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        f.total_likelihood(P)
    dt = (time.perf_counter() - t0) / reps
    f.enable_profile()
    lv = []
    for _ in range(5):
        f.total_likelihood(P)
        lv.append(f.launch_profile()[0])
    ms = np.median(np.array(lv), axis=0)
    print(f"rows/tree={rows}: {1e3 * dt:.4f} ms/eval, levels " + " ".join(f"{m:.4f}" for m in ms), flush=True)
    pts.append((rows, ms))
    f.close()
for lvl, steps_of in ((0, lambda r: r // 2), (1, lambda r: r // 4)):
    x = np.array([steps_of(r) for r, _ in pts], float)
    y = np.array([m[lvl] for _, m in pts]) * 1e3
    A = np.vstack([x, np.ones_like(x)]).T
    s, c = np.linalg.lstsq(A, y, rcond=None)[0]
    print(f"level {lvl}: {s:.3f} us per step + {c:.1f} us per launch")
