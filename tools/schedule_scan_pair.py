"""The wave / lane-pair crossover on the final lane bodies (diagnostic): C2-shaped forests of growing
size, ms per evaluation and per level launch for the wave schedule, the lane-pair schedule and auto
(the wave schedule up to 5 cells per SIMD, then lane-pair).  python tools/schedule_scan_pair.py [TREES...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
for n in [int(x) for x in sys.argv[1:]] or [1000, 1500, 2000, 2500, 3000, 4000, 5000]:
    hf = g.HostForest.synthetic(n, 200)
    res = []
    for k in ("wave", "pair", "auto"):
        f = g.Forest(hf, kernel=k)
        for _ in range(3):
            f.total_likelihood(P)
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            f.total_likelihood(P)
        dt = (time.perf_counter() - t0) / reps
        f.enable_profile()
        f.total_likelihood(P)
        ms, rows, names = f.launch_profile()
        res.append(f"{k} {1e3 * dt:.3f} ms [" + " ".join(f"{nm}:{m:.3f}" for nm, m in zip(names, ms)) + "]")
        f.close()
    print(f"trees={n} (levels {n}, {2 * n} cells): " + " | ".join(res), flush=True)
