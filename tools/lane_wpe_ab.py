"""A/B of the lane-schedule kernels' register budget (diagnostic): python tools/lane_wpe_ab.py LIB_DIR
loads libggp.so from LIB_DIR; times the lane schedule on a 40k-tree C2-shaped forest, the batched
484-point Hessian on C2, and the -p smoother on a 20k-tree C5-shaped forest."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native  # noqa: E402

_native.LIB_DIR = os.path.abspath(sys.argv[1])
import gfp_gaussian_process_amd as g  # noqa: E402
from gfp_gaussian_process_amd import optimize as opt  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def timed(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        v = fn()
    return 1e3 * (time.perf_counter() - t0) / reps, v


f = g.Forest(g.HostForest.synthetic(40000, 200), kernel="lane")
t_lane, v = timed(lambda: f.total_likelihood(P), 10)
f.close()
f = g.Forest(g.HostForest.synthetic(1000, 200))
pts, _ = opt.hessian_points(P, list(range(11)), 1e-2)
t_batch, _ = timed(lambda: f.total_likelihood_batch(pts), 3)
f.close()
f = g.Forest(g.HostForest.synthetic(20000, 500))
t_pred, _ = timed(lambda: f.predict(P, outputs=(False, False, False)), 3)
import hashlib  # noqa: E402
h = hashlib.sha1(f.predict_rows(0, 400000).tobytes()).hexdigest()[:12]   # the combined rows, bitwise
print(f"{sys.argv[1]}: lane 40k {t_lane:.3f} ms  batch484 {t_batch:.3f} ms  predict 20k x 500 {t_pred:.3f} ms  ll={v!r}"
      f"  rows sha1 {h}", flush=True)
