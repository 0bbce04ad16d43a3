"""A/B of the lane smoother (diagnostic): python tools/smoother_lane_ab.py LIB_DIR [TREES]
loads libggp.so from LIB_DIR; -p on TREES C5-shaped trees (500 rows; levels above 32k cells run the
lane smoother, k_fwd_level / k_bwd_level<true> with the combine fused): level and combine ms from the
engine's events, wall ms per predict, and a hash of the combined rows (bitwise check across builds)."""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native  # noqa: E402

_native.LIB_DIR = os.path.abspath(sys.argv[1])
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
trees = int(sys.argv[2]) if len(sys.argv) > 2 else 125000
f = g.Forest(g.HostForest.synthetic(trees, 500))
f.predict(P, outputs=(False, False, False))
t0 = time.perf_counter()
for _ in range(3):
    f.predict(P, outputs=(False, False, False))
wall = 1e3 * (time.perf_counter() - t0) / 3
sm, cb = f.predict_profile()
h = hashlib.sha1(f.predict_rows(0, 400000).tobytes()).hexdigest()[:12]
print(f"{sys.argv[1]}: -p {trees} x 500: wall {wall:.3f} ms  levels {sm:.3f} ms  combine {cb:.3f} ms  rows sha1 {h}", flush=True)
f.close()
