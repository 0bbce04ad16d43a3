"""A/B of engine builds on a C5 per-GPU shard (diagnostic): python tools/lane_ab_c5.py LIB_DIR
125k trees x 500 rows (6.25e7 rows): the -p smoother (forward + backward levels, combine) and the
total log-likelihood on the lane schedule; ms and a checksum of the smoother's first rows."""
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
hp = g.HostForest.synthetic(trees, 500)
out = [sys.argv[1]]
fp = g.Forest(hp, kernel="lane")
for _ in range(2):
    v = fp.total_likelihood(P)
t0 = time.perf_counter()
for _ in range(5):
    v = fp.total_likelihood(P)
out.append(f"ll lane {1e3 * (time.perf_counter() - t0) / 5:.3f} ms ll={v!r}")
fp.predict(P, outputs=(False, False, False))
sm = cb = 0.0
for _ in range(3):
    fp.predict(P, outputs=(False, False, False))
    a_, b_ = fp.predict_profile()
    sm += a_
    cb += b_
rows = fp.predict_rows(0, 100000)
out.append(f"smooth {sm / 3:.3f} ms combine {cb / 3:.3f} ms sha={hashlib.sha256(rows.tobytes()).hexdigest()[:16]}")
fp.close()
print(" | ".join(out), flush=True)
