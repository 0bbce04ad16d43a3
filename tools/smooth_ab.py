"""-p smoother A/B of two engine builds (diagnostic): python tools/smooth_ab.py LIB_DIR [TREES]
times ggp_predict on a C5-shaped forest (500 rows per tree) with libggp.so from LIB_DIR and
prints the forward/backward and combine device times and a hash of sampled output rows (forward,
backward, combined), so two builds can be compared for identical bits."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native  # noqa: E402

_native.LIB_DIR = os.path.abspath(sys.argv[1])
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
trees = int(sys.argv[2]) if len(sys.argv) > 2 else 125000
hf = g.HostForest.synthetic(trees, 500)
f = g.Forest(hf)
f.predict(P, outputs=(False, False, False))
sm, cb = [], []
for _ in range(3):
    f.predict(P, outputs=(False, False, False))
    a, b = f.predict_profile()
    sm.append(a)
    cb.append(b)
os.environ["GGP_SMOOTHER_LANE"] = "1"   # the hashed rows from the lane smoother on every level
small = g.Forest(g.HostForest.synthetic(200, 500)).predict(P)
h = hashlib.sha256(b"".join(x.tobytes() for x in small)).hexdigest()[:16]
print(json.dumps({"lib": sys.argv[1], "trees": trees, "smooth_ms": min(sm), "combine_ms": min(cb), "rows_hash": h}), flush=True)
