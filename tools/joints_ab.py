"""A/B of the -j walk kernel (diagnostic): python tools/joints_ab.py LIB_DIR
loads libggp.so from LIB_DIR; times ggp_joints over every start row of 20 C5-shaped trees (one call,
single pass) and prints a hash of the joints."""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native  # noqa: E402

_native.LIB_DIR = os.path.abspath(sys.argv[1])
import numpy as np  # noqa: E402

import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
hf = g.HostForest.synthetic(20, 500, seed=20261015, first_tree=2 * 10 ** 6)
f = g.Forest(hf)
buf = (np.zeros((1 << 21, 2), np.int64), np.zeros((1 << 21, 72)))
i, v = f.joints(P, 1e-10, 0, hf.n_rows, out=buf)
h = hashlib.sha1(i.tobytes() + v.tobytes()).hexdigest()[:12]
t0 = time.perf_counter()
for _ in range(5):
    f.joints(P, 1e-10, 0, hf.n_rows, out=buf)
ms = 1e3 * (time.perf_counter() - t0) / 5
print(f"{sys.argv[1]}: {len(i)} joints {ms:.2f} ms per call  hash {h}", flush=True)
f.close()
