"""A/B of the lane-pair likelihood kernel (diagnostic): python tools/pair_ab.py LIB_DIR
loads libggp.so from LIB_DIR; times a C4 shard (12.5k trees x 200, auto: lane-pair levels) and the
C3 forest (10k x 200), prints the per-level launch times, the total and a hash of the carried state."""
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

for trees in (12500, 10000):
    f = g.Forest(g.HostForest.synthetic(trees, 200))
    vals = [f.total_likelihood(P) for _ in range(3)]
    h = hashlib.sha1(f.state().tobytes()).hexdigest()[:12]
    t0 = time.perf_counter()
    for _ in range(40):
        f.total_likelihood(P)
    ms = 1e3 * (time.perf_counter() - t0) / 40
    f.enable_profile()
    f.total_likelihood(P)
    lv = " ".join(f"{x:.4f}" for x in f.launch_profile()[0])
    f.close()
    print(f"{sys.argv[1]}: {trees} trees {ms:.4f} ms  levels {lv}  ll={vals[-1]!r}  state sha1 {h}", flush=True)
