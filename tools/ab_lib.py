"""A/B timing of engine builds (diagnostic): python tools/ab_lib.py LIB_DIR [kernel] [trees; 0 = the example]
loads libggp.so from LIB_DIR instead of the package's lib/ and prints ms per evaluation of
C2-shaped forests and the per-level kernel times; run it alternately for two builds."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native  # noqa: E402

_native.LIB_DIR = os.path.abspath(sys.argv[1])
import gfp_gaussian_process_amd as g  # noqa: E402

kern = sys.argv[2] if len(sys.argv) > 2 else "auto"
trees = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
if trees > 0:
    hf = g.HostForest.synthetic(trees, 200)
else:   # 0: the reference's example (one tree, critical path 3,759 of 22,065 rows)
    import gzip, shutil, tempfile
    tmp = os.path.join(tempfile.gettempdir(), "ab_example.csv")
    with gzip.open(os.path.join(ROOT, "tests", "golden", "example_input.csv.gz"), "rb") as fi, open(tmp, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    hf = g.HostForest.from_csv(tmp, os.path.join(ROOT, "tests", "golden", "example_csv_config.txt"))
if os.environ.get("AB_PREHEAT_MS"):   # full-chip work first: the timed calls at the sustained clock
    hp = g.Forest(g.HostForest.synthetic(12500, 200, seed=7))
    t_end = time.perf_counter() + float(os.environ["AB_PREHEAT_MS"]) / 1e3
    while time.perf_counter() < t_end:
        hp.total_likelihood(P)
    hp.close()
f = g.Forest(hf, kernel=kern)
for _ in range(3):
    v = f.total_likelihood(P)
reps = 40
t0 = time.perf_counter()
for _ in range(reps):
    f.total_likelihood(P)
dt = (time.perf_counter() - t0) / reps
f.enable_profile()
lv = []
for _ in range(5):
    f.total_likelihood(P)
    lv.append(f.launch_profile()[0])
import numpy as np
ms = np.median(np.array(lv), axis=0)
kus = ""
try:   # the path launch's own device time (ggp_call_trace; builds from round 6 on)
    f2 = g.Forest(hf, kernel=kern)
    for _ in range(3 + reps):
        f2.total_likelihood(P)
    tr = f2.call_trace(reps)
    if len(tr) and np.all(tr[:, 3] > 0):
        kus = f"  kernel_us {np.median(tr[:, 3]):.2f} enqueue_us {np.median(tr[:, 0]):.2f} mhz {np.median(tr[:, 4]):.0f}"
except Exception:
    pass
print(f"{sys.argv[1]} {kern} trees={trees}: {1e3 * dt:.4f} ms/eval  levels " + " ".join(f"{m:.4f}" for m in ms)
      + f"  ll={v!r}" + kus, flush=True)
