"""Stress check of the path launch (diagnostic): many evaluations with varying parameters on
C2 and on the reference's example forest, each compared bitwise with a level-launch handle
(GGP_WAVE_PATHS_MAX=0) of the same forest -- a race in the in-launch flags or counters would
show as a mismatch or a hang.  python tools/path_stress.py [N]"""
import gzip
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
G = os.path.join(ROOT, "tests", "golden")
tmp = tempfile.mkdtemp()
csv = os.path.join(tmp, "input.csv")
with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
    shutil.copyfileobj(fi, fo)
P0 = np.array(g.ParameterSet.load(os.path.join(G, "example_parameter_file.txt")).get_init())
forests = {"C2": g.HostForest.synthetic(1000, 200),
           "example": g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"), -1, "scaled", "binomial")}
rng = np.random.default_rng(11)
for name, hf in forests.items():
    a = g.Forest(hf, kernel="auto")
    os.environ["GGP_WAVE_PATHS_MAX"] = "0"
    b = g.Forest(hf, kernel="auto")
    del os.environ["GGP_WAVE_PATHS_MAX"]
    n = N if name == "C2" else max(1, N // 50)
    t0 = time.perf_counter()
    bad = 0
    for k in range(n):
        P = P0 * (1 + 0.05 * rng.standard_normal(11))
        P[2] = abs(P[2])
        try:
            va = a.total_likelihood(P)
        except g.LikelihoodIsNan as e:
            va = ("nan", e.cell, e.row)
            a.reset_state()
        try:
            vb = b.total_likelihood(P)
        except g.LikelihoodIsNan as e:
            vb = ("nan", e.cell, e.row)
            b.reset_state()
        if va != vb:
            bad += 1
            if bad < 5:
                print(f"{name} eval {k}: path {va!r} level {vb!r}", flush=True)
        if k % 1000 == 999:
            print(f"{name}: {k + 1} evaluations, {bad} mismatches", flush=True)
    print(f"{name}: {n} evaluations in {time.perf_counter() - t0:.1f} s, {bad} mismatches; "
          f"states equal: {np.array_equal(a.state(), b.state())}", flush=True)
    assert bad == 0
