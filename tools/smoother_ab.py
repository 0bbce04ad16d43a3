"""-p smoother on the lane-pair split against the lane smoother (diagnostic): ms per ggp_predict
(outputs left in HBM) on C5-shaped forests (500 rows a tree) and the example, per schedule.
python tools/smoother_ab.py"""
import gzip
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def t_predict(hf, lane, reps=3):
    os.environ["GGP_SMOOTHER_LANE"] = "1" if lane else "0"
    f = g.Forest(hf)
    f.predict(P, outputs=(False, False, False))
    t0 = time.perf_counter()
    for _ in range(reps):
        f.predict(P, outputs=(False, False, False))
    ms = 1e3 * (time.perf_counter() - t0) / reps
    f.close()
    return ms


d = tempfile.mkdtemp()
with gzip.open(os.path.join(ROOT, "tests", "golden", "example_input.csv.gz"), "rb") as fi, open(d + "/in.csv", "wb") as fo:
    shutil.copyfileobj(fi, fo)
forests = [("example (77 cells, depth 12)", g.HostForest.from_csv(d + "/in.csv", os.path.join(ROOT, "tests", "golden",
                                                                                              "example_csv_config.txt")))]
forests += [(f"{t} trees x 500", g.HostForest.synthetic(t, 500)) for t in (1000, 5000, 12500, 20000, 125000)]
for name, hf in forests:
    print(f"{name}: lane {t_predict(hf, True):.3f} ms  split {t_predict(hf, False):.3f} ms", flush=True)
