"""Schedule policy scan beyond C2 (VERDICT r1 "untested dispatch thresholds"): ms per evaluation
of each schedule and of auto, and per-level ms, on
  * the C5 tree shape (500 rows: root 250 + 2 x 125) at several tree counts,
  * C2-shaped forests (200 rows) around the thresholds,
  * example-like deep trees: the reference's example tree (77 cells, depth 12, 188-446 rows a
    cell) replicated K times.
python tools/schedule_scan_shapes.py > profiles/rNN_schedule_scan_shapes.txt (GPU box)"""
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

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def replicate(hf, k):
    """k copies of a forest as one (cells and rows concatenated, indices shifted)"""
    a = hf.a
    nc, nr = hf.n_cells, hf.n_rows
    out = dict(a)
    ro = a["row_offset"]
    out["row_offset"] = np.concatenate([[0]] + [ro[1:] + i * nr for i in range(k)]).astype(np.int64)
    for key in ("parent", "daughter1", "daughter2"):
        v = a[key]
        out[key] = np.concatenate([np.where(v >= 0, v + i * nc, -1) for i in range(k)]).astype(np.int32)
    for key in ("time", "log_length", "fp", "segment"):
        out[key] = np.concatenate([a[key]] * k)
    return g.HostForest(out)


def scan(name, hf):
    res = []
    for k in ("wave", "group", "pair", "lane", "auto"):
        f = g.Forest(hf, kernel=k)
        for _ in range(2):
            f.total_likelihood(P)
        reps = 8
        t0 = time.perf_counter()
        for _ in range(reps):
            f.total_likelihood(P)
        dt = (time.perf_counter() - t0) / reps
        f.enable_profile()
        f.total_likelihood(P)
        ms, rows, names = f.launch_profile()
        lv = " ".join(f"{m:.3f}" for m in ms[:6]) + (" ..." if len(ms) > 6 else "")
        res.append((k, 1e3 * dt, lv, names))
        f.close()
    best = min(res[:4], key=lambda r: r[1])
    auto = res[4]
    print(f"{name} cells={hf.n_cells} rows={hf.n_rows}: " + " | ".join(f"{k} {t:.3f} ms [{lv}]" for k, t, lv, _ in res)
          + f" || best fixed: {best[0]} {best[1]:.3f}; auto/best = {auto[1] / best[1]:.3f}", flush=True)


d = tempfile.mkdtemp()
with gzip.open(os.path.join(ROOT, "tests", "golden", "example_input.csv.gz"), "rb") as fi, open(d + "/in.csv", "wb") as fo:
    shutil.copyfileobj(fi, fo)
ex = g.HostForest.from_csv(d + "/in.csv", os.path.join(ROOT, "tests", "golden", "example_csv_config.txt"))
for k in (1, 32, 128, 512):
    scan(f"example x{k}", replicate(ex, k) if k > 1 else ex)
for t in (1000, 2500, 4000, 6000, 12500):
    scan(f"C5-shape {t} trees x 500", g.HostForest.synthetic(t, 500))
for t in (1000, 4000, 6000, 12500, 20000, 40000):
    scan(f"C2-shape {t} trees x 200", g.HostForest.synthetic(t, 200))
