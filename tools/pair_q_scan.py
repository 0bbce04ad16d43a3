"""Lane-pair Q choice on r32+ lane bodies (diagnostic): ms per level launch on C3/C4-shaped forests
for Q by level size (default), Q = 4 everywhere and Q = 2 everywhere (GGP_PAIR_Q), values bitwise
equal.  python tools/pair_q_scan.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
for trees in (10000, 12500, 16000):
    hf = g.HostForest.synthetic(trees, 200)
    line = [f"{trees} trees:"]
    vals = set()
    for q in ("0", "4", "2"):
        os.environ["GGP_PAIR_Q"] = q
        f = g.Forest(hf)
        for _ in range(3):
            f.total_likelihood(P)
        f.enable_profile()
        f.total_likelihood(P)
        ms, rows, kinds = f.launch_profile()
        t0 = time.perf_counter()
        for _ in range(30):
            v = f.total_likelihood(P)
        el = 1e3 * (time.perf_counter() - t0) / 30
        vals.add(v)
        line.append(f"Q={q or 'auto'}: {el:.4f} ms/eval levels " + " ".join(f"{k}:{m:.3f}" for k, m in zip(kinds, ms)))
        f.close()
    line.append(f"bitwise {len(vals) == 1}")
    print(" | ".join(line), flush=True)
