"""Chained objective against call-by-call: num_hessian_ll's 400 points (10 free parameters) on
the reference's example and on C2, wall ms, and whether the values agree bitwise.  One JSON line.

  python tools/chain_time.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402
from gfp_gaussian_process_amd import optimize as opt  # noqa: E402

P = np.array([2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01,
              1.63e-04, 7.48e-01])


def case(hf, name, idx):
    pts, _ = opt.hessian_points(P, idx, 1e-2)
    res = {"points": len(pts), "rows": hf.n_rows}
    f = g.Forest(hf)
    f.total_likelihood(P)
    st0 = f.state()
    f.total_likelihood_chain(pts[:8])                   # workspace + code warm-up
    for rep in range(2):
        f.set_state(st0)
        t0 = time.perf_counter()
        seq = np.array([f.total_likelihood(p) for p in pts])
        t_seq = time.perf_counter() - t0
        st_seq = f.state()
        f.set_state(st0)
        t0 = time.perf_counter()
        ch = f.total_likelihood_chain(pts)
        t_ch = time.perf_counter() - t0
        st_ch = f.state()
    res.update(seq_ms=1e3 * t_seq, chain_ms=1e3 * t_ch, speedup=t_seq / t_ch,
               bitwise=bool(np.array_equal(seq, ch) and np.array_equal(st_seq, st_ch)))
    print(name, res, file=sys.stderr, flush=True)
    return res


def main():
    out = {}
    import tempfile, gzip, shutil
    d = tempfile.mkdtemp()
    csv = os.path.join(d, "input.csv")
    with gzip.open(os.path.join(ROOT, "tests", "golden", "example_input.csv.gz"), "rb") as a, open(csv, "wb") as b:
        shutil.copyfileobj(a, b)
    ex = g.HostForest.from_csv(csv, os.path.join(ROOT, "tests", "golden", "example_csv_config.txt"))
    idx = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9]
    out["example"] = case(ex, "example", idx)
    out["c2"] = case(g.HostForest.synthetic(1000, 200), "c2", idx)
    out["note"] = "num_hessian_ll's 4k^2 points (k=10, eps 1e-2) from the same carried state: one-by-one ggp_total_loglik vs one ggp_total_loglik_chain"
    shutil.rmtree(d, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
