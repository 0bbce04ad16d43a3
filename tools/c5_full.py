"""BASELINE configs[4] at its full size on ONE MI355X: the synthetic forest of 1M trees x 500
timepoints (5e8 rows), resident in HBM through the chunked layout (-chunk /
max_shard_rows: 8 chunks of the per-GPU shard size smoothed one after another through one
forward/backward workspace).

  1. the total log-likelihood of all 5e8 rows, timed, and against the CPU oracle over the whole
     forest (16 whole-tree shards, one oracle thread each) at the 1e-9 north-star bar;
  2. -p (forward + backward + combine, outputs resident), timed;
  3. every combined row streamed back by range (what the _prediction.csv writer reads): finite,
     and a per-column sum as a checksum; 1000 trees spread over the forest against the oracle
     smoother at PRED_TOL (tests/test_gpu_parity.py).

Progress lines go to stderr; one JSON line to stdout.

  python tools/c5_full.py [TREES=1000000] [CHUNKS=8]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def log(msg):
    print(f"[c5_full {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    trees = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rows = 500
    res = {"trees": trees, "rows_per_tree": rows, "chunks": chunks}
    t0 = time.perf_counter()
    hf = g.HostForest.synthetic(trees, rows)
    n = hf.n_rows
    res["rows"] = n
    res["synth_s"] = time.perf_counter() - t0
    log(f"synthetic forest: {n} rows, {hf.n_cells} cells in {res['synth_s']:.1f} s")

    t0 = time.perf_counter()
    f = g.Forest(hf, max_shard_rows=-(-n // chunks))
    res["create_s"] = time.perf_counter() - t0
    res["shards"] = len(f.shards())
    log(f"forest on the device: {res['shards']} chunks in {res['create_s']:.1f} s")

    ll = f.total_likelihood(P)                  # first (fresh-state) evaluation: the oracle's
    f.reset_state()
    times = []
    for _ in range(5):
        f.reset_state()
        t0 = time.perf_counter()
        v = f.total_likelihood(P)
        times.append(time.perf_counter() - t0)
        assert v == ll, (v, ll)
    res["ll"] = ll
    res["ll_ms"] = 1e3 * min(times)
    res["ll_updates_per_s"] = n / min(times)
    log(f"total log-likelihood {ll!r}: {res['ll_ms']:.1f} ms ({res['ll_updates_per_s']:.3g} updates/s)")
    # the split an 8-GPU run uses: each chunk is one GPU's whole-tree shard (LPT over reduction
    # blocks); per chunk its rows, cells and the device time of its launches in one evaluation
    res["shard_split"] = [{"device": d, "rows": r, "cells": c} for d, r, c in f.shards()]
    f.enable_profile()
    f.reset_state()
    f.total_likelihood(P)
    ms, lrows, kern = f.launch_profile()
    res["ll_launches"] = [{"ms": a, "rows": b, "kernel": k} for a, b, k in zip(ms, lrows, kern)]
    res["ll_device_ms_sum"] = float(sum(ms))

    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        f.predict(P, outputs=(False, False, False))
        times.append(time.perf_counter() - t0)
    res["predict_device_ms"] = dict(zip(("smooth", "combine"), f.predict_profile()))
    res["predict_ms"] = 1e3 * min(times)
    res["predict_rows_per_s"] = n / min(times)
    log(f"-p: {res['predict_ms']:.1f} ms ({res['predict_rows_per_s']:.3g} rows/s)")

    t0 = time.perf_counter()
    span = 1 << 22
    colsum = np.zeros(20)
    finite = True
    for lo in range(0, n, span):
        r = f.predict_rows(lo, min(n, lo + span))
        finite &= bool(np.isfinite(r).all())
        colsum += r.sum(axis=0)
        if (lo // span) % 16 == 0:
            log(f"rows streamed: {lo + r.shape[0]} / {n}")
    res["stream_s"] = time.perf_counter() - t0
    res["stream_rows_per_s"] = n / res["stream_s"]
    res["rows_finite"] = finite
    res["row_checksum"] = colsum.tolist()
    log(f"streamed every row in {res['stream_s']:.1f} s, finite={finite}")

    from oracle import oracle as O
    from test_gpu_parity import PRED_TOL, _smoother_err
    picks = list(range(0, trees, max(1, trees // 1000)))[:1000]   # 1000 trees spread over the forest
    sub = hf.subset_trees(hf.roots[picks])
    ref = O.OracleForest(sub.a).predict(P)[2]
    got = np.concatenate([f.predict_rows(rows * k, rows * k + rows) for k in picks])
    em, ec = _smoother_err(got, ref)
    res["predict_sample"] = {"trees": len(picks), "mean_err": em, "cov_err": ec, "tol": PRED_TOL}
    log(f"-p on {len(picks)} sampled trees vs the oracle: {em:.2e} / {ec:.2e} (tol {PRED_TOL})")
    assert em < PRED_TOL and ec < PRED_TOL
    f.close()

    # the whole forest's total on the CPU oracle, 16 whole-tree shards in parallel
    from concurrent.futures import ThreadPoolExecutor
    from gfp_gaussian_process_amd.distributed import shard
    nth = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    t0 = time.perf_counter()
    parts = [O.OracleForest(shard(hf, r, nth).a) for r in range(nth)]
    with ThreadPoolExecutor(nth) as ex:
        vals = list(ex.map(lambda o: o.total_likelihood(P)[0], parts))
    ref_ll = float(np.sum(vals))
    res["oracle_s"] = time.perf_counter() - t0
    res["oracle_threads"] = nth
    res["oracle_ll"] = ref_ll
    res["ll_rel_err"] = abs(ll - ref_ll) / abs(ref_ll)
    log(f"oracle total {ref_ll!r} in {res['oracle_s']:.1f} s on {nth} threads: rel err {res['ll_rel_err']:.2e}")
    assert res["ll_rel_err"] < 1e-9
    print(json.dumps(res))


if __name__ == "__main__":
    main()
