"""BASELINE.json's configs on the HIP path, at their stated sizes:

  C4  -s 1-D scan, 100k trees x 200 tp: the CLI on the whole forest (2e7 rows, one GPU; a
      binary dataset -- the CSV would be 1 GB), gamma_lambda bound (4.36E-02, 1.0E-03, 2.0E-02,
      8.0E-02): 60 chained samples (run_bound_1dscan, main.cpp:77-112).  Checks: the scan file
      is byte-identical with the forest on 8 logical shards (-g 0,...,0: the 8-GPU layout);
      every sample equals the Python handle's chained value bitwise; a 200-tree sub-forest
      keeping the full forest's init statistics follows the oracle's chain to 1e-9.
  C5  -p on a per-GPU shard of 1M trees x 500 tp (125k trees, 6.25e7 rows): 400 sampled trees
      against the oracle smoother at 2x its measured distance (test_gpu_parity.py pred_bound); the same forest in 8
      chunks through a capped workspace (max_shard_rows) bitwise equal to the one-shard run.
  C3  -m with all 11 parameters free (beta added as in SURVEY §8(d)), log space, LN_NELDERMEAD,
      on a reduced forest (300 trees x 200): the CLI's iteration log follows the restatement
      driven by the oracle objective for the first 60 evaluations.
"""
import os

import numpy as np
import pytest

from test_gpu_cli import CLI, INIT, NAMES, _ll_table, _param_file, _run
from test_gpu_parity import _smoother_err, pred_bound

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]
REL = 1e-9


@pytest.mark.timeout(400)
def test_c4_scan_100k_trees(tmp_path):
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.optimize import arange
    from oracle import oracle as O
    hf = g.HostForest.synthetic(100_000, 200, with_ids=True)
    assert hf.n_rows == 20_000_000
    data = str(tmp_path / "c4.ggpd")
    g.Dataset.from_forest(hf).save(data)
    pf = _param_file(tmp_path / "p.txt", {1: "4.36E-02, 1.0E-03, 2.0E-02, 8.0E-02"})
    samples = arange(2.0e-02, 8.0e-02, 1.0e-03)
    assert len(samples) == 60
    for tag, gl in (("one", "1"), ("eight", "0,0,0,0,0,0,0,0")):
        _run(["-i", data, "-b", pf, "-s", "-g", gl, "-o", str(tmp_path / tag)], tmp_path)
    name = "c4_scan_gamma_lambda.csv"
    one, eight = (open(tmp_path / t / name).read() for t in ("one", "eight"))
    assert one == eight
    rows = _ll_table(tmp_path / "one" / name)
    assert [r[2] for r in rows] == samples
    # the CLI's values are the engine's: the same chain through the Python handle, bitwise
    f = g.Forest(hf)
    p = list(INIT)
    for r, v in zip(rows, samples):
        p[1] = v
        assert f.total_likelihood(p) == r[-1]
    f.close()
    # 200 trees with the full forest's init statistics: the oracle's chain
    sub = hf.subset_trees(hf.roots[::500])
    assert sub.n_cells == 600
    fs, of = g.Forest(sub), O.OracleForest(sub.a)
    for v in samples:
        p[1] = v
        vg, vo = fs.total_likelihood(p), of.total_likelihood(p)[0]
        assert abs(vg - vo) / abs(vo) < REL, (v, vg, vo)


@pytest.mark.timeout(400)
def test_c5_predict_shard_125k_trees():
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(125_000, 500)
    n = hf.n_rows
    assert n == 62_500_000
    f = g.Forest(hf)
    f.predict(INIT, outputs=(False, False, False))
    picks = list(range(0, 125_000, 312))[:400]               # 400 trees; tree k: rows [500 k, 500 k + 500)
    sub = hf.subset_trees(hf.roots[picks])
    ref = O.OracleForest(sub.a).predict(INIT)[2]
    got = np.concatenate([f.predict_rows(500 * k, 500 * k + 500) for k in picks])
    em, ec = _smoother_err(got, ref)
    print(f"PRED_ERR c5_shard combined mean {em:.3e} cov {ec:.3e}")
    bm, bc = pred_bound("c5_shard", "combined")
    assert em < bm and ec < bc, (em, ec)
    # 8 chunks through a workspace of 1/8 of the rows (8 shards on the one device): bitwise
    c = g.Forest(hf, max_shard_rows=n // 8)
    assert len(c.shards()) >= 8 and max(r for _, r, _ in c.shards()) <= n // 8
    c.predict(INIT, outputs=(False, False, False))
    for lo in range(0, n, n // 16):
        hi = min(n, lo + 250_000)
        assert np.array_equal(c.predict_rows(lo, hi), f.predict_rows(lo, hi)), lo
    c.close()
    f.close()


@pytest.mark.timeout(400)
def test_c3_minimize_11_free_parameters(tmp_path):
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as Opt
    from oracle import oracle as O
    from test_gpu_cli import _small_csv
    csv = _small_csv(tmp_path / "c3.csv", n_trees=300, rows=200)
    cfg = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "example_csv_config.txt")
    pf = _param_file(tmp_path / "p.txt", {i: f"{INIT[i]!r}, {0.1 * INIT[i]!r}" for i in range(11)})
    _run(["-i", csv, "-b", pf, "-c", cfg, "-m", "-t", "1e-6", "-o", str(tmp_path / "o")], tmp_path)
    rows = _ll_table(tmp_path / "o" / "c3_f012345678910_b_iterations.csv")
    hf = g.HostForest.from_csv(csv, cfg)
    of = O.OracleForest(hf.a)
    seen = []

    def objective(p):
        v = of.total_likelihood(p)[0]
        seen.append((p.copy(), v))
        return v

    P = g.ParameterSet.load(pf)
    assert P.kind == ["free"] * 11
    Opt.minimize_wrapper(objective, P, tolerance=1e-6, search_space="log", maxeval=60)
    assert len(seen) == 60 and len(rows) > 60
    for k in range(60):
        assert np.allclose(rows[k][1:12], seen[k][0], rtol=1e-9, atol=0), k
        assert abs(rows[k][12] - seen[k][1]) / abs(seen[k][1]) < REL, k
