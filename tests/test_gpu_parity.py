"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

Tolerance (BASELINE north star): total log-likelihood within 1e-9 relative; topology
bit-exact (host ingest, tests/test_host.py).  Observed: <= 3e-10 on the example, ~1e-11 on the
synthetic forests (libm ulp differences, the products and contraction of the schedules' bodies;
profiles/r32_parity_margin.txt, DESIGN.md "Parity").
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]

REL = 1e-9
PARAMS = json.load(open(os.path.join(GOLDEN, "oracle_example.json")))
CONFIGS = [(k.split("/")[0], k.split("/")[1], [float.fromhex(x) for x in v["params"]]) for k, v in PARAMS.items()]


def _rel(a, b):
    return abs(a - b) / abs(b)


@pytest.fixture(scope="module")
def example_forests(example_paths):
    import gfp_gaussian_process_amd as g
    out = {}
    for noise, div, _ in CONFIGS:
        out[(noise, div)] = g.HostForest.from_csv(example_paths["csv"], example_paths["config"], -1, noise, div)
    return out


# every schedule against the oracle: lane (throughput), group (latency, bitwise = lane), wave
# (latency; outputs summed in another order, ~3e-10 on the example), pair (mid-size levels, a step
# over two waves, bitwise = lane).  Lane, group and pair form 22 exponentials as products and
# contract within expressions, as the wave schedule does: ~3e-10 on the example too
KERNELS = ["lane", "group", "wave", "pair"]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("noise,div,params", CONFIGS, ids=[f"{a}-{b}" for a, b, _ in CONFIGS])
def test_example_carried_state_chain(example_forests, noise, div, params, kernel):
    """fresh call + two calls on carried root state (predictions.h:63-78), vs the oracle"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = example_forests[(noise, div)]
    fg = g.Forest(hf, kernel=kernel)
    of = O.OracleForest(hf.a)
    for call in range(3):
        vg = fg.total_likelihood(params)
        vo, nc, nr = of.total_likelihood(params)
        assert nc == -1
        assert _rel(vg, vo) < REL, (call, vg, vo)


REF_DAWSON = json.load(open(os.path.join(GOLDEN, "oracle_example_refdawson.json")))


@pytest.mark.parametrize("kernel", KERNELS)
def test_example_chain_vs_reference_dawson_totals(example_forests, kernel):
    """the same chains against the oracle run on the reference's own Faddeeva::Dawson
    (tests/golden/oracle_example_refdawson.json, make_refdawson.py): the device holds the 1e-9
    bar against the reference's Dawson arithmetic as well as against the oracle's table"""
    import gfp_gaussian_process_amd as g
    worst = 0.0
    for key, v in REF_DAWSON.items():
        noise, div, _ = key.split("/")
        fg = g.Forest(example_forests[(noise, div)], kernel=kernel)
        params = [float.fromhex(x) for x in v["params"]]
        for call in range(3):
            vg = fg.total_likelihood(params)
            vr = float.fromhex(v["ll"][call])
            worst = max(worst, _rel(vg, vr))
            assert _rel(vg, vr) < REL, (key, call, vg, vr)
    print(f"{kernel}: worst rel vs the reference-Dawson totals {worst:.2e}")


@pytest.mark.parametrize("kernel", KERNELS)
def test_example_state_matches_oracle(example_forests, kernel):
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = example_forests[("scaled", "binomial")]
    P = CONFIGS[0][2]
    fg, of = g.Forest(hf, kernel=kernel), O.OracleForest(hf.a)
    for _ in range(2):
        fg.total_likelihood(P)
        of.total_likelihood(P)
    sg, so = fg.state(), of.state
    assert np.all(np.isfinite(sg))
    # means relative; covariances relative to sqrt(Cii Cjj).  The latent q is weakly
    # observed: perturbing every exp() of the oracle itself by +-1 ulp moves mean_q by
    # 1.5e-7 and the normalised cov by 4e-7 (DESIGN.md "Parity"), so the bound is 2e-6.
    assert np.max(np.abs(sg[:, :4] - so[:, :4]) / np.abs(so[:, :4]).clip(1e-300)) < 2e-6
    Cg, Co = sg[:, 4:].reshape(-1, 4, 4), so[:, 4:].reshape(-1, 4, 4)
    d = np.sqrt(np.abs(np.einsum("nii->ni", Co)))
    scale = d[:, :, None] * d[:, None, :]
    assert np.max(np.abs(Cg - Co) / scale) < 2e-6


def test_reset_state_and_determinism(example_forests):
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")]
    P = CONFIGS[0][2]
    a, b = g.Forest(hf), g.Forest(hf)
    first = a.total_likelihood(P)
    assert b.total_likelihood(P) == first            # bitwise reproducible
    second = a.total_likelihood(P)
    assert second != first                            # carried state changes the objective
    a.reset_state()
    assert a.total_likelihood(P) == first             # "fresh cells" again
    assert a.total_likelihood(P) == second


@pytest.mark.parametrize("kernel", KERNELS)
def test_nan_reported_like_reference(example_forests, kernel):
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = example_forests[("scaled", "binomial")]
    P = list(CONFIGS[0][2])
    P[2] = -1.0                                       # var_lambda < 0: sqrt(a<0) in the propagator
    _, oc, orow = O.OracleForest(hf.a).total_likelihood(P)
    with pytest.raises(g.LikelihoodIsNan) as e:
        g.Forest(hf, kernel=kernel).total_likelihood(P)
    assert (e.value.cell, e.value.row) == (oc, orow)
    assert e.value.cell_id == hf.ids[oc]


@pytest.mark.parametrize("kernel", ["auto"] + KERNELS)
@pytest.mark.parametrize("n_trees,rows", [(1000, 200), (37, 4), (5, 9), (3, 300)])
def test_synthetic_forest_vs_oracle(n_trees, rows, kernel):
    """(3, 300): 150-row roots cross the wave schedule's 64-row chunks and ll ring twice"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(n_trees, rows)
    P = CONFIGS[0][2]
    fg, of = g.Forest(hf, kernel=kernel), O.OracleForest(hf.a)
    for _ in range(2):
        vg = fg.total_likelihood(P)
        vo = of.total_likelihood(P)[0]
        assert _rel(vg, vo) < REL


def _ragged_roots(n_cells=40, seed=3):
    """roots only, 1..13 rows each, irregular time steps: rows of synthetic root cells with
    every 5th row dropped (dt = 2 gaps) -- data stay consistent with the model"""
    import gfp_gaussian_process_amd as g
    base = g.HostForest.synthetic(n_cells, 40)
    ro_b = base.a["row_offset"]
    a = dict(base.a)
    rows, lens = [], []
    for i in range(n_cells):
        r0 = ro_b[3 * i]                                  # the root cell of tree i (20 rows)
        keep = [r0 + k for k in range(20) if k % 5 != 3][: 1 + (i * 7) % 13]
        rows += keep
        lens.append(len(keep))
    rows = np.array(rows)
    a["row_offset"] = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    a["parent"] = np.full(n_cells, -1, np.int32)
    a["daughter1"] = np.full(n_cells, -1, np.int32)
    a["daughter2"] = np.full(n_cells, -1, np.int32)
    for k in ("time", "log_length", "fp", "segment"):
        a[k] = base.a[k][rows].copy()
    return g.HostForest(a)


@pytest.mark.parametrize("kernel", KERNELS)
def test_single_cells_and_ragged_rows(kernel):
    """1-row cells (no propagation) and dt = 2 steps (t != 1 exercises every t-power term and
    the wave schedule's per-dt cache)"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = _ragged_roots()
    assert np.any(np.diff(hf.a["time"]) == 2.0) and np.any(np.diff(hf.a["row_offset"]) == 1)
    P = CONFIGS[0][2]
    fg, of = g.Forest(hf, kernel=kernel), O.OracleForest(hf.a)
    for _ in range(2):
        assert _rel(fg.total_likelihood(P), of.total_likelihood(P)[0]) < REL


@pytest.mark.parametrize("kernel", KERNELS)
def test_rescaled_time_units(kernel):
    """time in hours (rescale_time = 60): dt = 1/60, a non-integer step"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(50, 40)
    hf.a["time"] = hf.a["time"] / 60.0
    P = list(CONFIGS[0][2])
    for i in (0, 1, 2, 4, 5, 6):                          # rates per hour
        P[i] *= 60.0 if i in (0, 1, 4, 6) else 1.0
    P[2] *= 60.0 ** 3
    P[5] *= 60.0
    fg, of = g.Forest(hf, kernel=kernel), O.OracleForest(hf.a)
    vg, vo = fg.total_likelihood(P), of.total_likelihood(P)[0]
    assert math.isfinite(vo) and _rel(vg, vo) < REL


def _irregular_times(hf, seed):
    """every cell sampled at irregular steps (0.3-2.5 time units apart), a daughter's first row
    0.5-2 units after its parent's last: a different dt at almost every step"""
    a = hf.a
    rng = np.random.default_rng(seed)
    ro, par = a["row_offset"], a["parent"]
    t = np.zeros(len(a["time"]))
    for c in range(len(par)):
        r0, r1 = ro[c], ro[c + 1]
        start = 0.0 if par[c] < 0 else t[ro[par[c] + 1] - 1] + rng.uniform(0.5, 2.0)
        assert par[c] < c
        t[r0:r1] = start + np.concatenate([[0.0], np.cumsum(rng.uniform(0.3, 2.5, r1 - r0 - 1))])
    a["time"] = t


@pytest.mark.parametrize("kernel", KERNELS)
def test_irregular_sampling_chain_vs_oracle(kernel):
    """irregular time steps (no two steps share a dt: the wave schedule's dt cache misses, every
    exp(s t) and product factor differs from step to step), three chained calls against the oracle"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(60, 40, seed=9)
    _irregular_times(hf, 1)
    P = CONFIGS[0][2]
    fg, of = g.Forest(hf, kernel=kernel), O.OracleForest(hf.a)
    for call in range(3):
        vg, vo = fg.total_likelihood(P), of.total_likelihood(P)[0]
        assert math.isfinite(vo) and _rel(vg, vo) < REL, (call, vg, vo)


def test_irregular_sampling_predict_vs_oracle():
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(30, 40, seed=4)
    _irregular_times(hf, 2)
    _check_predict(hf, CONFIGS[0][2], "irregular")


def test_empty_forest():
    import gfp_gaussian_process_amd as g
    a = dict(g.HostForest.synthetic(1, 8).a)
    for k in ("parent", "daughter1", "daughter2", "segment"):
        a[k] = np.zeros(0, np.int32)
    for k in ("time", "log_length", "fp"):
        a[k] = np.zeros(0)
    a["row_offset"] = np.zeros(1, np.int64)
    assert g.Forest(g.HostForest(a)).total_likelihood(CONFIGS[0][2]) == 0.0


def test_invalid_forest_rejected():
    import gfp_gaussian_process_amd as g
    a = dict(g.HostForest.synthetic(2, 8).a)
    a["parent"] = a["parent"].copy()
    a["parent"][1] = 99
    with pytest.raises(g.GGPError, match="out of range"):
        g.Forest(g.HostForest(a))


def test_shards_on_one_device_sum_to_whole():
    """additivity over trees (the multi-GPU invariant), here with 3 shards on cuda:0"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import combine_partials, shard
    full = g.HostForest.synthetic(300, 60)
    P = CONFIGS[0][2]
    whole = g.Forest(full)
    parts = [g.Forest(shard(full, r, 3)) for r in range(3)]
    for _ in range(2):
        w = whole.total_likelihood(P)
        s, _ = combine_partials([p.total_likelihood(P) for p in parts], [False] * 3)
        assert _rel(s, w) < 1e-12


def test_sharded_predict_on_one_device_equals_whole():
    """-p sharded by whole trees (distributed.ShardedPredictor), 3 shards on cuda:0 assembled
    in input order: bitwise equal to the unsharded smoother (same per-cell kernels)"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedPredictor, shard_rows
    full = g.HostForest.synthetic(300, 60)
    P = CONFIGS[0][2]
    want = g.Forest(full).predict(P)
    got = [np.empty_like(w) for w in want]
    n = 0
    for r in range(3):
        sub, rows = shard_rows(full, r, 3)
        sp = ShardedPredictor(g.Forest(sub), rows, full.n_rows)
        for k, part in enumerate(sp.predict(P)):
            got[k][rows] = part
        n += len(rows)
    assert n == full.n_rows
    for w, x in zip(want, got):
        assert np.array_equal(w, x)


def test_baseline_size_properties():
    """BASELINE C2 / C3 sizes: oracle agreement on C2, additivity + finiteness on C3"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    P = CONFIGS[0][2]
    c2 = g.HostForest.synthetic(1000, 200)
    assert _rel(g.Forest(c2).total_likelihood(P), O.OracleForest(c2.a).total_likelihood(P)[0]) < REL
    c3 = g.HostForest.synthetic(10000, 200)
    # one schedule for the whole and the halves (auto would run the halves' 5000-cell levels on
    # the wave schedule and the whole's 10000-cell levels on the lane schedule: ~1e-10 apart)
    f3 = g.Forest(c3, kernel="lane")
    v = f3.total_likelihood(P)
    assert math.isfinite(v)
    lo, hi = g.HostForest.synthetic(5000, 200), g.HostForest.synthetic(5000, 200, first_tree=5000)
    # shards carry the full forest's init statistics
    for h in (lo, hi):
        for k in ("root_mean_xg", "root_var_xg", "leaf_mean_xg", "leaf_var_xg"):
            h.a[k] = c3.a[k]
    s = g.Forest(lo, kernel="lane").total_likelihood(P) + g.Forest(hi, kernel="lane").total_likelihood(P)
    assert _rel(s, v) < 1e-12


@pytest.mark.timeout(300)
def test_c3_full_size_chain_vs_oracle():
    """BASELINE configs[2]'s forest at full size (10k trees x 200 = 2e6 rows) on the default
    (auto) schedule -- the one -m runs on it -- against the oracle: three chained evaluations
    (carried state, SURVEY finding 0.2) with different parameters, each at the 1e-9 bar"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    c3 = g.HostForest.synthetic(10000, 200)
    assert c3.n_rows == 2_000_000
    fg, of = g.Forest(c3), O.OracleForest(c3.a)
    P = CONFIGS[0][2]
    for k, scale in enumerate((1.0, 1.1, 0.9)):
        p = list(P)
        p[8] *= scale                            # var_g
        p[1] *= 2.0 - scale                      # gamma_lambda
        vg, vo = fg.total_likelihood(p), of.total_likelihood(p)[0]
        assert _rel(vg, vo) < REL, (k, vg, vo)


@pytest.mark.parametrize("which", ["example", "synthetic", "ragged"])
@pytest.mark.parametrize("other", ["group", "pair-q2", "pair-q4", "pair-q2-c32", "pair-q4-c32"])
def test_lane_group_pair_schedules_bitwise_equal(example_forests, which, other, monkeypatch):
    """the schedules run the same task expressions (csrc/ggp_prop.h): identical bits (pair-qQ:
    the lane schedule split over Q waves; -c32: 32 cells per workgroup, half its lanes empty)"""
    import gfp_gaussian_process_amd as g
    hf = {"example": lambda: example_forests[("scaled", "binomial")],
          "synthetic": lambda: g.HostForest.synthetic(300, 40),
          "ragged": _ragged_roots}[which]()
    P = CONFIGS[0][2]
    monkeypatch.setenv("GGP_PAIR_CPW", "32" if other.endswith("c32") else "64")
    monkeypatch.setenv("GGP_PAIR_Q", "4" if "q4" in other else "2")
    lane, o = g.Forest(hf, kernel="lane"), g.Forest(hf, kernel=other.split("-")[0])
    for _ in range(3):
        assert lane.total_likelihood(P) == o.total_likelihood(P)
    assert np.array_equal(lane.state(), o.state())


def test_pair_schedule_c4_shard_bitwise_and_auto():
    """a C4-shard-sized forest (12.5k trees x 200 rows): auto takes the lane-pair schedule for
    both levels (12.5k cells over four waves per cell, 25k over two), bitwise the lane schedule
    over a chain, and a NaN is located as the lane schedule locates it"""
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(12500, 200)
    P = CONFIGS[0][2]
    auto, lane = g.Forest(hf), g.Forest(hf, kernel="lane")
    for _ in range(2):
        assert auto.total_likelihood(P) == lane.total_likelihood(P)
    assert np.array_equal(auto.state(), lane.state())
    auto.enable_profile()
    auto.total_likelihood(P)
    assert auto.launch_profile()[2] == ["k_loglik_pair<4>", "k_loglik_pair<2>"]
    bad = list(P)
    bad[2] = -1.0
    errs = []
    for f in (g.Forest(hf), g.Forest(hf, kernel="lane")):
        with pytest.raises(g.LikelihoodIsNan) as e:
            f.total_likelihood(bad)
        errs.append((e.value.cell, e.value.row))
    assert errs[0] == errs[1]


# ------------------------------------------------------------------------------------------
# -p smoother (predictions.h:93-499) against the oracle's ora_predict
# ------------------------------------------------------------------------------------------
# Tolerance: means relative to (|m| + sd), covariances relative to sqrt(Cii Cjj).  The
# smoother inherits the latent-q sensitivity of the propagator (+-1 ulp on every exp moves
# the normalised state by ~4e-7, see test_example_state_matches_oracle) and adds five 4x4
# inverses per row.  PRED_TOL is the ceiling; each case is held at twice the distance measured on
# the MI355X for its (output, mean / covariance), capped by the ceiling (profiles/r36_pred_err.txt:
# the engine is deterministic, so the factor 2 is room for an ulp-level change of the kernels, not
# for run-to-run noise).  The example's const/gauss combined covariance (8.8e-6) keeps the ceiling.
PRED_TOL = 1e-5
PRED_MEASURED = {   # case: {output: (mean, covariance)} worst normalised distance from the oracle, r36
    "irregular": {"forward": (1.358e-08, 9.024e-08), "backward": (3.600e-08, 4.114e-07),
                  "combined": (3.248e-08, 3.249e-07)},
    "example/scaled/binomial": {"forward": (8.247e-07, 8.968e-07), "backward": (1.407e-06, 3.496e-06),
                                "combined": (2.370e-06, 3.799e-06)},
    "example/const/gauss": {"forward": (1.023e-06, 1.398e-06), "backward": (3.339e-06, 7.092e-06),
                            "combined": (3.598e-06, 8.794e-06)},
    "segments": {"forward": (4.134e-09, 7.250e-08), "backward": (1.686e-08, 2.431e-07),
                 "combined": (1.164e-08, 2.164e-07)},
    "four_segments": {"forward": (6.272e-09, 6.180e-08), "backward": (1.251e-08, 3.304e-07),
                      "combined": (1.215e-08, 2.871e-07)},
    "ragged": {"forward": (1.190e-09, 2.430e-08), "backward": (1.608e-09, 6.001e-08),
               "combined": (1.976e-09, 4.275e-08)},
    "fixture": {"forward": (1.797e-07, 3.975e-07), "backward": (7.091e-07, 1.284e-06),
                "combined": (2.146e-07, 1.194e-06)},
    "c5_shard": {"combined": (1.431e-06, 1.893e-06)},
}


def pred_bound(case: str, output: str):
    """(mean, covariance) bound of one case's output: 2x its measured distance, at most PRED_TOL"""
    em, ec = PRED_MEASURED[case][output]
    return min(PRED_TOL, 2 * em), min(PRED_TOL, 2 * ec)


def _smoother_err(a, b):
    m_a, m_b = a[:, :4], b[:, :4]
    C_a, C_b = a[:, 4:].reshape(-1, 4, 4), b[:, 4:].reshape(-1, 4, 4)
    sd = np.sqrt(np.abs(np.einsum("nii->ni", C_b)))
    em = np.max(np.abs(m_a - m_b) / (np.abs(m_b) + sd).clip(1e-300))
    ec = np.max(np.abs(C_a - C_b) / (sd[:, :, None] * sd[:, None, :]).clip(1e-300))
    return float(em), float(ec)


_NOISE_SEEDS = (12345, 777, 4242)
_NOISE_CACHE = {}


def _oracle_noise(hf, params, case):
    """per output (forward, backward, combined): the ORACLE's own largest (mean, covariance) movement
    under +-1 ulp random noise on every exp() over three seeds (cached per case)"""
    if case not in _NOISE_CACHE:
        from oracle import oracle as O
        ref = O.OracleForest(hf.a).predict(params)
        moves = [O.OracleForest(hf.a, exp_ulp_noise=sd).predict(params) for sd in _NOISE_SEEDS]
        _NOISE_CACHE[case] = [(max(_smoother_err(mv[k], ref[k])[0] for mv in moves),
                               max(_smoother_err(mv[k], ref[k])[1] for mv in moves)) for k in range(3)]
    return _NOISE_CACHE[case]


def example_pred_bound(hf, params, case, output):
    """an example case's bound: pred_bound, or 3x the oracle's own +-1 ulp movement where larger"""
    bm, bc = pred_bound(case, output)
    nm, nc = _oracle_noise(hf, params, case)[("forward", "backward", "combined").index(output)]
    return max(bm, 3 * nm), max(bc, 3 * nc)


def _check_predict(hf, params, case, noise_seeds=()):
    """the device's -p rows against the oracle's: each output within its case's bound, or -- with
    noise_seeds -- within 3x the ORACLE's own movement under +-1 ulp random noise on every exp()
    (those seeds) where that is larger: the reference's filter on the example is conditioned so that
    an ulp anywhere moves the smoothed covariances by ~1e-5 of a standard deviation (measured
    2026-10: the oracle moves by up to 8.4e-6 by itself), so the device's distance is held against
    the reference algorithm's own rounding sensitivity rather than a fixed number"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    got = g.Forest(hf).predict(params)
    ref = O.OracleForest(hf.a).predict(params)
    for name, x, y in zip(("forward", "backward", "combined"), got, ref):
        assert np.all(np.isfinite(y)), name
        assert np.all(np.isfinite(x)), name
        em, ec = _smoother_err(x, y)
        bm, bc = example_pred_bound(hf, params, case, name) if noise_seeds else pred_bound(case, name)
        print(f"PRED_ERR {case} {name} mean {em:.3e} (bound {bm:.1e}) cov {ec:.3e} (bound {bc:.1e})")
        assert em < bm and ec < bc, (case, name, em, ec)


@pytest.mark.parametrize("noise,div", [("scaled", "binomial"), ("const", "gauss")])
def test_predict_example_vs_oracle(example_forests, noise, div):
    params = next(p for n, d, p in CONFIGS if (n, d) == (noise, div))
    _check_predict(example_forests[(noise, div)], params, f"example/{noise}/{div}", noise_seeds=_NOISE_SEEDS)


def test_predict_segments_vs_oracle():
    """two parameter segments switching along time (get_segment_indices, main.cpp:120-151)"""
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(40, 40)
    t = hf.a["time"]
    hf.a["segment"] = (t >= np.median(t)).astype(np.int32)
    P0 = np.array(CONFIGS[0][2])
    P1 = P0.copy()
    P1[0] *= 1.1
    P1[3] *= 0.95
    P1[7] *= 1.2
    _check_predict(hf, np.stack([P0, P1]), "segments")


@pytest.mark.parametrize("lane_smoother", [False, True])
def test_predict_four_segments_vs_oracle(lane_smoother, monkeypatch):
    """four parameter segments by time quartile, every parameter of each moved: the default
    schedule (lane-pair levels, k_combine after the backward pass) and the lane smoother with the
    combine fused into the backward pass, both against the oracle"""
    import gfp_gaussian_process_amd as g
    if lane_smoother:
        monkeypatch.setenv("GGP_SMOOTHER_LANE", "1")
    hf = g.HostForest.synthetic(50, 60, seed=11)
    t = hf.a["time"]
    hf.a["segment"] = np.searchsorted(np.quantile(t, [0.25, 0.5, 0.75]), t, side="right").astype(np.int32)
    assert set(np.unique(hf.a["segment"])) == {0, 1, 2, 3}
    P0 = np.array(CONFIGS[0][2])
    rng = np.random.default_rng(5)
    params = np.stack([P0 * np.exp(rng.uniform(-0.1, 0.1, 11)) if k else P0 for k in range(4)])
    _check_predict(hf, params, "four_segments")


@pytest.mark.parametrize("which", ["example", "segments", "ragged", "wide"])
def test_predict_split_smoother_bitwise_lane(example_forests, which, monkeypatch):
    """the smoother's levels on the lane-pair split (k_fwd_pair / k_bwd_pair, four or two waves
    per cell) give the lane smoother's bits: forward, backward and combined rows (the example's
    deep small levels, two parameter segments, ragged cells, and a forest whose 6000-cell and
    12000-cell levels take Q = 4 and Q = 2)"""
    import gfp_gaussian_process_amd as g
    P0 = np.array(CONFIGS[0][2])
    if which == "example":
        hf, params = example_forests[("scaled", "binomial")], P0
    elif which == "segments":
        hf = g.HostForest.synthetic(40, 40)
        hf.a["segment"] = (hf.a["time"] >= np.median(hf.a["time"])).astype(np.int32)
        P1 = P0.copy()
        P1[0] *= 1.1
        P1[7] *= 1.2
        params = np.stack([P0, P1])
    elif which == "ragged":
        hf, params = _ragged_roots(), P0
    else:
        hf, params = g.HostForest.synthetic(6000, 40), P0
    got = g.Forest(hf).predict(params)
    monkeypatch.setenv("GGP_SMOOTHER_LANE", "1")
    ref = g.Forest(hf).predict(params)
    for name, x, y in zip(("forward", "backward", "combined"), got, ref):
        assert np.array_equal(x, y), name


@pytest.mark.parametrize("which", ["segments", "example"])
def test_combine_fused_into_backward_pass_bitwise(example_forests, which, monkeypatch):
    """with every level on the lane smoother the backward pass forms the combined rows itself
    (k_bwd_level<true>); GGP_COMBINE_FUSED=0 runs k_combine after it: the same rows bitwise,
    whether or not the backward rows are asked for (the fused pass then does not store them)"""
    import gfp_gaussian_process_amd as g
    if which == "segments":
        hf = g.HostForest.synthetic(60, 40)
        hf.a["segment"] = (hf.a["time"] >= np.median(hf.a["time"])).astype(np.int32)
        P0 = np.array(CONFIGS[0][2])
        P1 = P0.copy()
        P1[0] *= 1.1
        P1[7] *= 1.2
        params = np.stack([P0, P1])
    else:
        hf, params = example_forests[("scaled", "binomial")], CONFIGS[0][2]
    monkeypatch.setenv("GGP_SMOOTHER_LANE", "1")
    fused = g.Forest(hf)
    full = fused.predict(params)
    comb_only = fused.predict(params, outputs=(False, False, True))[2]
    rows = fused.predict_rows(0, hf.n_rows)
    monkeypatch.setenv("GGP_COMBINE_FUSED", "0")
    sep = g.Forest(hf).predict(params)
    for name, x, y in zip(("forward", "backward", "combined"), full, sep):
        assert np.array_equal(x, y), name
    assert np.array_equal(comb_only, sep[2]) and np.array_equal(rows, sep[2])


@pytest.mark.parametrize("noise,div", [("scaled", "binomial"), ("const", "gauss")])
def test_combine_fast_form_vs_exact(example_forests, noise, div, monkeypatch):
    """k_combine's fast form (the default: reciprocal pivots, reassociated mean) against the
    same kernel with the oracle's operations (GGP_COMBINE_EXACT=1): forward and backward rows
    bitwise (only the combine differs), combined rows within 1e-9 in the smoother check's
    normalisation, and both within the example's combined-row bound of the oracle (pred_bound)"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = example_forests[(noise, div)]
    params = next(p for n, d, p in CONFIGS if (n, d) == (noise, div))
    got = g.Forest(hf).predict(params)
    monkeypatch.setenv("GGP_COMBINE_EXACT", "1")
    exact = g.Forest(hf).predict(params)
    assert np.array_equal(got[0], exact[0]) and np.array_equal(got[1], exact[1])
    em, ec = _smoother_err(got[2], exact[2])
    assert em < 1e-9 and ec < 1e-9, (em, ec)
    ref = O.OracleForest(hf.a).predict(params)[2]
    bm, bc = example_pred_bound(hf, params, f"example/{noise}/{div}", "combined")
    for x in (got[2], exact[2]):
        em, ec = _smoother_err(x, ref)
        print(f"PRED_ERR combine_form mean {em:.3e} cov {ec:.3e}")
        assert em < bm and ec < bc, (em, ec)


def test_predict_ragged_and_single_rows():
    _check_predict(_ragged_roots(), CONFIGS[0][2], "ragged")


def test_predict_leaves_carried_state_alone(example_forests):
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")]
    P = CONFIGS[0][2]
    a, b = g.Forest(hf), g.Forest(hf)
    a.total_likelihood(P)
    b.total_likelihood(P)
    a.predict(P)
    assert a.total_likelihood(P) == b.total_likelihood(P)


def test_predict_workspace_reuse_and_partial_outputs():
    """the handle keeps the -p workspace across calls (ggp_predict): a second predict with other
    segments, then a repeat of the first, give bitwise the first results; outputs that are not
    requested come back as None and the rest are unchanged; the profile hook reports device time"""
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(30, 40)
    P0 = np.array(CONFIGS[0][2])
    P1 = P0.copy()
    P1[0] *= 1.1
    f = g.Forest(hf)
    first = f.predict(P0)
    f.predict(np.stack([P0, P1]))
    again = f.predict(P0)
    for x, y in zip(first, again):
        assert np.array_equal(x, y)
    part = f.predict(P0, outputs=(False, False, True))
    assert part[0] is None and part[1] is None
    assert np.array_equal(part[2], first[2])
    sm, cb = f.predict_profile()
    assert sm > 0.0 and cb > 0.0
    f.close()


def _points(P, n, seed=11):
    rng = np.random.default_rng(seed)
    base = np.asarray(P, np.float64)
    return np.stack([base * (1.0 + 0.02 * rng.standard_normal(base.size)) for _ in range(n)])


def test_batch_bitwise_equals_lane_evaluations(example_forests):
    """ggp_total_loglik_batch: every point from the same carried state, bitwise a lane-schedule
    ggp_total_loglik from that state; the handle's carried state is left unchanged"""
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")]
    P0 = CONFIGS[0][2]
    pts = _points(P0, 6)
    a = g.Forest(hf, kernel="lane")
    a.total_likelihood(P0)                            # carried state after one call
    ll, nan = a.total_likelihood_batch(pts)
    assert not nan.any()
    for k, pt in enumerate(pts):
        b = g.Forest(hf, kernel="lane")
        b.total_likelihood(P0)
        assert b.total_likelihood(pt) == ll[k], k
        b.close()
    c = g.Forest(hf, kernel="lane")
    c.total_likelihood(P0)
    assert a.total_likelihood(P0) == c.total_likelihood(P0)   # batch did not touch the state


@pytest.mark.parametrize("n_trees,rows", [(40, 40), (3, 300)])
def test_batch_vs_oracle_fresh(n_trees, rows):
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(n_trees, rows)
    pts = _points(CONFIGS[0][2], 5, seed=n_trees)
    ll, nan = g.Forest(hf).total_likelihood_batch(pts)
    assert not nan.any()
    for k, pt in enumerate(pts):
        vo = O.OracleForest(hf.a).total_likelihood(pt)[0]
        assert _rel(ll[k], vo) < REL, k


def test_batch_nan_point_and_chunking(example_forests):
    """a NaN point is flagged without disturbing the others; many points (chunks of the lane
    schedule's grid.y) agree with the few-point call"""
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")]
    P0 = CONFIGS[0][2]
    pts = _points(P0, 3)
    bad = pts.copy()
    bad[1, 2] = -1.0                                  # var_lambda < 0 (as test_nan_reported_like_reference)
    f = g.Forest(hf)
    ll, nan = f.total_likelihood_batch(bad)
    assert list(nan) == [False, True, False]
    assert math.isnan(ll[1])
    ref, _ = f.total_likelihood_batch(pts)
    assert ll[0] == ref[0] and ll[2] == ref[2]
    many = np.repeat(pts, 200, axis=0)
    llm, nanm = f.total_likelihood_batch(many)
    assert not nanm.any()
    assert np.array_equal(llm, np.repeat(ref, 200))


def test_batched_hessian_matches_point_formula(example_forests):
    """num_hessian_batched = num_hessian_ll's expression over lane evaluations of the same points
    from the same state (ll_error_bars' batched mode)"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as opt
    hf = example_forests[("scaled", "binomial")]
    P0 = np.asarray(CONFIGS[0][2])
    idx = [0, 1, 3, 7]
    f = g.Forest(hf)
    H = opt.num_hessian_batched(f, P0, idx, 1e-2)
    pts, h = opt.hessian_points(P0, idx, 1e-2)
    ll = np.array([g.Forest(hf, kernel="lane").total_likelihood(p) for p in pts]).reshape(4, 4, 4)
    for i in range(4):
        for j in range(4):
            want = (ll[i, j, 0] - ll[i, j, 1] - ll[i, j, 2] + ll[i, j, 3]) / (4 * h[i] * h[j])
            assert H[i, j] == want


def _tests_h_cell():
    """the reference's own likelihood test cell (src/tests.h:263-300, commented out there): one
    root, 3 rows at t = 0, 15, 30, a prior covariance whose off-diagonals the root keeps
    (init_sc_distribution resets only the mean and the diagonal, predictions.h:63-78)"""
    import gfp_gaussian_process_amd as g
    cov = np.array([[4.25476409e-02, 4.81488709e+01, -6.17116203e-05, -1.25892662e-01],
                    [4.81488709e+01, 1.67680116e+06, 2.59861605e-01, 7.45274531e+02],
                    [-6.17116203e-05, 2.59861605e-01, 8.48575294e-07, 8.44383560e-05],
                    [-1.25892662e-01, 7.45274531e+02, 8.44383560e-05, 1.63738212e+00]])
    mean = np.array([6.93147181e-01, 6.03801845e+03, 1.00811380e-02, 9.56031050e+00])
    a = dict(row_offset=np.array([0, 3], np.int64), parent=np.array([-1], np.int32),
             daughter1=np.array([-1], np.int32), daughter2=np.array([-1], np.int32),
             segment=np.zeros(3, np.int32), time=np.array([0.0, 15.0, 30.0]),
             log_length=np.array([0.6621376048238568, 0.8057995840040671, 1.016156660637409]),
             fp=np.array([6031.236638936349, 6179.754023612084, 6351.815340631341]),
             root_mean_xg=mean[:2].copy(), root_var_xg=np.array([cov[0, 0], cov[1, 1]]),
             leaf_mean_xg=mean[:2].copy(), leaf_var_xg=np.array([cov[0, 0], cov[1, 1]]),
             noise_scaled=1, division_binomial=1, fp_auto=0.0)
    state = np.concatenate([mean, cov.ravel()])[None, :]
    params = [0.01, 0.01, 1e-05, 10, 0.01, 0.1, 0.001, 0.001, 5000.0, 0.001, 5000.0]
    return g.HostForest(a), state, params


@pytest.mark.parametrize("kernel", KERNELS)
def test_tests_h_cell_with_carried_covariance(kernel):
    """ggp_set_state puts the test cell's covariance in the carried state; the GPU then follows
    the oracle on it for three chained calls (parity unpinned against the reference binary: its
    test prints the value but records none)"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf, state, params = _tests_h_cell()
    fg, of = g.Forest(hf, kernel=kernel), O.OracleForest(hf.a)
    fg.set_state(state)
    of.state[:] = state
    assert np.array_equal(fg.state(), state)
    for call in range(3):
        vg = fg.total_likelihood(params)
        vo, nc, _ = of.total_likelihood(params)
        assert nc == -1 and math.isfinite(vo)
        assert _rel(vg, vo) < REL, (call, vg, vo)


def test_set_state_resumes_the_chain(example_forests):
    """checkpoint / resume: a forest given another's carried state continues its chain bitwise"""
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")]
    P = CONFIGS[0][2]
    a = g.Forest(hf)
    a.total_likelihood(P)
    a.total_likelihood(P)
    ckpt = a.state()
    b = g.Forest(hf)
    b.set_state(ckpt)
    for _ in range(2):
        assert b.total_likelihood(P) == a.total_likelihood(P)
    with pytest.raises(ValueError):
        b.set_state(ckpt[:-1])


def test_predict_example_vs_committed_fixture(example_forests):
    """GPU -p against the committed oracle fixture (first and last row of every cell), so the
    GPU box checks the smoother without rerunning the oracle"""
    import gfp_gaussian_process_amd as g
    gold = np.load(os.path.join(GOLDEN, "oracle_example_predict.npz"))
    hf = example_forests[("scaled", "binomial")]
    got = g.Forest(hf).predict(list(gold["params"]))
    rows = gold["rows"]
    for name, x in zip(("fwd", "bwd", "comb"), got):
        em, ec = _smoother_err(x[rows], gold[name])
        bm, bc = pred_bound("fixture", {"fwd": "forward", "bwd": "backward", "comb": "combined"}[name])
        print(f"PRED_ERR fixture {name} mean {em:.3e} cov {ec:.3e}")
        assert em < bm and ec < bc, (name, em, ec)


def test_tests_h_cell_vs_committed_fixture():
    import gfp_gaussian_process_amd as g
    gold = json.load(open(os.path.join(GOLDEN, "oracle_tests_h_cell.json")))
    hf, state, params = _tests_h_cell()
    assert np.array_equal(state.ravel(), [float.fromhex(x) for x in gold["state"]])
    f = g.Forest(hf)
    f.set_state(state)
    for want in gold["ll"]:
        assert _rel(f.total_likelihood(params), float.fromhex(want)) < REL


_GATHER_CHILD = r'''
import os, sys, time, json, math
sys.path.insert(0, ROOT)
import torch, torch.distributed as dist
import numpy as np
import gfp_gaussian_process_amd as g
from gfp_gaussian_process_amd.distributed import ShardedObjective
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
P = PARAMS
hf = g.HostForest.synthetic(1000, 200)
same, nan_ok, t, mode = True, True, {}, {}
b = g.Forest(hf)
keep = []   # comm-attached handles kept to the teardown below (the loop destroys the rest as it goes)
for name, ec in (("engine", True), ("torch", False)):   # RCCL inside the engine; torch's all_gather
    a = g.Forest(hf)
    obj = ShardedObjective(a, always_gather=True, engine_comm=ec)
    if ec: keep.append(a)
    mode[name] = obj.engine
    b.reset_state()
    same = same and all(obj.total_likelihood(P) == b.total_likelihood(P) for _ in range(3))
    for _ in range(5):   # fresh objectives: their first collective is ordered after the engine
        a2, b2 = g.Forest(hf), g.Forest(hf)
        same = same and ShardedObjective(a2, always_gather=True, engine_comm=ec).total_likelihood(P) == b2.total_likelihood(P)
        if ec and len(keep) < 3: keep.append(a2)
    # the chain (-s scan): with the engine's collective each chained call already returns the total
    pts = np.repeat(np.array(P)[None, :], 3, axis=0); pts[:, 1] = [0.02, 0.03, 0.04]
    a3, b3 = g.Forest(hf), g.Forest(hf)
    o3 = ShardedObjective(a3, always_gather=True, engine_comm=ec)
    if ec: keep.append(a3)
    same = same and np.array_equal(o3.total_likelihood_chain(pts), b3.total_likelihood_chain(pts))
    bad = list(P); bad[2] = -1.0
    try:   # on its own forest: a NaN evaluation leaves NaN in the carried state, as in the reference
        ShardedObjective(g.Forest(hf), always_gather=True, engine_comm=ec).total_likelihood(bad); nan_ok = False
    except g.LikelihoodIsNan as e:
        nan_ok = nan_ok and e.cell >= 0
    for nm, fn in (("direct", b.total_likelihood), (name, obj.total_likelihood)):
        for _ in range(20): fn(P)
        t0 = time.perf_counter()
        for _ in range(200): fn(P)
        t[nm] = 1e3 * (time.perf_counter() - t0) / 200
# teardown of comm-attached handles in a defined order (ORDER): each engine communicator is
# destroyed by its handle (ggp_forest_destroy: the shard's stream synchronised, ncclCommDestroy,
# then the streams), before or after torch's process group
attached = [o for o in keep if getattr(o, "_comm_rank", None) is not None]
if ORDER == "close_first":
    for o in attached: o.close()
    dist.destroy_process_group()
elif ORDER == "group_first":
    dist.destroy_process_group()
    for o in attached: o.close()
else:   # "exit": the group destroyed, the handles left to the interpreter's teardown
    dist.destroy_process_group()
print(json.dumps({"same": same, "nan_ok": nan_ok, "ms": t, "engine_mode": mode, "attached": len(attached)}), flush=True)
'''


@pytest.mark.parametrize("order", ["close_first", "group_first", "exit"])
def test_sharded_objective_collective_path_on_rccl(order):
    """ShardedObjective's two RCCL paths on a 1-rank nccl group in a child process -- the
    engine's own (ggp_comm_attach: partial, all-gather and rank-order sum on the engine's stream)
    and torch's (pinned staging, all_gather_into_tensor, combine_partials): bitwise the direct
    objective over a carried-state chain, NaN raised with this rank's cell; prints the per-call
    cost of each.  Then every comm-attached handle is destroyed explicitly before torch's process
    group, after it, or left to the interpreter's exit: the child exits 0 in every order (DESIGN
    §5: the round-3 SIGSEGV came from torch using an engine stream its owner had destroyed)."""
    import socket
    import subprocess
    import sys
    from conftest import ROOT
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    code = f"ROOT={ROOT!r}\nPARAMS={list(CONFIGS[0][2])!r}\nORDER={order!r}\n" + _GATHER_CHILD
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print("collective path ms/call:", out["ms"])
    assert out["engine_mode"] == {"engine": True, "torch": False}
    assert out["same"] and out["nan_ok"] and out["attached"] >= 1


def test_chain_stall_is_a_timeout_not_a_nan(monkeypatch):
    """A second daughter whose parent does not finish within the chain-wait limit (forced here:
    GGP_CHAIN_SPIN_MAX=0, the parent root still running) ends the evaluation with GGP_ETIMEOUT
    (EvaluationStalled), never as LikelihoodIsNan (likelihood.h:71-93 semantics are for real NaN
    only); the carried state is then unspecified, so the handle refuses the next evaluation until
    reset_state().  A handle made without the limit evaluates the same forest normally."""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import _native as N
    from oracle import oracle as O
    P = CONFIGS[0][2]
    hf = g.HostForest.synthetic(64, 200)          # path launch: roots of 100 rows, two daughters each
    monkeypatch.setenv("GGP_CHAIN_SPIN_MAX", "0")
    f = g.Forest(hf, kernel="wave")
    monkeypatch.delenv("GGP_CHAIN_SPIN_MAX")
    with pytest.raises(g.EvaluationStalled) as ei:
        f.total_likelihood(P)
    assert not isinstance(ei.value, g.LikelihoodIsNan)
    assert "stall" in str(ei.value)
    # the raw C-ABI: GGP_ETIMEOUT, no NaN location
    import ctypes
    lib = N.engine()
    ll, nc, nr = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
    p = np.ascontiguousarray(P, np.float64)
    rc = lib.ggp_total_loglik(f._h, p.ctypes.data_as(N.c_double_p), ctypes.byref(ll), ctypes.byref(nc), ctypes.byref(nr))
    assert rc == N.GGP_ETIMEOUT and nr.value == -1
    with pytest.raises(g.GGPError, match="unspecified"):
        f.total_likelihood(P)
    ok = g.Forest(hf, kernel="wave")
    ref = O.OracleForest(hf.a).total_likelihood(P)[0]
    assert _rel(ok.total_likelihood(P), ref) < REL


_DEVICE_CHILD = r"""
import json, sys
sys.path.insert(0, ROOT)
import torch                                   # torch's HIP runtime first (as in bench.py)
n = torch.cuda.device_count()
torch.cuda.set_device(n - 1)
import gfp_gaussian_process_amd as g
hf = g.HostForest.synthetic(32, 40)
seen = []
for devs in ([0], [0, 0], list(range(n))):
    f = g.Forest(hf, devices=devs)
    seen.append(torch.cuda.current_device())
    f.total_likelihood(PARAMS)
    seen.append(torch.cuda.current_device())
    f.predict([PARAMS])
    f.state()
    f.reset_state()
    seen.append(torch.cuda.current_device())
    f.close()
    seen.append(torch.cuda.current_device())
print(json.dumps({"n": n, "seen": seen}))
"""


def test_caller_device_restored_across_calls():
    """Every C-ABI entry point restores the caller's current HIP device (include/ggp.h): Forests on
    device 0, on two logical shards of it and on every device, driven from a process whose current
    device is the last visible one, leave it there after create / evaluate / predict / state /
    destroy (on a one-GPU box the last device is device 0: every entry point still runs once).
    In a child process: torch initialises its runtime before the engine, as bench.py does."""
    import subprocess
    import sys
    from conftest import ROOT
    code = f"ROOT={ROOT!r}\nPARAMS={list(CONFIGS[0][2])!r}\n" + _DEVICE_CHILD
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["seen"] and all(d == out["n"] - 1 for d in out["seen"]), out


def _row_err(a, b):
    """per row: max normalised mean / covariance difference (_smoother_err's normalisation)"""
    m_a, m_b = a[:, :4], b[:, :4]
    C_a, C_b = a[:, 4:].reshape(-1, 4, 4), b[:, 4:].reshape(-1, 4, 4)
    sd = np.sqrt(np.abs(np.einsum("nii->ni", C_b)))
    em = np.max(np.abs(m_a - m_b) / (np.abs(m_b) + sd).clip(1e-300), axis=1)
    ec = np.max(np.abs(C_a - C_b) / (sd[:, :, None] * sd[:, None, :]).clip(1e-300), axis=(1, 2))
    return np.maximum(em, ec)


@pytest.mark.parametrize("which", ["example", "c5_shape_2k"])
def test_predict_every_row_within_the_oracles_own_noise(example_forests, which):
    """-p row by row against a bar calibrated on the reference algorithm itself: the oracle under
    +-1 ulp noise on every exp() moves each row by some amount; EVERY GPU row (forward, backward,
    combined) must lie within max(FLOOR, 10 x that movement) of the oracle.  On the example the
    movement is measured here (three seeds); on 2,000 C5-shaped trees (1e6 rows) it comes from the
    committed calibration over twelve seeds (tests/golden/smoother_noise_c5shape_2k.npz,
    make_smoother_noise.py: three seeds had underestimated 29 rows' sensitivity by up to 1.7x, and
    round 4's test had been relaxed to 30x for them; twelve seeds cover them, and the 10x bar holds
    for every row again).  Everywhere the GPU's median error must not exceed the oracle's own median
    movement.  FLOOR = 1e-10 covers the combine's reciprocal pivots (<= 1.2e-11 from the exact form,
    test_combine_fast_form_vs_exact).  The exact-arithmetic engine holds every row at 1e-12
    (test_gpu_exact.py)."""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    FLOOR = 1e-10
    P = CONFIGS[0][2]
    if which == "example":
        hf = example_forests[("scaled", "binomial")]
        ref = O.OracleForest(hf.a).predict(P)
        noisy = [O.OracleForest(hf.a, exp_ulp_noise=s).predict(P) for s in (12345, 777, 4242)]
        moves = [np.max([_row_err(z[k], ref[k]) for z in noisy], axis=0) for k in range(3)]
    else:
        hf = g.HostForest.synthetic(2000, 500)
        ref = O.OracleForest(hf.a).predict(P)
        cal = np.load(os.path.join(GOLDEN, "smoother_noise_c5shape_2k.npz"))
        moves = [10.0 ** (cal[n].astype(np.float64) / 16.0 - 16.0) for n in ("forward", "backward", "combined")]
    got = g.Forest(hf).predict(P)
    for k, name in enumerate(("forward", "backward", "combined")):
        move = moves[k]
        assert len(move) == len(ref[k])
        e = _row_err(got[k], ref[k])
        bound = np.maximum(FLOOR, 10 * move)
        print(f"{which} {name}: rows {len(e)}, gpu err median {np.median(e):.2e} max {e.max():.2e}; "
              f"oracle noise median {np.median(move):.2e} max {move.max():.2e}; worst err/bound "
              f"{np.max(e / bound):.2f}")
        assert np.median(e) <= np.median(move), name
        bad = np.nonzero(~(e <= bound))[0]
        assert len(bad) == 0, (name, len(bad), bad[:5], e[bad[:5]], bound[bad[:5]])


@pytest.mark.parametrize("kernel", KERNELS)
def test_long_dt_forests_vs_oracle(kernel):
    """time steps of 1e3-1.6e4 units (gl dt up to ~700, where exp(-gl dt) nears the underflow and
    the lane schedules' product exponentials could meet 0 x inf; they then form the 22 products from
    their own arguments, ggp_prop.h lane_guard_products): two chained calls against the oracle --
    within the bar while the oracle is finite; where the reference algorithm itself breaks down (its
    tauint integrals overflow first: at 1.6e4 the second call) the GPU raises LikelihoodIsNan as
    well -- at which row is not determined there: the first call's carried off-diagonals are in the
    overflow regime (the exact engine, which rounds as the oracle does, reports the oracle's cell
    and row: test_gpu_exact.py)"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    P = CONFIGS[0][2]
    for scale in (1000.0, 5000.0, 16000.0):
        hf = g.HostForest.synthetic(20, 40, seed=5)
        hf.a["time"] = hf.a["time"] * scale
        fg, of = g.Forest(hf, kernel=kernel), O.OracleForest(hf.a)
        for call in range(2):
            vo, nc, nr = of.total_likelihood(P)
            if math.isnan(vo):
                with pytest.raises(g.LikelihoodIsNan):
                    fg.total_likelihood(P)
                break
            vg = fg.total_likelihood(P)
            assert _rel(vg, vo) < REL, (scale, call, vg, vo)
        fg.close()


@pytest.mark.parametrize("kernel", ["lane", "pair", "group"])
def test_mixed_long_dt_waves_bitwise(kernel, monkeypatch):
    """every fourth tree's times stretched x2000 (its steps risky: |gq dt| > 700, ggp_prop.h
    products_risky): a lane-schedule wave holding such a cell runs the step with its products
    materialised and guarded (propagate_lane's wave-uniform branch), a wave without one forms them at
    the integrals' reads.  The ordinary trees' carried state and -p rows (lane smoother) in the mixed
    forest equal, bitwise, the same trees evaluated alone (every wave ordinary); the mixed total is
    within the bar of the oracle"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    monkeypatch.setenv("GGP_SMOOTHER_LANE", "1")
    P = CONFIGS[0][2]
    hf = g.HostForest.synthetic(256, 40, seed=3)
    tree = hf.tree_of_cell()
    roots = hf.roots
    long_roots, plain_roots = roots[::4], np.setdiff1d(roots, roots[::4])
    ro = hf.a["row_offset"]
    for c in np.nonzero(np.isin(tree, long_roots))[0]:
        hf.a["time"][ro[c]:ro[c + 1]] = hf.a["time"][ro[c]:ro[c + 1]] * 2000.0
    sub = hf.subset_trees(plain_roots)
    fm, fs = g.Forest(hf, kernel=kernel), g.Forest(sub, kernel=kernel)
    vm = fm.total_likelihood(P)
    fs.total_likelihood(P)
    vo = O.OracleForest(hf.a).total_likelihood(P)[0]
    assert math.isfinite(vo) and _rel(vm, vo) < REL, (vm, vo)
    keep = np.nonzero(np.isin(tree, plain_roots))[0]
    assert np.array_equal(fm.state()[keep], fs.state())
    rows = np.concatenate([np.arange(ro[c], ro[c + 1]) for c in keep])
    for a, b in zip(fm.predict(P), fs.predict(P)):
        assert np.array_equal(a[rows], b)
    fm.close()
    fs.close()


def test_predict_many_segments_parameter_rows_from_global(monkeypatch):
    """40 parameter segments (time quantiles), more than the 32 rows the lane smoother stages in LDS
    (ggp_engine.hip kSegLds): the lane smoother reads them from global memory (k_fwd_level<false>,
    k_bwd_level<true, false>); its rows equal the lane-pair smoother's bitwise (every level of this
    forest fits the split) and lie within the smoother bar of the oracle"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(30, 60, seed=21)
    t = hf.a["time"]
    nseg = 40
    hf.a["segment"] = np.searchsorted(np.quantile(t, np.linspace(0, 1, nseg + 1)[1:-1]), t, side="right").astype(np.int32)
    assert len(np.unique(hf.a["segment"])) > 32   # (the times are whole minutes: some quantiles coincide)
    P0 = np.array(CONFIGS[0][2])
    rng = np.random.default_rng(8)
    params = np.stack([P0 * np.exp(rng.uniform(-0.05, 0.05, 11)) for _ in range(nseg)])
    split = g.Forest(hf).predict(params)
    monkeypatch.setenv("GGP_SMOOTHER_LANE", "1")
    lane = g.Forest(hf).predict(params)
    for name, x, y in zip(("forward", "backward", "combined"), lane, split):
        assert np.array_equal(x, y), name
    ref = O.OracleForest(hf.a).predict(params)
    for name, x, y in zip(("forward", "backward", "combined"), lane, ref):
        em, ec = _smoother_err(x, y)
        print(f"PRED_ERR 40 segments {name} mean {em:.3e} cov {ec:.3e}")
        assert em < PRED_TOL and ec < PRED_TOL, (name, em, ec)


def test_total_likelihood_parameter_forms(example_forests):
    """the 11 parameters as a list, a tuple or a numpy array give the same bits; any other count,
    or a non-number, is a ValueError before anything runs (the carried state is untouched)"""
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")]
    P = CONFIGS[0][2]
    vals = []
    for form in (list(P), tuple(P), np.asarray(P)):
        f = g.Forest(hf)
        vals.append(f.total_likelihood(form))
    assert vals[0] == vals[1] == vals[2]
    f = g.Forest(hf)
    for bad in (P[:10], list(P) + [1.0], [None] * 11, "abcdefghijk"):
        with pytest.raises(ValueError):
            f.total_likelihood(bad)
    assert f.total_likelihood(P) == vals[0]   # the failed calls ran nothing: still the first call
