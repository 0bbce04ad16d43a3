"""The lane queue (k_loglik_lane_queue, csrc/ggp_engine.hip): a run of consecutive lane-schedule
levels in one persistent launch whose workgroups take 64-cell chunks from a counter, a later
level's chunk waiting for its cells' parents' done flags.  The cell body is the lane schedule's,
so every total, carried state and NaN location is bitwise what the level-by-level launches give
(GGP_LANE_QUEUE=0); those are checked against the oracle in test_gpu_parity.py.  Reference:
likelihood.h:110-122 (a daughter after its parent, nothing else ordered)."""
import numpy as np
import pytest

from test_gpu_parity import CONFIGS, REL, _ragged_roots, _rel, example_forests  # noqa: F401

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]


def _pair(hf, monkeypatch, kernel="lane"):
    import gfp_gaussian_process_amd as g
    monkeypatch.setenv("GGP_LANE_QUEUE", "0")
    lv = g.Forest(hf, kernel=kernel)
    monkeypatch.setenv("GGP_LANE_QUEUE", "1")
    q = g.Forest(hf, kernel=kernel)
    monkeypatch.delenv("GGP_LANE_QUEUE")
    return lv, q


@pytest.mark.parametrize("which", ["example", "synthetic", "example-const-gauss"])
def test_queue_bitwise_level_launches(example_forests, which, monkeypatch):
    """three chained calls and the carried state: the queue's bits are the level launches'"""
    import gfp_gaussian_process_amd as g
    hf = {"example": lambda: example_forests[("scaled", "binomial")],
          "example-const-gauss": lambda: example_forests[("const", "gauss")],
          "synthetic": lambda: g.HostForest.synthetic(300, 40)}[which]()
    P = next(c[2] for c in CONFIGS if (c[0], c[1]) == ("const", "gauss")) if which.endswith("gauss") else CONFIGS[0][2]
    lv, q = _pair(hf, monkeypatch)
    for _ in range(3):
        assert q.total_likelihood(P) == lv.total_likelihood(P)
    assert np.array_equal(q.state(), lv.state())
    q.enable_profile()
    q.total_likelihood(P)
    names = q.launch_profile()[2]
    assert names == ["k_loglik_lane_queue"], names   # every level of these forests in one run
    lv.enable_profile()
    lv.total_likelihood(P)
    assert set(lv.launch_profile()[2]) == {"k_loglik_level"}


def test_queue_single_level_forest_takes_level_launch(monkeypatch):
    """a forest of roots only has no run of two levels: one k_loglik_level launch, as before"""
    hf = _ragged_roots()
    P = CONFIGS[0][2]
    lv, q = _pair(hf, monkeypatch)
    assert q.total_likelihood(P) == lv.total_likelihood(P)
    q.enable_profile()
    q.total_likelihood(P)
    assert q.launch_profile()[2] == ["k_loglik_level"]


def test_queue_c4_shape_auto_bitwise(monkeypatch):
    """C4-shaped levels (40k roots of 100 rows, 80k daughters of 50): auto takes the lane
    schedule for both, in one queue launch, bitwise the level launches; the oracle on a slice of
    the same trees"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(40000, 200)
    P = CONFIGS[0][2]
    lv, q = _pair(hf, monkeypatch, kernel="auto")
    for _ in range(2):
        assert q.total_likelihood(P) == lv.total_likelihood(P)
    assert np.array_equal(q.state(), lv.state())
    q.enable_profile()
    q.total_likelihood(P)
    ms, rows, names = q.launch_profile()
    assert names == ["k_loglik_lane_queue"] and rows == [40000 * 200]
    sub = g.HostForest.synthetic(200, 200)              # the first 200 trees of the same stream
    fs = g.Forest(sub, kernel="lane")
    assert _rel(fs.total_likelihood(P), O.OracleForest(sub.a).total_likelihood(P)[0]) < REL


def test_queue_nan_location_is_the_level_launches(example_forests, monkeypatch):
    """var_lambda < 0: the first NaN (cell, row) in reference order, as the levels and the oracle"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = example_forests[("scaled", "binomial")]
    bad = list(CONFIGS[0][2])
    bad[2] = -1.0
    lv, q = _pair(hf, monkeypatch)
    got = []
    for f in (lv, q):
        with pytest.raises(g.LikelihoodIsNan) as e:
            f.total_likelihood(bad)
        got.append((e.value.cell, e.value.row))
    _, oc, orow = O.OracleForest(hf.a).total_likelihood(bad)
    assert got[0] == got[1] == (oc, orow)


def test_queue_wait_limit_is_a_stall(monkeypatch):
    """GGP_CHAIN_SPIN_MAX=0: a daughter chunk taken while its roots still run (64 trees: one root
    chunk, two daughter chunks on other workgroups) stops waiting at once and reports a stall
    (GGP_ETIMEOUT, EvaluationStalled), never a value or a NaN; without the limit the same forest
    evaluates to the level launches' bits"""
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(64, 200)
    P = CONFIGS[0][2]
    monkeypatch.setenv("GGP_CHAIN_SPIN_MAX", "0")
    f = g.Forest(hf, kernel="lane")
    monkeypatch.delenv("GGP_CHAIN_SPIN_MAX")
    with pytest.raises(g.EvaluationStalled) as ei:
        f.total_likelihood(P)
    assert not isinstance(ei.value, g.LikelihoodIsNan)
    lv, q = _pair(hf, monkeypatch)
    assert q.total_likelihood(P) == lv.total_likelihood(P)
