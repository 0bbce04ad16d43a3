"""Armed objective calls (ggp_arm, include/ggp.h; csrc/ggp_engine.hip arm_wait / arm_ring): each
call enqueues the next call's path launch, which stages its call-independent tables and waits for
the parameters the next call writes through a door in mapped host memory.  The evaluation after the
door is the plain path launch's, so every total, carried state and NaN location is bitwise the plain
calls' (those are checked against the oracle in test_gpu_parity.py).  Reference: the objective call
sequence of the optimiser, gaussian_process.cpp / minimizer (one total per parameter point)."""
import time

import numpy as np
import pytest

from test_gpu_parity import CONFIGS, example_forests  # noqa: F401

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]


def _points(P, k):
    """k parameter points near P (the first parameter scaled by 1 + 0.01 i)"""
    out = []
    for i in range(k):
        q = list(P)
        q[0] = q[0] * (1.0 + 0.01 * i)
        out.append(q)
    return out


def _pair(hf):
    import gfp_gaussian_process_amd as g
    plain = g.Forest(hf, kernel="wave")
    armed = g.Forest(hf, kernel="wave")
    armed.arm(True)
    return plain, armed


@pytest.mark.parametrize("which", ["example", "c2"])
def test_armed_calls_bitwise_plain(example_forests, which):
    """five chained calls at different parameters, the carried state, then a call after another
    entry point (the armed launch left): the plain calls' bits, and the calls ran armed"""
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")] if which == "example" else g.HostForest.synthetic(1000, 200)
    plain, armed = _pair(hf)
    pts = _points(CONFIGS[0][2], 5)
    # the plain handle's calls first: a waiting armed launch holds the compute units it occupies
    want = [plain.total_likelihood(q) for q in pts]
    want_state = plain.state()
    want2 = [plain.total_likelihood(q) for q in pts[:2]]
    want3 = plain.total_likelihood(pts[3])
    assert [armed.total_likelihood(q) for q in pts] == want
    assert armed.arm(None) == 4          # the first call is plain (nothing was armed yet)
    assert np.array_equal(armed.state(), want_state)
    assert [armed.total_likelihood(q) for q in pts[:2]] == want2
    assert armed.arm(None) == 5
    armed.arm(False)
    assert armed.total_likelihood(pts[3]) == want3
    assert armed.arm(None) == 5


def test_armed_expiry_runs_plain():
    """a call more than 50 ms after the previous one finds its armed launch expired: it runs as a
    plain launch (same bits), the next call is plain and arms the one after it"""
    import gfp_gaussian_process_amd as g
    plain, armed = _pair(g.HostForest.synthetic(300, 200))
    pts = _points(CONFIGS[0][2], 4)
    want = [plain.total_likelihood(q) for q in pts]
    assert armed.total_likelihood(pts[0]) == want[0]
    time.sleep(0.15)
    assert armed.total_likelihood(pts[1]) == want[1]
    assert armed.arm(None) == 0
    assert armed.total_likelihood(pts[2]) == want[2]
    assert armed.total_likelihood(pts[3]) == want[3]
    assert armed.arm(None) == 1


def test_armed_nan_location(example_forests):
    """var_lambda < 0 through the door: the first NaN (cell, row) of the plain launch"""
    import gfp_gaussian_process_amd as g
    hf = example_forests[("scaled", "binomial")]
    plain, armed = _pair(hf)
    P = CONFIGS[0][2]
    bad = list(P)
    bad[2] = -1.0
    got = []
    for f in (plain, armed):
        f.total_likelihood(P)
        with pytest.raises(g.LikelihoodIsNan) as e:
            f.total_likelihood(bad)
        got.append((e.value.cell, e.value.row))
    assert got[0] == got[1]
    assert armed.arm(None) == 1


def test_armed_then_other_entry_points(example_forests):
    """batch, chain, predict and state after armed calls: each makes the armed launch leave first,
    so each gives the plain handle's values at once (no 50 ms wait behind the armed launch)"""
    hf = example_forests[("scaled", "binomial")]
    plain, armed = _pair(hf)
    pts = _points(CONFIGS[0][2], 3)
    for f in (plain, armed):
        f.total_likelihood_batch(pts)    # (the batch's first-call allocations, outside the timing)
        f.total_likelihood(pts[0])
        f.total_likelihood(pts[1])
    t0 = time.perf_counter()
    b_a = armed.total_likelihood_batch(pts)
    t_a = time.perf_counter() - t0
    t0 = time.perf_counter()
    b_p = plain.total_likelihood_batch(pts)
    t_p = time.perf_counter() - t0
    assert t_a < t_p + 0.02, (t_a, t_p)   # not behind a waiting launch's 50 ms
    assert np.array_equal(np.asarray(b_a[0]), np.asarray(b_p[0]))
    for f in (plain, armed):
        f.total_likelihood(pts[2])
    assert np.array_equal(armed.total_likelihood_chain(pts), plain.total_likelihood_chain(pts))
    for f in (plain, armed):
        f.total_likelihood(pts[0])
    pa, pp = armed.predict(pts[0]), plain.predict(pts[0])
    for x, y in zip(pa, pp):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    want = plain.total_likelihood(pts[1])
    assert armed.total_likelihood(pts[1]) == want
