"""The -j oracle (oracle/ggp_oracle_joints.c) checked by an identity of the model: with the
constant noise model every joint's target marginal is the smoothed marginal of -p (both
are P(z_target | all data)), computed here through a different chain of operations.  With
the scaled model the reference uses the cell's post -p mean in the noise term
(correlation_tree.h:485-490), so the identity does not hold there; that case is covered by
the GPU comparison (tests/test_gpu_joints.py).  Parity with a reference binary: unpinned.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.usefixtures("built")
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 2.6e4, 1.63e-04, 7.48e-01]


@pytest.mark.parametrize("div", [1, 0])
def test_joint_target_marginal_is_the_smoothed_marginal(div):
    """binomial: everywhere, across divisions too.  gauss: within the start's cell only -- the
    reference's gauss branch of consecutive_*_cell_division joins the forward marginal of the
    last row to the division map without the propagation over the division's dt
    (correlation_tree.h:203-229), so past a division it is a different distribution from the
    smoother's (which propagates, predictions.h:28-31); the restatement keeps that."""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(3, 40)
    a = dict(hf.a)
    a["noise_scaled"] = 0
    a["division_binomial"] = div
    of = O.OracleForest(a)
    idx, val = of.joints(P, 1e-10)
    _, _, comb = of.predict(P)
    assert len(idx) > 500
    cell = np.searchsorted(a["row_offset"], np.arange(len(a["time"])), "right") - 1
    crossed, worst = 0, 0.0
    for (s, t), v in zip(idx, val):
        across = cell[s] != cell[t]
        crossed += int(across)
        if across and not div:
            continue
        rm, rC = comb[t, :4], comb[t, 4:].reshape(4, 4)
        sd = np.sqrt(np.abs(np.diag(rC)))
        e = max(np.max(np.abs(v[:4] - rm) / (np.abs(rm) + sd)),
                np.max(np.abs(v[8:].reshape(8, 8)[:4, :4] - rC) / np.outer(sd, sd)))
        worst = max(worst, e)
    assert worst < 1e-9, worst
    assert crossed > 0                        # walks do cross divisions


def test_joint_walk_structure():
    """targets follow the start in the walk order: the rest of the start's cell, then the
    daughter1 subtree before the daughter2 subtree; a leaf's last row starts nothing"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(2, 40)
    idx, _ = O.OracleForest(hf.a).joints(P, 1e-10)
    ro = hf.a["row_offset"]
    starts = set(idx[:, 0].tolist())
    for c in range(len(ro) - 1):
        if hf.a["daughter1"][c] < 0:
            assert int(ro[c + 1]) - 1 not in starts
    for s in list(starts)[:10]:
        t = idx[idx[:, 0] == s, 1]
        assert np.all(t > s) and np.all(np.diff(t) > 0)   # synthetic rows: d1 rows precede d2 rows
