"""-j on the GPU (ggp_joints) against the CPU oracle (oracle/ggp_oracle_joints.c).

The oracle restatement itself is validated on CPU (tests/test_oracle_joints.py) by an
identity of the model: with the constant noise model, the target marginal of every joint
equals the smoothed marginal of -p to ~1e-11.  Here the GPU joints are compared with the
oracle's: the set of (start, target) pairs (the walk stops where |C_ij / (m_i m_j)| falls
below the tolerance, so a pair whose ratio sits within rounding of the threshold may differ;
the test allows 0.1% of pairs) and the values of common pairs, normalised by the standard
deviations, at 1e-6.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def _compare(ig, vg, io, vo):
    kg = {tuple(k): n for n, k in enumerate(ig.tolist())}
    ko = {tuple(k): n for n, k in enumerate(io.tolist())}
    common = sorted(set(kg) & set(ko))
    diff = set(kg) ^ set(ko)
    assert len(common) > 0
    assert len(diff) <= max(2, 1e-3 * len(ko)), (len(diff), len(ko))
    a = vg[[kg[k] for k in common]]
    b = vo[[ko[k] for k in common]]
    sd = np.sqrt(np.abs(b[:, 8:].reshape(-1, 8, 8)[:, range(8), range(8)]))
    em = np.max(np.abs(a[:, :8] - b[:, :8]) / (np.abs(b[:, :8]) + sd))
    ec = np.max(np.abs(a[:, 8:].reshape(-1, 8, 8) - b[:, 8:].reshape(-1, 8, 8)) / (sd[:, :, None] * sd[:, None, :]))
    return em, ec, len(common)


@pytest.mark.parametrize("noise,div", [(1, 1), (0, 0), (1, 0)])
def test_joints_synthetic_vs_oracle(noise, div):
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(4, 40)
    hf.a["noise_scaled"] = noise
    hf.a["division_binomial"] = div
    ig, vg = g.Forest(hf).joints(P, 1e-10)
    io, vo = O.OracleForest(hf.a).joints(P, 1e-10)
    em, ec, n = _compare(ig, vg, io, vo)
    assert em < 1e-6 and ec < 1e-6, (em, ec, n)


def test_joints_example_subset_vs_oracle(example_paths):
    """the reference's example, start rows in the first root cell and around a division"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.from_csv(example_paths["csv"], example_paths["config"], -1, "scaled", "binomial")
    fg, of = g.Forest(hf), O.OracleForest(hf.a)
    ro = hf.a["row_offset"]
    last = int(ro[1]) - 1                       # the first cell's last row (a division if it has daughters)
    for lo, hi in ((0, 40), (max(0, last - 20), last + 1)):
        ig, vg = fg.joints(P, 1e-10, lo, hi, cap=1 << 21)
        io, vo = of.joints(P, 1e-10, lo, hi, cap=1 << 21)
        em, ec, n = _compare(ig, vg, io, vo)
        assert em < 1e-6 and ec < 1e-6, (lo, hi, em, ec, n)
