"""-j on the GPU (ggp_joints) against the CPU oracle (oracle/ggp_oracle_joints.c).

The oracle restatement itself is validated on CPU (tests/test_oracle_joints.py) by an
identity of the model: with the constant noise model, the target marginal of every joint
equals the smoothed marginal of -p to ~1e-11.  Here the GPU joints are compared with the
oracle's: the set of (start, target) pairs (the walk stops where |C_ij / (m_i m_j)| falls
below the tolerance, so a pair whose ratio sits within rounding of the threshold may stop one
walk and not the other; every pair present on one side only must follow such a near-threshold
pair, one whose cross ratio is within 1e3 x tol -- see _compare) and the values of common pairs, normalised by the standard
deviations, at 1e-6.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
# The constant noise model on the synthetic forest (simulated with the scaled model, g ~ 3e4)
# needs a g noise variance of the data's order: with var_g = 0.826 the filter is overconfident
# by ~4 orders of magnitude and chaotic -- the ORACLE ITSELF moves by 0.2-0.9 sd of the smoothed
# marginals under +-1 ulp noise on exp() (tools/joints_diag.py; measured 2026-10), so no
# device/CPU comparison is meaningful there.  var_g = 2.6e4 makes it well conditioned (oracle
# self-sensitivity 9e-9), the same choice as tests/test_oracle_joints.py.
P_CONST = P[:8] + [2.6e4] + P[9:]


def _ratio(v):
    """max |C_ij / (m_i m_j)| over the cross block: the stop test of crosscovariance_is_small"""
    m, C = v[:8], v[8:].reshape(8, 8)
    return np.max(np.abs(C[:4, 4:] / np.outer(m[:4], m[4:])))


def _unexplained(ix, vx, other, tol, band):
    """pairs emitted by one side only must follow a threshold event: the walk of the other
    side stopped at a pair whose cross ratio is below band * tol (the noise floor of the tiny
    cross-covariances), and the diverging pairs run until the two walks meet again (the next
    sibling subtree).  Returns the pairs no such event explains and the largest event ratio."""
    bad, worst = [], 0.0
    starts = ix[:, 0]
    for s in np.unique(starts):
        boundary = False
        for n in np.nonzero(starts == s)[0]:
            key = (int(ix[n, 0]), int(ix[n, 1]))
            if key in other:
                boundary = False
                continue
            if boundary:
                continue
            d = _ratio(vx[n]) / tol
            worst = max(worst, d)
            if d < band:
                boundary = True
            else:
                bad.append((key, d))
    return bad, worst


def _norm_err(a, b):
    """per pair: max normalised mean and covariance difference (by the oracle's sds)"""
    sd = np.sqrt(np.abs(b[:, 8:].reshape(-1, 8, 8)[:, range(8), range(8)]))
    em = np.max(np.abs(a[:, :8] - b[:, :8]) / (np.abs(b[:, :8]) + sd), axis=1)
    ec = np.max(np.abs(a[:, 8:].reshape(-1, 8, 8) - b[:, 8:].reshape(-1, 8, 8))
                / (sd[:, :, None] * sd[:, None, :]), axis=(1, 2))
    return np.maximum(em, ec)


def _stable(io, vo, ip, vp, bound=1e-6):
    """pairs of the oracle that +-1 ulp noise on exp() moves by less than `bound`: the
    well-conditioned joints (the reference algorithm loses positive variances far along some
    walks, and those values are rounding noise in the reference itself)"""
    kp = {tuple(k): n for n, k in enumerate(ip.tolist())}
    keys = [tuple(k) for k in io.tolist()]
    both = [n for n, k in enumerate(keys) if k in kp]
    e = _norm_err(vp[[kp[keys[n]] for n in both]], vo[both])
    return {keys[n] for n, x in zip(both, e) if x < bound}


def _compare(ig, vg, io, vo, tol=1e-10, band=1e3, only=None):
    kg = {tuple(k): n for n, k in enumerate(ig.tolist())}
    ko = {tuple(k): n for n, k in enumerate(io.tolist())}
    common = sorted(set(kg) & set(ko))
    assert len(common) > 0
    # The stop rule compares a ratio of tiny cross-covariances (~1e-10 of m_i m_j, far below
    # the rounding noise of C - K S^-1 K^T at the scale of sd_i sd_j) with tol, so where a walk
    # ends is itself rounding-dominated: the ORACLE against itself with +-1 ulp noise on exp()
    # diverges on 4% of the example's pairs, each divergence starting at a pair whose ratio is
    # 1-64 x tol (tools/joints_diag.py).  Every divergence must start below band * tol, and the
    # pair sets must agree to within 10%.
    assert len(set(kg) ^ set(ko)) <= 0.1 * len(ko), (len(set(kg) ^ set(ko)), len(ko))
    bad_g, wg = _unexplained(ig, vg, ko, tol, band)
    bad_o, wo = _unexplained(io, vo, kg, tol, band)
    assert not bad_g and not bad_o, (bad_g[:5], bad_o[:5], len(kg), len(ko))
    if only is not None:
        common = [k for k in common if k in only]
    e = _norm_err(vg[[kg[k] for k in common]], vo[[ko[k] for k in common]])
    return float(e.max()), float(np.median(e)), len(common)


@pytest.mark.parametrize("noise,div", [(1, 1), (0, 0), (1, 0), (0, 1)])
def test_joints_synthetic_vs_oracle(noise, div):
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.synthetic(4, 40)
    hf.a["noise_scaled"] = noise
    hf.a["division_binomial"] = div
    p = P if noise else P_CONST
    ig, vg = g.Forest(hf).joints(p, 1e-10)
    io, vo = O.OracleForest(hf.a).joints(p, 1e-10)
    err, _, n = _compare(ig, vg, io, vo)
    assert err < 1e-6, (err, n)


def test_joints_example_subset_vs_oracle(example_paths):
    """the reference's example, start rows in the first root cell and around a division.
    The example's joints are far less well conditioned than the synthetic forest's: the oracle
    against itself under +-1 ulp exp() noise moves them by 5e-7 (median, normalised), and two
    noise seeds differ by up to 3e-5 on the pairs either seed moves < 1e-6 (measured).  Values
    are compared on those stable pairs (at least half; the rest are rounding noise in the
    reference algorithm itself, some with negative variances): max < 1e-4, median < 1e-5."""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.from_csv(example_paths["csv"], example_paths["config"], -1, "scaled", "binomial")
    fg, of, op = g.Forest(hf), O.OracleForest(hf.a), O.OracleForest(hf.a, exp_ulp_noise=12345)
    ro = hf.a["row_offset"]
    last = int(ro[1]) - 1                       # the first cell's last row (a division if it has daughters)
    for lo, hi in ((0, 40), (max(0, last - 20), last + 1)):
        ig, vg = fg.joints(P, 1e-10, lo, hi, cap=1 << 21)
        io, vo = of.joints(P, 1e-10, lo, hi, cap=1 << 21)
        ip, vp = op.joints(P, 1e-10, lo, hi, cap=1 << 21)
        stable = _stable(io, vo, ip, vp)
        assert len(stable) >= 0.5 * len(io), (lo, hi, len(stable), len(io))
        err, med, n = _compare(ig, vg, io, vo, only=stable)
        assert err < 1e-4 and med < 1e-5, (lo, hi, err, med, n)
