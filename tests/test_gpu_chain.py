"""ggp_total_loglik_chain: a known sequence of objective calls, each from the carried state the
previous one left (num_hessian_ll's 4k^2 calls, likelihood.h:211-258; the -s scan, main.cpp:80-114),
in one chained launch.  The bar is bitwise: every value, the NaN location and the carried state
afterwards equal those of the same calls made one by one through ggp_total_loglik (which the
parity tests hold against the oracle at 1e-9); one oracle check on top.
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]

PARAMS = json.load(open(os.path.join(GOLDEN, "oracle_example.json")))
P0 = np.array([float.fromhex(x) for x in PARAMS["scaled/binomial/example"]["params"]])


def _points(n, seed=5, scale=0.02):
    rng = np.random.default_rng(seed)
    return np.stack([P0 * (1.0 + scale * rng.standard_normal(P0.size)) for _ in range(n)])


@pytest.fixture(scope="module")
def example(example_paths):
    import gfp_gaussian_process_amd as g
    return g.HostForest.from_csv(example_paths["csv"], example_paths["config"])


def _sequential(hf, pts, warm=1, **kw):
    import gfp_gaussian_process_amd as g
    f = g.Forest(hf, **kw)
    for _ in range(warm):
        f.total_likelihood(P0)
    ll = np.array([f.total_likelihood(p) for p in pts])
    return ll, f.state()


def _chained(hf, pts, warm=1, **kw):
    import gfp_gaussian_process_amd as g
    f = g.Forest(hf, **kw)
    for _ in range(warm):
        f.total_likelihood(P0)
    ll = f.total_likelihood_chain(pts)
    return ll, f.state(), f


def test_chain_bitwise_sequential_on_the_example(example):
    """the reference's example (one tree, 77 cells, path launch): 40 points chained through the
    root's carried state; values and the state afterwards bitwise the one-by-one calls, and the
    handle continues the chain like a handle that made the calls itself"""
    pts = _points(40)
    want, st_want = _sequential(example, pts)
    got, st_got, f = _chained(example, pts)
    assert np.array_equal(got, want)
    assert np.array_equal(st_got, st_want)
    import gfp_gaussian_process_amd as g
    h = g.Forest(example)
    h.set_state(st_want)
    assert f.total_likelihood(P0) == h.total_likelihood(P0)


def test_chain_fresh_state_vs_oracle(example):
    """from fresh cells (read_data's zero state), the chained values against the oracle's own
    chained calls at 1e-9"""
    from oracle import oracle as O
    pts = _points(6, seed=9)
    got, _, _ = _chained(example, pts, warm=0)
    of = O.OracleForest(example.a)
    for k, p in enumerate(pts):
        vo, nc, _ = of.total_likelihood(p)
        assert nc == -1
        assert abs(got[k] - vo) / abs(vo) < 1e-9, k


@pytest.mark.parametrize("devices", [(0,), (0, 0, 0)])
def test_chain_many_trees_and_shards(devices):
    """a 48-tree forest (roots, first and second daughters: waits within a point and across
    points), whole or in three logical shards: bitwise the sequential calls"""
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(48, 120)
    pts = _points(25, seed=2)
    want, st_want = _sequential(hf, pts, devices=list(devices))
    got, st_got, _ = _chained(hf, pts, devices=list(devices))
    assert np.array_equal(got, want)
    assert np.array_equal(st_got, st_want)


def test_chain_chunks(example, monkeypatch):
    """points split over launches (GGP_BATCH_CHUNK=7: the carried state handed from one chunk's
    last point to the next chunk's first) give the same bits"""
    pts = _points(23, seed=4)
    want, st_want = _sequential(example, pts)
    monkeypatch.setenv("GGP_BATCH_CHUNK", "7")
    got, st_got, _ = _chained(example, pts)
    assert np.array_equal(got, want)
    assert np.array_equal(st_got, st_want)


def test_chain_level_launch_handles_run_one_by_one(example, monkeypatch):
    """handles without the path launch (lane schedule; GGP_CHAIN_FUSED=0) take the call-by-call
    form: the same values"""
    pts = _points(5, seed=8)
    want, _ = _sequential(example, pts, kernel="lane")
    got, _, _ = _chained(example, pts, kernel="lane")
    assert np.array_equal(got, want)
    want_w, _ = _sequential(example, pts)
    monkeypatch.setenv("GGP_CHAIN_FUSED", "0")
    got_w, _, _ = _chained(example, pts)
    assert np.array_equal(got_w, want_w)


def test_chain_stops_at_the_first_nan_point(example):
    """a NaN point (var_lambda < 0) raises LikelihoodIsNan with the sequential call's cell and
    row; .point is its index and .ll the values before it, bitwise the sequential ones; the
    handle then refuses to evaluate until its state is reset (include/ggp.h "Errors")"""
    import gfp_gaussian_process_amd as g
    pts = _points(9, seed=3)
    pts[6, 2] = -1.0
    f = g.Forest(example)
    f.total_likelihood(P0)
    seq = []
    with pytest.raises(g.LikelihoodIsNan) as es:
        for p in pts:
            seq.append(f.total_likelihood(p))
    c = g.Forest(example)
    c.total_likelihood(P0)
    with pytest.raises(g.LikelihoodIsNan) as ec:
        c.total_likelihood_chain(pts)
    assert ec.value.point == 6 and len(seq) == 6
    assert np.array_equal(ec.value.ll, np.array(seq))
    assert (ec.value.cell, ec.value.row) == (es.value.cell, es.value.row)
    with pytest.raises(g.GGPError, match="unspecified"):
        c.total_likelihood(P0)
    c.reset_state()
    assert math.isfinite(c.total_likelihood(P0))


def test_chain_empty_and_bad_shapes(example):
    import gfp_gaussian_process_amd as g
    f = g.Forest(example)
    assert f.total_likelihood_chain(np.zeros((0, 11))).shape == (0,)
    with pytest.raises(ValueError):
        f.total_likelihood_chain(np.zeros((2, 10)))


def test_hessian_chained_equals_num_hessian(example):
    """optimize.num_hessian on a Forest's objective (the chained call) is bitwise num_hessian_ll
    over one-by-one calls (ggp_num_hessian with a callback), carried state included"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as opt
    idx = [0, 1, 3, 7]
    a = g.Forest(example)
    a.total_likelihood(P0)
    H_chain = opt.num_hessian(a.total_likelihood, P0, idx, 1e-2)
    b = g.Forest(example)
    b.total_likelihood(P0)
    H_seq = opt.num_hessian(lambda p: b.total_likelihood(p), P0, idx, 1e-2)
    assert np.array_equal(H_chain, H_seq)
    assert np.array_equal(a.state(), b.state())


def test_python_minimize_lookahead_is_the_same_run(example, tmp_path, monkeypatch):
    """optimize.minimize_wrapper on a Forest objective takes the lookahead
    (ggp_nldrmd_minimize_ahead + ggp_total_loglik_tree): the same result, evaluation count and
    carried state as the call-by-call run (GGP_NM_LOOKAHEAD=0)"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as opt
    names = ["mean_lambda", "gamma_lambda", "var_lambda", "mean_q", "gamma_q", "var_q", "beta",
             "var_x", "var_g", "var_dx", "var_dg"]
    free = {0: "2.31E-03, 2.31E-04", 7: "3.35E-04, 3.35E-05", 8: "8.26E-01, 8.26E-02"}
    pf = tmp_path / "p.txt"
    pf.write_text("".join(f"{n} = {free.get(i, repr(float(P0[i])))}\n" for i, n in enumerate(names)))
    P = g.ParameterSet.load(str(pf))
    runs = {}
    for tag in ("seq", "ahead"):
        if tag == "seq":
            monkeypatch.setenv("GGP_NM_LOOKAHEAD", "0")
        else:
            monkeypatch.delenv("GGP_NM_LOOKAHEAD", raising=False)
        f = g.Forest(example)
        calls = []
        orig = f.total_likelihood

        def counted(p, orig=orig, calls=calls):   # the calls the run makes (not the speculated ones)
            calls.append(np.array(p, copy=True))
            return orig(p)
        x, ll, rc = opt.minimize_wrapper(f.total_likelihood if tag == "ahead" else counted, P, tolerance=1e-3,
                                         search_space="log", maxeval=400)
        runs[tag] = (x, ll, rc, f.state(), len(calls))
    a, b = runs["seq"], runs["ahead"]
    assert np.array_equal(a[0], b[0]) and a[1] == b[1] and a[2] == b[2]
    assert np.array_equal(a[3], b[3])
    assert a[4] > 50


def test_python_scan_chained_equals_calls(example, tmp_path):
    """optimize.bound_1dscan on a Forest objective (one chained call per parameter) gives the
    call-by-call values bitwise, and leaves the same carried state"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as opt
    names = ["mean_lambda", "gamma_lambda", "var_lambda", "mean_q", "gamma_q", "var_q", "beta",
             "var_x", "var_g", "var_dx", "var_dg"]
    bound = {8: "8.26E-01, 1.0E-01, 4.0E-01, 1.3E+00", 7: "3.35E-04, 1.0E-04, 1.0E-04, 9.0E-04"}
    pf = tmp_path / "p.txt"
    pf.write_text("".join(f"{n} = {bound.get(i, repr(float(P0[i])))}\n" for i, n in enumerate(names)))
    P = g.ParameterSet.load(str(pf))
    a, b = g.Forest(example), g.Forest(example)
    ra = opt.bound_1dscan(a.total_likelihood, P)
    rb = opt.bound_1dscan(lambda p: b.total_likelihood(p), P)
    assert ra == rb and sum(len(v) for v in ra.values()) > 10
    assert np.array_equal(a.state(), b.state())


@pytest.mark.parametrize("devices", [(0,), (0, 0, 0)])
def test_tree_points_bitwise_their_call_sequences(devices):
    """ggp_total_loglik_tree: every point's value is bitwise a ggp_total_loglik call made after
    the calls of its predecessor chain (emulated with state snapshots), the carried state is left
    alone, and keep_point_state(i) adopts exactly the state point i's call leaves -- on one shard
    and on three logical shards of a 48-tree forest"""
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(48, 120)
    pts = _points(7, seed=12)
    pred = np.array([-1, 0, 0, 1, 1, 2, 4], np.int32)
    f = g.Forest(hf, devices=list(devices))
    f.total_likelihood(P0)
    st0 = f.state()
    ll, status, nc, nr = f.total_likelihood_tree(pts, pred)
    assert (status == 0).all() and (nc == -1).all()
    assert np.array_equal(f.state(), st0)                      # nothing adopted yet
    e = g.Forest(hf, devices=list(devices))
    after = {}
    for i in range(len(pts)):
        e.set_state(st0 if pred[i] < 0 else after[pred[i]])
        assert e.total_likelihood(pts[i]) == ll[i], i
        after[i] = e.state()
    for i in (6, 3, 0):
        f.keep_point_state(i)
        assert np.array_equal(f.state(), after[i]), i


# ---- stalls of the chained and speculative schedules (include/ggp.h ggp_total_loglik_chain) ----
# GGP_CHAIN_SPIN_MAX=0 (read when a handle is created) makes every wait that finds its cell not
# done time out at once: a point's roots waiting for the previous point's, a second daughter for
# its parent.  A forest of roots only has no wait inside a point, so its one-by-one calls never
# stall there while its chained and tree launches do.

def _roots_only(hf):
    import gfp_gaussian_process_amd as g
    a = hf.a
    ro = a["row_offset"]
    roots = np.nonzero(a["parent"] == -1)[0]
    rows = np.concatenate([np.arange(ro[c], ro[c + 1]) for c in roots])
    b = dict(a)
    b["row_offset"] = np.concatenate([[0], np.cumsum(ro[roots + 1] - ro[roots])]).astype(np.int64)
    for k in ("parent", "daughter1", "daughter2"):
        b[k] = np.full(len(roots), -1, np.int32)
    for k in ("segment", "time", "log_length", "fp"):
        b[k] = np.ascontiguousarray(a[k][rows])
    return g.HostForest(b)


def _stalling(hf, monkeypatch, **kw):
    import gfp_gaussian_process_amd as g
    monkeypatch.setenv("GGP_CHAIN_SPIN_MAX", "0")
    f = g.Forest(hf, kernel="wave", **kw)
    monkeypatch.delenv("GGP_CHAIN_SPIN_MAX")
    return f


def test_chain_stall_finishes_call_by_call(monkeypatch):
    """a chained launch whose waits time out (point 1's roots find point 0's still running) is
    the schedule's failure, not the calls': the chain adopts the last completed point's state and
    runs the rest one by one -- values and carried state bitwise the sequential calls', no
    EvaluationStalled, one fallback counted"""
    import gfp_gaussian_process_amd as g
    hf = _roots_only(g.HostForest.synthetic(48, 400))   # 48 roots of 200 rows: point 0 is still running
    pts = _points(12)
    want, st_want = _sequential(hf, pts, kernel="wave")
    f = _stalling(hf, monkeypatch)
    f.total_likelihood(P0)
    got = f.total_likelihood_chain(pts)
    assert np.array_equal(got, want)
    assert np.array_equal(f.state(), st_want)
    assert f.chain_fallbacks() == 1
    more = _points(3, seed=9)   # the handle goes on like one that made the calls itself
    w2 = g.Forest(hf, kernel="wave")
    w2.set_state(st_want)
    assert np.array_equal(f.total_likelihood_chain(more), np.array([w2.total_likelihood(p) for p in more]))


def test_chain_stall_raises_when_the_calls_stall_too(monkeypatch):
    """with second daughters the one-by-one calls wait too: the chain ends as EvaluationStalled
    (GGP_ETIMEOUT), never LikelihoodIsNan, at point 0 with no values"""
    import ctypes
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import _native as N
    f = _stalling(g.HostForest.synthetic(64, 200), monkeypatch)
    with pytest.raises(g.EvaluationStalled) as ei:
        f.total_likelihood_chain(_points(5))
    assert not isinstance(ei.value, g.LikelihoodIsNan)
    assert ei.value.point == 0 and ei.value.ll.size == 0
    f2 = _stalling(g.HostForest.synthetic(64, 200), monkeypatch)
    pts = np.ascontiguousarray(_points(5), np.float64)
    ll = np.zeros(5)
    n_ok, nc, nr = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
    rc = N.engine().ggp_total_loglik_chain(f2._h, 5, pts.ctypes.data_as(N.c_double_p), ll.ctypes.data_as(N.c_double_p),
                                           ctypes.byref(n_ok), ctypes.byref(nc), ctypes.byref(nr))
    assert rc == N.GGP_ETIMEOUT and n_ok.value == 0 and nr.value == -1


def test_tree_stall_statuses(monkeypatch):
    """ggp_total_loglik_tree under stalls: points from the carried state (pred -1) complete,
    bitwise the one-by-one call; points that wait on another point report GGP_ETIMEOUT, never
    GGP_ENAN"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import _native as N
    hf = _roots_only(g.HostForest.synthetic(48, 400))
    pts = _points(6, seed=3)
    pred = np.array([-1, 0, 0, 1, -1, 4], np.int32)
    f = _stalling(hf, monkeypatch)
    f.total_likelihood(P0)
    ll, st, nc, nr = f.total_likelihood_tree(pts, pred)
    assert st[0] == N.GGP_OK and st[4] == N.GGP_OK
    assert all(int(v) in (N.GGP_OK, N.GGP_ETIMEOUT) for v in st)
    assert st[1] == N.GGP_ETIMEOUT and st[5] == N.GGP_ETIMEOUT
    ref = g.Forest(hf, kernel="wave")
    ref.total_likelihood(P0)
    st0 = ref.state()
    assert ll[0] == ref.total_likelihood(pts[0])
    ref.set_state(st0)
    assert ll[4] == ref.total_likelihood(pts[4])


def test_minimize_lookahead_with_stalls_matches_call_by_call(monkeypatch):
    """-m's lookahead on a handle whose speculative launches stall: a stalled node is not served,
    its call runs as usual from the last served node's state -- the optimiser's result and the
    carried state are those of the call-by-call run"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as opt
    hf = _roots_only(g.HostForest.synthetic(16, 80))
    P = g.ParameterSet.load(os.path.join(GOLDEN, "example_parameter_file.txt"))
    a = _stalling(hf, monkeypatch)
    xa, lla, rca = opt.minimize_wrapper(a.total_likelihood, P, tolerance=1e-6, maxeval=120)
    monkeypatch.setenv("GGP_NM_LOOKAHEAD", "0")
    b = g.Forest(hf, kernel="wave")
    xb, llb, rcb = opt.minimize_wrapper(b.total_likelihood, P, tolerance=1e-6, maxeval=120)
    assert rca == rcb and lla == llb and np.array_equal(xa, xb)
    assert np.array_equal(a.state(), b.state())


def test_chain_rows_cap_chunks_bitwise(monkeypatch, example):
    """the cap on chained root rows per launch (2^22; here 1000 rows: four of the example's
    243-row root per launch) splits a chain into launches with the same values and state"""
    pts = _points(11, seed=8)
    want, st_want = _sequential(example, pts)
    monkeypatch.setenv("GGP_CHAIN_ROWS_PER_LAUNCH", "1000")
    got, st_got, _ = _chained(example, pts)
    assert np.array_equal(got, want) and np.array_equal(st_got, st_want)
