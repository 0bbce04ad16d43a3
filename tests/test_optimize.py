"""-m / -s numerics on the CPU: the NLopt 2.7.1 Nelder-Mead restatement, the Hessian error
bars, arange, and the CLI's argument checks (no GPU needed).

NLopt is not in this image, so these tests pin the restatement's documented behaviour
(initial simplex, bound pinning, fixed-dimension elimination, ftol_abs stop, exception
path) rather than an NLopt trajectory: "parity unpinned" for the optimiser.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.usefixtures("built")


def test_quadratic_with_a_fixed_dimension():
    from gfp_gaussian_process_amd import optimize as O
    seen = []

    def f(x):
        seen.append(x.copy())
        return (x[0] - 1) ** 2 + 10 * (x[1] + 2) ** 2 + 0.5 * x[2] ** 2

    x, fm, rc, nev = O.nldrmd_minimize(f, [0, 0, 3], [-5, -5, 3], [5, 5, 3], [0.5, 0.5, 1], 1e-12)
    assert rc == O.FTOL_REACHED and nev == len(seen)
    assert abs(x[0] - 1) < 1e-5 and abs(x[1] + 2) < 1e-5 and x[2] == 3
    assert all(s[2] == 3.0 for s in seen)                 # lb == ub: eliminated, never moved
    assert fm == min(f(s) for s in seen[:-1] + [seen[-1]])


def test_initial_simplex_and_step_turned_back_inside_bounds():
    from gfp_gaussian_process_amd import optimize as O
    seen = []

    def f(x):
        seen.append(x.copy())
        return float(np.sum(x ** 2))

    O.nldrmd_minimize(f, [1.0, 0.95, 0.0], [-1, -1, -1], [1, 1, 1], [0.3, 0.3, 0.3], 1e-3, maxeval=4)
    assert np.array_equal(seen[0], [1.0, 0.95, 0.0])            # the start point first
    assert np.array_equal(seen[1], [0.7, 0.95, 0.0])            # x + step beyond ub, ub too close: go back
    # nldrmd builds each vertex from x, which its CHECK_EVAL has already moved to the best
    # point so far ([0.7, 0.95, 0] is better than the start)
    assert np.array_equal(seen[2], [0.7, 1.0, 0.0])             # ub farther than step/10: pin to ub
    assert np.array_equal(seen[3], [0.7, 0.95, 0.3])


def test_points_stay_inside_bounds_and_rosenbrock_converges():
    from gfp_gaussian_process_amd import optimize as O
    lb, ub = np.array([-2.0, -1.0]), np.array([2.0, 3.0])
    seen = []

    def rb(x):
        seen.append(x.copy())
        return 100 * (x[1] - x[0] ** 2) ** 2 + (1 - x[0]) ** 2

    x, fm, rc, _ = O.nldrmd_minimize(rb, [-1.2, 1.0], lb, ub, [0.1, 0.1], 1e-14)
    assert rc == O.FTOL_REACHED
    assert np.all([np.all((s >= lb) & (s <= ub)) for s in seen])
    assert np.allclose(x, [1, 1], atol=1e-3) and fm < 1e-8


def test_objective_exception_propagates():
    from gfp_gaussian_process_amd import optimize as O
    calls = []

    def f(x):
        calls.append(1)
        if len(calls) == 5:
            raise FloatingPointError("Likelihood is Nan")
        return float(np.sum(x ** 2))

    with pytest.raises(FloatingPointError):
        O.nldrmd_minimize(f, [1.0, 1.0], [-2, -2], [2, 2], [0.1, 0.1], 1e-12)
    assert len(calls) == 5


def test_hessian_and_pplu_inverse():
    from gfp_gaussian_process_amd import optimize as O
    f = lambda x: 3 * x[0] ** 2 + 2 * x[0] * x[1] + 5 * x[1] ** 2 + x[2]   # noqa: E731
    H = O.num_hessian(f, [1.0, 2.0, 3.0], [0, 1], 1e-3)
    assert np.allclose(H, [[6, 2], [2, 10]], rtol=1e-6)
    A = np.random.default_rng(7).normal(size=(9, 9))
    assert np.allclose(O.inverse_pplu(A), np.linalg.inv(A), rtol=1e-10, atol=1e-12)
    # partial pivoting picks the first max |a|: a zero leading pivot is swapped out
    P = np.array([[0.0, 2.0], [3.0, 1.0]])
    assert np.allclose(O.inverse_pplu(P), np.linalg.inv(P))


def test_arange_accumulates_like_utils_h():
    from gfp_gaussian_process_amd import optimize as O
    assert O.arange(0.1, 0.4, 0.1) == [0.1, 0.2, 0.30000000000000004]
    assert O.arange(0.0, 1.0, 0.25) == [0.0, 0.25, 0.5, 0.75]


def test_minimize_wrapper_on_the_oracle_objective(example_paths):
    """-m in log space with two free parameters on a small synthetic forest, the CPU oracle
    as the objective: converges (FTOL), improves the likelihood, keeps fixed ones fixed"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as O
    from oracle import oracle as Or
    hf = g.HostForest.synthetic(20, 40)
    of = Or.OracleForest(hf.a)
    P = g.ParameterSet.load(example_paths["params"])
    P.kind = ["fixed"] * 11
    P.kind[7] = P.kind[8] = "free"                      # var_x, var_g
    P.lower[:] = 0.0
    P.upper[:] = np.inf
    objective = lambda p: of.total_likelihood(p)[0]     # noqa: E731
    ll0 = Or.OracleForest(hf.a).total_likelihood(P.init)[0]
    x, ll, rc = O.minimize_wrapper(objective, P, tolerance=1e-6, search_space="log")
    assert rc == O.FTOL_REACHED
    assert ll > ll0
    fixed = [i for i in range(11) if i not in (7, 8)]
    assert np.allclose(x[fixed], P.init[fixed], rtol=1e-15)
    err = O.ll_error_bars(objective, x, P, 1e-2)
    assert err.shape == (2,) and np.all(err > 0)


# ---- the CLI binary: argument handling (no device needed) ----------------------------------
CLI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gfp_gaussian_process_amd", "lib", "ggp")


def _cli(*args, cwd=None):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=120, cwd=cwd)


def test_cli_help_and_argument_errors(tmp_path, example_paths):
    r = _cli("-h")
    assert r.returncode == 0 and "Usage: ./gfp_gaussian [-options]" in r.stdout and "--parameter_bounds" in r.stdout
    r = _cli("-b", example_paths["params"])
    assert r.returncode == 1 and "Required infile flag not set" in r.stdout
    r = _cli("-i", str(tmp_path / "missing.csv"), "-b", example_paths["params"])
    assert r.returncode == 1 and "not found" in r.stdout
    r = _cli("-i", example_paths["csv"], "-b", example_paths["params"], "-space", "cubic")
    assert r.returncode == 1 and "search_space must be either 'log' or 'linear'" in r.stdout


def test_cli_fails_loudly_without_a_device(tmp_path, example_paths):
    """no CPU fallback: with no GPU the evaluation stops with an error, it does not compute"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    r = _cli("-i", example_paths["csv"], "-b", example_paths["params"], "-c", example_paths["config"], "-e",
             "-o", str(tmp_path / "out"))
    assert r.returncode == 1 and "Quit because of an error" in r.stdout
    assert os.path.exists(tmp_path / "out" / "input_error.log")


def test_hessian_points_match_num_hessian_visits():
    """the batched Hessian's points are exactly (bitwise, in order) those num_hessian_ll visits,
    and its expression over them gives num_hessian's matrix bitwise"""
    from gfp_gaussian_process_amd import optimize as O

    class Batch:
        def total_likelihood_batch(self, pts):
            return np.array([f(p) for p in pts]), np.zeros(len(pts), bool)

    seen = []

    def f(x):
        x = np.asarray(x, np.float64)
        return float(-3 * x[0] ** 2 + 2 * x[0] * x[1] - 5 * x[1] ** 2 + np.sin(x[3]) * x[0])

    def rec(x):
        seen.append(np.array(x, np.float64))
        return f(x)

    x = np.array([1.3, 0.2, 7.0, 0.4, 2e-13])
    idx = [0, 1, 3, 4]                                 # x[4] tiny: the 1e-12 step floor
    H = O.num_hessian(rec, x, idx, 1e-2)
    pts, h = O.hessian_points(x, idx, 1e-2)
    assert np.array_equal(np.array(seen), pts)
    assert np.array_equal(O.num_hessian_batched(Batch(), x, idx, 1e-2), H)
    assert h[3] == 1e-12


@pytest.mark.parametrize("n,fixed", [(10, -1), (4, 1), (2, -1)])
def test_lookahead_serves_the_same_calls(tmp_path, n, fixed):
    """the -m lookahead (ggp_nelder_mead.h Machine + speculate): the run makes the same calls with
    the same values as without it, and every call after the first is served from a speculated
    tree (parents listed before children, at most Lookahead::max_nodes points per tree)"""
    import shutil
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "nm_ahead_check")
    subprocess.run([cxx, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "gfp_gaussian_process_amd", "csrc", "host"),
                    "-o", exe, os.path.join(ROOT, "tests", "nm_ahead_check.cpp")], check=True)
    out = subprocess.run([exe, str(n), str(fixed)], capture_output=True, text=True, check=True).stdout.split()
    assert out[0] == "same", out
    calls, served, launches, max_nodes = map(int, out[1:])
    assert calls > 50 and served == calls - 1, out
    assert launches * 2 < calls and max_nodes <= 40, out


def test_chain_dispatch_only_for_the_forest_objective():
    """num_hessian / bound_1dscan / minimize_wrapper take the chained and lookahead engine calls
    only for a Forest or its own bound total_likelihood; a subclass overriding total_likelihood
    (a prior, a logging wrapper) or any other callable is called one call at a time"""
    from gfp_gaussian_process_amd import Forest
    from gfp_gaussian_process_amd.optimize import _chain_forest

    class WithPrior(Forest):
        def total_likelihood(self, params):
            return super().total_likelihood(params) - 1.0

    f = Forest.__new__(Forest)       # no device handle: only the dispatch is under test
    w = WithPrior.__new__(WithPrior)
    assert _chain_forest(f) is f
    assert _chain_forest(f.total_likelihood) is f
    assert _chain_forest(w) is None
    assert _chain_forest(w.total_likelihood) is None
    assert _chain_forest(lambda p: f.total_likelihood(p)) is None
    assert _chain_forest(f.state) is None


@pytest.mark.parametrize("name", ["fixed_dimension", "bound_pinned", "rugged_shrinks"])
def test_nelder_mead_call_sequences_are_pinned(name):
    """every objective call of three recorded runs of the restatement (a fixed dimension, a bound
    the optimum lies on, a rugged function whose simplex shrinks 3 times), bit for bit, and each
    run's result: tests/golden/make_nm_sequences.py froze the machine the GPU CLI's -m trajectory
    is checked against, so an edit of the machine or its lookahead cannot move it unnoticed"""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_nm_sequences as M
    want = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "nm_call_sequences.json")))[name]
    got = M.run(name)
    assert len(got["calls"]) == len(want["calls"])
    assert got["calls"] == want["calls"]
    assert (got["x"], got["minf"], got["rc"], got["nevals"]) == (want["x"], want["minf"], want["rc"], want["nevals"])
