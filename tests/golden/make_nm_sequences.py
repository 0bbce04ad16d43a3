"""Recorded call sequences of the Nelder-Mead restatement (csrc/host/ggp_nelder_mead.h), the
machine the GPU CLI's -m trajectory is checked against (tests/test_gpu_cli.py): every objective
call of three runs -- a fixed dimension eliminated, a bound the optimum lies on (points pinned),
and a rugged function whose run shrinks the simplex 3 times -- plus each run's result.
tests/test_optimize.py::test_nelder_mead_call_sequences_are_pinned replays them bit for bit, so a
later edit of the machine (or of its lookahead, which must make the same calls) cannot move the
trajectory unnoticed.  Regenerate only for a deliberate change of the algorithm:

    python tests/golden/make_nm_sequences.py   # -> tests/golden/nm_call_sequences.json
"""
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

PROBLEMS = {
    "fixed_dimension": dict(x0=[0.0, 0.0, 3.0], lb=[-5, -5, 3], ub=[5, 5, 3], dx=[0.5, 0.5, 1.0], tol=1e-12, maxeval=0),
    "bound_pinned": dict(x0=[-1.2, 1.0], lb=[-2.0, -1.0], ub=[0.8, 3.0], dx=[0.1, 0.1], tol=1e-14, maxeval=0),
    "rugged_shrinks": dict(x0=[1.5, -2.0, 0.9], lb=[-4, -4, -4], ub=[4, 4, 4], dx=[0.7, 0.7, 0.7], tol=1e-10,
                           maxeval=2000),
}


def objective(name, x):
    if name == "fixed_dimension":
        return (x[0] - 1) ** 2 + 10 * (x[1] + 2) ** 2 + 0.5 * x[2] ** 2
    if name == "bound_pinned":
        return 100 * (x[1] - x[0] ** 2) ** 2 + (1 - x[0]) ** 2
    return sum(x[i] * x[i] + 0.3 * math.sin(40 * x[i]) for i in range(3))


def run(name):
    from gfp_gaussian_process_amd import optimize as O
    p = PROBLEMS[name]
    calls = []

    def f(x):
        calls.append([float(v).hex() for v in x])
        return objective(name, [float(v) for v in x])
    x, fm, rc, nev = O.nldrmd_minimize(f, p["x0"], p["lb"], p["ub"], p["dx"], p["tol"], p["maxeval"])
    return {"calls": calls, "x": [float(v).hex() for v in x], "minf": float(fm).hex(), "rc": int(rc), "nevals": int(nev)}


if __name__ == "__main__":
    out = {name: run(name) for name in PROBLEMS}
    with open(os.path.join(HERE, "nm_call_sequences.json"), "w") as fh:
        json.dump(out, fh, indent=0)
    print({k: len(v["calls"]) for k, v in out.items()})
