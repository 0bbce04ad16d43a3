"""Lane-pair stress check (diagnostic): random parameter sets (log-uniform around the example's,
as an optimiser explores them) on forests whose levels take the lane-pair schedule with Q = 4 and
Q = 2, chained evaluations through the auto policy (GGP_AUTO_SMALL=group: every schedule bitwise
lane) against the lane schedule -- totals, NaN
locations and carried states bitwise equal; then -p on the split smoother against the lane one.
python tools/pair_stress.py [N_PARAM_SETS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gfp_gaussian_process_amd as g  # noqa: E402

P0 = np.array([2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01,
               1.63e-04, 7.48e-01])
n_sets = int(sys.argv[1]) if len(sys.argv) > 1 else 200
rng = np.random.default_rng(20261017)
bad = 0
for trees, rows in ((6000, 200), (3000, 80), (12000, 40)):
    hf = g.HostForest.synthetic(trees, rows)
    os.environ["GGP_SMOOTHER_LANE"] = "0"
    os.environ["GGP_AUTO_SMALL"] = "group"   # small levels on the group schedule: all bitwise lane
    auto = g.Forest(hf)
    os.environ["GGP_SMOOTHER_LANE"] = "1"
    lane = g.Forest(hf, kernel="lane")
    auto.enable_profile()
    auto.total_likelihood(P0)
    kinds = auto.launch_profile()[2]
    auto.reset_state()
    n_nan = 0
    for k in range(n_sets):
        p = P0 * np.exp(rng.normal(0.0, 0.3 if k % 2 else 1.5, size=11))   # wide sets hit NaNs
        try:
            a = auto.total_likelihood(p)
        except g.LikelihoodIsNan as e:
            a = ("nan", e.cell, e.row)
            auto.reset_state()
        try:
            b = lane.total_likelihood(p)
        except g.LikelihoodIsNan as e:
            b = ("nan", e.cell, e.row)
            lane.reset_state()
        n_nan += isinstance(b, tuple)
        if a != b:
            bad += 1
            print("MISMATCH", trees, rows, k, a, b, flush=True)
    same_state = bool(np.array_equal(auto.state(), lane.state()))
    bad += not same_state
    pa, pl = auto.predict(P0), lane.predict(P0)
    same_pred = all(np.array_equal(x, y) for x, y in zip(pa, pl))
    bad += not same_pred
    print(f"{trees} trees x {rows}: schedules {kinds}, {n_sets} chained sets ({n_nan} NaN), states equal {same_state}, "
          f"-p equal {same_pred}", flush=True)
print("mismatches:", bad)
sys.exit(1 if bad else 0)
