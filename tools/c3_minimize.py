"""BASELINE configs[2] (C3) on one GPU: the 10k trees x 200 tp synthetic forest, a log-space
Nelder-Mead run with all 11 parameters free (the -m loop: optimize.nldrmd_minimize, the NLopt
LN_NELDERMEAD restatement, over the GPU objective), bounded at a fixed evaluation count.
Prints one JSON line: evaluations/s, updates/s, the objective before and after."""
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import gfp_gaussian_process_amd as g  # noqa: E402
from gfp_gaussian_process_amd import optimize as opt  # noqa: E402

P = np.array([2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01,
              1.63e-04, 7.48e-01])
maxeval = int(sys.argv[1]) if len(sys.argv) > 1 else 400
t0 = time.perf_counter()
hf = g.HostForest.synthetic(10000, 200)
f = g.Forest(hf)
t_build = time.perf_counter() - t0
n_eval = [0]


def obj(x):          # minimize_wrapper's log-space form: exp() first, then -ll (likelihood.h:161-167)
    n_eval[0] += 1
    return -f.total_likelihood(np.exp(x))


x0 = np.log(P)
first = obj(x0)
t1 = time.perf_counter()
xb, fb, rc, ne = opt.nldrmd_minimize(obj, x0, x0 - math.log(10.0), x0 + math.log(10.0),
                                     np.full(11, math.log(1.1)), 1e-10, maxeval)
el = time.perf_counter() - t1
print(json.dumps({"config": "C3: synthetic 10000 trees x 200 tp, -m log-space Nelder-Mead, 11 free parameters",
                  "rows": hf.n_rows, "evaluations": ne, "seconds": el, "evals_per_s": ne / el,
                  "updates_per_s": ne * hf.n_rows / el, "ms_per_eval": 1e3 * el / ne,
                  "neg_ll_start": first, "neg_ll_best": fb, "nlopt_result": rc,
                  "forest_build_s": t_build, "note": "bounded at maxeval; the optimiser steps are sequential "
                  "(carried state), each one GPU evaluation"}))
