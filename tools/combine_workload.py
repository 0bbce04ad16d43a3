"""-p workload for PMC passes (diagnostic): one warm-up and one timed ggp_predict on a C5-shaped
forest (500 rows per tree), outputs left in HBM.  python tools/combine_workload.py [TREES]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
trees = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
hf = g.HostForest.synthetic(trees, 500)
f = g.Forest(hf)
f.predict(P, outputs=(False, False, False))
f.predict(P, outputs=(False, False, False))
sm, cb = f.predict_profile()
print(json.dumps({"trees": trees, "rows": hf.n_rows, "cells": f.n_cells, "smooth_ms": sm, "combine_ms": cb}))
