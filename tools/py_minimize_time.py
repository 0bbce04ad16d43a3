"""optimize.minimize_wrapper on the example (the example parameter file: 10 free parameters, log
space) with a Forest objective: call by call (a plain function objective) against the lookahead
(the Forest's bound total_likelihood).  One JSON line: wall seconds, calls, identical result."""
import gzip
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402
from gfp_gaussian_process_amd import optimize as opt  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
d = tempfile.mkdtemp()
csv = os.path.join(d, "input.csv")
with gzip.open(os.path.join(GOLD, "example_input.csv.gz"), "rb") as a, open(csv, "wb") as b:
    shutil.copyfileobj(a, b)
hf = g.HostForest.from_csv(csv, os.path.join(GOLD, "example_csv_config.txt"))
P = g.ParameterSet.load(os.path.join(GOLD, "example_parameter_file.txt"))
res = {}
for tag in ("call_by_call", "lookahead"):
    f = g.Forest(hf)
    n = [0]

    def plain(p, f=f, n=n):
        n[0] += 1
        return f.total_likelihood(p)
    t0 = time.perf_counter()
    x, ll, rc = opt.minimize_wrapper(plain if tag == "call_by_call" else f.total_likelihood, P, tolerance=1e-10,
                                     search_space="log")
    res[tag] = {"wall_s": time.perf_counter() - t0, "ll": ll, "rc": rc, "x": [float(v) for v in x],
                "state_sha": __import__("hashlib").sha256(f.state().tobytes()).hexdigest()[:16]}
    if tag == "call_by_call":
        res[tag]["calls"] = n[0]
    print(tag, res[tag]["wall_s"], file=sys.stderr, flush=True)
res["identical"] = all(res["call_by_call"][k] == res["lookahead"][k] for k in ("ll", "rc", "x", "state_sha"))
res["speedup"] = res["call_by_call"]["wall_s"] / res["lookahead"]["wall_s"]
shutil.rmtree(d, ignore_errors=True)
print(json.dumps(res))
