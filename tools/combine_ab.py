"""A/B of a -p build against another (diagnostic): python tools/combine_ab.py OLD_LIB_DIR
runs the C5-shard smoother with the package's libggp.so and with OLD_LIB_DIR's in two
processes, and compares device times and the combined rows bitwise on a small forest."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, hashlib
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native
if LIB: _native.LIB_DIR = LIB
import numpy as np
import gfp_gaussian_process_amd as g
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
small = g.Forest(g.HostForest.synthetic(300, 60))
f, b, c = small.predict(P)
h = hashlib.sha256(f.tobytes() + b.tobytes() + c.tobytes()).hexdigest()
big = g.Forest(g.HostForest.synthetic(125000, 500))
big.predict(P, outputs=(False, False, False))
sm, cb = [], []
for _ in range(5):
    big.predict(P, outputs=(False, False, False))
    a_, b_ = big.predict_profile()
    sm.append(a_); cb.append(b_)
print(json.dumps({"sha": h, "smooth_ms": sorted(sm)[2], "combine_ms": sorted(cb)[2]}))
'''
out = {}
for tag, lib in (("new", ""), ("old", os.path.abspath(sys.argv[1])), ("new2", ""), ("old2", os.path.abspath(sys.argv[1]))):
    code = f"ROOT={ROOT!r}\nLIB={lib!r}\n" + CHILD
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(tag, "failed", r.stderr[-2000:])
        sys.exit(1)
    out[tag] = json.loads(r.stdout.strip().splitlines()[-1])
    print(tag, out[tag], flush=True)
print("bitwise equal:", out["new"]["sha"] == out["old"]["sha"])
