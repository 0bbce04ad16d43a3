"""Lane-pair schedule probe (diagnostic): bitwise equality of k_loglik_pair<CPW> with the lane
schedule (totals over a carried-state chain and the carried state), then per-level launch
times against the lane and auto schedules on C2, C3 and C4-shard shaped forests.
  python tools/pair_probe.py [TREES ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def forest(hf, kernel, cpw=64, q=0):
    os.environ["GGP_PAIR_CPW"] = str(cpw)
    os.environ["GGP_PAIR_Q"] = str(q)
    return g.Forest(hf, kernel=kernel)


def bitwise(trees):
    hf = g.HostForest.synthetic(trees, 200)
    ref = forest(hf, "lane")
    want = [ref.total_likelihood(P) for _ in range(3)]
    st = ref.state()
    out = {}
    for q in (2, 4):
        for cpw in (32, 64):
            f = forest(hf, "pair", cpw, q)
            got = [f.total_likelihood(P) for _ in range(3)]
            out[f"{trees} q{q} cpw{cpw}"] = {"same_ll": got == want, "same_state": bool(np.array_equal(f.state(), st))}
    return out


def timing(trees, reps=20):
    hf = g.HostForest.synthetic(trees, 200)
    res = {}
    for name, kernel, cpw, q in (("lane", "lane", 64, 0), ("auto", "auto", 64, 0), ("q2c64", "pair", 64, 2),
                                 ("q4c64", "pair", 64, 4), ("q4c32", "pair", 32, 4)):
        f = forest(hf, kernel, cpw, q)
        for _ in range(3):
            f.total_likelihood(P)
        t0 = time.perf_counter()
        for _ in range(reps):
            v = f.total_likelihood(P)
        ms = 1e3 * (time.perf_counter() - t0) / reps
        f.enable_profile()
        f.total_likelihood(P)
        res[name] = {"ms": round(ms, 4), "levels_ms": [round(x, 4) for x in f.launch_profile()[0]], "ll": v}
        f.close()
    return res


if __name__ == "__main__":
    sizes = [int(x) for x in sys.argv[1:]] or [12500, 10000, 4000, 30000]
    print(json.dumps({"bitwise": {**bitwise(300), **bitwise(5000)}}), flush=True)
    for t in sizes:
        print(json.dumps({"trees": t, "t": timing(t)}), flush=True)
