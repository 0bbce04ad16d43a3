"""Wave-G schedule probe (diagnostic): parity of k_loglik_wg<G> against the oracle, then
per-level launch times against the lane / wave / auto schedules on C2, C3 and C4-shard
forests.  python tools/wg_probe.py [G ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gfp_gaussian_process_amd as g  # noqa: E402
from oracle import oracle as O  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
Gs = [int(x) for x in sys.argv[1:]] or [8, 16, 32]


def forest(hf, kernel, G=16):
    os.environ["GGP_WG_G"] = str(G)
    return g.Forest(hf, kernel=kernel)


def parity():
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_example.json")))
    import gzip
    import shutil
    import tempfile
    csv = os.path.join(tempfile.mkdtemp(), "input.csv")
    with gzip.open(os.path.join(ROOT, "tests", "golden", "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    cfg = os.path.join(ROOT, "tests", "golden", "example_csv_config.txt")
    out = {}
    for key, v in gold.items():
        noise, div = key.split("/")[:2]
        params = [float.fromhex(x) for x in v["params"]]
        hf = g.HostForest.from_csv(csv, cfg, -1, noise, div)
        of = O.OracleForest(hf.a)
        want = [of.total_likelihood(params)[0] for _ in range(3)]
        for G in Gs:
            f = forest(hf, "wg", G)
            got = [f.total_likelihood(params) for _ in range(3)]
            out[f"example {key} G={G}"] = max(abs(a - b) / abs(b) for a, b in zip(got, want))
    for trees in (300, 2000):
        hf = g.HostForest.synthetic(trees, 200)
        of = O.OracleForest(hf.a)
        want = [of.total_likelihood(P)[0] for _ in range(2)]
        for G in Gs:
            f = forest(hf, "wg", G)
            got = [f.total_likelihood(P) for _ in range(2)]
            out[f"synthetic {trees} G={G}"] = max(abs(a - b) / abs(b) for a, b in zip(got, want))
    return out


def timing(trees, rows=200, reps=20):
    hf = g.HostForest.synthetic(trees, rows)
    res = {}
    for name, kernel, G in [("lane", "lane", 16), ("auto", "auto", 16), ("wave", "wave", 16)] + \
            [(f"wg{G}", "wg", G) for G in Gs]:
        if name == "wave" and trees > 3000:
            continue
        f = forest(hf, kernel, G)
        for _ in range(3):
            f.total_likelihood(P)
        t0 = time.perf_counter()
        for _ in range(reps):
            v = f.total_likelihood(P)
        ms = 1e3 * (time.perf_counter() - t0) / reps
        f.enable_profile()
        f.total_likelihood(P)
        lv = [round(x, 4) for x in f.launch_profile()[0]]
        res[name] = {"ms": round(ms, 4), "levels_ms": lv, "ll": v}
        f.close()
    return res


if __name__ == "__main__":
    print(json.dumps({"parity": parity()}, indent=1), flush=True)
    for trees in (1000, 10000, 12500, 4000):
        print(json.dumps({"trees": trees, "t": timing(trees)}), flush=True)
