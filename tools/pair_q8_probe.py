"""Lane-pair Q = 8 probe (diagnostic): eight waves per 64-cell workgroup (two per SIMD) against
Q = 4 and the auto policy on C4-shard / C3 shaped forests: bitwise equality with the lane schedule
(totals over a carried-state chain and the carried state), then per-level launch times, alternated.
  python tools/pair_q8_probe.py [TREES ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def forest(hf, kernel, q=0):
    os.environ["GGP_PAIR_Q"] = str(q)
    return g.Forest(hf, kernel=kernel)


def main(sizes, reps=30, rounds=3):
    for trees in sizes:
        hf = g.HostForest.synthetic(trees, 200)
        ref = forest(hf, "lane")
        want = [ref.total_likelihood(P) for _ in range(3)]
        st = ref.state()
        ref.close()
        out = {"trees": trees}
        fs = {}
        for name, kernel, q in (("auto", "auto", 0), ("pair_q4", "pair", 4), ("pair_q8", "pair", 8)):
            f = forest(hf, kernel, q)
            got = [f.total_likelihood(P) for _ in range(3)]
            out[name + "_bitwise"] = bool(got == want and np.array_equal(f.state(), st))
            fs[name] = f
        ms = {k: [] for k in fs}
        lv = {}
        for _ in range(rounds):
            for name, f in fs.items():
                for _ in range(3):
                    f.total_likelihood(P)
                t0 = time.perf_counter()
                for _ in range(reps):
                    f.total_likelihood(P)
                ms[name].append(1e3 * (time.perf_counter() - t0) / reps)
        for name, f in fs.items():
            f.enable_profile()
            f.total_likelihood(P)
            lv[name] = [round(x, 4) for x in f.launch_profile()[0]]
            f.close()
        out["ms"] = {k: [round(x, 4) for x in v] for k, v in ms.items()}
        out["levels_ms"] = lv
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [12500, 10000, 6000])
