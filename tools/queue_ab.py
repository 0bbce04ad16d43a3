"""A/B of the lane queue (GGP_LANE_QUEUE=1, k_loglik_lane_queue) against level-by-level lane
launches on C4 (BASELINE configs[3]: 1e5 trees x 200 rows, one GPU): ms per evaluation and the
profiled launches, after a full-chip preheat: python tools/queue_ab.py [trees]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
trees = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
hf = g.HostForest.synthetic(trees, 200)
fs = {}
for q in ("0", "1"):
    os.environ["GGP_LANE_QUEUE"] = q
    fs[q] = g.Forest(hf)
vals = {}
for rnd in range(3):
    for q, f in fs.items():
        f.reset_state()
        for _ in range(2):
            f.total_likelihood(P)
        t0 = time.perf_counter()
        for _ in range(10):
            v = f.total_likelihood(P)
        dt = (time.perf_counter() - t0) / 10
        vals.setdefault(q, []).append(v)
        f.enable_profile()
        f.total_likelihood(P)
        ms, rows, names = f.launch_profile()
        f.disable_profile()
        print(f"queue={q} trees={trees} {dt * 1e3:.3f} ms/eval  launches " +
              ", ".join(f"{n} {m:.3f} ms ({r / 1e6:.1f}M rows)" for m, r, n in zip(ms, rows, names)), flush=True)
print("bitwise equal:", vals["0"] == vals["1"])
