"""In-process A/B of an engine switch read at forest creation (diagnostic):
python tools/env_ab.py VAR [trees] -- forests built with VAR=0 and VAR=1 on the same C2-shaped
forest, alternating timed blocks; prints ms/eval (median of 6 blocks) and whether the values
agree."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gfp_gaussian_process_amd as g  # noqa: E402

var = sys.argv[1]
trees = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
hf = g.HostForest.synthetic(trees, 200)
forests = {}
for v in ("0", "1"):
    os.environ[var] = v
    forests[v] = g.Forest(hf, device=0)
res, vals = {"0": [], "1": []}, {"0": [], "1": []}
for rep in range(6):
    for v, f in forests.items():
        for _ in range(5):
            f.total_likelihood(P)
        t0 = time.perf_counter()
        for _ in range(50):
            x = f.total_likelihood(P)
        res[v].append(1e3 * (time.perf_counter() - t0) / 50)
        vals[v].append(x)
for v in res:
    r = sorted(res[v])
    print(f"{var}={v} trees={trees}: ms/eval median {r[len(r) // 2]:.4f} min {r[0]:.4f}")
rel = max(abs(a - b) / abs(b) for a, b in zip(vals["0"], vals["1"]))
print("same values:", vals["0"] == vals["1"], f"max rel diff {rel:.2e}")
