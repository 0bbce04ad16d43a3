"""A/B of the completion wait (GGP_SPIN=1 poll the sequence slot vs 0 hipStreamSynchronize) on
the C2 forest: ms per evaluation, alternating blocks, same process."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
hf = g.HostForest.synthetic(1000, 200, seed=20261015)
forests = {}
for spin in ("0", "1"):
    os.environ["GGP_SPIN"] = spin
    forests[spin] = g.Forest(hf, device=0)
res = {"0": [], "1": []}
vals = {}
for rep in range(6):
    for spin, f in forests.items():
        for _ in range(3):
            f.total_likelihood(P)
        t0 = time.perf_counter()
        for _ in range(50):
            v = f.total_likelihood(P)
        res[spin].append(1e3 * (time.perf_counter() - t0) / 50)
        vals.setdefault(spin, []).append(v)
for spin in res:
    r = sorted(res[spin])
    print(f"GGP_SPIN={spin}: ms/eval median {r[len(r)//2]:.4f} min {r[0]:.4f}  blocks {['%.4f' % x for x in res[spin]]}")
print("same values:", vals["0"] == vals["1"])
