"""-j compute timing ("-j is timed on a <= 10k-row subset"): ggp_joints over
every start row of a synthetic forest, in start-row chunks, joints per second.  Prints one
JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
trees = int(sys.argv[1]) if len(sys.argv) > 1 else 50
hf = g.HostForest.synthetic(trees, 200)
f = g.Forest(hf)
nr = hf.n_rows
chunk = 500
f.joints(P, 1e-10, 0, min(chunk, nr), cap=1 << 20)            # warm-up
t0 = time.perf_counter()
total, cap = 0, 1 << 20
for lo in range(0, nr, chunk):
    hi = min(nr, lo + chunk)
    while True:
        try:
            idx, val = f.joints(P, 1e-10, lo, hi, cap=cap)
            break
        except g.GGPError:
            cap *= 2
    total += len(idx)
el = time.perf_counter() - t0
print(json.dumps({"config": f"-j compute, synthetic {trees} trees x 200 tp ({nr} rows), tol 1e-10, "
                            f"start-row chunks of {chunk}, joints copied to the host",
                  "rows": nr, "joints": total, "seconds": el, "joints_per_s": total / el,
                  "start_rows_per_s": nr / el}))
