"""A/B timing of the lane and group schedules across forest sizes (one process)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
sizes = [int(x) for x in (sys.argv[1:] or ["100", "1000", "4000", "10000", "30000"])]
for n in sizes:
    hf = g.HostForest.synthetic(n, 200)
    row = [f"trees={n:6d} rows={hf.n_rows:8d}"]
    for k in ("lane", "group", "auto"):
        f = g.Forest(hf, kernel=k)
        for _ in range(2):
            f.total_likelihood(P)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            v = f.total_likelihood(P)
        dt = (time.perf_counter() - t0) / reps
        row.append(f"{k}: {1e3*dt:8.3f} ms {hf.n_rows/dt:9.3e}/s")
        f.close()
    print(" | ".join(row), flush=True)
