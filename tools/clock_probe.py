"""Diagnostic: the shader clock (ggp_launch_clock) of C2 path launches after a full-chip preheat,
call by call, in the spin-wait mode and in the event-profile mode (hipStreamSynchronize per call):
python tools/clock_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
hp = g.Forest(g.HostForest.synthetic(12500, 200, seed=7))
f = g.Forest(g.HostForest.synthetic(1000, 200))
t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:
    hp.total_likelihood(P)


def run(tag, n, profile=False):
    out = []
    for _ in range(n):
        t0 = time.perf_counter()
        f.total_likelihood(P)
        w = (time.perf_counter() - t0) * 1e6
        ev = f.launch_profile()[0][0] * 1e3 if profile else 0.0
        out.append((round(f.launch_clock()[0]), round(w, 1), round(ev, 1)))
    print(tag, out, flush=True)


run("spin", 20)
f.enable_profile()
run("profile", 10, profile=True)
run("profile", 10, profile=True)
f2 = g.Forest(g.HostForest.synthetic(1000, 200))
f, f2 = f2, f
run("spin-after", 20)
time.sleep(0.05)
run("spin-after-50ms-idle", 20)
