"""scan lane-schedule cells-per-wave and group cells-per-wave on a few forest sizes"""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys, time
sys.path.insert(0, %r)
import gfp_gaussian_process_amd as g
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
n = int(sys.argv[1]); k = sys.argv[2]
hf = g.HostForest.synthetic(n, 200)
f = g.Forest(hf, kernel=k)
f.total_likelihood(P); f.total_likelihood(P)
t0 = time.perf_counter()
for _ in range(4): f.total_likelihood(P)
dt = (time.perf_counter() - t0) / 4
print("%%.3f" %% (1e3 * dt))
''' % ROOT
for n in [int(x) for x in sys.argv[1:]] or [1000, 10000, 30000]:
    res = []
    for cpw in (1, 2, 4, 8, 16, 32, 64):
        env = dict(os.environ, GGP_LANE_CPW=str(cpw))
        out = subprocess.run([sys.executable, "-c", code, str(n), "lane"], env=env, capture_output=True, text=True, timeout=300)
        res.append(f"lane{cpw}:{out.stdout.strip()}")
    for cpw in (1, 2, 4, 8):
        env = dict(os.environ, GGP_GROUP_CPW=str(cpw))
        out = subprocess.run([sys.executable, "-c", code, str(n), "group"], env=env, capture_output=True, text=True, timeout=300)
        res.append(f"grp{cpw}:{out.stdout.strip()}")
    print(f"trees={n}: " + " ".join(res), flush=True)
