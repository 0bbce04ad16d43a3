"""A/B of the engine builds (GPU box): parity on the example and time per call, for the library
GGP_ENGINE_LIB names (libggp.so = the fast arithmetic, libggp_exact.so = GGP_EXACT).

  GGP_ENGINE_LIB=libggp_exact.so python tools/exact_ab.py [--quick]

Prints one JSON line: per schedule the worst relative distance of the example's 5 configurations x
3 chained calls from tests/golden/oracle_example.json, and ms per call of the timed legs."""
import gzip, json, os, shutil, sys, tempfile, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g
from gfp_gaussian_process_amd import _native as N

G = os.path.join(ROOT, "tests", "golden")
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
quick = "--quick" in sys.argv
out = {"lib": N.engine_name()}

tmp = tempfile.mkdtemp()
csv = os.path.join(tmp, "input.csv")
with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
    shutil.copyfileobj(fi, fo)
own = json.load(open(os.path.join(G, "oracle_example.json")))
par = {}
for kern in ("lane", "pair", "group", "wave", "auto"):
    w = 0.0
    for key, v in own.items():
        noise, div = key.split("/")[:2]
        hf = g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"), -1, noise, div)
        try:
            f = g.Forest(hf, kernel=kern)
        except g.GGPError as e:   # the exact engine has no wave schedule
            w = str(e)
            break
        p = [float.fromhex(x) for x in v["params"]]
        ll = np.array([f.total_likelihood(p) for _ in range(3)])
        ref = np.array([float.fromhex(x) for x in v["ll"]])
        w = max(w, float(np.max(np.abs(ll - ref) / np.abs(ref))))
        f.close()
    par[kern] = w
out["example_rel_vs_oracle"] = par
print(json.dumps(out), flush=True)


def timed(f, reps, fn):
    for _ in range(3):
        fn(f)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn(f)
    return 1e3 * (time.perf_counter() - t0) / reps


legs = {}
hf = g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"))
for kern in ("lane", "pair", "auto"):
    f = g.Forest(hf, kernel=kern)
    legs[f"example_{kern}"] = timed(f, 20, lambda f: f.total_likelihood(P))
    f.close()
for n, kern in ((1000, "auto"), (1000, "lane"), (10000, "auto"), (12500, "auto"), (40000, "auto")):
    hs = g.HostForest.synthetic(n, 200)
    f = g.Forest(hs, kernel=kern)
    legs[f"c2shape_{n}_{kern}"] = timed(f, 20 if n < 20000 else 10, lambda f: f.total_likelihood(P))
    f.close()
print(json.dumps({"lib": out["lib"], "ms": legs}), flush=True)
if not quick:
    n = 20000
    hs = g.HostForest.synthetic(n, 500)
    f = g.Forest(hs)
    legs[f"predict_c5shape_{n}"] = timed(f, 5, lambda f: f.predict(P, outputs=(False, False, False)))
    f.close()
    hs = g.HostForest.synthetic(125000, 500)
    f = g.Forest(hs)
    legs["loglik_c5shard"] = timed(f, 5, lambda f: f.total_likelihood(P))
    legs["predict_c5shard"] = timed(f, 3, lambda f: f.predict(P, outputs=(False, False, False)))
    f.close()
out["ms"] = legs
print(json.dumps(out), flush=True)
shutil.rmtree(tmp)
