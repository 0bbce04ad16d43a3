"""GPU check of the wave schedule: parity against the oracle on the example configs and a
synthetic forest, then C2 timing of every schedule (one process)."""
import gzip, json, os, shutil, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g
from oracle import oracle as O

G = os.path.join(ROOT, "tests", "golden")
tmp = tempfile.mkdtemp()
csv = os.path.join(tmp, "input.csv")
with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
    shutil.copyfileobj(fi, fo)
kern = sys.argv[1] if len(sys.argv) > 1 else "wave"
worst = 0.0
for k, v in json.load(open(os.path.join(G, "oracle_example.json"))).items():
    noise, div = k.split("/")[:2]
    p = [float.fromhex(x) for x in v["params"]]
    hf = g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"), -1, noise, div)
    fg, of = g.Forest(hf, kernel=kern), O.OracleForest(hf.a)
    errs = []
    for call in range(3):
        a, b = fg.total_likelihood(p), of.total_likelihood(p)[0]
        errs.append(abs(a - b) / abs(b))
    worst = max(worst, max(errs))
    print(f"{k:28s} rel {max(errs):.2e}", flush=True)
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
hf = g.HostForest.synthetic(1000, 200)
vo = O.OracleForest(hf.a).total_likelihood(P)[0]
for k in ("auto", "group", kern):
    f = g.Forest(hf, kernel=k)
    v = f.total_likelihood(P)
    for _ in range(3):
        f.total_likelihood(P)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        f.total_likelihood(P)
    dt = (time.perf_counter() - t0) / reps
    f.enable_profile()
    f.total_likelihood(P)
    ms, rows, names = f.launch_profile()
    print(f"C2 {k:6s}: {1e3*dt:.3f} ms/eval {hf.n_rows/dt:.3e} updates/s  rel {abs(v-vo)/abs(vo):.2e}  launches "
          + ", ".join(f"{n} {m:.3f}ms" for n, m in zip(names, ms)), flush=True)
    f.close()
print("worst example rel", worst)
