"""Quick GPU sanity run: example forest parity vs the CPU oracle + a synthetic timing."""
import gzip, os, shutil, sys, tempfile, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g
from oracle import oracle as O

G = os.path.join(ROOT, "tests", "golden")
tmp = tempfile.mkdtemp()
csv = os.path.join(tmp, "input.csv")
with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
    shutil.copyfileobj(fi, fo)
hf = g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"))
P0 = g.ParameterSet.load(os.path.join(G, "example_parameter_file.txt")).get_init()
of = O.OracleForest(hf.a)
fg = g.Forest(hf)
for k in range(3):
    t0 = time.time(); vg = fg.total_likelihood(P0); t1 = time.time()
    vo = of.total_likelihood(P0)[0]
    print(f"call {k}: gpu {vg!r} oracle {vo!r} rel {abs(vg-vo)/abs(vo):.3e}  gpu {1e3*(t1-t0):.2f} ms", flush=True)
st_g = fg.state(); st_o = of.state
print("state max rel diff", np.nanmax(np.abs(st_g - st_o) / (np.abs(st_o) + 1e-300)))
for n_trees in (1000, 10000):
    hs = g.HostForest.synthetic(n_trees, 200)
    fs = g.Forest(hs)
    fs.total_likelihood(P0)
    ts = []
    for _ in range(5):
        t0 = time.time(); v = fs.total_likelihood(P0); ts.append(time.time() - t0)
    ofs = O.OracleForest(hs.a)
    vo = ofs.total_likelihood(P0)[0]
    vg0 = g.Forest(hs).total_likelihood(P0)
    print(f"synthetic {n_trees}x200: rows {hs.n_rows} best {1e3*min(ts):.3f} ms -> {hs.n_rows/min(ts):.3e} updates/s; fresh gpu {vg0!r} oracle {vo!r} rel {abs(vg0-vo)/abs(vo):.2e}", flush=True)
