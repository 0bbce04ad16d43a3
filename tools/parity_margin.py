"""Parity margins (diagnostic): python tools/parity_margin.py LIB_DIR
The largest relative error against the oracle of the total log-likelihood for each schedule
over the example's five configurations x three carried-state calls (tests/test_gpu_parity.py's
cases), and of the -p smoother's rows (normalised as the tests do), one line per schedule."""
import gzip
import json
import os
import shutil
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gfp_gaussian_process_amd import _native  # noqa: E402

_native.LIB_DIR = os.path.abspath(sys.argv[1])
import gfp_gaussian_process_amd as g  # noqa: E402
from oracle import oracle as O  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
PARAMS = json.load(open(os.path.join(G, "oracle_example.json")))
CONFIGS = [(k.split("/")[0], k.split("/")[1], [float.fromhex(x) for x in v["params"]]) for k, v in PARAMS.items()]
tmp = tempfile.mkdtemp()
csv = os.path.join(tmp, "input.csv")
with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
    shutil.copyfileobj(fi, fo)
forests = {(n, d): g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"), -1, n, d) for n, d, _ in CONFIGS}
ref = []   # per configuration (two share a noise/division pair with other parameters)
for n, d, p in CONFIGS:
    of = O.OracleForest(forests[(n, d)].a)
    ref.append([of.total_likelihood(p)[0] for _ in range(3)])
out = [sys.argv[1]]
for kern in ("lane", "group", "pair", "wave"):
    worst = 0.0
    for ci, (n, d, p) in enumerate(CONFIGS):
        f = g.Forest(forests[(n, d)], kernel=kern)
        for call in range(3):
            worst = max(worst, abs(f.total_likelihood(p) - ref[ci][call]) / abs(ref[ci][call]))
        f.close()
    out.append(f"{kern} {worst:.2e}")
# the smoother against the oracle's, normalised as tests/test_gpu_parity.py::_smoother_err
def smoother_err(a, b):
    m_a, m_b = a[:, :4], b[:, :4]
    C_a, C_b = a[:, 4:].reshape(-1, 4, 4), b[:, 4:].reshape(-1, 4, 4)
    sd = np.sqrt(np.abs(np.einsum("nii->ni", C_b)))
    em = np.max(np.abs(m_a - m_b) / (np.abs(m_b) + sd).clip(1e-300))
    ec = np.max(np.abs(C_a - C_b) / (sd[:, :, None] * sd[:, None, :]).clip(1e-300))
    return max(float(em), float(ec))


n, d, p = CONFIGS[0]
hf = forests[(n, d)]
ref_p = O.OracleForest(hf.a).predict(p)
for kern in ("lane", "auto"):
    f = g.Forest(hf) if kern == "auto" else g.Forest(hf, kernel=kern)
    got = f.predict(p)
    out.append(f"predict[{kern}] " + " ".join(f"{nm} {smoother_err(x, y):.2e}"
                                               for nm, x, y in zip(("fwd", "bwd", "comb"), got, ref_p)))
    f.close()
print(" | ".join(out), flush=True)
