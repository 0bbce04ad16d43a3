"""Numerical experiment (diagnostic): the total log-likelihood of the oracle with its own
mean_cov_model, with the device lane expressions (tools/libhostsim.so hs_mcm_lane) and with
the wave schedule's table-driven outputs (hs_mcm_tab), on the example (5 configs, fresh +
2 carried-state calls) and a synthetic forest.  Relative differences are what the parity
tests must absorb beyond libm."""
import ctypes
import gzip
import os
import shutil
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402
from oracle import oracle as O  # noqa: E402

HS = ctypes.CDLL(os.path.join(ROOT, "tools", "libhostsim.so"))
L = O.lib(sens=True)
FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p)
L.ora_set_mcm_hook.argtypes = [ctypes.c_void_p]
HOOKS = {"oracle": None, "lane": ctypes.cast(HS.hs_mcm_lane, ctypes.c_void_p).value,
         "tab": ctypes.cast(HS.hs_mcm_tab, ctypes.c_void_p).value,
         "wave": ctypes.cast(HS.hs_mcm_wave, ctypes.c_void_p).value}

G = os.path.join(ROOT, "tests", "golden")
tmp = tempfile.mkdtemp()
csv = os.path.join(tmp, "input.csv")
with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
    shutil.copyfileobj(fi, fo)
P0 = g.ParameterSet.load(os.path.join(G, "example_parameter_file.txt")).get_init()
P1 = list(P0)
P1[8] = 2.6e4
cases = []
for noise, div, p in (("scaled", "binomial", P0), ("const", "gauss", P1), ("scaled", "gauss", P0),
                      ("const", "binomial", P1)):
    cases.append((f"example {noise}/{div}", g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"), -1, noise, div).a, p))
cases.append(("synthetic 200x200", g.HostForest.synthetic(200, 200).a, P0))


def run(a, p, hook):
    L.ora_set_mcm_hook(HOOKS[hook])
    of = O.OracleForest(a, exp_ulp_noise=0)
    of._noise = -1     # use the sens build without exp noise
    L.ora_set_exp_ulp_noise(0)
    out = []
    for _ in range(3):
        f = O.OracleForest.__new__(O.OracleForest)
    return out


for name, a, p in cases:
    res = {}
    for hook in HOOKS:
        L.ora_set_mcm_hook(HOOKS[hook])
        L.ora_set_exp_ulp_noise(0)
        f = O.make_forest(a)
        st = np.zeros((f.n_cells, 20))
        cl = np.zeros(f.n_cells)
        nc, nr = ctypes.c_int64(), ctypes.c_int64()
        pp = np.ascontiguousarray(p, np.float64)
        vals = [L.ora_total_loglik(ctypes.byref(f), O._dp(pp), O._dp(st), ctypes.byref(nc), ctypes.byref(nr), O._dp(cl))
                for _ in range(3)]
        res[hook] = np.array(vals)
    L.ora_set_mcm_hook(None)
    base = res["oracle"]
    print(f"{name:28s} ll {base[0]:.10g}  lane rel {np.max(np.abs(res['lane'] - base) / np.abs(base)):.2e}"
          f"  tab rel {np.max(np.abs(res['tab'] - base) / np.abs(base)):.2e}"
          f"  wave rel {np.max(np.abs(res['wave'] - base) / np.abs(base)):.2e}")
