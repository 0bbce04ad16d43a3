"""BASELINE configs[3] at full size on one GPU (diagnostic record): the 100k-tree x 200 tp forest
(2e7 rows), the -s scan SURVEY 8(d) restates (gamma_lambda bound at 1.0E-03 .. 8.0E-02 step 2.0E-02
around its init: arange gives the samples; the reference's 60-sample file steps finer), each sample
on the carried state of the previous one.
  * one handle over the whole forest (auto schedule) and one per 12.5k-tree shard (what each of
    8 GPUs holds): ms per evaluation;
  * the scan as one chained call (ggp_total_loglik_chain, as the CLI's -s runs it) and call by call
    -- bitwise equal;
  * the first three samples against the 16-thread CPU oracle.
Prints one JSON line."""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402
from gfp_gaussian_process_amd.distributed import shard  # noqa: E402
from gfp_gaussian_process_amd.optimize import arange  # noqa: E402
from oracle import oracle as O  # noqa: E402

P = np.array([2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04,
              7.48e-01])
t0 = time.perf_counter()
hf = g.HostForest.synthetic(100000, 200)
out = {"trees": 100000, "rows": hf.n_rows, "synth_s": time.perf_counter() - t0}
samples = arange(1.0e-03, 8.0e-02, 1.0e-03 * 1.3)   # 61 samples across the bound interval
pts = np.repeat(P[None, :], len(samples), axis=0)
pts[:, 1] = samples
out["samples"] = len(samples)

f = g.Forest(hf)
for _ in range(3):
    f.total_likelihood(P)
f.reset_state()
t1 = time.perf_counter()
for _ in range(20):
    f.total_likelihood(P)
out["eval_ms_whole_forest"] = 1e3 * (time.perf_counter() - t1) / 20
f.reset_state()
t1 = time.perf_counter()
chain = f.total_likelihood_chain(pts)
out["scan_chain_s"] = time.perf_counter() - t1
f.reset_state()
t1 = time.perf_counter()
seq = np.array([f.total_likelihood(p) for p in pts])
out["scan_call_by_call_s"] = time.perf_counter() - t1
out["chain_bitwise_call_by_call"] = bool(np.array_equal(chain, seq))
f.close()

fs = g.Forest(shard(hf, 0, 8))   # one GPU's whole-tree share of an 8-GPU run (global init statistics)
for _ in range(3):
    fs.total_likelihood(P)
t1 = time.perf_counter()
for _ in range(50):
    fs.total_likelihood(P)
out["eval_ms_per_gpu_shard"] = 1e3 * (time.perf_counter() - t1) / 50
fs.close()

# the first three scan samples against the oracle (16 whole-tree shards, one thread each)
ors = [O.OracleForest(shard(hf, r, 16).a) for r in range(16)]
t1 = time.perf_counter()
ref = []
with ThreadPoolExecutor(16) as ex:
    for p in pts[:3]:
        vals = list(ex.map(lambda o: o.total_likelihood(p)[0], ors))
        ref.append(float(np.sum(vals)))
out["oracle_s"] = time.perf_counter() - t1
out["rel_err_first3"] = [abs(a - b) / abs(b) for a, b in zip(chain[:3], ref)]
print(json.dumps(out), flush=True)
