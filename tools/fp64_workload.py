"""Workload for the FP64 counter pass (tools/measure.sh): a few evaluations of
  * C2 (1000 trees x 200) under the default (auto) schedule -- k_loglik_wave, whose counters
    give the ISSUED FP64 work per update (every lane of every wave-instruction counted), and
  * 1024 trees x 200 under the lane schedule -- k_loglik_level, one cell per lane and every
    wave full (levels of 1024 and 2048 cells), whose counters give the USEFUL FP64 work of one
    update: what a single thread executing the algorithm once issues;
  * bench.py's large_forest leg (12.5k trees x 200, auto: k_loglik_pair) and predict leg (125k
    trees x 500: k_fwd_* / k_bwd_* / k_combine), so every timed leg states its FP64 and VALU-issue
    fractions from counters of the same build.
Rows per launch are printed for the summary (tools/fp64_summary.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
out = {}
for name, trees, kernel in (("wave", 1000, "auto"), ("lane", 1024, "lane")):
    hf = g.HostForest.synthetic(trees, 200)
    # the lane figure is one lane running whole updates: the level launches (k_loglik_level), not
    # the lane queue, whose waiting chunks would add their polls to the counts
    os.environ["GGP_LANE_QUEUE"] = "0" if name == "lane" else "1"
    f = g.Forest(hf, kernel=kernel)
    for _ in range(3):
        f.total_likelihood(P)
    out[name] = {"trees": trees, "rows": hf.n_rows, "evals": 3}
    f.close()
hf = g.HostForest.synthetic(12500, 200)                 # bench.py large_forest (its seed is irrelevant here)
f = g.Forest(hf)
for _ in range(3):
    f.total_likelihood(P)
out["pair"] = {"trees": 12500, "rows": hf.n_rows, "evals": 3}
f.close()
hf = g.HostForest.synthetic(125000, 500)                # bench.py predict
os.environ["GGP_COMBINE_FUSED"] = "0"   # the smoother and the combine counted apart (the bench fuses them)
f = g.Forest(hf)
for _ in range(2):
    f.predict(P, outputs=(False, False, False))
out["smooth"] = {"trees": 125000, "rows": hf.n_rows, "evals": 2}
out["combine"] = out["smooth"]
f.close()
print(json.dumps(out))
