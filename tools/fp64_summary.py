"""FP64 work per update from one rocprofv3 --pmc pass over tools/fp64_workload.py:

  python3 tools/fp64_summary.py PMC_DIR OUT_JSON

flops of a launch = 64 lanes x (ADD + MUL + TRANS + 2 FMA) F64 wave-instructions (FMA = 2 flops),
summed over the launches of a kernel and divided by the rows those launches processed:
  issued_flops_per_update  k_loglik_wave (C2): every lane of every wave-instruction -- the wave
                           schedule runs the update's scalar work in all 64 lanes and forms
                           every task candidate, so this is issue, not useful work
  useful_flops_per_update  k_loglik_level (1024 trees, full waves): one lane runs one cell's
                           whole update -- the FP64 work the algorithm itself needs
  pair / smooth / combine  bench.py's large_forest (k_loglik_pair) and predict legs (forward +
                           backward smoother kernels per row, k_combine per row)
The engine library's sha256 is recorded: bench.py uses the figures only for that same build."""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
d, out_path = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(float))
n_disp = defaultdict(set)
for fn in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        k = row["Kernel_Name"]
        if "k_loglik_wave" in k:
            kind = "wave"
        elif "k_loglik_level" in k and "batch" not in k:
            kind = "lane"
        elif "k_loglik_pair" in k:
            kind = "pair"
        elif "k_fwd_" in k or "k_bwd_" in k:
            kind = "smooth"
        elif "k_combine" in k:
            kind = "combine"
        else:
            continue
        acc[kind][row["Counter_Name"]] += float(row["Counter_Value"])
        n_disp[kind].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
work = json.loads(open(os.path.join(d, "workload.json")).read())
res = {"engine_sha256": hashlib.sha256(open(os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", "libggp.so"),
                                            "rb").read()).hexdigest(),
       "source": "rocprofv3 --pmc SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 SQ_INSTS_VALU SQ_WAVES over tools/fp64_workload.py"}
for kind, c in acc.items():
    if kind not in work:
        continue
    w = work[kind]
    rows = w["rows"] * w["evals"]
    f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_TRANS_F64"] + 2 * c["SQ_INSTS_VALU_FMA_F64"]
    res[kind] = {"rows": rows, "launches": len(n_disp[kind]), "valu_wave_insts": c["SQ_INSTS_VALU"],
                 "f64_wave_insts": c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] +
                 c["SQ_INSTS_VALU_TRANS_F64"] + c["SQ_INSTS_VALU_FMA_F64"],
                 "flops_per_update": 64.0 * f64 / rows, "valu_wave_insts_per_update": c["SQ_INSTS_VALU"] / rows,
                 "f64_wave_insts_per_update": (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] +
                                               c["SQ_INSTS_VALU_TRANS_F64"] + c["SQ_INSTS_VALU_FMA_F64"]) / rows}
res["issued_flops_per_update"] = res.get("wave", {}).get("flops_per_update")
res["useful_flops_per_update"] = res.get("lane", {}).get("flops_per_update")
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res, indent=1))
