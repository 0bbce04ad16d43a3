"""Per-row PMC figures of the -p kernels (diagnostic) from three rocprofv3 --pmc passes over
tools/combine_workload.py: HBM bytes (FETCH_SIZE + WRITE_SIZE, KiB per dispatch, uncorrected) and
VALU wave-instructions per row.  python3 tools/smoother_pmc.py FETCH_DIR WRITE_DIR VALU_DIR WORKLOAD_JSON OUT"""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_kernel(d, counter, scale=1.0):
    acc = defaultdict(float)
    for fn in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(fn)):
            if row["Counter_Name"] == counter:
                n = row["Kernel_Name"]
                for k in ("k_fwd_level", "k_bwd_level", "k_fwd_pair", "k_bwd_pair", "k_combine"):
                    if k in n:
                        acc[k] += float(row["Counter_Value"]) * scale
    return acc


wl = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
rows = wl["rows"]
fetch = per_kernel(sys.argv[1], "FETCH_SIZE", 1024.0)
write = per_kernel(sys.argv[2], "WRITE_SIZE", 1024.0)
valu = per_kernel(sys.argv[3], "SQ_INSTS_VALU")
out = {"workload": wl, "note": "two predicts (warm-up + timed): per-row figures divide by 2 x rows; "
       "bytes uncorrected (FETCH_SIZE+WRITE_SIZE KiB x 1024)", "kernels": {}}
for k in sorted(set(fetch) | set(write) | set(valu)):
    out["kernels"][k] = {"hbm_bytes_per_row": (fetch.get(k, 0.0) + write.get(k, 0.0)) / (2 * rows),
                         "valu_wave_insts_per_row": valu.get(k, 0.0) / (2 * rows)}
json.dump(out, open(sys.argv[5], "w"), indent=1)
print(json.dumps(out, indent=1))
