"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

  python3 tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON

Both counters are in KiB per dispatch (rocprofv3 derived counters).  MI355X_MICROARCH.md:
FETCH_SIZE reads exactly half the bytes of a 16-B/lane coalesced streaming read on gfx950;
the engine's reads are 8-B scalar-per-cell loads, for which the guide has no calibration,
so the value is reported uncorrected and labelled so.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_kernel(d, counter):
    acc = defaultdict(list)
    for fn in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(fn)):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def short(name):
    if "k_loglik_group<" in name:
        return "k_loglik_group<" + name.split("k_loglik_group<")[1].split(">")[0] + ">"
    for k in ("k_loglik_wave", "k_loglik_level", "k_reduce", "k_fwd_level", "k_bwd_level", "k_combine"):
        if k in name:
            return k
    return name[:40]


fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
out = {}
for k in set(fetch) | set(write):
    s = short(k)
    if s.startswith("k_"):
        out[s] = {"fetch_bytes": fetch.get(k), "write_bytes": write.get(k),
                  "bytes_per_launch": (fetch.get(k) or 0.0) + (write.get(k) or 0.0)}
import hashlib
import os
lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gfp_gaussian_process_amd", "lib", "libggp.so")
json.dump({"note": "FETCH_SIZE+WRITE_SIZE (KiB*1024) per dispatch, mean over dispatches; uncorrected "
                   "(8-B loads: the guide's x2 FETCH_SIZE correction is for 16-B/lane streams only)",
           "engine_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
           "workload": "bench.py defaults (C2: 1000 trees x 200)",
           "kernels": out}, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
