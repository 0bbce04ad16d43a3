"""Gaps between consecutive kernels of one evaluation (diagnostic): reads a rocprofv3
--kernel-trace CSV and prints, for the last few evaluations, each kernel's duration and the
idle gap before it (us)."""
import csv
import glob
import sys

rows = []
for fn in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]))
rows.sort()
tail = rows[-int(sys.argv[2]) if len(sys.argv) > 2 else -30:]
prev_end = None
for s, e, n in tail:
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print(f"{n:40s} dur {(e - s) / 1e3:8.2f} us   gap before {gap:8.2f} us")
    prev_end = e
