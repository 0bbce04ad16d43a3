"""Summarise rocprofv3 counter_collection.csv files: per kernel name, mean of each counter."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    acc = defaultdict(lambda: defaultdict(list))
    for fn in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(fn)):
            k = row.get("Kernel_Name", "?")[:60]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(f"== {d}")
    for k, cs in acc.items():
        print("  " + k)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
