"""gaps between consecutive k_loglik_wave dispatches in a rocprofv3 kernel trace (armed vs plain
blocks of tools/arm_ab.py): start(k+1) - end(k) and durations, medians per template variant"""
import csv
import glob
import re
import statistics
import sys

rows = []
for fn in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(fn) as f:
        for r in csv.DictReader(f):
            m = re.search(r"k_loglik_wave<(\w+), ?(\w+)>", r["Kernel_Name"])
            if m:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(2) == "true"))
rows.sort()
gaps = {False: [], True: []}
durs = {False: [], True: []}
for (s0, e0, a0), (s1, e1, a1) in zip(rows, rows[1:]):
    if a0 == a1:
        gaps[a1].append((s1 - e0) / 1e3)
        durs[a1].append((e1 - s1) / 1e3)
for a in (False, True):
    if gaps[a]:
        g = sorted(gaps[a])
        print(f"armed={a}: n {len(g)} gap start(k+1)-end(k) median {statistics.median(g):.2f} us "
              f"p10 {g[len(g)//10]:.2f} p90 {g[9*len(g)//10]:.2f}; duration median {statistics.median(durs[a]):.2f} us")
