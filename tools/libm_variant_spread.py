#!/usr/bin/env python3
"""How far the reference's own total moves with the machine it runs on (diagnostic; build container).

The reference is built for plain x86-64 (src/Makefile:2) and calls glibc's exp/log/pow; glibc picks
an implementation of each at load time from the CPU's features (its FMA build on an FMA CPU, its
SSE2 build otherwise).  The oracle (oracle/liboracle.so, the reference's path restated in C with the
same libm calls) is run here twice on the example's 5 configurations x 3 chained calls: as this CPU
selects (FMA) and with the FMA/AVX2 builds masked (GLIBC_TUNABLES=glibc.cpu.hwcaps=-AVX2_Usable,
-FMA_Usable: what an x86-64 CPU without FMA runs), each in a process of its own.  The worst relative
distance between the two is the reference's own machine-to-machine spread on the bar's config.

Usage: python tools/libm_variant_spread.py [--out profiles/rNN_libm_variant_spread.json]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import gzip, json, os, shutil, sys, tempfile
import numpy as np
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g
from oracle import oracle as O
G = os.path.join(ROOT, "tests", "golden")
tmp = tempfile.mkdtemp(); csv = os.path.join(tmp, "input.csv")
with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
    shutil.copyfileobj(fi, fo)
own = json.load(open(os.path.join(G, "oracle_example.json")))
out = {}
for key, v in own.items():
    noise, div = key.split("/")[:2]
    hf = g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"), -1, noise, div)
    of = O.OracleForest(hf.a)
    p = [float.fromhex(x) for x in v["params"]]
    out[key] = [of.total_likelihood(p)[0].hex() for _ in range(3)]
shutil.rmtree(tmp)
print(json.dumps(out))
'''


def run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", f"ROOT={ROOT!r}\n" + CHILD], capture_output=True, text=True, env=env,
                       check=True)
    return {k: [float.fromhex(x) for x in v] for k, v in json.loads(r.stdout.strip().splitlines()[-1]).items()}


def main() -> int:
    fma = run({})
    nofma = run({"GLIBC_TUNABLES": "glibc.cpu.hwcaps=-AVX2_Usable,-FMA_Usable,-FMA4_Usable,-AVX2,-FMA"})
    own = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_example.json")))
    worst = max(abs(a - b) / abs(b) for k in fma for a, b in zip(nofma[k], fma[k]))
    fixture = max(abs(a - float.fromhex(b)) / abs(float.fromhex(b)) for k in fma for a, b in zip(fma[k], own[k]["ll"]))
    res = {"calls": 15, "worst_rel_fma_vs_sse2_glibc": worst, "fma_run_vs_fixture": fixture,
           "per_config": {k: [abs(a - b) / abs(b) for a, b in zip(nofma[k], fma[k])] for k in fma},
           "note": "the oracle (the reference path restated in C, the same glibc calls) on the example's 15 "
                   "chained totals, glibc's FMA builds of exp/log/pow (this CPU) against its SSE2 builds "
                   "(GLIBC_TUNABLES hwcaps masked): the reference binary's own spread between x86-64 machines"}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2 and sys.argv[1] == "--out":
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)
            f.write("\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
