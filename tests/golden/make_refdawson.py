#!/usr/bin/env python3
"""Regenerate tests/golden/oracle_example_refdawson.json (build container only: it needs the
reference's own Faddeeva.cc compiled in place into oracle/_ref by `make -C oracle ref`).

The example's carried-state chains of oracle_example.json (five configurations x three calls),
with every Dawson value taken from the reference's Faddeeva::Dawson instead of the oracle's
regenerated table (oracle.OracleForest(ref_dawson=True)): the totals the reference's own Dawson
arithmetic gives under the oracle's restatement of the rest of the path.  Doubles as float.hex.
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import gfp_gaussian_process_amd as g  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main() -> None:
    tmp = tempfile.mkdtemp()
    csv = os.path.join(tmp, "input.csv")
    with gzip.open(os.path.join(HERE, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    cases = json.load(open(os.path.join(HERE, "oracle_example.json")))
    out = {}
    for key, v in cases.items():
        noise, div = key.split("/")[:2]
        params = [float.fromhex(x) for x in v["params"]]
        hf = g.HostForest.from_csv(csv, os.path.join(HERE, "example_csv_config.txt"), -1, noise, div)
        of = O.OracleForest(hf.a, ref_dawson=True)
        ll = [of.total_likelihood(params)[0] for _ in range(3)]
        own = [float.fromhex(x) for x in v["ll"]]
        out[key] = {"params": v["params"], "ll": [x.hex() for x in ll],
                    "rel_vs_oracle_table_dawson": [abs(a - b) / abs(b) for a, b in zip(ll, own)]}
    shutil.rmtree(tmp)
    with open(os.path.join(HERE, "oracle_example_refdawson.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
