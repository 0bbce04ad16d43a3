#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ (run in the build container only:
it reads /root/reference, which does not exist on the GPU box).

  example_input.csv.gz, example_csv_config.txt, example_parameter_file.txt
        the reference's own example data set (example_data_set/), data files only
  dawson_ref.json      x -> Faddeeva::Dawson(x) from the reference's Faddeeva.cc compiled
                       in place into oracle/_ref (`make -C oracle ref`)
  dawson_maple.json    the real-axis Dawson cases of Faddeeva.cc's own self-test
                       (inputs and Maple reference values, Faddeeva.cc:2378-2511)
  example_topology.json  cell ids / genealogy / row counts / init statistics of the
                       example, from an independent brute-force restatement of
                       read_data + build_cell_genealogy + init_cells (O(N^2), as the
                       reference does it) -- pins the C++ host ingest bit-exactly
  oracle_example.json  total log-likelihoods of the CPU oracle on the example (carried
                       state chain of 3 calls) -- regression pin of the oracle itself
                       (self-generated: "parity unpinned" against a reference run)

  oracle_example_predict.npz  -p of the CPU oracle on the example: forward / backward /
                       combined state of every cell's first and last row + sha256 of all rows
  oracle_tests_h_cell.json   the oracle's 3-call chain on the reference's tests.h:263-300 cell

Doubles are stored as float.hex strings (exact) or in .npz (exact, loaded without pickle).
`--oracle-only` regenerates just the two oracle fixtures from the committed example data.
"""
from __future__ import annotations

import gzip
import json
import math
import os
import re
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)


def hx(v: float) -> str:
    return float(v).hex()


def dawson_fixtures():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    from oracle import oracle as O
    ref = O.faddeeva_ref()
    rng = np.random.default_rng(20261015)
    xs = list(np.logspace(-300, 8, 1500)) + list(rng.uniform(0, 50, 1500)) + list(rng.uniform(0, 0.05, 300))
    xs += [100.0 / k - 1.0 for k in range(1, 101)]                  # y100 interval edges
    xs += [45.0, math.nextafter(45.0, 100), 5e7, math.nextafter(5e7, 1e9), 0.0, 1e-310]
    xs += [-x for x in xs if x > 0]
    out = {"x": [hx(x) for x in xs], "dawson": [hx(ref(float(x))) for x in xs]}
    json.dump(out, open(os.path.join(HERE, "dawson_ref.json"), "w"))

    # self-test values of Faddeeva.cc (TST(Dawson) block): keep purely real inputs
    src = open(os.path.join(REF, "src", "Faddeeva.cc")).read()
    i = src.index("TST(Dawson")
    j = src.rfind("cmplx z[NTST]", 0, i)
    block = src[j:i]
    zs_txt, ws_txt = block.split("cmplx w[NTST]")
    num = r"([-+]?(?:Inf|NaN|[0-9.]+(?:e[-+]?[0-9]+)?))"
    pat = re.compile(r"C\(\s*" + num + r"\s*,\s*" + num + r"\s*\)")

    def conv(s):
        return {"Inf": math.inf, "-Inf": -math.inf, "NaN": math.nan}.get(s, None) if s in ("Inf", "-Inf", "NaN") else float(s)
    zs = [(conv(a), conv(b)) for a, b in pat.findall(zs_txt)]
    ws = [(conv(a), conv(b)) for a, b in pat.findall(ws_txt)]
    assert len(zs) == len(ws), (len(zs), len(ws))
    real = [(z[0], w[0]) for z, w in zip(zs, ws) if z[1] == 0 and math.isfinite(z[0])]
    json.dump({"x": [hx(a) for a, _ in real], "dawson": [hx(b) for _, b in real],
               "note": "real-axis Dawson cases of Faddeeva.cc self-test (Maple values)"},
              open(os.path.join(HERE, "dawson_maple.json"), "w"))
    return len(xs), len(real)


def brute_force_topology(csv_path: str):
    """independent restatement of read_data + build_cell_genealogy + init_cells for the
    example's csv_config (cell_tags = lane, cell_id; parent_tags = lane, parent_id)."""
    lines = open(csv_path).read().split("\n")
    hdr = lines[0].split(",")
    H = {}
    for i, h in enumerate(hdr):
        H.setdefault(h.strip(), i)

    def rld(s):
        if all(ch.isdigit() or ch == "." for ch in s):
            if all(ch == "0" for ch in s.split(".")[-1]):
                return str(int(s.split(".")[0] or "0"))
        return s
    cells = []
    last = None
    for ln in lines[1:]:
        if ln == "":
            continue
        f = ln.split(",")
        cid = rld(f[H["lane"]]) + "." + rld(f[H["cell_id"]])
        if cid != last:
            cells.append({"id": cid, "pid": rld(f[H["lane"]]) + "." + rld(f[H["parent_id"]]), "t": [], "x": [], "g": []})
            last = cid
        c = cells[-1]
        c["t"].append(float(f[H["time_min"]]) / 1.0)
        c["x"].append(math.log(float(f[H["length"]])))
        c["g"].append(float(f[H["gfp"]]))
    n = len(cells)
    parent, d1, d2 = [-1] * n, [-1] * n, [-1] * n
    for k in range(n):
        for j in range(n):
            if cells[j]["id"] == cells[k]["pid"]:
                parent[k] = j
                if d1[j] == -1:
                    d1[j] = k
                elif d2[j] == -1:
                    d2[j] = k
                else:
                    raise ValueError("third daughter")

    def stats(v):
        s = 0.0
        for a in v:
            s = s + a
        m = s / len(v)
        sq = 0.0
        for a in v:
            sq = sq + a * a
        return m, sq / len(v) - m * m
    multi = [c for c in cells if len(c["t"]) > 1]
    rs = [stats([c["x"][0] for c in multi]), stats([c["g"][0] for c in multi])]
    ls = [stats([c["x"][-1] for c in multi]), stats([c["g"][-1] for c in multi])]
    dfs = []

    def rec(c):
        if c < 0:
            return
        dfs.append(c)
        rec(d1[c])
        rec(d2[c])
    for r in range(n):
        if parent[r] == -1:
            rec(r)
    return {
        "ids": [c["id"] for c in cells], "parent_ids": [c["pid"] for c in cells],
        "parent": parent, "daughter1": d1, "daughter2": d2, "rows": [len(c["t"]) for c in cells],
        "dfs_order": dfs,
        "root_mean_xg": [hx(rs[0][0]), hx(rs[1][0])], "root_var_xg": [hx(rs[0][1]), hx(rs[1][1])],
        "leaf_mean_xg": [hx(ls[0][0]), hx(ls[1][0])], "leaf_var_xg": [hx(ls[0][1]), hx(ls[1][1])],
        "time_sum": hx(sum(sum(c["t"]) for c in cells)),
        "log_length_sum": hx(sum(sum(c["x"]) for c in cells)),
        "fp_sum": hx(sum(sum(c["g"]) for c in cells)),
    }


# parameter sets used by the parity tests (index 0: the example's own parameter file)
PARAM_SETS = {
    "example": [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01],
    # 'const' noise needs var_g on the scale of g (the example's var_g is per unit of g)
    "const_noise": [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 2.6e+04, 1.63e-04, 7.48e-01],
    "perturbed": [2.5e-03, 5.0e-02, 1.2e-07, 8.5e+01, 1.4e-02, 2.2e+01, 5.5e-04, 3.0e-04, 9.0e-01, 1.8e-04, 6.5e-01],
}


def oracle_fixture(csv_path: str):
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    out = {}
    cfg = os.path.join(HERE, "example_csv_config.txt")
    for noise, div, pname in [("scaled", "binomial", "example"), ("scaled", "gauss", "example"),
                              ("const", "binomial", "const_noise"), ("const", "gauss", "const_noise"),
                              ("scaled", "binomial", "perturbed")]:
        hf = g.HostForest.from_csv(csv_path, cfg, -1, noise, div)
        of = O.OracleForest(hf.a)
        vals = [of.total_likelihood(PARAM_SETS[pname]) for _ in range(3)]
        out[f"{noise}/{div}/{pname}"] = {"ll": [hx(v[0]) for v in vals], "nan": [v[1:] for v in vals],
                                         "params": [hx(p) for p in PARAM_SETS[pname]]}
    json.dump(out, open(os.path.join(HERE, "oracle_example.json"), "w"), indent=1)
    return out


def oracle_predict_fixture(csv_path: str):
    """-p of the CPU oracle on the example (scaled / binomial, the example parameters): the
    forward, backward and combined state of the first and last row of every cell, plus a
    sha256 of the full [n_rows, 20] arrays (SURVEY.md §8(c) golden vector 7)"""
    import hashlib
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.from_csv(csv_path, os.path.join(HERE, "example_csv_config.txt"), -1, "scaled", "binomial")
    fwd, bwd, comb = O.OracleForest(hf.a).predict(PARAM_SETS["example"])
    ro = hf.a["row_offset"]
    rows = np.unique(np.concatenate([ro[:-1], ro[1:] - 1])).astype(np.int64)
    sha = hashlib.sha256(b"".join(np.ascontiguousarray(x).tobytes() for x in (fwd, bwd, comb))).hexdigest()
    np.savez_compressed(os.path.join(HERE, "oracle_example_predict.npz"), rows=rows, fwd=fwd[rows], bwd=bwd[rows],
                        comb=comb[rows], params=np.array(PARAM_SETS["example"]),
                        sha256=np.frombuffer(bytes.fromhex(sha), np.uint8))
    return len(rows), sha


def oracle_tests_h_fixture():
    """the reference's own likelihood test cell (src/tests.h:263-300) with its covariance as
    the carried state: the oracle's chain of 3 calls (SURVEY.md §8(c) golden vector 4)"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import pytest  # noqa: F401  (test module imports)
    from oracle import oracle as O
    src = open(os.path.join(ROOT, "tests", "test_gpu_parity.py")).read()
    i = src.index("def _tests_h_cell")
    j = src.index("@pytest.mark.parametrize", i)
    ns = {"np": np}
    exec(src[i:j], ns)
    hf, state, params = ns["_tests_h_cell"]()
    of = O.OracleForest(hf.a)
    of.state[:] = state
    vals = [of.total_likelihood(params)[0] for _ in range(3)]
    out = {"params": [hx(p) for p in params], "state": [hx(v) for v in state.ravel()], "ll": [hx(v) for v in vals]}
    json.dump(out, open(os.path.join(HERE, "oracle_tests_h_cell.json"), "w"), indent=1)
    return vals


def main():
    if "--oracle-only" in sys.argv:   # fixtures that need only the committed example data
        import tempfile
        with tempfile.TemporaryDirectory() as td:
            csv = os.path.join(td, "input.csv")
            with gzip.open(os.path.join(HERE, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
                shutil.copyfileobj(fi, fo)
            print("predict rows:", oracle_predict_fixture(csv))
        print("tests.h cell:", oracle_tests_h_fixture())
        return
    src = os.path.join(REF, "example_data_set")
    with open(os.path.join(src, "input.csv"), "rb") as fi, gzip.open(os.path.join(HERE, "example_input.csv.gz"), "wb", 9) as fo:
        shutil.copyfileobj(fi, fo)
    shutil.copy(os.path.join(src, "csv_config.txt"), os.path.join(HERE, "example_csv_config.txt"))
    shutil.copy(os.path.join(src, "parameter_file.txt"), os.path.join(HERE, "example_parameter_file.txt"))
    for f in ("example_csv_config.txt", "example_parameter_file.txt"):
        os.chmod(os.path.join(HERE, f), 0o644)
    print("dawson fixtures:", dawson_fixtures())
    topo = brute_force_topology(os.path.join(src, "input.csv"))
    json.dump(topo, open(os.path.join(HERE, "example_topology.json"), "w"))
    print("topology: cells", len(topo["ids"]))
    o = oracle_fixture(os.path.join(src, "input.csv"))
    for k, v in o.items():
        print(k, [float.fromhex(x) for x in v["ll"]], v["nan"])
    print("predict rows:", oracle_predict_fixture(os.path.join(src, "input.csv")))
    print("tests.h cell:", oracle_tests_h_fixture())


if __name__ == "__main__":
    main()
