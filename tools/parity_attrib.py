#!/usr/bin/env python3
"""Attribute the example's GPU-vs-oracle gap (diagnostic; build container only).

Runs tools/parity_attrib.cpp -- the lane schedule's total log-likelihood emulated on the host from
the device source -- on the example's five configurations x three chained calls
(tests/golden/oracle_example.json) with the device's departures from the oracle switched on one at
a time, and prints the worst relative distance of each configuration from

  * the oracle fixture (oracle_example.json: the oracle on its own Dawson table), and
  * the reference-Dawson fixture (oracle_example_refdawson.json: the oracle on the reference's own
    Faddeeva::Dawson, compiled in place into oracle/_ref).

Usage: python tools/parity_attrib.py [--out profiles/rNN_parity_attrib.txt]
"""
from __future__ import annotations

import argparse
import ctypes
import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402
from oracle import oracle as O  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
CLANG = "/opt/rocm/llvm/bin/clang++"
ALL_PRODUCTS = (1 << 22) - 1


def build(contract: bool, outdir: str, exact: bool = False) -> ctypes.CDLL:
    so = os.path.join(outdir, f"libpa_{'c' if contract else 'nc'}{'_exact' if exact else ''}.so")
    cmd = [CLANG, "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
           "-I", os.path.join(ROOT, "gfp_gaussian_process_amd", "csrc"), "-I", os.path.join(ROOT, "oracle"),
           "-o", so, os.path.join(ROOT, "tools", "parity_attrib.cpp")]
    if contract:
        cmd[1:1] = ["-DGGP_HOST_CONTRACT", "-mfma"]
    if exact:
        cmd[1:1] = ["-DGGP_EXACT"]
    subprocess.run(cmd, check=True)
    L = ctypes.CDLL(so)
    L.pa_configure.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_void_p]
    L.pa_configure.restype = None
    L.pa_total.argtypes = [ctypes.POINTER(O.OraForest), ctypes.c_void_p, ctypes.c_void_p]
    L.pa_total.restype = ctypes.c_double
    assert L.pa_contracted() == int(contract)
    return L


def load_cases():
    tmp = tempfile.mkdtemp()
    csv = os.path.join(tmp, "input.csv")
    with gzip.open(os.path.join(G, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    own = json.load(open(os.path.join(G, "oracle_example.json")))
    ref = json.load(open(os.path.join(G, "oracle_example_refdawson.json")))
    cases = []
    for key, v in own.items():
        noise, div = key.split("/")[:2]
        hf = g.HostForest.from_csv(csv, os.path.join(G, "example_csv_config.txt"), -1, noise, div)
        cases.append((key, hf.a, [float.fromhex(x) for x in v["params"]],
                      np.array([float.fromhex(x) for x in v["ll"]]),
                      np.array([float.fromhex(x) for x in ref[key]["ll"]])))
    shutil.rmtree(tmp)
    return cases


def run(L, cases, exp_kind, mask, pow_libm, dawson):
    L.pa_configure(exp_kind, mask, pow_libm, dawson)
    out = {}
    for key, a, p, _, _ in cases:
        f = O.make_forest(a)
        st = np.zeros((f.n_cells, 20))
        pp = np.ascontiguousarray(p, np.float64)
        out[key] = np.array([L.pa_total(ctypes.byref(f), pp.ctypes.data, st.ctypes.data) for _ in range(3)])
    return out


def worst(res, cases, which):
    return max(float(np.max(np.abs(res[k] - (own if which == 0 else ref)) / np.abs(own)))
               for k, _, _, own, ref in cases)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    tmp = tempfile.mkdtemp()
    Lnc, Lc, Lx = build(False, tmp), build(True, tmp), build(False, tmp, exact=True)
    fad = O.faddeeva_ref()
    fad_ptr = ctypes.cast(fad, ctypes.c_void_p).value if fad is not None else None
    cases = load_cases()
    lines = []

    def row(name, L, exp_kind, mask, pow_libm, dawson=None):
        r = run(L, cases, exp_kind, mask, pow_libm, dawson)
        s = f"{name:58s} {worst(r, cases, 0):9.2e} {worst(r, cases, 1):9.2e}"
        print(s, flush=True)
        lines.append(s)
        return r

    hdr = f"{'configuration (lane schedule, host emulation)':58s} {'vs oracle':>9s} {'vs refDaw':>9s}"
    print(hdr)
    lines.append(hdr)
    row("oracle's arithmetic (glibc exp, no products/fma, pow)", Lnc, 0, 0, 1)
    row("  + 22 product exponentials", Lnc, 0, ALL_PRODUCTS, 1)
    row("  + fma contraction per expression", Lc, 0, 0, 1)
    row("  + exp_ocml (ocml's exp)", Lnc, 1, 0, 1)
    row("  + pow(a, k+1/2) as a^k sqrt(a)", Lnc, 0, 0, 0)
    if fad_ptr:
        row("  + the reference's Faddeeva::Dawson", Lnc, 0, 0, 1, fad_ptr)
    row("device lane body (all of the above but Faddeeva)", Lc, 1, ALL_PRODUCTS, 0)
    row("  - products", Lc, 1, 0, 0)
    row("  - fma contraction", Lnc, 1, ALL_PRODUCTS, 0)
    row("  - exp_ocml", Lc, 0, ALL_PRODUCTS, 0)
    row("  - a^k sqrt(a)", Lc, 1, ALL_PRODUCTS, 1)
    row("  - products, fma", Lnc, 1, 0, 0)
    row("  - products, fma, a^k sqrt(a)", Lnc, 1, 0, 1)
    if fad_ptr:
        row("device lane body on Faddeeva::Dawson", Lc, 1, ALL_PRODUCTS, 0, fad_ptr)
    row("GGP_EXACT lane body (exp_glibc, 74 exps, no fma, a^k sqrt(a))", Lx, 0, 0, 0)
    if fad_ptr:
        row("GGP_EXACT lane body on Faddeeva::Dawson", Lx, 0, 0, 0, fad_ptr)
    shutil.rmtree(tmp)
    if args.out:
        with open(args.out, "w") as f:
            f.write("# tools/parity_attrib.py: worst relative distance over the example's 5 configurations x 3 chained\n"
                    "# calls, host emulation of the lane schedule (device source, GGP_HOST_SIM)\n")
            f.write("\n".join(lines) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
