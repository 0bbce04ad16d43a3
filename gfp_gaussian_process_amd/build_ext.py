"""Compile the native libraries in-tree (no JIT cache, no pip install).

  lib/libggp.so       HIP engine for gfx950 (hipcc --offload-arch=gfx950)   include/ggp.h
  lib/libggp_exact.so the same engine in the oracle's arithmetic (GGP_EXACT)  include/ggp.h
  lib/libggp_host.so  host ingest, plain C++17 (g++)                        include/ggp_host.h
  lib/ggp             C++ CLI mirroring the reference's main.cpp modes
  lib/ggp_exact       the same CLI on libggp_exact.so

``python -m gfp_gaussian_process_amd.build_ext`` or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
INC = os.path.join(ROOT, "include")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = "gfx950"

# -ffp-contract=off: evaluate the reference's expressions without FMA contraction (the
# reference is built for plain x86-64, src/Makefile:2); DESIGN.md "Parity".
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
             "-Wall", "-Wno-unused-function"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall"]


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ...")


def _newer(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in deps)


def build(verbose: bool = False, force: bool = False) -> dict:
    os.makedirs(LIB, exist_ok=True)
    out = {}
    # --- device engine ---
    eng_src = os.path.join(CSRC, "ggp_engine.hip")
    eng_deps = [eng_src, os.path.join(CSRC, "ggp_device.h"), os.path.join(CSRC, "dawson_table.inc"),
                os.path.join(CSRC, "exp_table.inc"), os.path.join(INC, "ggp.h")]
    for extra in ("ggp_prop.h", "ggp_group.h", "ggp_predict.h", "ggp_joints.h", "ggp_outtab.h",
                  "ggp_out_tables.inc", "ggp_wave.h"):
        p = os.path.join(CSRC, extra)
        if os.path.exists(p):
            eng_deps.append(p)
    eng = os.path.join(LIB, "libggp.so")
    eng_x = os.path.join(LIB, "libggp_exact.so")
    # -cuid: a fixed offload compilation-unit id (clang derives it from the source path by
    # default), so the same sources give the same bytes in any checkout -- the PMC stamps in
    # profiles/ are keyed on this library's sha256 (bench.py).  The second library is the same
    # engine in the oracle's arithmetic (-DGGP_EXACT: glibc's exp, no products, no fma
    # contraction; DESIGN.md §2 "Exact arithmetic"), selected with GGP_ENGINE_LIB=libggp_exact.so.
    # The two compile concurrently (one hipcc each).
    jobs = []
    if force or not _newer(eng, eng_deps):
        jobs.append([HIPCC, *HIP_FLAGS, "-cuid=ggp_engine", "-shared", f"-I{INC}", f"-I{CSRC}", "-o", eng, eng_src,
                     "-ldl"])
    if force or not _newer(eng_x, eng_deps):
        jobs.append([HIPCC, *HIP_FLAGS, "-DGGP_EXACT", "-cuid=ggp_engine", "-shared", f"-I{INC}", f"-I{CSRC}", "-o",
                     eng_x, eng_src, "-ldl"])
    if jobs:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(len(jobs)) as ex:
            for fut in [ex.submit(_run, j, verbose) for j in jobs]:
                fut.result()
    out["libggp"] = eng
    out["libggp_exact"] = eng_x
    # --- host ingest ---
    host_src = os.path.join(CSRC, "host", "ggp_host.cpp")
    host = os.path.join(LIB, "libggp_host.so")
    host_deps = [host_src, os.path.join(CSRC, "host", "ggp_nelder_mead.h"), os.path.join(INC, "ggp_host.h"),
                 os.path.join(INC, "ggp.h")]
    if force or not _newer(host, host_deps):
        cxx = shutil.which("g++") or "g++"
        _run([cxx, *CXX_FLAGS, "-shared", f"-I{INC}", "-o", host, host_src, "-lpthread"], verbose)
    out["libggp_host"] = host
    # --- CLI ---
    cli_src = os.path.join(CSRC, "host", "ggp_cli.cpp")
    if os.path.exists(cli_src):
        cli = os.path.join(LIB, "ggp")
        deps = [cli_src, host_src, os.path.join(INC, "ggp.h"), os.path.join(INC, "ggp_host.h"),
                os.path.join(CSRC, "host", "ggp_text.h")]
        nm = os.path.join(CSRC, "host", "ggp_nelder_mead.h")
        if os.path.exists(nm):
            deps.append(nm)
        if force or not _newer(cli, deps + [eng]):
            _run([HIPCC, "-O2", "-std=c++17", f"-I{INC}", "-o", cli, cli_src, host_src,
                  f"-L{LIB}", "-lggp", "-Wl,-rpath,$ORIGIN", "-lpthread"], verbose)
        out["cli"] = cli
        # the same CLI on the exact-arithmetic engine (every output in the oracle's arithmetic)
        cli_x = os.path.join(LIB, "ggp_exact")
        if force or not _newer(cli_x, deps + [eng_x]):
            _run([HIPCC, "-O2", "-std=c++17", f"-I{INC}", "-o", cli_x, cli_src, host_src,
                  f"-L{LIB}", "-l:libggp_exact.so", "-Wl,-rpath,$ORIGIN", "-lpthread"], verbose)
        out["cli_exact"] = cli_x
    return out


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
