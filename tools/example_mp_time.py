"""The reference's published command (`-m -p` on the example, example_data_set/README.txt:1-3)
through lib/ggp, call by call (GGP_NM_LOOKAHEAD=0 GGP_CHAIN_FUSED=0) and with the optimiser's
lookahead and the chained Hessian (default): wall seconds each, and whether every output file is
byte-identical.  One JSON line.

  python tools/example_mp_time.py
"""
import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", "ggp")
GOLD = os.path.join(ROOT, "tests", "golden")


def main():
    d = tempfile.mkdtemp(prefix="ggp_exmp_")
    csv = os.path.join(d, "input.csv")
    with gzip.open(os.path.join(GOLD, "example_input.csv.gz"), "rb") as a, open(csv, "wb") as b:
        shutil.copyfileobj(a, b)
    res, files = {}, {}
    runs = [("call_by_call", {"GGP_NM_LOOKAHEAD": "0", "GGP_CHAIN_FUSED": "0"}), ("default", {"GGP_TIMING": "1"})]
    for spec in filter(None, os.environ.get("EXMP_EXTRA", "").split(";")):   # name:K=V,K=V
        name, kv = spec.split(":")
        runs.append((name, dict([e.split("=") for e in kv.split(",")], GGP_TIMING="1")))
    for tag, env in runs:
        out = os.path.join(d, tag)
        t0 = time.perf_counter()
        r = subprocess.run([CLI, "-i", csv, "-b", os.path.join(GOLD, "example_parameter_file.txt"), "-c",
                            os.path.join(GOLD, "example_csv_config.txt"), "-m", "-p", "-g", "1", "-o", out],
                           capture_output=True, text=True, timeout=280, env=dict(os.environ, **env))
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            raise SystemExit(r.stdout[-2000:] + r.stderr[-2000:])
        files[tag] = {n: open(os.path.join(out, n), "rb").read() for n in sorted(os.listdir(out))
                      if not n.endswith(".log")}
        its = [n for n in files[tag] if n.endswith("_iterations.csv")]
        res[tag] = {"wall_s": wall, "nelder_mead_calls": files[tag][its[0]].count(b"\n") - 1 if its else None}
        timing = [ln for ln in r.stderr.splitlines() if ln.startswith("[ggp timing]")]
        if timing:
            res[tag]["phases"] = timing
        print(tag, res[tag], file=sys.stderr, flush=True)
    res["identical_files"] = all(sorted(files[t]) == sorted(files["call_by_call"]) and all(
        files[t][n] == files["call_by_call"][n] for n in files[t]) for t in files)
    res["files"] = sorted(files["default"])
    res["speedup"] = res["call_by_call"]["wall_s"] / res["default"]["wall_s"]
    shutil.rmtree(d, ignore_errors=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
