"""-js over the whole reference example (22,065 start rows, collect_joint_distributions,
correlation_tree.h:629-648) through the CLI, timed: wall seconds of `lib/ggp -i input.csv -b
parameter_file.txt -c csv_config.txt -js` (ingest, -p, the joints, both files), the sparse
file's size and joint lines.  The file is deleted afterwards.  Also -p alone, so the joints'
share is visible.  Prints one JSON line.

  python tools/joints_example_full.py [OUT_BASE_DIR]
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
GOLD = os.path.join(ROOT, "tests", "golden")
CLI = os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", "ggp")


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else tempfile.gettempdir()
    free = shutil.disk_usage(base).free
    d = tempfile.mkdtemp(prefix="ggp_js_", dir=base)
    try:
        csv = os.path.join(d, "input.csv")
        with gzip.open(os.path.join(GOLD, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
            shutil.copyfileobj(fi, fo)
        par = os.path.join(GOLD, "example_parameter_file.txt")
        cfg = os.path.join(GOLD, "example_csv_config.txt")
        res = {"free_disk_gb": free / 1e9, "io_threads": os.environ.get("GGP_IO_THREADS") or os.environ.get("OMP_NUM_THREADS")}
        for tag, flag in (("p", "-p"), ("js", "-js")):
            out = os.path.join(d, tag)
            t0 = time.perf_counter()
            r = subprocess.run([CLI, "-i", csv, "-b", par, "-c", cfg, flag, "-g", "1", "-o", out],
                               capture_output=True, text=True, timeout=900)
            wall = time.perf_counter() - t0
            if r.returncode != 0:
                raise SystemExit(r.stdout[-2000:] + r.stderr[-2000:])
            res[f"{tag}_wall_s"] = wall
            if tag == "js":
                sp = [f for f in os.listdir(out) if f.endswith("_joints_sparse.csv")][0]
                path = os.path.join(out, sp)
                lines, body = 0, False
                with open(path, "rb") as f:
                    for line in f:
                        if body:
                            lines += 1
                        elif line.startswith(b"start_row,column,"):
                            body = True
                res["sparse_bytes"] = os.path.getsize(path)
                res["joint_lines"] = lines
                os.remove(path)
        res["joints_wall_s"] = res["js_wall_s"] - res["p_wall_s"]
        res["joint_lines_per_s"] = res["joint_lines"] / res["js_wall_s"]
        res["note"] = ("lib/ggp -i input.csv -b parameter_file.txt -c csv_config.txt -js -g 1 on the reference example "
                       "(all 22,065 start rows); the dense -j file would be ~21 GB (44 fields x rows^2)")
        print(json.dumps(res))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
