"""The CLI's -p writer at scale: `lib/ggp -i c5.ggpd -b params -p` on a per-GPU shard of
BASELINE configs[4] (125k trees x 500 = 6.25e7 rows; the whole C5 file would be ~100 GB,
SURVEY §8 a15), wall seconds and bytes of _prediction.csv.

The file goes to /dev/null (a symlink in the output directory: formatting + the ordered
write, no disk), and -- when the disk has room -- to a real file, deleted afterwards.  Also
-pbin (binary rows) for the device-to-host floor.  Prints one JSON line.

  python tools/writer_c5.py [TREES=125000] [OUT_BASE_DIR] [CHUNK_ROWS=0]

TREES=1000000 CHUNK_ROWS=62500000 is the whole C5 forest (5e8 rows) through -chunk on one GPU; the
binary rows then go to /dev/null as well when the disk cannot hold them (56 GB).
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfp_gaussian_process_amd as g  # noqa: E402

CLI = os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", "ggp")
NAMES = ["mean_lambda", "gamma_lambda", "var_lambda", "mean_q", "gamma_q", "var_q", "beta",
         "var_x", "var_g", "var_dx", "var_dg"]
P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def run(args):
    t0 = time.perf_counter()
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=900)
    print(f"{' '.join(args[4:])}: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    for ln in r.stderr.splitlines():   # the CLI's phase timings (GGP_TIMING=1)
        if ln.startswith("[ggp timing]"):
            print("   " + ln, file=sys.stderr, flush=True)
    if r.returncode != 0:
        raise SystemExit(r.stdout[-2000:] + r.stderr[-2000:])
    return time.perf_counter() - t0


def main():
    trees = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
    base = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] else tempfile.gettempdir()
    chunk = ["-chunk", sys.argv[3]] if len(sys.argv) > 3 and int(sys.argv[3]) > 0 else []
    d = tempfile.mkdtemp(prefix="ggp_wr_", dir=base)
    try:
        t0 = time.perf_counter()
        hf = g.HostForest.synthetic(trees, 500, with_ids=True)
        data = os.path.join(d, "c5.ggpd")
        g.Dataset.from_forest(hf).save(data)
        print(f"dataset {hf.n_rows} rows written in {time.perf_counter() - t0:.1f} s ({os.path.getsize(data) / 1e9:.1f} GB)",
              file=sys.stderr, flush=True)
        pf = os.path.join(d, "p.txt")
        with open(pf, "w") as f:
            for n, v in zip(NAMES, P):
                f.write(f"{n} = {v!r}\n")
        res = {"trees": trees, "rows": hf.n_rows, "dataset_bytes": os.path.getsize(data),
               "io_threads": os.environ.get("GGP_IO_THREADS") or os.environ.get("OMP_NUM_THREADS")}
        del hf
        res["chunk_rows"] = int(chunk[1]) if chunk else 0
        # the device-to-host floor: binary rows (to /dev/null when the disk cannot hold them)
        out = os.path.join(d, "bin")
        if shutil.disk_usage(d).free < 2 * 120 * res["rows"]:
            os.makedirs(out)
            os.symlink("/dev/null", os.path.join(out, "c5_f_b_prediction.bin"))
            res["pbin_to"] = "/dev/null"
        res["pbin_wall_s"] = run(["-i", data, "-b", pf, "-p", "-pbin", "-g", "1", *chunk, "-o", out])
        shutil.rmtree(out)
        # formatting + ordered write into /dev/null
        out = os.path.join(d, "null")
        os.makedirs(out)
        os.symlink("/dev/null", os.path.join(out, "c5_f_b_prediction.csv"))
        res["csv_null_wall_s"] = run(["-i", data, "-b", pf, "-p", "-g", "1", *chunk, "-o", out])
        shutil.rmtree(out)
        # a real file, if the disk holds it (~200 B a row)
        need = 250 * res["rows"]
        res["free_disk_gb"] = shutil.disk_usage(d).free / 1e9
        if shutil.disk_usage(d).free > 3 * need:
            out = os.path.join(d, "file")
            res["csv_file_wall_s"] = run(["-i", data, "-b", pf, "-p", "-g", "1", *chunk, "-o", out])
            path = os.path.join(out, "c5_f_b_prediction.csv")
            res["csv_bytes"] = os.path.getsize(path)
            res["csv_file_gb_per_s"] = res["csv_bytes"] / res["csv_file_wall_s"] / 1e9
            shutil.rmtree(out)
        res["note"] = ("wall seconds of the whole CLI run (dataset load, forest upload, -p on the GPU, the writer); "
                       "csv_null: _prediction.csv symlinked to /dev/null")
        print(json.dumps(res))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
