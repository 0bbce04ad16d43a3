#!/usr/bin/env python3
"""Benchmark: cell-timepoint Kalman updates/s of the lineage-tree log-likelihood.

Workload (BASELINE.json configs[1], "C2"): a synthetic forest of 1,000 trees x 200 rows
per GPU (root 100 rows + two daughters of 50, dt = 1 min, simulated from the model SDE with
the example parameters, Philox4x32 keyed by (seed, tree)); one step = one full
total-log-likelihood evaluation (likelihood.h:125-174 semantics, carried root state) with
the inputs resident in HBM, plus -- for N > 1 -- the one exchange of the per-rank partials
(host shared memory for the ranks of one node, distributed.NodeExchange; torch's all_gather over
RCCL otherwise, and timed beside it in `collective`).  Weak scaling: rank r evaluates trees
[r*T, (r+1)*T).

  python bench.py [--gpus N --steps K --warmup W --trees T --rows P --kernel auto|lane|group|wave]

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel (the one with the
largest share of the evaluation), timed with HIP events on the engine's own stream; `fp64` sets
that launch time against the FP64 work per update counted by PMC on this same build
(profiles/fp64_counts.json); `cpu_baseline` is the CPU oracle (oracle/, a C port of the
reference path) timed on this host, single-threaded (as the reference) and tree-parallel.

Order: the C2 forest is made resident, then the C4 strong-scaling leg runs (BASELINE configs[3],
~0.3 s of full-chip work), then the W warm-up and the K timed C2 steps, then the other legs.  The
C4 leg first means the headline runs at the shader clock the path sustains in a minimisation, not
the lower clock the first tens of milliseconds after idle hold (DESIGN.md §6 "The clock"); the
line's `clock` field reports the clock of the timed launches either way.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_UPDATE = 24          # time + log_length + fp doubles
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector (AMD spec)
COMBINE_BYTES_PER_ROW = 484   # k_combine: fwd + bwd rows (2 x 160 B) + prior segment (4 B) read, 160 B written
VALU_ISSUE_CYCLES = 4          # cycles a SIMD takes per 64-lane FP64 VALU wave-instruction (16 lanes/cycle)
VALU32_ISSUE_CYCLES = 2        # ... per 32-bit VALU wave-instruction (32-wide SIMD, MI355X_MICROARCH.md)
CLOCK_HZ = 2.4e9               # MI355X peak engine clock (MI355X_MICROARCH.md)
P_EXAMPLE = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04,
             3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]   # example_data_set/parameter_file.txt
SEED = 20261015


def _engine_sha() -> str:
    import hashlib
    return hashlib.sha256(open(os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", "libggp.so"), "rb").read()).hexdigest()


def _profile_json(name: str, args):
    """a committed PMC summary (profiles/<name>) -- only if it was taken on this same default
    workload AND on this very engine build (its recorded sha256): never a stale figure"""
    path = os.path.join(ROOT, "profiles", name)
    if args.trees != 1000 or args.rows != 200 or args.kernel != "auto" or not os.path.exists(path):
        return None
    d = json.load(open(path))
    return d if d.get("engine_sha256") == _engine_sha() else None


def traffic_for(kernel: str, args):
    """HBM bytes per launch of `kernel` from the PMC passes (profiles/traffic.json,
    tools/pmc_traffic.py), same workload and build only; else None"""
    d = _profile_json("traffic.json", args)
    k = None if d is None else d.get("kernels", {}).get(kernel)
    return None if k is None else k["bytes_per_launch"]


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_threads() -> int:
    """the host cores this process may use; on the GPU box the job's CPU share is 16
    (OMP_NUM_THREADS), while os.cpu_count() reports the whole machine"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def cpu_baseline(hf, budget_s: float):
    """time the CPU oracle on the same forest: whole evaluations until `budget_s` elapsed"""
    from oracle import oracle as O
    of = O.OracleForest(hf.a)
    first = None
    n_eval, t0 = 0, time.perf_counter()
    while True:
        v = of.total_likelihood(P_EXAMPLE)[0]
        if first is None:
            first = v
        n_eval += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return first, n_eval * hf.n_rows / el, n_eval, el


def cpu_baseline_parallel(hf, budget_s: float, threads: int):
    """the same oracle, tree-parallel: the forest in `threads` whole-tree shards (LPT, the
    global init statistics kept), one thread each (ctypes drops the GIL in the C oracle);
    whole evaluations of the forest until `budget_s` elapsed"""
    from concurrent.futures import ThreadPoolExecutor
    from gfp_gaussian_process_amd.distributed import shard
    from oracle import oracle as O
    parts = [O.OracleForest(shard(hf, r, threads).a) for r in range(threads)]
    n_eval, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while True:
            list(ex.map(lambda o: o.total_likelihood(P_EXAMPLE), parts))
            n_eval += 1
            el = time.perf_counter() - t0
            if el >= budget_s:
                break
    return n_eval * hf.n_rows / el, n_eval, el


def example_mp(tmp: str, cpu_budget: float):
    """The reference's published workload (example_data_set/README.txt:1-3: `-m -p` on the example,
    "around 5min"): the drop-in CLI lib/ggp with the reference's own arguments on the committed
    example files, one GPU.  Evaluations = the Nelder-Mead objective calls (one _iterations.csv row
    each, likelihood.h:142-148) + the chained Hessian error bars (3 epsilons x 4 k^2 points,
    likelihood.h:211-258, k = free parameters).  cpu_estimate_s = evaluations x the 1-core oracle's
    ms per evaluation of the same example forest, measured here."""
    import gzip
    import shutil
    import subprocess
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    gold = os.path.join(ROOT, "tests", "golden")
    os.makedirs(tmp, exist_ok=True)
    csv = os.path.join(tmp, "input.csv")
    with gzip.open(os.path.join(gold, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    par = os.path.join(gold, "example_parameter_file.txt")
    cfg = os.path.join(gold, "example_csv_config.txt")
    out = os.path.join(tmp, "out")
    cli = os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", "ggp")
    t0 = time.perf_counter()
    r = subprocess.run([cli, "-i", csv, "-b", par, "-c", cfg, "-m", "-p", "-g", "1", "-o", out],
                       capture_output=True, text=True, timeout=1200)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        return {"error": (r.stdout + r.stderr)[-400:]}
    its = [f for f in os.listdir(out) if f.endswith("_iterations.csv")]
    n_nm = sum(1 for _ in open(os.path.join(out, its[0]))) - 1 if its else 0
    ps = g.ParameterSet.load(par)
    k = len(ps.non_fixed())
    n_hess = 3 * 4 * k * k
    n_eval = n_nm + n_hess
    # the 1-core oracle on the same forest (init values), evaluations until the budget is spent
    hf = g.HostForest.from_csv(csv, cfg, -1, "scaled", "binomial")
    of = O.OracleForest(hf.a)
    pinit = ps.get_init()
    n, t1 = 0, time.perf_counter()
    while True:
        of.total_likelihood(pinit)
        n += 1
        if time.perf_counter() - t1 >= cpu_budget:
            break
    cpu_ms = 1e3 * (time.perf_counter() - t1) / n
    return {"wall_s": wall, "n_evals": n_eval, "n_nelder_mead": n_nm, "n_hessian": n_hess, "free_params": k,
            "ms_per_eval": 1e3 * wall / n_eval, "rows": hf.n_rows,
            "cpu_ms_per_eval_1core": cpu_ms, "cpu_estimate_s": n_eval * cpu_ms / 1e3,
            "reference_published": "around 5min (example_data_set/README.txt:1-3, hardware not stated)",
            "note": "lib/ggp -i input.csv -b parameter_file.txt -c csv_config.txt -m -p -g 1 (the reference's "
                    "command), wall time of the whole CLI run incl. ingest, -p and output files; the optimiser "
                    "evaluates its possible next calls ahead and the Hessians run chained (every output file "
                    "byte-identical to the call-by-call run: tools/example_mp_time.py); ms_per_eval = wall / "
                    "evaluations"}


def inprocess_child(argv) -> int:
    """`bench.py --inprocess-child TREES ROWS STEPS WARMUP KERNEL DEV[,DEV...]`: the drop-in CLI's
    multi-GPU path (Forest(hf, devices=[...]), what `-g all` runs) timed in a process of its own,
    so a failure there never takes the bench line with it; prints one JSON line"""
    trees, rows, steps, warmup = (int(x) for x in argv[:4])
    kernel, devs = argv[4], [int(d) for d in argv[5].split(",")]
    import gfp_gaussian_process_amd as g
    ha = g.HostForest.synthetic(trees, rows, seed=SEED)
    fa = g.Forest(ha, devices=devs, kernel=kernel)
    for _ in range(warmup):
        fa.total_likelihood(P_EXAMPLE)
    t1 = time.perf_counter()
    for _ in range(steps):
        v = fa.total_likelihood(P_EXAMPLE)
    iel = time.perf_counter() - t1
    print(json.dumps({"devices": devs, "trees": trees, "rows": ha.n_rows, "steps": steps,
                      "ms_per_step": 1e3 * iel / steps, "value": ha.n_rows * steps / iel,
                      "shards": len(fa.shards()), "total_log_likelihood": v}))
    fa.close()
    return 0


def example_parity(kernels=("auto", "lane")) -> dict:
    """North star's parity config: the example's total log-likelihood against the CPU oracle.  The
    five committed configurations x three chained calls (tests/golden/oracle_example.json, the oracle
    on its own Dawson table) and the same chains with the reference's own Faddeeva::Dawson
    (oracle_example_refdawson.json); worst relative distance per schedule, on the engine this
    process loaded (_native.engine_name())"""
    import gzip
    import shutil
    import tempfile
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import _native as N
    gold = os.path.join(ROOT, "tests", "golden")
    own = json.load(open(os.path.join(gold, "oracle_example.json")))
    ref = json.load(open(os.path.join(gold, "oracle_example_refdawson.json")))
    tmp = tempfile.mkdtemp()
    csv = os.path.join(tmp, "input.csv")
    with gzip.open(os.path.join(gold, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    out = {"engine": N.engine_name(), "calls": 3 * len(own), "bar": 1e-9}
    for kern in kernels:
        w_own = w_ref = 0.0
        for key, v in own.items():
            noise, div = key.split("/")[:2]
            hf = g.HostForest.from_csv(csv, os.path.join(gold, "example_csv_config.txt"), -1, noise, div)
            f = g.Forest(hf, kernel=kern)
            p = [float.fromhex(x) for x in v["params"]]
            ll = np.array([f.total_likelihood(p) for _ in range(3)])
            f.close()
            a = np.array([float.fromhex(x) for x in v["ll"]])
            b = np.array([float.fromhex(x) for x in ref[key]["ll"]])
            w_own = max(w_own, float(np.max(np.abs(ll - a) / np.abs(a))))
            w_ref = max(w_ref, float(np.max(np.abs(ll - b) / np.abs(b))))
        out[kern] = {"rel_vs_oracle": w_own, "rel_vs_refdawson": w_ref}
    shutil.rmtree(tmp)
    return out


def example_parity_child() -> int:
    """`bench.py --example-parity-child`: example_parity in a process of its own (the engine named by
    GGP_ENGINE_LIB, e.g. the exact-arithmetic libggp_exact.so); prints one JSON line"""
    from gfp_gaussian_process_amd import _native as N
    kern = ("auto", "lane", "pair") if "exact" in N.engine_name() else ("auto", "lane")
    print(json.dumps(example_parity(kern)))
    return 0


def run_example_parity() -> dict:
    """The example's parity (north star's parity config) on this process's engine and, in a child
    process, on the exact-arithmetic engine; errors are reported in the result, not raised"""
    import subprocess
    try:
        out = {"default_engine": example_parity(("auto", "lane"))}
    except Exception as e:
        out = {"default_engine": {"error": repr(e)[-300:]}}
    envx = dict(os.environ, GGP_ENGINE_LIB="libggp_exact.so")
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--example-parity-child"],
                           capture_output=True, text=True, timeout=600, env=envx)
        out["exact_engine"] = (json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else
                               {"error": (r.stdout + r.stderr)[-400:]})
    except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
        out["exact_engine"] = {"error": repr(e)[-300:]}
    return out


def host_split(step_t, trace) -> dict:
    """the timed steps' wall times and, per step, the engine's host split (ggp_call_trace: enqueue,
    wait for the completion, result; the path launch's own device time and clock), so the line shows
    where a step's time goes beyond the kernel: min / median / max over the steps and the first step
    on its own"""
    wall = np.diff(np.asarray(step_t)) * 1e6

    def stats(x):
        x = np.asarray(x, float)
        return {"min": float(x.min()), "median": float(np.median(x)), "max": float(x.max()), "first": float(x[0]),
                "mean": float(x.mean())}
    out = {"wall_us": stats(wall)}
    if trace is not None and len(trace) == len(wall):
        enq, wait, res, kern, mhz = (trace[:, k] for k in range(5))
        out.update({"enqueue_us": stats(enq), "wait_us": stats(wait), "result_us": stats(res)})
        out["python_us"] = stats(wall - enq - wait - res)
        if np.all(kern > 0):
            out.update({"kernel_us": stats(kern), "shader_mhz": stats(mhz),
                        "host_us": stats(wall - kern),
                        "dispatch_and_completion_us": stats(wait - kern)})
        out["note"] = ("per timed step: wall = python + enqueue + wait + result; wait = the launch's dispatch + kernel "
                       "(its first block start to its publishing block's end on the device's 100 MHz counter) + the "
                       "completion's trip to the host; ggp_call_trace")
    return out


def leg_fp64(cnt, kind: str, rows_per_s: float, n_simd: int, per_row_useful: bool = False, note: str = ""):
    """FP64 and VALU-issue fractions of a bench leg from the PMC pass of this build
    (profiles/fp64_counts.json, tools/fp64_summary.py kind `kind`): achieved FP64 = flops per row x
    rows/s against the FP64 peak (per_row_useful: the lane schedule's useful flops per update
    instead of the kernel's issued ones), and the class-weighted VALU issue cycles the rate needs
    per SIMD against the clock.  None without counters for this build."""
    if not cnt or not cnt.get(kind) or rows_per_s <= 0:
        return None
    c = cnt[kind]
    fpr = cnt.get("useful_flops_per_update") if per_row_useful else c.get("flops_per_update")
    if not fpr:
        return None
    vpu, f64pu = c.get("valu_wave_insts_per_update"), c.get("f64_wave_insts_per_update")
    out = {"kernel_counters": kind, "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS, "flops_per_row": fpr,
           "achieved": fpr * rows_per_s / 1e12, "frac": fpr * rows_per_s / 1e12 / FP64_PEAK_TFLOPS,
           "source": "profiles/fp64_counts.json (rocprofv3 PMC of this build)", "note": note}
    if vpu and f64pu is not None:
        cyc = VALU_ISSUE_CYCLES * f64pu + VALU32_ISSUE_CYCLES * (vpu - f64pu)
        out["valu_issue"] = {"valu_wave_insts_per_row": vpu, "f64_wave_insts_per_row": f64pu,
                             "issue_cycles_per_row": cyc, "frac": cyc * rows_per_s / n_simd / CLOCK_HZ}
    return out


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--inprocess-child":
        return inprocess_child(sys.argv[2:])
    if len(sys.argv) > 1 and sys.argv[1] == "--example-parity-child":
        return example_parity_child()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--trees", type=int, default=1000, help="trees per GPU")
    ap.add_argument("--rows", type=int, default=200, help="rows per tree")
    ap.add_argument("--kernel", default="auto", choices=["auto", "lane", "group", "wave", "pair"])
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU oracle work (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--large-trees", type=int, default=12500,
                    help="also time a C4-shard-sized forest (0 = skip)")
    ap.add_argument("--predict-trees", type=int, default=125000,
                    help="also time the -p smoother on a C5-shard forest: trees per GPU (0 = skip)")
    ap.add_argument("--hessian", type=int, default=1, help="also time the batched 11-parameter Hessian (0 = skip)")
    ap.add_argument("--predict-rows", type=int, default=500, help="rows per tree of the -p forest")
    ap.add_argument("--example-mp", type=int, default=1,
                    help="also time the reference's published workload: the CLI's -m -p on the example (N=1; 0 = skip)")
    ap.add_argument("--c3-evals", type=int, default=400,
                    help="also time BASELINE configs[2]: -m on 10k trees x 200 tp, this many evaluations (N=1; 0 = skip)")
    ap.add_argument("--joints-trees", type=int, default=20,
                    help="also time -j over every start row of this many C5-shaped trees (N=1; 0 = skip)")
    ap.add_argument("--inprocess", type=int, default=1,
                    help="N > 1: also time the CLI's in-process device-list path (one process, every rank's trees "
                         "sharded over devices 0..N-1, include/ggp.h) on rank 0 while the others wait (0 = skip)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo: rehearsal of the "
                         "multi-rank path on one GPU, the per-call 16 B through host memory)")
    ap.add_argument("--device", type=int, default=None,
                    help="HIP ordinal of this rank (default LOCAL_RANK; rehearsal: several ranks on one GPU)")
    ap.add_argument("--c4-trees", type=int, default=100000,
                    help="strong-scaling leg: BASELINE configs[3]'s forest (trees x --rows) split over the N ranks, "
                         "one evaluation per step plus the -s scan (0 = skip)")
    ap.add_argument("--c4-steps", type=int, default=20, help="evaluations timed in the C4 leg")
    ap.add_argument("--c4-scan", type=int, default=61, help="samples of the C4 leg's chained -s scan (0 = skip)")
    ap.add_argument("--c5-trees", type=int, default=1000000,
                    help="strong-scaling leg: BASELINE configs[4]'s -p on this many trees x --predict-rows split "
                         "over the N ranks (0 = skip)")
    ap.add_argument("--c5-chunk-rows", type=int, default=62500000,
                    help="rows per shard of the C5 leg's handle (a rank's share above it is smoothed in chunks)")
    ap.add_argument("--engine-comm-leg", type=int, default=1,
                    help="N > 1 with nccl: also time the C4 leg with the engine's own RCCL all-gather "
                         "(ggp_comm_attach), after the headline; a failure is reported in the line (0 = skip)")
    ap.add_argument("--example-parity", type=int, default=1,
                    help="N = 1: the example's 15 totals against the committed oracle fixtures, on this engine "
                         "and on the exact-arithmetic engine (libggp_exact.so, a child process) (0 = skip)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedObjective

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if args.device is not None:
        local = args.device
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    # the max-over-ranks of the timings: device tensors for RCCL, host tensors for gloo
    red_dev = "cuda" if args.backend == "nccl" else "cpu"

    # ---- this rank's forest (weak scaling), resident on the GPU before timing ----
    hf = g.HostForest.synthetic(args.trees, args.rows, seed=SEED, first_tree=rank * args.trees)
    fg = g.Forest(hf, device=local, kernel=args.kernel)
    obj = ShardedObjective(fg) if world > 1 else fg
    rows_rank = hf.n_rows

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---- strong scaling, BASELINE configs[3] (C4): ONE forest of --c4-trees x --rows split over the
    # N ranks by whole trees (contiguous blocks: every tree has the same rows, so this is the LPT
    # split), the init statistics of the whole forest on every rank (one all_reduce at setup); one
    # evaluation per step with one all_gather of the partials; then the chained -s scan
    # (main.cpp:77-112) -- every rank chains its shard, one all_gather of the per-sample partials.
    # It runs before the C2 headline: ~0.3 s of full-chip work, after which the headline's K steps
    # run at the shader clock the path sustains in a minimisation (2.37-2.39 GHz) rather than the
    # ~2.2 GHz the first tens of milliseconds after idle hold (DESIGN.md §6 "The clock"; the line's
    # `clock` field records it either way; --c4-trees 0 skips it) ----
    c4s = None
    if args.c4_trees > 0:
        from gfp_gaussian_process_amd.distributed import global_init_stats
        from gfp_gaussian_process_amd.optimize import arange
        T4 = args.c4_trees
        lo4, hi4 = rank * T4 // world, (rank + 1) * T4 // world
        h4 = g.HostForest.synthetic(hi4 - lo4, args.rows, seed=SEED, first_tree=3 * 10 ** 6 + lo4)
        if world > 1:
            global_init_stats(h4)
        f4 = g.Forest(h4, device=local, kernel=args.kernel)
        o4 = ShardedObjective(f4)
        for _ in range(3):
            o4.total_likelihood(P_EXAMPLE)
        barrier()
        t1 = time.perf_counter()
        for _ in range(args.c4_steps):
            ll4 = o4.total_likelihood(P_EXAMPLE)
        barrier()
        el4 = max_over_ranks((time.perf_counter() - t1) / args.c4_steps)
        rows4 = torch.tensor([h4.n_rows], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(rows4)
        rows4 = int(rows4.item())
        c4s = {"config": f"BASELINE configs[3] (C4): {T4} trees x {args.rows} tp, one forest split over "
                         f"{world} rank(s) by whole trees; the init statistics of the whole forest",
               "trees": T4, "rows": rows4, "trees_per_rank": hi4 - lo4, "steps": args.c4_steps,
               "ms_per_eval": 1e3 * el4, "updates_per_s": rows4 / el4, "scaling": "strong",
               "total_log_likelihood": ll4, "levels": f4.info()["levels"],
               "collective": {"kind": o4.exchange_kind if world > 1 else None,
                              "backend": args.backend if world > 1 else None,
                              "ranks": dist.get_world_size() if world > 1 else 1}}
        if args.c4_scan > 0:
            P4 = np.array(P_EXAMPLE)
            samples = arange(1.0e-03, 8.0e-02, (8.0e-02 - 1.0e-03) / args.c4_scan)[: args.c4_scan]
            pts = np.repeat(P4[None, :], len(samples), axis=0)
            pts[:, 1] = samples
            f4.reset_state()
            barrier()
            t1 = time.perf_counter()
            scan = o4.total_likelihood_chain(pts)
            barrier()
            sel4 = max_over_ranks(time.perf_counter() - t1)
            c4s["scan"] = {"parameter": "gamma_lambda", "samples": len(samples), "seconds": sel4,
                           "updates_per_s": len(samples) * rows4 / sel4, "first": float(scan[0]),
                           "last": float(scan[-1]),
                           "note": "-s: each sample from the carried state the previous left; every rank "
                                   "chains its trees (ggp_total_loglik_chain), one all_gather of the partials"}
        # the C4 handle is released after the headline: freeing its device memory here would put
        # an idle gap between the leg's full-chip work and the headline's steps
    for _ in range(args.warmup):
        obj.total_likelihood(P_EXAMPLE)

    # ---- roofline of the dominant kernel, HIP events on the engine's stream: a profiled window of
    # the same evaluations right after the warm-up, while the clock is the one the timed steps run at
    # (a gap of tens of ms before it would drop the clock to ~2.2 GHz for milliseconds, DESIGN.md §6
    # "The clock"); the events leave the handle's spin wait for a stream synchronisation, so the
    # window is separate from the timed steps, which follow it after W more warm-up calls ----
    fg.enable_profile()
    per = {}                                   # kernel name -> [ms, rows, launches]
    clocks = []
    n_prof = max(3, min(args.steps, 10))
    for _ in range(n_prof):
        fg.total_likelihood(P_EXAMPLE)
        ck = fg.launch_clock()
        if ck:
            clocks.append(ck[0])
        for ms, rows, name in zip(*fg.launch_profile()):
            acc = per.setdefault(name, [0.0, 0, 0])
            acc[0] += ms
            acc[1] += rows
            acc[2] += 1
    fg.disable_profile()
    # the profiled window synchronised on the stream, so the host thread slept between its calls;
    # the same number of calls on every rank (each is a collective at N > 1), at least 300 of them
    # (~50 ms of spin-waited calls), bring the host's enqueue back to its steady cost before the
    # timed steps: with only W = 5 the timed steps' median enqueue was 5.9 us against 2.9 us
    # (profiles/r6h_bench.json against profiles/r6g_bench.json), with 100 settling calls 4.1 us
    # (profiles/r6i_bench_driver_cmd.txt)
    n_settle = max(args.warmup, 300)
    for _ in range(n_settle):
        obj.total_likelihood(P_EXAMPLE)

    # ---- timed region: exactly K steps (each step's wall time kept: the line's `steps_us`; the
    # collector paused so no collection lands inside a step) ----
    import gc
    gc.disable()
    step_t = [0.0] * (args.steps + 1)
    barrier()
    t0 = time.perf_counter()
    step_t[0] = t0
    for k in range(args.steps):
        ll = obj.total_likelihood(P_EXAMPLE)
        step_t[k + 1] = time.perf_counter()
    barrier()
    el = time.perf_counter() - t0
    gc.enable()
    clock_timed = fg.launch_clock()   # the last timed launch's shader clock (wave schedule only)
    steps_us = host_split(step_t, fg.call_trace(args.steps) if hasattr(fg, "call_trace") else None)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_rows = rows_rank * world * args.steps
    value = total_rows / el

    # ---- N > 1: what the one exchange per call costs: the same K steps without it
    # (each rank's own evaluation only), with the headline's exchange (host shared memory when the
    # ranks share a node, else torch's all_gather), with torch's all_gather over RCCL, and, nccl
    # only, with the engine's RCCL all-gather (ggp_comm_attach, its own handle; a failure is
    # reported, not raised); microseconds per call = the difference of the max-over-ranks times ----
    coll = None
    if world > 1:
        def timed_steps(fn):
            for _ in range(3):
                fn(P_EXAMPLE)
            barrier()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                fn(P_EXAMPLE)
            barrier()
            tt = time.perf_counter() - t1
            t = torch.tensor([tt], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item()) / args.steps
        local_s = timed_steps(fg.total_likelihood)
        coll = {"ranks": dist.get_world_size(), "backend": args.backend, "headline_exchange": obj.exchange_kind,
                "local_only_ms_per_step": 1e3 * local_s, "headline_ms_per_step": 1e3 * el / args.steps,
                "headline_us_per_call": 1e6 * (el / args.steps - local_s)}
        ot = ShardedObjective(fg, node_exchange=False)
        tor_s = timed_steps(ot.total_likelihood)
        coll.update({"torch_all_gather_ms_per_step": 1e3 * tor_s,
                     "torch_all_gather_us_per_call": 1e6 * (tor_s - local_s)})
        if args.backend == "nccl" and args.engine_comm_leg:
            os.environ.setdefault("GGP_COMM_TIMEOUT_S", "60")
            try:
                fe2 = g.Forest(hf, device=local, kernel=args.kernel)
                oe2 = ShardedObjective(fe2, engine_comm=True)
                if oe2.engine:
                    eng_s = timed_steps(oe2.total_likelihood)
                    coll.update({"engine_rccl_ms_per_step": 1e3 * eng_s,
                                 "engine_rccl_us_per_call": 1e6 * (eng_s - local_s),
                                 "engine_rccl_value": rows_rank * world / eng_s,
                                 "rccl_comm_count": fe2.comm_size()})
                else:
                    coll["engine_rccl_error"] = "the engine's RCCL path was unavailable on some rank"
                fe2.close()
            except Exception as e:   # reported in the line: the headline stands either way
                coll["engine_rccl_error"] = repr(e)[-400:]

    if c4s is not None:
        if world > 1 and args.backend == "nccl" and args.engine_comm_leg:
            # the engine's own RCCL path (include/ggp.h ggp_comm_attach), after the headline and the
            # torch leg; a wait inside it is bounded by GGP_COMM_TIMEOUT_S and reported, not raised
            os.environ.setdefault("GGP_COMM_TIMEOUT_S", "60")
            eng = {}
            try:
                fe = g.Forest(h4, device=local, kernel=args.kernel)
                oe = ShardedObjective(fe, engine_comm=True)
                if not oe.engine:
                    eng["error"] = "the engine's RCCL path was unavailable on some rank (torch's path kept)"
                else:
                    eng["rccl_comm_count"] = fe.comm_size()
                    for _ in range(3):
                        oe.total_likelihood(P_EXAMPLE)
                    barrier()
                    t1 = time.perf_counter()
                    for _ in range(args.c4_steps):
                        lle = oe.total_likelihood(P_EXAMPLE)
                    barrier()
                    ele = max_over_ranks((time.perf_counter() - t1) / args.c4_steps)
                    eng.update({"ms_per_eval": 1e3 * ele, "updates_per_s": rows4 / ele,
                                "total_log_likelihood": lle, "same_total_as_torch_path": lle == ll4})
                fe.close()
            except Exception as e:   # reported in the line: the headline stands either way
                eng["error"] = repr(e)[-400:]
            eng["kind"] = "engine RCCL (ggp_comm_attach): partial, ncclAllGather, rank-order sum on the engine's stream"
            c4s["engine_rccl"] = eng

    # ---- roofline of the dominant kernel: HIP events on the engine's stream, recorded before the
    # timed region (above) ----
    if c4s is not None:   # released only now: freeing a 2e7-row forest (host and device) idles the GPU
        # long enough for its clock to fall, so neither the headline's steps nor its profiled launches
        # may follow it (DESIGN.md §6 "The clock")
        if world > 1:
            o4.close()
        f4.close()
        del h4
    dom = max(per, key=lambda k: per[k][0])
    d_ms, d_rows, d_n = per[dom]
    avg_ms = d_ms / d_n
    bytes_per_launch = BYTES_PER_UPDATE * d_rows / d_n
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    info = fg.info()
    # FP64 rates of the dominant kernel (profiles/fp64_counts.json, tools/fp64_summary.py; same
    # workload and build only).  useful: the FP64 work one update needs (one lane running the
    # whole update, the lane schedule on full waves) -- the figure to set against peak; issued:
    # every lane of every FP64 wave-instruction of the wave schedule, scalar work run in all 64
    # lanes and unused task candidates included -- an issue rate, not work done
    fp64 = None
    cnt = _profile_json("fp64_counts.json", args)
    n_simd_chip = 4 * torch.cuda.get_device_properties(local).multi_processor_count
    if cnt and dom.startswith("k_loglik_wave") and avg_ms > 0 and cnt.get("useful_flops_per_update"):
        upd_s = (d_rows / d_n) / (avg_ms * 1e-3)
        useful = cnt["useful_flops_per_update"] * upd_s / 1e12
        issued = (cnt.get("issued_flops_per_update") or 0.0) * upd_s / 1e12
        fp64 = {"kernel": dom, "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
                "useful_flops_per_update": cnt["useful_flops_per_update"], "achieved_useful": useful,
                "frac_useful": useful / FP64_PEAK_TFLOPS,
                "issued_lane_flops_per_update": cnt.get("issued_flops_per_update"), "issued_lane_rate": issued,
                "source": "profiles/fp64_counts.json (rocprofv3 PMC of this build) x the live launch time"}
        # the bound the kernel actually meets: VALU issue.  A SIMD issues at most one 64-lane FP64
        # wave-instruction per 4 cycles (16 lanes/cycle); the PMC pass counts the wave's VALU
        # instructions per update (SQ_INSTS_VALU), so their issue time over every SIMD of the chip
        # for one launch, against the launch time at the 2.4 GHz peak clock
        wv = cnt.get("wave") or {}
        vpu = wv.get("valu_wave_insts_per_update")
        f64pu = wv.get("f64_wave_insts_per_update")
        if vpu:
            n_simd = 4 * torch.cuda.get_device_properties(local).multi_processor_count
            # issue cycles by class: 4 per FP64 wave-instruction (16 FP64 lanes/cycle), 2 per 32-bit one
            # (32-wide SIMD); without the split (an older summary) every instruction at 4
            cyc = (VALU_ISSUE_CYCLES * f64pu + VALU32_ISSUE_CYCLES * (vpu - f64pu)) if f64pu is not None \
                else VALU_ISSUE_CYCLES * vpu
            need = cyc * (d_rows / d_n) / n_simd
            have = avg_ms * 1e-3 * CLOCK_HZ
            fp64["valu_issue"] = {"valu_wave_insts_per_update": vpu, "f64_wave_insts_per_update": f64pu,
                                  "issue_cycles_per_update": cyc, "simds": n_simd,
                                  "cycles_per_f64_inst": VALU_ISSUE_CYCLES, "cycles_per_32bit_inst": VALU32_ISSUE_CYCLES,
                                  "clock_ghz": CLOCK_HZ / 1e9, "frac": need / have,
                                  "note": "VALU issue cycles the launch needs per SIMD (class-weighted) / the launch's "
                                          "cycles: the root level runs one wave per SIMD (latency), the daughters two"}

    # ---- the same path on a C4-shard-sized forest (BASELINE configs[3]: 100k trees over 8
    # GPUs = 12.5k trees per GPU), reported beside the C2 headline ----
    large = None
    if args.large_trees > 0:
        hl = g.HostForest.synthetic(args.large_trees, args.rows, seed=SEED,
                                    first_tree=world * args.trees + rank * args.large_trees)
        fl = g.Forest(hl, device=local, kernel=args.kernel)
        for _ in range(2):
            fl.total_likelihood(P_EXAMPLE)
        barrier()
        t1 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            fl.total_likelihood(P_EXAMPLE)
        torch.cuda.synchronize()
        lel = (time.perf_counter() - t1) / reps
        large = {"trees_per_gpu": args.large_trees, "rows_per_gpu": hl.n_rows,
                 "ms_per_eval": 1e3 * lel, "updates_per_s_per_gpu": hl.n_rows / lel,
                 "note": "same path, per-GPU shard of BASELINE configs[3] (C4); not the headline value"}
        large["fp64"] = leg_fp64(cnt, "pair", hl.n_rows / lel, n_simd_chip, per_row_useful=True,
                                 note="k_loglik_pair counters x the leg's wall rate per evaluation")
        fl.close()

    # ---- opt-in batched objective on the C2 forest: the 4 k^2 = 484 points of an 11-parameter
    # Hessian (likelihood.h:211-258) in one ggp_total_loglik_batch call ----
    hess = None
    if args.hessian:
        from gfp_gaussian_process_amd import optimize as opt
        pts, _ = opt.hessian_points(P_EXAMPLE, list(range(11)), 1e-2)
        fg.total_likelihood_batch(pts)                     # warm-up + workspace
        barrier()
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            fg.total_likelihood_batch(pts)
        barrier()
        hel = (time.perf_counter() - t1) / reps
        # the same points with the reference's semantics (each from the state the previous left),
        # as the CLI's error bars make them: one ggp_total_loglik_chain call, bitwise the calls
        st0 = fg.state()
        fg.total_likelihood_chain(pts[:8])
        cel = 0.0
        for _ in range(reps):
            fg.set_state(st0)
            barrier()
            t1 = time.perf_counter()
            fg.total_likelihood_chain(pts)
            barrier()
            cel += (time.perf_counter() - t1) / reps
        hess = {"points": len(pts), "rows_per_point": rows_rank, "ms_per_batch": 1e3 * hel,
                "updates_per_s_per_gpu": len(pts) * rows_rank / hel,
                "sequential_ms_estimate": len(pts) * 1e3 * el / args.steps,
                "chained": {"ms_per_chain": 1e3 * cel, "updates_per_s_per_gpu": len(pts) * rows_rank / cel,
                            "note": "the same points chained through the carried state as the reference "
                                    "calls them (ggp_total_loglik_chain: bitwise the one-by-one calls)"},
                "note": "batched objective (opt-in, points independent) on the C2 forest; not the headline value"}

    # ---- the -p smoother on a per-GPU shard of BASELINE configs[4] (C5: 1M trees x 500 tp over
    # 8 GPUs = 125k trees per GPU): forward + backward levels and k_combine, device-resident
    # (outputs stay in HBM; the host copies are the CLI's I/O, not the smoother) ----
    pred = None
    if args.predict_trees > 0:
        hp = g.HostForest.synthetic(args.predict_trees, args.predict_rows, seed=SEED,
                                    first_tree=world * (args.trees + args.large_trees) + rank * args.predict_trees)
        fp_ = g.Forest(hp, device=local)
        fp_.predict(P_EXAMPLE, outputs=(False, False, False))        # warm-up + workspace
        barrier()
        t1 = time.perf_counter()
        reps, sm, cb = 3, 0.0, 0.0
        for _ in range(reps):
            fp_.predict(P_EXAMPLE, outputs=(False, False, False))
            a_, b_ = fp_.predict_profile()
            sm += a_
            cb += b_
        barrier()
        pel = (time.perf_counter() - t1) / reps
        if world > 1:
            t = torch.tensor([pel], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            pel = float(t.item())
        nr = hp.n_rows
        cb_ms = cb / reps
        # every level of a C5 shard runs the lane smoother, so the backward pass forms the combined
        # rows itself (k_bwd_level<true>): the events then see no separate combine
        fused = cb_ms < 0.01 * (sm / reps)
        pred = {"trees_per_gpu": args.predict_trees, "rows_per_gpu": nr, "ms_per_predict": 1e3 * pel,
                "rows_per_s": nr * world / pel, "smooth_ms": sm / reps,
                "combine_ms": None if fused else cb_ms, "combine_fused_into_backward": fused,
                "combine_bytes_per_row": COMBINE_BYTES_PER_ROW,
                "combine_gbs": None if fused else COMBINE_BYTES_PER_ROW * nr / (cb_ms * 1e-3) / 1e9,
                "note": "-p forward+backward+combine per GPU shard of BASELINE configs[4] (C5), outputs "
                        "resident in HBM; smooth_ms includes the combine when it is fused into the "
                        "backward pass; rows_per_s is whole-job; not the headline value"}
        if sm > 0 and not fused:
            pred["fp64_smooth"] = leg_fp64(cnt, "smooth", nr / (sm / reps * 1e-3), n_simd_chip,
                                           note="forward + backward smoother kernels (one row per lane: issued "
                                                "= the work) x the device time of the levels")
        elif sm > 0 and cnt and cnt.get("smooth") and cnt.get("combine"):
            # the fused pass issues the smoother's and the combine's instructions (counted apart,
            # tools/fp64_workload.py runs the predict with GGP_COMBINE_FUSED=0)
            both = {k: cnt["smooth"][k] + cnt["combine"][k]
                    for k in ("flops_per_update", "valu_wave_insts_per_update", "f64_wave_insts_per_update")}
            pred["fp64_smooth_and_combine"] = leg_fp64({"both": both}, "both", nr / (sm / reps * 1e-3), n_simd_chip,
                                                       note="forward + backward smoother with the combine fused in: "
                                                            "the smoother's and k_combine's counters per row x the "
                                                            "device time of the levels")
        if not fused and cb_ms > 0:
            pred["fp64_combine"] = leg_fp64(cnt, "combine", nr / (cb_ms * 1e-3), n_simd_chip,
                                            note="k_combine counters x its device time")
        fp_.close()

    # ---- N > 1: the drop-in CLI's own multi-GPU path (-g all): ONE process, the whole job's trees
    # sharded over devices 0..N-1 inside the C-ABI (include/ggp.h), timed on rank 0 while the other
    # ranks wait on the store (no GPU work of theirs meanwhile) ----
    inproc = None
    if world > 1 and args.inprocess:
        store = dist.distributed_c10d._get_default_store()
        devs = [None] * world                      # the devices the ranks use (a rehearsal: all 0)
        dist.all_gather_object(devs, local)
        barrier()
        if rank == 0:
            import subprocess
            # a child process of its own (started, not exec'd): a fault on any device there is
            # reported in the line instead of ending this rank before it prints
            cmd = [sys.executable, os.path.abspath(__file__), "--inprocess-child", str(args.trees * world),
                   str(args.rows), str(args.steps), str(args.warmup), args.kernel, ",".join(str(int(d)) for d in devs)]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
                if r.returncode == 0:
                    inproc = json.loads(r.stdout.strip().splitlines()[-1])
                else:
                    inproc = {"error": f"exit {r.returncode}: " + (r.stdout + r.stderr)[-400:]}
            except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
                inproc = {"error": repr(e)[-400:]}
            inproc["note"] = ("one process drives every device (Forest(hf, devices=range(N)), the CLI's -g all), "
                              "in a child process: the whole job's forest, bitwise the single-device total; the "
                              "same metric as value")
            store.set("ggp_inprocess_done", "1")
        else:
            store.wait(["ggp_inprocess_done"])
        barrier()
    # ---- BASELINE configs[2] (C3): the -m loop on the 10k trees x 200 tp forest, all 11 parameters
    # free (the example's file with beta = 4.95E-04, 4.95E-05), log space, LN_NELDERMEAD at
    # tol 1e-10 through optimize.minimize_wrapper (the product's optimiser and objective), bounded
    # at a fixed evaluation count ----
    c3 = None
    if world == 1 and args.c3_evals > 0:
        from gfp_gaussian_process_amd import optimize as opt
        P3 = g.ParameterSet.load(os.path.join(ROOT, "tests", "golden", "example_parameter_file.txt"))
        P3.kind[6], P3.step[6] = "free", 4.95e-05
        h3 = g.HostForest.synthetic(10000, 200, seed=SEED, first_tree=10 ** 6)
        f3 = g.Forest(h3, device=local, kernel=args.kernel)
        calls = [0]

        def obj3(p):
            calls[0] += 1
            return f3.total_likelihood(p)
        obj3(P3.init)                               # warm-up (workspaces), not counted below
        f3.reset_state()
        calls[0] = 0
        barrier()
        t1 = time.perf_counter()
        x3, ll3, rc3 = opt.minimize_wrapper(obj3, P3, tolerance=1e-10, search_space="log", maxeval=args.c3_evals)
        barrier()
        c3el = time.perf_counter() - t1
        c3 = {"config": "C3: synthetic 10000 trees x 200 tp, -m log-space Nelder-Mead (minimize_wrapper), "
                        "11 free parameters, tol 1e-10, bounded at maxeval",
              "rows": h3.n_rows, "evaluations": calls[0], "seconds": c3el, "ms_per_eval": 1e3 * c3el / calls[0],
              "evals_per_s": calls[0] / c3el, "updates_per_s": calls[0] * h3.n_rows / c3el,
              "ll_best": ll3, "nlopt_result": rc3, "levels": f3.info()["levels"],
              "note": "BASELINE configs[2]; the optimiser's calls are sequential (carried state), each one "
                      "GPU evaluation with the optimiser's host step between; not the headline value"}
        f3.close()

    # ---- BASELINE configs[4]'s -j half on C5-shaped trees (the <= 10k-row subset): 20
    # trees x 500 tp (250 + 125 + 125 rows), ggp_joints over every start row in ranges as the CLI
    # streams them (ggp_cli.cpp: 4,096 start rows first, then ranges sized for about 2^20 joints at
    # the density seen), into one pair of host buffers reused from range to range as the CLI's
    # are, the joints copied to the host ----
    jc5 = None
    if world == 1 and args.joints_trees > 0:
        hj = g.HostForest.synthetic(args.joints_trees, args.predict_rows, seed=SEED, first_tree=2 * 10 ** 6)
        fj = g.Forest(hj, device=local)
        nrj = hj.n_rows
        jcap = 1 << 21   # the CLI's max_cap
        jbuf = (np.empty((jcap, 2), np.int64), np.empty((jcap, 44)))   # packed, as the CLI takes them
        for b_ in jbuf:
            b_.fill(0)   # paged in, as a long-running writer's buffers are
        fj.joints(P_EXAMPLE, 1e-10, 0, min(nrj, 256), out=jbuf, packed=True)   # warm-up: smoother tables cached
        barrier()
        t1 = time.perf_counter()
        nj, lo, chunk, n_calls = 0, 0, 4096, 0
        while lo < nrj:
            hi = min(nrj, lo + chunk)
            n_calls += 1
            try:
                idx_j, _ = fj.joints(P_EXAMPLE, 1e-10, lo, hi, out=jbuf, packed=True)
            except g.GGPError:   # more than the CLI's max_cap: split the range, as the CLI does
                chunk = max(1, (hi - lo) // 2)
                continue
            nj += len(idx_j)
            if len(idx_j):
                chunk = min(65536, max(256, (hi - lo) * (jcap // 2) // len(idx_j)))
            lo = hi
        barrier()
        jel = time.perf_counter() - t1
        jc5 = {"config": f"-j on {args.joints_trees} C5-shaped trees x {args.predict_rows} tp ({nrj} rows), "
                         "tol 1e-10, every start row, ranges as the CLI's (4,096 start rows, then sized for ~2^20 "
                         "joints), reused host buffers",
               "rows": nrj, "joints": nj, "calls": n_calls, "seconds": jel, "joints_per_s": nj / jel, "start_rows_per_s": nrj / jel,
               "note": "BASELINE configs[4]'s -j leg on its tree shape (SURVEY 8(d) subset); joints computed on "
                       "the GPU and copied to the host as the CLI takes them (ggp_joints_packed: 8 means and "
                       "the covariance's upper triangle, 44 doubles each), parameter tables cached per parameters"}
        fj.close()


    # ---- strong scaling, BASELINE configs[4] (C5): -p over ONE forest of --c5-trees x --predict-rows
    # split over the N ranks (no collective on the data path: every rank smooths its trees, the rows
    # stay in HBM); a rank's share above --c5-chunk-rows is smoothed in chunks through one workspace ----
    c5s = None
    if args.c5_trees > 0:
        from gfp_gaussian_process_amd.distributed import global_init_stats
        T5 = args.c5_trees
        lo5, hi5 = rank * T5 // world, (rank + 1) * T5 // world
        t1 = time.perf_counter()
        h5 = g.HostForest.synthetic(hi5 - lo5, args.predict_rows, seed=SEED, first_tree=4 * 10 ** 6 + lo5)
        if world > 1:
            global_init_stats(h5)
        synth5 = time.perf_counter() - t1
        chunk = args.c5_chunk_rows if h5.n_rows > args.c5_chunk_rows else 0
        f5 = g.Forest(h5, device=local, max_shard_rows=chunk)
        nsh5 = len(f5.shards())
        f5.predict(P_EXAMPLE, outputs=(False, False, False))    # warm-up + workspace
        barrier()
        t1 = time.perf_counter()
        reps5 = 2
        for _ in range(reps5):
            f5.predict(P_EXAMPLE, outputs=(False, False, False))
        barrier()
        el5 = max_over_ranks((time.perf_counter() - t1) / reps5)
        rows5 = torch.tensor([h5.n_rows], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(rows5)
        rows5 = int(rows5.item())
        c5s = {"config": f"BASELINE configs[4] (C5) -p: {T5} trees x {args.predict_rows} tp, one forest split over "
                         f"{world} rank(s) by whole trees, forward + backward + combine, rows resident in HBM",
               "trees": T5, "rows": rows5, "trees_per_rank": hi5 - lo5, "shards_per_rank": nsh5,
               "chunk_rows": chunk, "ms_per_predict": 1e3 * el5, "rows_per_s": rows5 / el5, "scaling": "strong",
               "synth_s_rank0": synth5}
        f5.close()
        del h5

    exmp = None
    if world == 1 and args.example_mp:
        exmp = example_mp(os.path.join("/tmp", f"ggp_example_mp_{os.getpid()}"), 3.0 if not args.no_cpu else 0.5)

    result = None
    if rank == 0:
        result = {
            "metric": "cell-timepoint Kalman updates/s",
            "value": value,
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * el / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (model-SDE simulated forest, Philox4x32 seed 20261015)",
            "config": {
                "workload": f"C2: synthetic forest {args.trees} trees x {args.rows} timepoints per GPU "
                            f"(root {args.rows // 2} + 2 x {args.rows // 4} rows), single total-log-likelihood "
                            "evaluation per step, scaled noise + binomial division, example parameters",
                "trees_per_gpu": args.trees, "rows_per_gpu": rows_rank, "levels": info["levels"],
                "kernel": args.kernel, "parallelism": f"forest sharded by whole trees, {world} rank(s)"
                                                      + ("" if world == 1 else f", {args.backend}"),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic_for(dom, args),
                "traffic_source": "rocprofv3 PMC FETCH_SIZE + WRITE_SIZE per launch (profiles/traffic.json, this build): "
                                  "bytes between L2 and the fabric, not HBM bytes -- part of the 4.8 MB forest stays "
                                  "in L2 / the Infinity Cache from one launch to the next, so the fetch side sits "
                                  "below the algorithmic reads",
                "bytes_per_update": BYTES_PER_UPDATE,
                "avg_launch_ms": avg_ms,
                "launches_timed": d_n,
                "per_kernel_ms": {k: v[0] / v[2] for k, v in per.items()},
                "note": "algorithmic bytes only; the path is FP64-latency/VALU bound (DESIGN.md)",
            },
            "fp64": fp64,
            "total_log_likelihood": ll,
            # the chained calls behind that total: W warm-up, the profiled window, the settling calls, the K steps
            "chained_calls": args.warmup + n_prof + n_settle + args.steps,
            "steps_us": steps_us,
            "clock": None if clock_timed is None else {
                "shader_mhz_last_timed_launch": clock_timed[0], "window_us": clock_timed[1],
                "shader_mhz_profiled_launches": clocks,
                "note": "the path launch's block 0: s_memtime cycles per s_memrealtime tick (100 MHz) over its "
                        "path (ggp_launch_clock), i.e. the DVFS clock the evaluation ran at; peak 2400 MHz"},
        }
        if large is not None:
            result["large_forest"] = large
        if pred is not None:
            result["predict"] = pred
        if hess is not None:
            result["hessian_batch"] = hess
        if exmp is not None:
            result["example_mp"] = exmp
        if c3 is not None:
            result["c3_minimize"] = c3
        if jc5 is not None:
            result["joints_c5_subset"] = jc5
        if inproc is not None:
            result["inprocess"] = inproc
        if coll is not None:
            result["collective"] = coll
        if c4s is not None:
            result["c4_strong"] = c4s
        if c5s is not None:
            result["c5_predict_split"] = c5s
        if world == 1 and args.example_parity:
            result["example_parity"] = run_example_parity()
        if world == 1 and not args.no_cpu:
            fresh = g.Forest(hf, device=local, kernel=args.kernel).total_likelihood(P_EXAMPLE)
            ref, rate, n_eval, cel = cpu_baseline(hf, args.cpu_budget)
            nth = cpu_threads()
            prate, pn, pel = cpu_baseline_parallel(hf, args.cpu_budget * 0.6, nth)
            result["cpu_baseline"] = {
                "value": rate, "unit": "updates/s", "cores": 1, "kind": "port",
                "sample": f"{n_eval} full evaluations of the same {rows_rank}-row forest "
                          f"({cel:.1f} s, single thread -- the reference is single-threaded -- "
                          f"oracle/ggp_oracle.c -O3)",
                "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
                "parallel": {"value": prate, "cores": nth,
                             "sample": f"{pn} full evaluations in {pel:.1f} s, forest split into {nth} "
                                       f"whole-tree shards, one oracle thread each"},
            }
            result["ll_rel_err_vs_cpu"] = abs(fresh - ref) / abs(ref)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    fg.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
