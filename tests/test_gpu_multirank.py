"""Multi-rank runs of the HIP engine on the one-GPU box: several processes, one group.

The driver's scaling run launches bench.py with one rank per GPU over RCCL (nccl).  A GPU
box here has one card, and RCCL does not put two ranks on one device, so these tests
rehearse the same code with the gloo backend and every rank on cuda:0:
  - bench.py under torch.distributed.run with 2 ranks: the JSON line's whole-job value,
    n_gpus and the gathered total (bitwise the rank-order sum of single-process evaluations);
  - ShardedObjective over whole-tree shards of ONE forest (distributed.shard), each rank's
    partial from the HIP engine: the sum against the whole forest and the oracle, and a NaN
    on one rank raised on every rank.
"""
import json
import math
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P0 = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo_rehearsal():
    """bench.py --gpus 2 as the driver launches it (torch.distributed.run, one process per
    rank), gloo and both ranks on cuda:0"""
    import gfp_gaussian_process_amd as g
    sys.path.insert(0, ROOT)
    import bench
    trees, rows, steps, warm = 200, 200, 20, 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", str(warm),
           "--trees", str(trees), "--rows", str(rows), "--no-cpu", "--large-trees", "0", "--predict-trees", "0",
           "--hessian", "0", "--backend", "gloo", "--device", "0",
           "--c4-trees", "2000", "--c4-steps", "5", "--c4-scan", "5", "--c5-trees", "2000",
           "--c5-chunk-rows", "300000"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]      # rank 0 prints ONE line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == steps and out["warmup"] == warm
    assert out["config"]["rows_per_gpu"] == trees * rows
    # whole-job value: rows of both ranks over the max-over-ranks time of the K steps
    assert out["value"] == pytest.approx(2 * trees * rows / (out["ms_per_step"] * 1e-3), rel=1e-9)
    # the gathered total after the line's chained calls (W warm-up, the profiled window, the settling
    # calls, the K steps): the rank-order sum of each rank's own chain
    calls = out["chained_calls"]
    assert calls >= 2 * warm + steps
    want = 0.0
    for rank in range(2):
        hf = g.HostForest.synthetic(trees, rows, seed=bench.SEED, first_tree=rank * trees)
        f = g.Forest(hf, device=0)
        for _ in range(calls):
            v = f.total_likelihood(bench.P_EXAMPLE)
        f.close()
        want = want + v
    assert out["total_log_likelihood"] == want
    # the drop-in's own multi-GPU path, in a child process of rank 0: one handle over the device
    # list of the ranks ([0, 0] here: two logical shards), the whole job's forest, W + K chained
    # calls -- bitwise the single-device chain of the same forest
    ip = out["inprocess"]
    assert "error" not in ip, ip
    assert ip["devices"] == [0, 0] and ip["shards"] == 2 and ip["value"] > 0
    hw = g.HostForest.synthetic(2 * trees, rows, seed=bench.SEED)
    fw = g.Forest(hw, device=0)
    for _ in range(warm + steps):
        vw = fw.total_likelihood(bench.P_EXAMPLE)
    fw.close()
    assert ip["total_log_likelihood"] == vw
    # the strong-scaling legs: ONE forest split over the ranks.  C4: 2000 trees x 200 in two halves,
    # the whole forest's init statistics on both (one all_reduce), 3 + 5 evaluations then the
    # 5-sample chained scan; the gathered total against one handle over the whole forest (the
    # statistics' sums cross ranks in another order: agreement to the path's conditioning, not bitwise)
    c4 = out["c4_strong"]
    assert c4["rows"] == 2000 * rows and c4["trees_per_rank"] == 1000 and c4["scaling"] == "strong"
    assert c4["collective"]["ranks"] == 2 and c4["scan"]["samples"] == 5
    h4 = g.HostForest.synthetic(2000, rows, seed=bench.SEED, first_tree=3 * 10 ** 6)
    f4 = g.Forest(h4, device=0)
    for _ in range(3 + 5):
        v4 = f4.total_likelihood(bench.P_EXAMPLE)
    f4.close()
    assert c4["total_log_likelihood"] == pytest.approx(v4, rel=1e-9)
    # C5 -p split: 2000 trees x 500 = 1e6 rows, 5e5 per rank smoothed in two chunks of <= 3e5 rows
    # the collective's cost per call, and the rank count (gloo here: torch's path only)
    co = out["collective"]
    assert co["ranks"] == 2 and co["backend"] == "gloo" and co["local_only_ms_per_step"] > 0
    # the headline's exchange: host shared memory (both ranks on this node), cheaper than torch's
    assert co["headline_exchange"].startswith("host shared memory"), co
    assert c4["collective"]["kind"].startswith("host shared memory"), c4
    # (both legs timed; on one shared card their difference is the ranks' kernels queueing behind
    # each other, not the exchange: no ordering asserted here)
    assert co["headline_ms_per_step"] > 0 and co["torch_all_gather_ms_per_step"] > 0, co
    print("collective:", co)
    c5 = out["c5_predict_split"]
    assert c5["rows"] == 2000 * 500 and c5["shards_per_rank"] == 2 and c5["rows_per_s"] > 0


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedObjective, shard
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        full = g.HostForest.synthetic(301, 120)
        mine = shard(full, rank, world)
        obj = ShardedObjective(g.Forest(mine, device=0))
        vals = [obj.total_likelihood(P0) for _ in range(3)]
        bad = list(P0)
        bad[2] = -1.0
        # a NaN on one rank only: rank 1 evaluates bad parameters, rank 0 good ones
        obj2 = ShardedObjective(g.Forest(mine, device=0))
        try:
            obj2.total_likelihood(bad if rank == 1 else P0)
            nan_ok = False
        except g.LikelihoodIsNan:
            nan_ok = True
        q.put((rank, vals, mine.n_cells, nan_ok))
    finally:
        dist.destroy_process_group()


def test_sharded_objective_hip_engine_two_ranks():
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = g.HostForest.synthetic(301, 120)
    whole = g.Forest(full, device=0)
    of = O.OracleForest(full.a)
    want = [whole.total_likelihood(P0) for _ in range(3)]
    ref = [of.total_likelihood(P0)[0] for _ in range(3)]
    assert res[0][2] + res[1][2] == full.n_cells and min(res[0][2], res[1][2]) > 0
    for rank, vals, ncells, nan_ok in res:
        assert nan_ok                              # both ranks raise
        for v, w, o in zip(vals, want, ref):
            assert math.isfinite(v)
            assert abs(v - w) <= 1e-12 * abs(w)    # another partition of the same sum
            assert abs(v - o) <= 1e-9 * abs(o)     # the parity bar against the oracle
    assert res[0][1] == res[1][1]                  # every rank holds the same total


def _worker_nan(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedObjective, shard
    from test_distributed import _nan_forest
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mine = shard(_nan_forest(), rank, world)
        out = {}
        for mode in ("1", "0"):
            os.environ["GGP_NODE_EXCHANGE"] = mode
            obj = ShardedObjective(g.Forest(mine, device=0))
            try:
                obj.total_likelihood(P0)
                out[mode] = None
            except g.LikelihoodIsNan as e:
                out[mode] = (e.cell, e.row, e.rank)
            obj.close()
        obj = ShardedObjective(g.Forest(mine, device=0))
        pts = np.repeat(np.array(P0)[None, :], 3, axis=0)
        try:
            obj.total_likelihood_chain(pts)
            out["chain"] = None
        except g.LikelihoodIsNan as e:
            out["chain"] = (e.cell, e.row, e.rank, e.point)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_first_nan_across_ranks_hip_engine():
    """the whole forest's first NaN in the reference's order (likelihood.h:71-93, 110-122) from two
    ranks' HIP evaluations when the HIGHER rank holds the earlier root (tests/test_distributed.py's
    forest): every rank raises the oracle's (cell, row) through the shared-memory exchange, torch's
    all_gather and the chained path"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O
    from test_distributed import _nan_forest
    world = 2
    v, c, r = O.OracleForest(_nan_forest().a).total_likelihood(P0)
    assert math.isnan(v)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_nan, args=(rk, world, port, q)) for rk in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in res:
        assert out["1"] == (c, r, 1) and out["0"] == (c, r, 1), (rank, out)
        assert out["chain"] == (c, r, 1, 0), (rank, out)


_NCCL_CHILD = r'''
import os, sys, json, math
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch, torch.distributed as dist
import gfp_gaussian_process_amd as g
from gfp_gaussian_process_amd.distributed import ShardedObjective, shard
from test_distributed import _nan_forest
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(rank)
dist.init_process_group("nccl", device_id=torch.device("cuda", rank))
P = PARAMS
full = g.HostForest.synthetic(301, 120)
mine = shard(full, rank, world)
res = {}
for name, ec in (("engine", True), ("node", False)):
    o = ShardedObjective(g.Forest(mine, device=rank), engine_comm=ec)
    res[name] = {"engine": o.engine, "comm": o.f.comm_size() if ec else 0,
                 "vals": [o.total_likelihood(P) for _ in range(3)]}
    pts = np.repeat(np.array(P)[None, :], 3, axis=0); pts[:, 1] = [0.02, 0.03, 0.04]
    res[name]["chain"] = [float(x) for x in o.total_likelihood_chain(pts)]
    bad = shard(_nan_forest(), rank, world)
    ob = ShardedObjective(g.Forest(bad, device=rank), engine_comm=ec)
    try:
        ob.total_likelihood(P); res[name]["nan"] = None
    except g.LikelihoodIsNan as e:
        res[name]["nan"] = [e.cell, e.row, e.rank]
dist.destroy_process_group()
print(json.dumps({"rank": rank, "res": res}), flush=True)
'''


def test_engine_rccl_two_devices():
    """the engine's own RCCL collective (ggp_comm_attach) across two ranks on two distinct GPUs, one
    process each (nccl): totals and chained totals bitwise the host exchange's, the communicator
    holding both ranks, and the reference's first NaN on every rank.  Needs two visible devices
    (skipped on a one-GPU box; the driver's multi-GPU node runs it unchanged)"""
    import subprocess
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible devices")
    from oracle import oracle as O
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_distributed import _nan_forest
    code = f"ROOT={ROOT!r}\nPARAMS={P0!r}\n" + _NCCL_CHILD
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True, env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 0, (so[-2000:], se[-3000:])
    res = [json.loads(so.strip().splitlines()[-1])["res"] for so, _ in outs]
    _, c, r = O.OracleForest(_nan_forest().a).total_likelihood(P0)
    for rr in res:
        assert rr["engine"]["engine"] and rr["engine"]["comm"] == 2
        assert rr["engine"]["vals"] == rr["node"]["vals"] == res[0]["node"]["vals"]
        assert rr["engine"]["chain"] == rr["node"]["chain"]
        assert rr["engine"]["nan"] == [c, r, 1] and rr["node"]["nan"] == [c, r, 1]
