"""World-size-2 gloo tests of the forest sharding + the one collective per objective call.

The per-rank partial comes from the CPU oracle here (no GPU in this container); on the
GPU box the same ShardedObjective wraps the HIP engine's Forest and runs over RCCL.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.usefixtures("built")

P0 = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


class _OracleShard:
    def __init__(self, hf):
        from oracle import oracle as O
        self.o = O.OracleForest(hf.a)

    def total_likelihood(self, params):
        from gfp_gaussian_process_amd import LikelihoodIsNan
        v, c, r = self.o.total_likelihood(params)
        if math.isnan(v):
            raise LikelihoodIsNan(c, r)
        return v


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedObjective, shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        full = g.HostForest.synthetic(12, 40)
        # make tree sizes uneven so LPT matters
        mine = shard(full, rank, world)
        obj = ShardedObjective(_OracleShard(mine))
        vals = [obj.total_likelihood(P0) for _ in range(3)]
        bad = list(P0)
        bad[2] = -1.0
        try:
            obj.total_likelihood(bad)
            nan_ok = False
        except g.LikelihoodIsNan:
            nan_ok = True
        q.put((rank, vals, mine.n_cells, nan_ok))
    finally:
        dist.destroy_process_group()


def test_sharded_sum_equals_unsharded_oracle():
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    full = g.HostForest.synthetic(12, 40)
    of = O.OracleForest(full.a)
    want = [of.total_likelihood(P0)[0] for _ in range(3)]
    for rank, vals, ncells, nan_ok in res:
        assert nan_ok
        assert ncells == 18                      # 12 equal trees -> 6 trees (18 cells) per rank
        for v, w in zip(vals, want):
            assert v == pytest.approx(w, rel=1e-13)
    assert res[0][1] == res[1][1]                # every rank holds the same total (rank-order sum)


def test_lpt_partition_balances_and_is_deterministic():
    from gfp_gaussian_process_amd.distributed import lpt_partition
    w = [100, 90, 80, 70, 60, 50, 40, 30, 20, 10]
    parts = lpt_partition(w, 3)
    loads = [sum(w[i] for i in p) for p in parts]
    assert sorted(i for p in parts for i in p) == list(range(10))
    assert max(loads) - min(loads) <= 10
    assert parts == lpt_partition(w, 3)
    assert lpt_partition(w, 1) == [list(range(10))]
    assert lpt_partition([], 2) == [[], []]


def test_shards_cover_the_forest_exactly():
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import shard
    full = g.HostForest.synthetic(7, 40, with_ids=True)
    ids = []
    for r in range(3):
        ids += shard(full, r, 3).ids
    assert sorted(ids) == sorted(full.ids)


class _OraclePredictor:
    def __init__(self, hf):
        from oracle import oracle as O
        self.o = O.OracleForest(hf.a)

    def predict(self, params):
        return self.o.predict(params)


def _worker_predict(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedPredictor, shard_rows
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        full = g.HostForest.synthetic(12, 40)
        mine, rows = shard_rows(full, rank, world)
        sp = ShardedPredictor(_OraclePredictor(mine), rows, full.n_rows)
        fwd, bwd, comb = sp.predict(P0)
        out = sp.gather(comb, dst=0)
        q.put((rank, len(rows), None if out is None else out.tobytes()))
    finally:
        dist.destroy_process_group()


def test_sharded_predict_equals_unsharded_oracle():
    """-p over two ranks (gloo): each rank smooths its own trees, one gather assembles the
    combined rows in input order; bitwise equal to the unsharded smoother (no term crosses
    a tree, root/leaf statistics are the full forest's)"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_predict, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = g.HostForest.synthetic(12, 40)
    want = O.OracleForest(full.a).predict(P0)[2]
    assert res[0][1] + res[1][1] == full.n_rows and res[1][2] is None
    got = np.frombuffer(res[0][2]).reshape(want.shape)
    assert np.array_equal(got, want)


class _OracleChainShard(_OracleShard):
    """the oracle with Forest's chain entry: points one after another on the carried state"""

    def total_likelihood_chain(self, points):
        return np.array([self.total_likelihood(p) for p in np.atleast_2d(points)])


def _strong_worker(rank, world, port, q):
    """bench.py's strong-scaling legs on CPU: one synthetic forest generated per rank by tree index,
    the whole forest's init statistics by global_init_stats, then a sharded chain (the -s scan)"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedObjective, global_init_stats
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        T = 10
        lo, hi = rank * T // world, (rank + 1) * T // world
        mine = g.HostForest.synthetic(hi - lo, 40, first_tree=lo)
        local_stats = {k: np.array(mine.a[k]) for k in ("root_mean_xg", "root_var_xg", "leaf_mean_xg", "leaf_var_xg")}
        global_init_stats(mine)
        stats = {k: np.array(mine.a[k]) for k in local_stats}
        obj = ShardedObjective(_OracleChainShard(mine))
        pts = np.repeat(np.array(P0)[None, :], 4, axis=0)
        pts[:, 1] = [0.02, 0.03, 0.04, 0.05]
        chain = obj.total_likelihood_chain(pts)
        q.put((rank, stats, local_stats, chain))
    finally:
        dist.destroy_process_group()


def test_strong_split_init_stats_and_sharded_chain():
    """global_init_stats gives each rank's share the statistics of the whole forest (within rounding of
    the single-process ones), and ShardedObjective.total_likelihood_chain the whole forest's chained
    totals (each rank chains its share, one all_gather)"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = g.HostForest.synthetic(10, 40)
    for k in ("root_mean_xg", "root_var_xg", "leaf_mean_xg", "leaf_var_xg"):
        for r in range(world):
            np.testing.assert_allclose(res[r][1][k], full.a[k], rtol=1e-12)
        assert not np.allclose(res[0][2][k], full.a[k], rtol=1e-9) or k.endswith("mean_xg")
    np.testing.assert_array_equal(res[0][3], res[1][3])   # every rank holds the same totals
    of = O.OracleForest(full.a)
    pts = np.repeat(np.array(P0)[None, :], 4, axis=0)
    pts[:, 1] = [0.02, 0.03, 0.04, 0.05]
    want = np.array([of.total_likelihood(p)[0] for p in pts])
    # the statistics differ from the single-process ones in the last bits, and the totals move by
    # ~5e-11 relative for that (the path's conditioning): the north star's bar
    np.testing.assert_allclose(res[0][3], want, rtol=1e-9)


def _worker_xchg(rank, world, port, q):
    import random
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import NodeExchange, ShardedObjective, shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        # the exchange itself: many back-to-back calls with ranks running at uneven speeds
        x = NodeExchange(dist, None, width=2)
        assert x.ok
        rnd = random.Random(rank)
        seen = []
        for k in range(300):
            if rnd.random() < 0.05:
                time.sleep(0.002 * rnd.random())
            got = x.exchange((rank * 1000.0 + k, -k))
            seen.append(bool(np.array_equal(got[:, 0], np.arange(world) * 1000.0 + k)
                             and np.all(got[:, 1] == -k)))
        # a rank that never publishes: the others time out instead of waiting forever
        y = NodeExchange(dist, None, width=1, timeout_s=0.5)
        timed_out = False
        if rank != world - 1:
            try:
                y.exchange((1.0,))
            except TimeoutError:
                timed_out = True
        dist.barrier()
        y.close()
        # the objective: the shared-memory path and torch's give the same bits, NaN included
        full = g.HostForest.synthetic(12, 40)
        mine = shard(full, rank, world)
        res = {}
        for mode in ("1", "0"):
            os.environ["GGP_NODE_EXCHANGE"] = mode
            obj = ShardedObjective(_OracleShard(mine))
            assert (obj.xchg is not None) == (mode == "1")
            vals = [obj.total_likelihood(P0) for _ in range(2)]
            bad = list(P0)
            bad[2] = -1.0
            try:
                obj.total_likelihood(bad)
                nan_ok = False
            except g.LikelihoodIsNan:
                nan_ok = True
            res[mode] = (vals, nan_ok)
        x.close()
        q.put((rank, all(seen), timed_out, res))
    finally:
        dist.destroy_process_group()


def test_node_exchange_four_ranks():
    """NodeExchange (host shared memory, the partials' exchange for ranks on one node): 300
    back-to-back all-gathers at uneven rank speeds, a bounded wait when a rank never publishes, and
    the sharded objective bitwise the same through it as through torch's all_gather, NaN included;
    nothing left in /dev/shm"""
    import glob
    world = 4
    before = set(glob.glob("/dev/shm/ggp_x_*"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_xchg, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, seen_ok, timed_out, r in res:
        assert seen_ok, rank
        assert timed_out == (rank != world - 1), rank
        assert r["1"] == r["0"], rank
        assert r["1"][1]
    assert res[0][3]["1"][0] == res[-1][3]["1"][0]
    assert set(glob.glob("/dev/shm/ggp_x_*")) == before


def _nan_forest():
    """12 trees x 40 rows (tree k: cells 3k, 3k+1, 3k+2); LPT deals the even trees to rank 0 and the
    odd ones to rank 1.  NaN data in tree 4's root (rank 0) and in tree 1's second daughter (rank 1):
    the reference's first NaN is tree 1's (roots in input order), on the HIGHER rank"""
    import gfp_gaussian_process_amd as g
    full = g.HostForest.synthetic(12, 40, with_ids=True)
    ro = full.a["row_offset"]
    full.a["fp"] = np.array(full.a["fp"])
    full.a["fp"][ro[12] + 5] = np.nan     # tree 4, root, row 5
    full.a["fp"][ro[5] + 3] = np.nan      # tree 1, daughter2, row 3
    full.a["fp"][ro[4] + 7] = np.nan      # tree 1, daughter1, row 7: before daughter2 in DFS order
    return full


def _worker_nan(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd.distributed import ShardedObjective, shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mine = shard(_nan_forest(), rank, world)
        out = {}
        for mode in ("1", "0"):
            os.environ["GGP_NODE_EXCHANGE"] = mode
            obj = ShardedObjective(_OracleChainShard(mine), host_forest=mine)
            try:
                obj.total_likelihood(P0)
                out[mode] = None
            except g.LikelihoodIsNan as e:
                out[mode] = (e.cell, e.row, e.rank)
            obj.close()
        # the chain: the first point already fails (the data are NaN)
        obj = ShardedObjective(_OracleChainShard(mine), host_forest=mine)
        pts = np.repeat(np.array(P0)[None, :], 3, axis=0)
        try:
            obj.total_likelihood_chain(pts)
            out["chain"] = None
        except g.LikelihoodIsNan as e:
            out["chain"] = (e.cell, e.row, e.rank, e.point, len(e.ll))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_first_nan_across_ranks_is_the_references():
    """the reference's first NaN (roots in input order, DFS pre-order, row; likelihood.h:71-93,
    110-122) when both ranks hit NaN and the HIGHER rank holds the earlier root: every rank raises
    the whole-forest oracle's (cell, row), through the shared-memory exchange, torch's all_gather
    and the chained path"""
    from oracle import oracle as O
    world = 2
    full = _nan_forest()
    v, c, r = O.OracleForest(full.a).total_likelihood(P0)
    assert math.isnan(v) and (c, r) == (4, 7)          # tree 1's daughter1 (rank 1)
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
        assert out["1"] == (c, r, 1), (rank, out)
        assert out["0"] == (c, r, 1), (rank, out)
        assert out["chain"] == (c, r, 1, 0, 0), (rank, out)


def test_nan_order_keys():
    """NanOrder: DFS pre-order ranks within a tree and the root's input position in the whole forest"""
    from gfp_gaussian_process_amd.distributed import NanOrder, shard
    full = _nan_forest()
    sub = shard(full, 1, 2)                  # trees 1, 3, 5, ...: cells 3, 4, 5, 9, 10, 11, ...
    o = NanOrder(sub, rank=1)
    assert o.key(0, 2) == (3.0, 0.0, 2.0, 3.0)
    assert o.key(1, 7) == (3.0, 1.0, 7.0, 4.0)
    assert o.key(2, 3) == (3.0, 2.0, 3.0, 5.0)
    assert o.key(3, 0) == (9.0, 0.0, 0.0, 9.0)
    assert o.key(-1, -1)[0] == math.inf
