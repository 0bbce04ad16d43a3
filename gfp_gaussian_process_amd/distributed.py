"""Multi-GPU forest sharding: one process per GPU, torch.distributed over RCCL (xGMI).

Trees are independent (no cross-tree term in total_likelihood, likelihood.h:125-159), so
the forest is split into whole trees, balanced by longest-processing-time bin packing on
row count (ties: critical-path length, then tree order).  Each rank keeps its shard's
device-resident data and carried root state; one objective call = every rank evaluates
its shard, then ONE collective exchanges one double per rank (all_gather), and the
partials are summed in rank order so the result is bitwise reproducible run to run.
For ranks on one node (every rank of a one-node torchrun) the exchange goes through host shared
memory (NodeExchange: the partials are already on the host, 16 bytes per rank is latency, not
bandwidth); across nodes, or with GGP_NODE_EXCHANGE=0, it is torch's all_gather_into_tensor (RCCL
for an nccl group); opt-in (engine_comm=True / GGP_ENGINE_COMM=1) it runs inside the engine
(include/ggp.h ggp_comm_attach: partial, RCCL all-gather and rank-order sum enqueued on the
engine's stream behind the evaluation).  All give the same bits.
The first NaN is resolved as the reference finds it: each rank sends the place of its own first NaN
in the whole forest's order (root input position, DFS rank, row; NanOrder) with its partial, and
every rank raises the smallest one's (cell, row).
Scan samples and optimiser steps stay sequential (carried state), only the forest is
parallel.

-p shards the same way (ShardedPredictor): the smoother has no term across trees either,
so every rank smooths its own trees with no collective on the data path; one gather at
the end assembles the rows in input order on one rank (or each rank writes its own rows).
"""
from __future__ import annotations

import heapq
import math
import os
import platform
import secrets
import socket
import time

import numpy as np

from .forest import Forest, HostForest, LikelihoodIsNan


def tree_sizes(hf: HostForest):
    """(roots, rows per tree, critical path rows per tree) in root order"""
    a = hf.a
    ro = a["row_offset"]
    rows_cell = np.diff(ro)
    d1, d2 = a["daughter1"], a["daughter2"]
    roots = hf.roots
    tot, crit = [], []
    for r in roots:
        stack = [(int(r), int(rows_cell[r]))]
        s, best = 0, 0
        while stack:
            c, path = stack.pop()
            s += int(rows_cell[c])
            best = max(best, path)
            for ch in (d1[c], d2[c]):
                if ch >= 0:
                    stack.append((int(ch), path + int(rows_cell[ch])))
        tot.append(s)
        crit.append(best)
    return roots, np.array(tot, np.int64), np.array(crit, np.int64)


def lpt_partition(weights, world: int, secondary=None):
    """Longest-processing-time bin packing: returns `world` lists of item indices.
    Deterministic: items by (-weight, -secondary, index), ties on bins by (load, rank)."""
    weights = np.asarray(weights, np.int64)
    sec = np.zeros_like(weights) if secondary is None else np.asarray(secondary, np.int64)
    order = sorted(range(len(weights)), key=lambda i: (-int(weights[i]), -int(sec[i]), i))
    heap = [(0, r) for r in range(world)]
    bins = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        bins[r].append(i)
        heapq.heappush(heap, (load + int(weights[i]), r))
    return [sorted(b) for b in bins]


def shard(hf: HostForest, rank: int, world: int) -> HostForest:
    """rank's whole-tree sub-forest (global init statistics kept)."""
    roots, tot, crit = tree_sizes(hf)
    parts = lpt_partition(tot, world, crit)
    return hf.subset_trees(roots[parts[rank]])


def global_init_stats(hf: HostForest, group=None, device=None) -> None:
    """Give this rank's forest the init statistics of the whole forest the ranks hold between them
    (init_cells_f / init_cells_r, moma_input.h:675-735: mean and E[v^2] - mean^2 of the first and
    last log_length / fp over every cell with more than one row), for ranks that generated or read
    only their own trees: one all_reduce of 9 sums.  The sums cross ranks in another order than one
    process adds them, so the statistics agree with the single-forest ones to the last bits, not
    bitwise."""
    import torch
    import torch.distributed as dist
    a = hf.a
    ro = np.asarray(a["row_offset"])
    sel = np.diff(ro) > 1
    first, last = ro[:-1][sel], ro[1:][sel] - 1
    cols = [a["log_length"][first], a["fp"][first], a["log_length"][last], a["fp"][last]]
    v = [float(sel.sum())] + [float(np.sum(c)) for c in cols] + [float(np.sum(c * c)) for c in cols]
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        backend = dist.get_backend(group)
        dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                 if backend == "nccl" else torch.device("cpu"))
        t = torch.tensor(v, dtype=torch.float64, device=dev)
        dist.all_reduce(t, group=group)
        v = [float(x) for x in t.cpu()]
    n = v[0]
    mean = [x / n for x in v[1:5]]
    var = [v[5 + k] / n - mean[k] * mean[k] for k in range(4)]
    a["root_mean_xg"] = np.array(mean[0:2])
    a["root_var_xg"] = np.array(var[0:2])
    a["leaf_mean_xg"] = np.array(mean[2:4])
    a["leaf_var_xg"] = np.array(var[2:4])


def combine_partials(partials, nan_flags, keys=None):
    """rank-order sum of the partials.  The first NaN: the rank whose first NaN comes first in the
    reference's order -- roots in input order, DFS pre-order within a tree, row (likelihood.h:71-93,
    125-159) -- by each rank's order key (NanOrder.key); without keys, the lowest
    rank that saw one.  Returns (total, first NaN rank or -1)."""
    bad = [r for r, flag in enumerate(nan_flags) if flag]
    if bad:
        if keys is None:
            return math.nan, bad[0]
        return math.nan, min(bad, key=lambda r: (tuple(float(k) for k in keys[r]), r))
    s = 0.0
    for v in partials:
        s = s + float(v)
    return s, -1


class NanOrder:
    """Where a rank's first NaN stands in the whole forest's reference order.

    The reference stops at the first row whose running total is NaN, walking the roots in input
    order, each tree in DFS pre-order (cell, daughter1's subtree, daughter2's subtree), each cell's
    rows in order (likelihood_recr, likelihood.h:110-122; sc_likelihood :71-93).  A rank holds
    whole trees of that forest, so its first NaN's place is the key (global position of its tree's
    root, DFS rank of the cell within the tree, row); the smallest key over the ranks is the
    reference's first NaN.  The global position of a root is its input-order cell index in the
    whole forest (HostForest.cells, kept by subset_trees); a shard without that mapping (each rank
    generated or read only its own trees, contiguous blocks in rank order) orders by rank first.
    key() returns four floats (exact integers below 2^53): the three key parts and the cell's index
    in the whole forest (its local index without the mapping), the cell the error reports."""

    def __init__(self, hf, rank: int = 0):
        self.rank = rank
        self.hf = hf
        self._root_pos = self._dfs = None

    def _build(self):
        a = self.hf.a
        d1, d2 = np.asarray(a["daughter1"]), np.asarray(a["daughter2"])
        n = len(d1)
        root_of = np.full(n, -1, np.int64)
        dfs = np.zeros(n, np.int64)
        for r in self.hf.roots:
            k, stack = 0, [int(r)]
            while stack:
                c = stack.pop()
                root_of[c], dfs[c] = r, k
                k += 1
                if d2[c] >= 0:
                    stack.append(int(d2[c]))
                if d1[c] >= 0:
                    stack.append(int(d1[c]))
        cells = self.hf.cells
        if cells is not None:
            pos = np.asarray(cells, np.int64)[root_of]
        else:
            pos = self.rank * (1 << 40) + root_of
        self._root_pos, self._dfs = pos, dfs

    def key(self, cell: int, row: int):
        if cell is None or cell < 0:          # no location (a peer's report, a stall): last in order
            return (math.inf, math.inf, math.inf, -1.0)
        if self.hf is None:
            return (float(self.rank * (1 << 40) + cell), 0.0, float(row), float(cell))
        if self._root_pos is None:
            self._build()
        gcell = cell if self.hf.cells is None else int(self.hf.cells[cell])
        return (float(self._root_pos[cell]), float(self._dfs[cell]), float(row), float(gcell))

    def error(self, owner: int, key, local_err):
        """the LikelihoodIsNan every rank raises: the whole forest's first NaN (cell, row), owned by
        rank `owner` (its cell id where this rank is the owner and knows it)"""
        mine = owner == self.rank and local_err is not None
        cid = getattr(local_err, "cell_id", None) if mine else None
        if mine and self.hf is not None and self.hf.ids and local_err.local_cell >= 0:
            cid = self.hf.ids[local_err.local_cell]
        e = LikelihoodIsNan(int(key[3]), int(key[2]), cid)
        e.rank = owner
        e.local_cell = getattr(local_err, "local_cell", -1) if local_err is not None else -1
        e.local_row = getattr(local_err, "local_row", -1) if local_err is not None else -1
        return e


class NodeExchange:
    """An all-gather of a few doubles per rank through host shared memory, for ranks on one node.

    Each call of the sharded objective exchanges 16 bytes per rank, values the ranks already hold
    on the host (the engine returns its partial through mapped memory).  Over RCCL that is two
    copies, a device collective and a stream synchronisation, ~36 us per call on the box
    (DESIGN.md §5); here each rank writes its values and a sequence number into its own 128-byte
    slot and polls the others' sequence numbers.  A slot holds two value sets used alternately: a
    rank can run one exchange ahead of a slower one (it has published its next values) but never
    two (it waits for every rank's number), so a set is never rewritten while being read.
    x86-64 only: its stores are not reordered with other stores, nor its loads with other loads,
    so the sequence number written after the values and read before them is a sufficient fence.
    The segment (a /dev/shm file mapped by every rank) is unlinked as soon as every rank has mapped
    it, so nothing is left behind whatever happens later.

    The constructor is collective (every rank of the group calls it, in the same order); on any
    failure every rank gets `ok == False` and the caller keeps torch's collective.
    """

    SLOT = 16   # float64 per rank: sequence number, two sets of up to 7 values

    def __init__(self, dist, group=None, width: int = 2, timeout_s: float | None = None):
        import mmap
        import torch
        assert 1 <= width <= (self.SLOT - 1) // 2
        self.width = width
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.timeout = float(os.environ.get("GGP_COMM_TIMEOUT_S", "600")) if timeout_s is None else timeout_s
        self.seq = 0
        self.mm = None
        self.a = None
        size = self.world * self.SLOT * 8
        backend = dist.get_backend(group)
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

        def agree(ok: bool) -> bool:
            f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MIN, group=group)
            return int(f.item()) == 1

        hosts = [None] * self.world
        dist.all_gather_object(hosts, (socket.gethostname(), platform.machine()), group=group)
        ok = len(set(hosts)) == 1 and hosts[0][1] in ("x86_64", "AMD64") and os.path.isdir("/dev/shm")
        name = [None]
        path = None
        if ok and self.rank == 0:
            path = f"/dev/shm/ggp_x_{os.getpid()}_{secrets.token_hex(6)}"
            try:
                self.mm = self._map(path, size, os.O_RDWR | os.O_CREAT | os.O_EXCL, mmap)
                name[0] = path
            except OSError:
                self.mm = None
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(name, src=src, group=group)
        ok = ok and name[0] is not None
        if ok and self.rank != 0:
            try:
                self.mm = self._map(name[0], size, os.O_RDWR, mmap)
            except OSError:
                self.mm = None
        self.ok = agree(ok and self.mm is not None)
        if path is not None and name[0] is not None:
            os.unlink(path)   # every rank has it mapped (or gave up): the name is no longer needed
        if not self.ok:
            self.close()
            return
        self.a = np.ndarray((self.world, self.SLOT), np.float64, buffer=self.mm)
        if self.rank == 0:
            self.a[:] = 0.0
        agree(True)   # the slots are zeroed before any rank publishes

    @staticmethod
    def _map(path, size, flags, mmap):
        fd = os.open(path, flags, 0o600)
        try:
            if flags & os.O_CREAT:
                os.ftruncate(fd, size)
            return mmap.mmap(fd, size)
        finally:
            os.close(fd)

    def exchange(self, vals) -> np.ndarray:
        """every rank's `width` values, [world, width], in rank order.  A waiting rank polls flat
        out for ~1 ms (an evaluation's skew between ranks), then yields its core between polls
        (sched_yield, then 50 us sleeps after ~0.1 s), so a rank waiting on a slower one's host work
        neither burns a core nor holds the GIL.  After a timeout the exchange is unusable: the
        ranks' sequence numbers are out of step, so every later call raises at once."""
        if self.a is None:
            raise RuntimeError("NodeExchange: unusable (closed, or a peer timed out earlier)")
        s = self.seq + 1
        lo = 1 + (s & 1) * self.width
        hi = lo + self.width
        mine = self.a[self.rank]
        mine[lo:hi] = vals
        mine[0] = s                     # published after the values
        a, deadline, t_wait = self.a, None, None
        for r in range(self.world):
            n = 0
            while a[r, 0] < s:
                n += 1
                if (n & 0xFFF) == 0:
                    now = time.monotonic()
                    if deadline is None:
                        deadline, t_wait = now + self.timeout, now
                    if now > deadline:
                        self.a = None
                        raise TimeoutError(f"NodeExchange: rank {r} did not publish call {s} in {self.timeout} s")
                    if now - t_wait > 0.1:
                        time.sleep(50e-6)
                    elif now - t_wait > 1e-3:
                        time.sleep(0)
        out = a[:, lo:hi].copy()        # read after the sequence numbers
        self.seq = s
        return out

    def close(self) -> None:
        self.a = None
        if self.mm is not None:
            try:
                self.mm.close()
            except BufferError:
                pass
            self.mm = None


class ShardedObjective:
    """total_likelihood over a forest sharded across the ranks of a process group.

    device_forest: this rank's Forest (or any object with .total_likelihood(params)).
    host_forest: this rank's HostForest, where device_forest does not carry it as .host (the first
    NaN's place in the whole forest, NanOrder).
    """

    # per rank and call: the partial, the NaN flag, and the first NaN's order key (NanOrder)
    WIDTH = 6

    def __init__(self, device_forest, group=None, device=None, always_gather: bool = False,
                 engine_comm: bool | None = None, node_exchange: bool | None = None, host_forest=None):
        import torch
        import torch.distributed as dist
        self.f = device_forest
        self.dist = dist
        self.torch = torch
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.always_gather = always_gather          # tests: the collective path at world size 1
        # this rank's trees (the first NaN's place in the whole forest): the Forest's own by default
        self.order = NanOrder(host_forest if host_forest is not None else getattr(device_forest, "host", None),
                              dist.get_rank(group) if dist.is_initialized() else 0)
        backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        # RCCL inside the engine (include/ggp.h ggp_comm_attach): the all-gather is enqueued on the
        # engine's stream behind the evaluation, no host round trip in between.  Opt-in
        # (engine_comm=True or GGP_ENGINE_COMM=1) for nccl groups whose per-rank objective is a HIP
        # Forest: it has run on a 1-rank group only (no multi-GPU box to the builder yet), so the
        # default is torch's all_gather path until a multi-rank run has passed
        if engine_comm is None:
            engine_comm = os.environ.get("GGP_ENGINE_COMM", "0") == "1"
        self.engine = False
        if (engine_comm and backend == "nccl" and (self.world > 1 or always_gather)
                and isinstance(device_forest, Forest)):
            self._attach_engine(torch, dist, group)
        self.dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                      if backend == "nccl" else torch.device("cpu"))
        # ranks on one node: the partials' exchange through host shared memory (GGP_NODE_EXCHANGE=0:
        # torch's collective)
        self.xchg = None
        if node_exchange is None:
            node_exchange = os.environ.get("GGP_NODE_EXCHANGE", "1") != "0"
        if not self.engine and (self.world > 1 or always_gather) and node_exchange:
            x = NodeExchange(dist, group, width=self.WIDTH)
            self.xchg = x if x.ok else None
        self._send = torch.zeros(self.WIDTH, dtype=torch.float64, device=self.dev)
        self._recv = torch.zeros(self.WIDTH * self.world, dtype=torch.float64, device=self.dev)
        # per call, RCCL moves 16 B per rank: stage them through pinned host tensors (one async
        # copy each way, numpy views for the element writes) instead of two element-fill
        # launches and a blocking .cpu()
        self._cuda = self.dev.type == "cuda"
        pin = self._cuda
        self._h_send = torch.zeros(self.WIDTH, dtype=torch.float64, pin_memory=pin)
        self._h_recv = torch.zeros(self.WIDTH * self.world, dtype=torch.float64, pin_memory=pin)
        self._h_send_np = self._h_send.numpy()
        self._h_recv_np = self._h_recv.numpy()

    def _attach_engine(self, torch, dist, group):
        """join the engine's RCCL communicator; every rank first checks it can (the library and
        its entry points) and the group agrees, so a rank that cannot never leaves the others
        waiting in ncclCommInitRank: then all keep torch's all_gather path"""
        import sys
        from .forest import GGPError, comm_unique_id
        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        lib = lib if os.path.exists(lib) else None      # the RCCL torch loaded: one RCCL per process
        rank = dist.get_rank(group)
        src = 0 if group is None else dist.get_global_rank(group, 0)
        try:   # rank 0 makes the id, the others only check the library (one bootstrap root)
            if len(self.f.shards()) != 1:   # ggp_comm_attach needs one shard (one device) per rank
                raise GGPError(f"{len(self.f.shards())} shards on this rank")
            mine = comm_unique_id(lib) if rank == 0 else (comm_unique_id(lib, probe=True) or bytes(128))
            ok = 1
        except GGPError as e:
            print(f"ShardedObjective: engine RCCL unavailable on rank {rank} ({e}); torch's all_gather instead",
                  file=sys.stderr)
            mine, ok = bytes(128), 0
        flag = torch.tensor([ok], dtype=torch.int32, device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if int(flag.item()) == 0:
            return
        uid = torch.frombuffer(bytearray(mine), dtype=torch.uint8).to("cuda")
        dist.broadcast(uid, src=src, group=group)
        self.f.comm_attach(self.world, rank, bytes(uid.cpu().numpy().tobytes()), lib)
        self.engine = True

    def local(self, params):
        try:
            return self.f.total_likelihood(params), False, None
        except LikelihoodIsNan as e:
            return math.nan, True, e

    def _allgather(self, vec) -> np.ndarray:
        """every rank's float64 vector (the same length on every rank), [world, len], through torch's
        collective (the NaN resolution and the chained partials: once per chain or per failure)"""
        torch = self.torch
        v = np.ascontiguousarray(vec, np.float64)
        send = torch.from_numpy(v.copy()).to(self.dev)
        recv = torch.zeros(len(v) * self.world, dtype=torch.float64, device=self.dev)
        self.dist.all_gather_into_tensor(recv, send, group=self.group)
        return recv.cpu().numpy().reshape(self.world, len(v))

    def _key(self, err):
        if err is None:
            return (math.inf, math.inf, math.inf, -1.0)
        return self.order.key(getattr(err, "local_cell", err.cell), getattr(err, "local_row", err.row))

    def _engine_nan(self, err):
        """the engine's collective reported a NaN on every rank: one exchange of each rank's own
        first NaN (its order key) names the whole forest's first one, the same on every rank"""
        own = err if getattr(err, "local_cell", -1) is not None and getattr(err, "local_cell", -1) >= 0 else None
        got = self._allgather((1.0 if own is not None else 0.0,) + self._key(own))
        _, owner = combine_partials(np.zeros(self.world), got[:, 0] != 0, got[:, 1:4])
        if owner < 0:   # no rank located it (cannot happen with a NaN on some rank): the engine's report
            return err
        e = self.order.error(owner, got[owner, 1:5], own)
        for k in ("point", "ll"):
            if hasattr(err, k):
                setattr(e, k, getattr(err, k))
        return e

    def total_likelihood_chain(self, points):
        """a known sequence of objective calls, each from the state the previous left (the -s scan,
        the Hessian points; ggp_total_loglik_chain): every rank chains its own shard -- the carried
        state is per tree, so the points need no exchange between them -- and ONE all_gather of the
        per-point partials follows; the totals are the rank-order sums, as total_likelihood's.
        A NaN raises, on every rank, what the one-process chain raises: LikelihoodIsNan at the
        first point any rank failed (.point, .ll = the totals before it), located at the whole
        forest's first NaN of that point (NanOrder).  With the engine's collective every chained
        call already returns the total over the ranks (ggp_comm_attach), so its results are the
        totals as they are."""
        pts = np.ascontiguousarray(np.atleast_2d(points), np.float64)
        n = pts.shape[0]
        if self.engine:
            try:
                return np.asarray(self.f.total_likelihood_chain(pts), np.float64)
            except LikelihoodIsNan as e:
                raise self._engine_nan(e) from None
        err = None
        try:
            local = np.asarray(self.f.total_likelihood_chain(pts), np.float64)
        except LikelihoodIsNan as e:
            if self.world == 1 and not self.always_gather:
                raise
            err = e
            local = np.asarray(getattr(e, "ll", []), np.float64)
        fail = len(local) if err is not None else n   # this rank's first failing point (n: none)
        if len(local) < n:
            local = np.concatenate([local, np.full(n - len(local), math.nan)])
        if self.world == 1 and not self.always_gather:
            return local
        got = self._allgather(np.concatenate([local, [float(fail)], self._key(err)]))
        out = np.empty(n)
        for k in range(n):
            s = 0.0
            for r in range(self.world):
                s = s + float(got[r, k])
            out[k] = s
        p = int(got[:, n].min())
        if p < n:
            _, owner = combine_partials(np.zeros(self.world), got[:, n] == p, got[:, n + 1:n + 4])
            e = self.order.error(owner, got[owner, n + 1:n + 5], err if err is not None and fail == p else None)
            e.point, e.ll = p, out[:p].copy()
            raise e
        return out

    @property
    def exchange_kind(self) -> str:
        if self.engine:
            return "engine RCCL (ggp_comm_attach): partial, ncclAllGather, rank-order sum on the engine's stream"
        if self.xchg is not None:
            return "host shared memory (NodeExchange): 48 B per rank, rank-order sum"
        return "torch all_gather_into_tensor of 48 B per rank, rank-order sum"

    def close(self) -> None:
        if self.xchg is not None:
            self.xchg.close()
            self.xchg = None

    def total_likelihood(self, params) -> float:
        if self.engine:   # the engine returns the rank-order sum (or a NaN on every rank)
            try:
                return self.f.total_likelihood(params)
            except LikelihoodIsNan as e:
                raise self._engine_nan(e) from None
        v, isnan, err = self.local(params)
        if self.world == 1 and not self.always_gather:
            if isnan:
                raise err
            return v
        mine = (v, 1.0 if isnan else 0.0) + self._key(err)
        if self.xchg is not None:
            got = self.xchg.exchange(mine)
        else:
            self._h_send_np[:] = mine
            if self._cuda:
                self._send.copy_(self._h_send, non_blocking=True)
                self.dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
                self._h_recv.copy_(self._recv, non_blocking=True)
                self.torch.cuda.current_stream(self.dev).synchronize()
            else:
                self.dist.all_gather_into_tensor(self._h_recv, self._h_send, group=self.group)
            got = self._h_recv_np.reshape(self.world, self.WIDTH)
        total, nan_rank = combine_partials(got[:, 0], got[:, 1] != 0, got[:, 2:5])
        if nan_rank >= 0:
            raise self.order.error(nan_rank, got[nan_rank, 2:6], err)
        return total


def shard_rows(hf: HostForest, rank: int, world: int):
    """rank's whole-tree sub-forest and the input-order index of each of its rows"""
    sub = shard(hf, rank, world)
    return sub, sub.rows


class ShardedPredictor:
    """-p over a forest sharded by whole trees.

    prediction_forward / prediction_backward / combine_predictions (predictions.h:166-173,
    438-444, 466-499) run cell by cell, parent to daughter and back; no term crosses a tree.
    So every rank runs the smoother over its own trees on its own GPU (no collective on the
    data path) and predict() returns this rank's rows; gather() assembles [n_rows, 20] in
    input order on rank `dst` with one gather of per-rank blocks (padded to the largest).

    predictor: this rank's Forest (or any object with .predict(params_per_segment)).
    rows: input-order index of each local row (HostForest.rows of the shard).
    """

    def __init__(self, predictor, rows, n_rows: int, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.p = predictor
        self.rows = np.asarray(rows, np.int64)
        self.n_rows = int(n_rows)
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        self.dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                      if backend == "nccl" else torch.device("cpu"))

    def predict(self, params_per_segment):
        """this rank's (forward, backward, combined) rows, [len(rows), 20] each"""
        return self.p.predict(params_per_segment)

    def gather(self, local, dst: int = 0):
        """assemble one [len(rows), 20] block per rank into input order on rank dst (None elsewhere)"""
        import torch
        local = np.asarray(local, np.float64)
        if self.world == 1:
            out = np.empty((self.n_rows, local.shape[1]))
            out[self.rows] = local
            return out
        n = torch.tensor([len(self.rows)], dtype=torch.int64, device=self.dev)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(sizes, n, group=self.group)
        sizes = [int(x.item()) for x in sizes]
        mx = max(sizes)
        buf = torch.zeros((mx, 1 + local.shape[1]), dtype=torch.float64, device=self.dev)
        buf[: len(self.rows), 0] = torch.from_numpy(self.rows.astype(np.float64))   # exact below 2**53
        buf[: len(self.rows), 1:] = torch.from_numpy(local)
        rank = self.dist.get_rank(self.group)
        parts = [torch.empty_like(buf) for _ in range(self.world)] if rank == dst else None
        self.dist.gather(buf, parts, dst=dst, group=self.group)
        if rank != dst:
            return None
        out = np.empty((self.n_rows, local.shape[1]))
        for k, part in zip(sizes, parts):
            a = part[:k].cpu().numpy()
            out[a[:, 0].astype(np.int64)] = a[:, 1:]
        return out
