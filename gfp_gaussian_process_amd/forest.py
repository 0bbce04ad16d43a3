"""Host-side mirror of the reference's data model and objective entry points.

Reference interface (C++), and what mirrors it here:

  CSVconfig(filename)                      CSVConfig.load             CSVconfig.h:26-98
  Parameter_set(filename)                  ParameterSet.load          Parameters.h:133-176
  read_data(file, config, noise, div)      Dataset.read               moma_input.h:401-527
  get_segment_indices(cells)               Dataset.segment_indices    moma_input.h:538-570
  get_segment + build_cell_genealogy       HostForest.build           moma_input.h:580-620,125-151
    + init_cells                                                      moma_input.h:738-741
  std::vector<MOMAdata> (on the device)    Forest                     moma_input.h:22-80
  total_likelihood(params, cells) -> +ll   total_likelihood           likelihood.h:170-174
  total_likelihood(x, grad, data) -> -ll   total_likelihood_nlopt     likelihood.h:125-159
  total_likelihood_log_params              total_likelihood_log_params likelihood.h:161-167

Every likelihood evaluation runs in the HIP engine (lib/libggp.so).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field

import numpy as np

from . import _native as N

NOISE_MODELS = {"scaled": 1, "const": 0}
DIVISION_MODELS = {"binomial": 1, "gauss": 0}
PARAM_NAMES = ["mean_lambda", "gamma_lambda", "var_lambda", "mean_q", "gamma_q", "var_q",
               "beta", "var_x", "var_g", "var_dx", "var_dg"]


class GGPError(RuntimeError):
    pass


class LikelihoodIsNan(GGPError):
    """std::domain_error("Likelihood is Nan") of likelihood.h:71-93."""

    def __init__(self, cell: int, row: int, cell_id: str | None = None):
        self.cell, self.row, self.cell_id = cell, row, cell_id
        # this process's own first NaN (its handle's cell index and row; -1 if its own evaluation
        # was clean): what distributed.ShardedObjective exchanges to find the reference's first NaN
        self.local_cell, self.local_row = cell, row
        super().__init__(f"Likelihood is Nan (cell {cell_id or cell}, row {row})")


class EvaluationStalled(GGPError):
    """GGP_ETIMEOUT: a wait inside one evaluation timed out (a daughter cell's wait for its parent,
    or a peer rank's collective) -- a scheduling failure, never reported as LikelihoodIsNan.  The
    carried state is unspecified afterwards, as after a NaN."""


def _host_err() -> str:
    return (N.host().ggp_host_last_error() or b"").decode()


# ------------------------------------------------------------------------------------------
class CSVConfig:
    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load(cls, path: str | None = None) -> "CSVConfig":
        h = ctypes.c_void_p()
        rc = N.host().ggp_csv_config_load(path.encode() if path else None, ctypes.byref(h))
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        return cls(h)

    def get(self, key: str) -> str:
        buf = ctypes.create_string_buffer(4096)
        if N.host().ggp_csv_config_get(self._h, key.encode(), buf, 4096) != N.GGP_OK:
            raise KeyError(key)
        return buf.value.decode()

    def __del__(self):
        if getattr(self, "_h", None):
            N.host().ggp_csv_config_free(self._h)
            self._h = None


@dataclass
class ParameterSet:
    names: list = field(default_factory=lambda: list(PARAM_NAMES))
    kind: list = field(default_factory=list)      # "fixed" | "free" | "bound"
    init: np.ndarray = None
    step: np.ndarray = None
    lower: np.ndarray = None
    upper: np.ndarray = None

    @classmethod
    def load(cls, path: str, check_complete: bool = True) -> "ParameterSet":
        ps = N.ParamSetC()
        rc = N.host().ggp_param_file_load(path.encode(), 1 if check_complete else 0, ctypes.byref(ps))
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        kinds = {0: "fixed", 1: "free", 2: "bound"}
        return cls(kind=[kinds[ps.kind[i]] for i in range(N.N_PARAMS)],
                   init=np.array(ps.init[:]), step=np.array(ps.step[:]),
                   lower=np.array(ps.lower[:]), upper=np.array(ps.upper[:]))

    def get_init(self) -> np.ndarray:
        return self.init.copy()

    def non_fixed(self) -> list:
        return [i for i, k in enumerate(self.kind) if k != "fixed"]

    def bound(self) -> list:
        return [i for i, k in enumerate(self.kind) if k == "bound"]


class Dataset:
    """read_data output: cells in input order (moma_input.h:401-527)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def read(cls, infile: str, config: CSVConfig | None = None) -> "Dataset":
        if N.host().ggp_dataset_is_binary(infile.encode()):
            return cls.load(infile)
        h = ctypes.c_void_p()
        rc = N.host().ggp_dataset_read(infile.encode(), config._h if config else None, ctypes.byref(h))
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        return cls(h)

    @classmethod
    def load(cls, path: str) -> "Dataset":
        """a binary dataset written by save() (ggp_dataset_load, "GGPD0001")"""
        h = ctypes.c_void_p()
        if N.host().ggp_dataset_load(path.encode(), ctypes.byref(h)) != N.GGP_OK:
            raise GGPError(_host_err())
        return cls(h)

    @classmethod
    def from_forest(cls, hf: "HostForest") -> "Dataset":
        """the dataset a flattened forest came from (cells, ids, rows; ggp_dataset_create) --
        e.g. a synthetic forest to save() for the CLI"""
        if hf.ids is None or hf.parent_ids is None:
            raise ValueError("the forest needs cell and parent ids (synthetic(..., with_ids=True))")
        a = hf.a
        n = hf.n_cells
        ids = (ctypes.c_char_p * max(1, n))(*[s.encode() for s in hf.ids])
        pids = (ctypes.c_char_p * max(1, n))(*[s.encode() for s in hf.parent_ids])
        arr = {k: np.ascontiguousarray(a[k]) for k in ("row_offset", "time", "log_length", "fp", "segment")}
        h = ctypes.c_void_p()
        rc = N.host().ggp_dataset_create(n, arr["row_offset"].ctypes.data_as(N.c_int64_p),
                                         arr["time"].ctypes.data_as(N.c_double_p),
                                         arr["log_length"].ctypes.data_as(N.c_double_p),
                                         arr["fp"].ctypes.data_as(N.c_double_p),
                                         arr["segment"].astype(np.int32).ctypes.data_as(N.c_int32_p),
                                         ids, pids, float(a["fp_auto"]), ctypes.byref(h))
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        return cls(h)

    def write_csv(self, csv_path: str, config_path: str) -> None:
        """the reference's input CSV (example column layout, %.17g) and the csv_config that reads
        it back bit for bit (ggp_dataset_write_csv): a synthetic forest the reference can read"""
        if N.host().ggp_dataset_write_csv(self._h, csv_path.encode(), config_path.encode()) != N.GGP_OK:
            raise GGPError(_host_err())

    def save(self, path: str) -> None:
        """binary dataset ("GGPD0001", ggp_dataset_save): the CLI's -i reads it directly"""
        if N.host().ggp_dataset_save(self._h, path.encode()) != N.GGP_OK:
            raise GGPError(_host_err())

    @property
    def n_cells(self) -> int:
        return int(N.host().ggp_dataset_n_cells(self._h))

    @property
    def n_rows(self) -> int:
        return int(N.host().ggp_dataset_n_rows(self._h))

    def segment_indices(self) -> list:
        n = ctypes.c_int32()
        rc = N.host().ggp_dataset_segments(self._h, None, 0, ctypes.byref(n))   # the count first
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        buf = (ctypes.c_int32 * max(1, n.value))()
        rc = N.host().ggp_dataset_segments(self._h, buf, n.value, ctypes.byref(n))
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        return list(buf[: n.value])

    def __del__(self):
        if getattr(self, "_h", None):
            N.host().ggp_dataset_free(self._h)
            self._h = None


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


class HostForest:
    """A flattened forest: the reference's std::vector<MOMAdata> after genealogy + init_cells,
    as structure-of-arrays (cells in input order, rows cell-major)."""

    def __init__(self, arrays: dict, ids=None, parent_ids=None, rows=None, cells=None):
        self.a = arrays
        self.ids = ids
        self.parent_ids = parent_ids
        self.rows = rows          # subset_trees: each row's index in the full forest
        self.cells = cells        # subset_trees: each cell's index in the full forest (input order)

    # -- constructors --
    @classmethod
    def _from_handle(cls, h, with_ids=True) -> "HostForest":
        H = N.host()
        d = N.ForestDesc()
        H.ggp_host_forest_desc(h, ctypes.byref(d))
        nc, nr = int(d.n_cells), int(d.n_rows)
        a = dict(
            row_offset=_arr(d.row_offset, nc + 1, np.int64), parent=_arr(d.parent, nc, np.int32),
            daughter1=_arr(d.daughter1, nc, np.int32), daughter2=_arr(d.daughter2, nc, np.int32),
            segment=_arr(d.segment, nr, np.int32), time=_arr(d.time, nr, np.float64),
            log_length=_arr(d.log_length, nr, np.float64), fp=_arr(d.fp, nr, np.float64),
            root_mean_xg=np.array(d.root_mean_xg[:]), root_var_xg=np.array(d.root_var_xg[:]),
            leaf_mean_xg=np.array(d.leaf_mean_xg[:]), leaf_var_xg=np.array(d.leaf_var_xg[:]),
            noise_scaled=int(d.noise_scaled), division_binomial=int(d.division_binomial),
            fp_auto=float(d.fp_auto))
        ids = pids = None
        if with_ids:
            ids = [H.ggp_host_forest_cell_id(h, i).decode() for i in range(nc)]
            pids = [H.ggp_host_forest_parent_id(h, i).decode() for i in range(nc)]
        H.ggp_host_forest_free(h)
        return cls(a, ids, pids)

    @classmethod
    def build(cls, dataset: Dataset, segment: int = -1, noise_model: str = "scaled",
              cell_division_model: str = "binomial") -> "HostForest":
        h = ctypes.c_void_p()
        rc = N.host().ggp_forest_build(dataset._h, segment, NOISE_MODELS[noise_model],
                                       DIVISION_MODELS[cell_division_model], ctypes.byref(h))
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        return cls._from_handle(h)

    @classmethod
    def from_csv(cls, infile: str, csv_config: str | None = None, segment: int = -1,
                 noise_model: str = "scaled", cell_division_model: str = "binomial") -> "HostForest":
        ds = Dataset.read(infile, CSVConfig.load(csv_config))
        return cls.build(ds, segment, noise_model, cell_division_model)

    @classmethod
    def synthetic(cls, n_trees: int, rows_per_tree: int = 200, seed: int = 20261015, first_tree: int = 0,
                  noise_model: str = "scaled", cell_division_model: str = "binomial",
                  with_ids: bool = False) -> "HostForest":
        h = ctypes.c_void_p()
        rc = N.host().ggp_synthetic_forest(n_trees, rows_per_tree, seed, first_tree,
                                           NOISE_MODELS[noise_model], DIVISION_MODELS[cell_division_model],
                                           ctypes.byref(h))
        if rc != N.GGP_OK:
            raise GGPError(_host_err())
        return cls._from_handle(h, with_ids=with_ids)

    # -- binary SoA in/out (forests far beyond CSV scale) --
    _SCALARS = ("noise_scaled", "division_binomial", "fp_auto")

    def save(self, path: str) -> None:
        """the flattened forest as one .npz (SoA arrays as stored, ids as fixed-width text)"""
        out = {k: np.asarray(v) for k, v in self.a.items()}
        if self.ids is not None:
            out["_ids"] = np.array(self.ids, dtype=np.str_)
            out["_parent_ids"] = np.array(self.parent_ids, dtype=np.str_)
        if self.rows is not None:
            out["_rows"] = np.asarray(self.rows, np.int64)
        if self.cells is not None:
            out["_cells"] = np.asarray(self.cells, np.int64)
        np.savez(path, **out)

    @classmethod
    def load(cls, path: str) -> "HostForest":
        """read a forest written by save() (numpy's loader with allow_pickle=False)"""
        with np.load(path, allow_pickle=False) as z:
            a = {k: z[k] for k in z.files if not k.startswith("_")}
            for k in cls._SCALARS:
                a[k] = a[k].item()
            ids = [str(x) for x in z["_ids"]] if "_ids" in z.files else None
            pids = [str(x) for x in z["_parent_ids"]] if "_parent_ids" in z.files else None
            rows = z["_rows"] if "_rows" in z.files else None
            cells = z["_cells"] if "_cells" in z.files else None
        return cls(a, ids, pids, rows, cells)

    # -- properties --
    @property
    def n_cells(self) -> int:
        return len(self.a["parent"])

    @property
    def n_rows(self) -> int:
        return len(self.a["time"])

    @property
    def roots(self) -> np.ndarray:
        return np.nonzero(self.a["parent"] == -1)[0]

    def tree_of_cell(self) -> np.ndarray:
        """root index of every cell"""
        p = self.a["parent"]
        tree = np.full(self.n_cells, -1, np.int64)
        for c in range(self.n_cells):
            r = c
            while p[r] != -1:
                r = p[r]
            tree[c] = r
        return tree

    def subset_trees(self, roots) -> "HostForest":
        """The sub-forest made of whole trees `roots` (cells keep input order); root/leaf
        statistics stay those of the full forest, as one MOMAdata vector would have them."""
        tree = self.tree_of_cell()
        keep = np.isin(tree, np.asarray(roots))
        idx = np.nonzero(keep)[0]
        remap = np.full(self.n_cells, -1, np.int64)
        remap[idx] = np.arange(len(idx))
        ro = self.a["row_offset"]
        rows = np.concatenate([np.arange(ro[c], ro[c + 1]) for c in idx]) if len(idx) else np.zeros(0, np.int64)
        lens = (ro[idx + 1] - ro[idx]).astype(np.int64)
        a = dict(self.a)
        a["row_offset"] = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)

        def rm(v):
            v = v[idx]
            return np.where(v >= 0, remap[np.maximum(v, 0)], -1).astype(np.int32)
        a["parent"], a["daughter1"], a["daughter2"] = rm(self.a["parent"]), rm(self.a["daughter1"]), rm(self.a["daughter2"])
        for k in ("segment", "time", "log_length", "fp"):
            a[k] = self.a[k][rows]
        ids = [self.ids[i] for i in idx] if self.ids else None
        pids = [self.parent_ids[i] for i in idx] if self.parent_ids else None
        grows = np.asarray(rows, np.int64) if self.rows is None else np.asarray(self.rows, np.int64)[rows]
        gcells = idx.astype(np.int64) if self.cells is None else np.asarray(self.cells, np.int64)[idx]
        return HostForest(a, ids, pids, rows=grows, cells=gcells)

    def desc(self, devices=(0,), kernel: str = "auto", max_shard_rows: int = 0) -> N.ForestDesc:
        """ggp_forest_desc; devices: HIP ordinals to shard over (repeats = logical shards on one
        device), None = every visible device"""
        a = self.a
        d = N.ForestDesc()
        d.n_cells, d.n_rows = self.n_cells, self.n_rows

        def ptr(name, ctype):
            arr = np.ascontiguousarray(a[name])
            a[name] = arr
            return arr.ctypes.data_as(ctypes.POINTER(ctype))
        d.row_offset = ptr("row_offset", ctypes.c_int64)
        d.parent = ptr("parent", ctypes.c_int32)
        d.daughter1 = ptr("daughter1", ctypes.c_int32)
        d.daughter2 = ptr("daughter2", ctypes.c_int32)
        d.segment = ptr("segment", ctypes.c_int32)
        d.time = ptr("time", ctypes.c_double)
        d.log_length = ptr("log_length", ctypes.c_double)
        d.fp = ptr("fp", ctypes.c_double)
        d.root_mean_xg[:] = list(a["root_mean_xg"])
        d.root_var_xg[:] = list(a["root_var_xg"])
        d.leaf_mean_xg[:] = list(a["leaf_mean_xg"])
        d.leaf_var_xg[:] = list(a["leaf_var_xg"])
        d.noise_scaled = a["noise_scaled"]
        d.division_binomial = a["division_binomial"]
        d.fp_auto = a["fp_auto"]
        if devices is None:
            d.n_devices, d.devices = N.GGP_ALL_DEVICES, None
        else:
            dv = np.ascontiguousarray(devices, np.int32)
            if dv.ndim != 1 or dv.size == 0:
                raise ValueError("devices: a non-empty list of HIP ordinals (or None for all)")
            self._devices = dv                      # keeps the array alive with the descriptor
            d.n_devices, d.devices = dv.size, dv.ctypes.data_as(N.c_int32_p)
        d.max_shard_rows = int(max_shard_rows)
        d.kernel = N.KERNELS[kernel]
        return d


# ------------------------------------------------------------------------------------------
def kernel_name(code: int) -> str:
    """the HIP kernel symbol behind a launch-profile code (include/ggp.h)"""
    kind, lanes = code >> 8, code & 0xFF
    if kind == N.KERNELS["lane"]:
        return "k_loglik_lane_queue" if lanes == 2 else "k_loglik_level"
    if kind == N.KERNELS["wave"]:
        return "k_loglik_wave"
    if kind == N.KERNELS["pair"]:
        return f"k_loglik_pair<{lanes}>"
    return f"k_loglik_group<{lanes}>"


def comm_unique_id(rccl_lib: str | None = None, probe: bool = False) -> bytes | None:
    """the 128-byte RCCL unique id (ncclGetUniqueId) rank 0 makes for Forest.comm_attach;
    probe=True only checks that the RCCL library and its entry points load (None)"""
    buf = None if probe else ctypes.create_string_buffer(128)
    lib = N.engine()
    rc = lib.ggp_comm_unique_id(rccl_lib.encode() if rccl_lib else None, buf)
    if rc != N.GGP_OK:
        raise GGPError(lib.ggp_strerror(rc).decode())
    return None if probe else buf.raw


class Forest:
    """Device-resident forest + carried state.  Owns a ggp_forest handle.

    device: one HIP ordinal; devices: a list of ordinals the forest is sharded over (whole
    trees, include/ggp.h "Sharding"; repeats = logical shards on one device; None = every
    visible device).  Results have the same bits for any device list."""

    def __init__(self, host_forest: HostForest, device: int = 0, kernel: str = "auto", devices=(),
                 max_shard_rows: int = 0, exact: bool = False):
        self.host = host_forest
        # exact=True: the engine built in the oracle's arithmetic (lib/libggp_exact.so, GGP_EXACT:
        # glibc's exp, every exponential from its own argument, no fma contraction, the combine's
        # IEEE inverses; no wave schedule), the reference's roundings step for step
        self._lib = N.engine(N.EXACT_ENGINE if exact else None)
        self.exact = bool(exact) or N.engine_name() == N.EXACT_ENGINE
        self._poisoned = False
        d = host_forest.desc([device] if devices == () else devices, kernel, max_shard_rows)
        h = ctypes.c_void_p()
        rc = self._lib.ggp_forest_create(ctypes.byref(d), ctypes.byref(h))
        if rc != N.GGP_OK:
            raise GGPError(self._lib.ggp_strerror(rc).decode())
        self._h = h
        self.n_rows = host_forest.n_rows
        self.n_cells = host_forest.n_cells
        # the per-call argument objects, made once (an evaluation is ~0.3 ms: ~5 us of ctypes
        # object creation per call showed up in the C2 rate)
        # the call's parameters: a ctypes array (a slice assignment from a list costs half a
        # numpy array's) and its pointer, made once
        self._p = (ctypes.c_double * N.N_PARAMS)()
        self._p_ptr = ctypes.cast(self._p, N.c_double_p)
        self._ll, self._nc, self._nr = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        self._out_refs = (ctypes.byref(self._ll), ctypes.byref(self._nc), ctypes.byref(self._nr))

    def _check(self, rc):
        if rc != N.GGP_OK:
            raise GGPError(self._lib.ggp_strerror(rc).decode())

    def _nan(self, nc: int, nr: int):
        # after a NaN the carried state is unspecified (include/ggp.h "Errors"): the next
        # evaluation needs reset_state() or set_state() first.  With the engine's collective, a
        # rank whose own evaluation was bad is marked even when a lower rank had the first NaN.
        if getattr(self, "_comm_rank", None) is not None:
            r = self._lib.ggp_comm_nan_rank(self._h)
            if self._lib.ggp_comm_local_nan(self._h):
                self._poisoned = True
            if r >= 0 and r != self._comm_rank:
                e = LikelihoodIsNan(-1, -1, f"rank {r}")
                e.local_cell, e.local_row = nc, nr
                return e
        self._poisoned = True
        cid = self.host.ids[nc] if (self.host.ids and nc >= 0) else None
        return LikelihoodIsNan(nc, nr, cid)

    def _usable(self):
        if self._poisoned:
            raise GGPError("carried state is unspecified after a NaN evaluation: call reset_state() or set_state()")

    def total_likelihood(self, params) -> float:
        try:
            self._p[:] = params   # (ctypes: ValueError unless exactly N_PARAMS values)
        except (TypeError, ValueError):
            raise ValueError("params must hold 11 values (Parameters.h:175 order)") from None
        self._usable()
        rc = self._lib.ggp_total_loglik(self._h, self._p_ptr, *self._out_refs)
        if rc == N.GGP_ENAN:
            raise self._nan(self._nc.value, self._nr.value)
        self._stalled(rc)
        self._check(rc)
        return self._ll.value

    def _stalled(self, rc):
        if rc == N.GGP_ETIMEOUT:
            if getattr(self, "_comm_rank", None) is None or self._lib.ggp_comm_local_nan(self._h):
                self._poisoned = True
            raise EvaluationStalled(self._lib.ggp_strerror(rc).decode())

    # -- one process per GPU: the engine's own RCCL collective (include/ggp.h ggp_comm_attach) --
    def comm_attach(self, nranks: int, rank: int, uid: bytes, rccl_lib: str | None = None) -> None:
        """join a group of one-GPU processes: every later total_likelihood returns the total over
        all ranks (this forest is this rank's whole-tree shard); `uid` from comm_unique_id() on
        rank 0.  Every rank of the group must call it."""
        if len(uid) != 128:
            raise ValueError("uid must be the 128-byte id of comm_unique_id()")
        self._check(self._lib.ggp_comm_attach(self._h, rccl_lib.encode() if rccl_lib else None, int(nranks),
                                              int(rank), bytes(uid)))
        self._comm_rank = int(rank)

    def launch_clock(self):
        """(shader MHz, window us) of the last path launch's block 0 (ggp_launch_clock), or None"""
        mhz, us = ctypes.c_double(), ctypes.c_double()
        if self._lib.ggp_launch_clock(self._h, ctypes.byref(mhz), ctypes.byref(us)) != N.GGP_OK:
            return None
        return mhz.value, us.value

    def call_trace(self, last: int = 512) -> np.ndarray:
        """the host split of the last `last` objective calls (ggp_call_trace), oldest first: [k, 6] =
        (enqueue_us, wait_us, result_us, kernel_us, shader_mhz, call index)"""
        out = np.zeros((max(1, last), 6))
        n = ctypes.c_int32()
        self._check(self._lib.ggp_call_trace(self._h, int(last), out.ctypes.data_as(N.c_double_p), ctypes.byref(n)))
        return out[: n.value]

    def comm_size(self) -> int:
        """ranks of the attached RCCL communicator as RCCL counts them (ncclCommCount); 0 if the handle
        is not attached"""
        return int(self._lib.ggp_comm_size(self._h))

    def submit(self, params) -> None:
        """enqueue one evaluation (ggp_total_loglik_async)"""
        self._usable()
        self._pending = np.ascontiguousarray(params, np.float64)
        self._check(self._lib.ggp_total_loglik_async(self._h, self._pending.ctypes.data_as(N.c_double_p)))

    def result(self) -> float:
        ll = ctypes.c_double()
        nc, nr = ctypes.c_int64(), ctypes.c_int64()
        rc = self._lib.ggp_loglik_result(self._h, ctypes.byref(ll), ctypes.byref(nc), ctypes.byref(nr))
        if rc == N.GGP_ENAN:
            raise self._nan(nc.value, nr.value)
        self._stalled(rc)
        self._check(rc)
        return ll.value

    def total_likelihood_batch(self, params_points):
        """+ll of every parameter point (rows of an [n, 11] array), each from the carried state as
        it is now; the carried state is left unchanged (ggp_total_loglik_batch).  Returns
        (ll [n], nan [n] bool); a NaN point has ll = nan instead of raising."""
        p = np.ascontiguousarray(np.atleast_2d(params_points), np.float64)
        if p.shape[1] != N.N_PARAMS:
            raise ValueError(f"expected [n, {N.N_PARAMS}] parameter points, got {p.shape}")
        ll = np.zeros(p.shape[0])
        st = np.zeros(p.shape[0], np.int32)
        self._check(self._lib.ggp_total_loglik_batch(self._h, p.shape[0], p.ctypes.data_as(N.c_double_p),
                                                     ll.ctypes.data_as(N.c_double_p),
                                                     st.ctypes.data_as(N.c_int32_p)))
        return ll, st == N.GGP_ENAN

    def total_likelihood_chain(self, params_points) -> np.ndarray:
        """+ll of every parameter point (rows of an [n, 11] array) in order, each from the carried
        state the previous one left (ggp_total_loglik_chain): bitwise n successive
        total_likelihood calls, run as one chained launch where the handle allows.  A failing
        point raises what total_likelihood would (LikelihoodIsNan / EvaluationStalled), with
        .point = its index and .ll = the values of the points before it."""
        p = np.ascontiguousarray(np.atleast_2d(params_points), np.float64)
        if p.ndim != 2 or p.shape[1] != N.N_PARAMS:
            raise ValueError(f"expected [n, {N.N_PARAMS}] parameter points, got {p.shape}")
        self._usable()
        ll = np.zeros(p.shape[0])
        n_ok, nc, nr = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        rc = self._lib.ggp_total_loglik_chain(self._h, p.shape[0], p.ctypes.data_as(N.c_double_p),
                                              ll.ctypes.data_as(N.c_double_p), ctypes.byref(n_ok),
                                              ctypes.byref(nc), ctypes.byref(nr))
        if rc in (N.GGP_ENAN, N.GGP_ETIMEOUT):
            try:
                if rc == N.GGP_ENAN:
                    raise self._nan(nc.value, nr.value)
                self._stalled(rc)
            except GGPError as e:
                e.point, e.ll = int(n_ok.value), ll[:n_ok.value].copy()
                raise
        self._check(rc)
        return ll

    def total_likelihood_tree(self, params_points, pred):
        """speculative evaluation (ggp_total_loglik_tree): point i (a row of an [n, 11] array) from
        the state point pred[i] leaves (-1: the carried state), in one launch; the carried state
        is unchanged until keep_point_state(i).  Returns (ll, status, nan_cell, nan_row) arrays
        (status: GGP_OK / GGP_ENAN / GGP_ETIMEOUT per point); None if the handle has no path
        launch (nothing was evaluated)."""
        p = np.ascontiguousarray(np.atleast_2d(params_points), np.float64)
        pr = np.ascontiguousarray(pred, np.int32)
        if p.ndim != 2 or p.shape[1] != N.N_PARAMS or pr.shape != (p.shape[0],):
            raise ValueError("expected [n, 11] points and n predecessors")
        self._usable()
        n = p.shape[0]
        ll, st = np.zeros(n), np.zeros(n, np.int32)
        nc, nr = np.zeros(n, np.int64), np.zeros(n, np.int64)
        rc = self._lib.ggp_total_loglik_tree(self._h, n, p.ctypes.data_as(N.c_double_p), pr.ctypes.data_as(N.c_int32_p),
                                             ll.ctypes.data_as(N.c_double_p), st.ctypes.data_as(N.c_int32_p),
                                             nc.ctypes.data_as(N.c_int64_p), nr.ctypes.data_as(N.c_int64_p))
        if rc == N.GGP_EINVAL:
            return None
        self._check(rc)
        return ll, st, nc, nr

    def chain_fallbacks(self) -> int:
        """chained calls (total_likelihood_chain) of this handle that finished one by one after a
        stall of the chained schedule (ggp_chain_fallbacks)"""
        n = ctypes.c_int64()
        self._check(self._lib.ggp_chain_fallbacks(self._h, ctypes.byref(n)))
        return n.value

    def keep_point_state(self, point: int) -> None:
        """make the state point `point` of the last total_likelihood_tree left the carried state"""
        self._check(self._lib.ggp_keep_point_state(self._h, int(point)))

    def reset_state(self) -> None:
        self._check(self._lib.ggp_reset_state(self._h))
        self._poisoned = False

    def state(self) -> np.ndarray:
        out = np.zeros((self.n_cells, N.STATE))
        self._check(self._lib.ggp_get_state(self._h, out.ctypes.data_as(N.c_double_p)))
        return out

    def set_state(self, state) -> None:
        """restore a carried state read by state() (checkpoint / resume of a chain)"""
        st = np.ascontiguousarray(state, np.float64)
        if st.shape != (self.n_cells, N.STATE):
            raise ValueError(f"state must be [{self.n_cells}, {N.STATE}], got {st.shape}")
        self._check(self._lib.ggp_set_state(self._h, st.ctypes.data_as(N.c_double_p)))
        self._poisoned = False

    def predict(self, params_per_segment, outputs=(True, True, True)):
        """-p smoother (ggp_predict): (forward, backward, combined) [n_rows, 20] arrays; an output
        whose flag in `outputs` is False is not copied back and comes back as None"""
        p = np.ascontiguousarray(np.atleast_2d(params_per_segment), np.float64)
        out = [np.zeros((self.n_rows, N.STATE)) if want else None for want in outputs]
        self._check(self._lib.ggp_predict(self._h, p.ctypes.data_as(N.c_double_p), p.shape[0],
                                          *(o.ctypes.data_as(N.c_double_p) if o is not None else None
                                            for o in out)))
        return tuple(out)

    def predict_rows(self, r_lo: int, r_hi: int) -> np.ndarray:
        """combined rows [r_lo, r_hi) of the last predict (ggp_predict_rows), [r_hi - r_lo, 20]"""
        out = np.zeros((max(0, r_hi - r_lo), N.STATE))
        self._check(self._lib.ggp_predict_rows(self._h, r_lo, r_hi, out.ctypes.data_as(N.c_double_p)))
        return out

    def shards(self):
        """[(device, rows, cells)] of the handle's shards"""
        n = ctypes.c_int32()
        self._check(self._lib.ggp_forest_shards(self._h, ctypes.byref(n), None, None, None, 0))
        dv = (ctypes.c_int32 * max(1, n.value))()
        rows = (ctypes.c_int64 * max(1, n.value))()
        cells = (ctypes.c_int64 * max(1, n.value))()
        self._check(self._lib.ggp_forest_shards(self._h, ctypes.byref(n), dv, rows, cells, n.value))
        return [(dv[k], rows[k], cells[k]) for k in range(n.value)]

    def predict_profile(self):
        """device ms of the last predict: (forward + backward levels, k_combine)"""
        a, b = ctypes.c_float(), ctypes.c_float()
        self._check(self._lib.ggp_predict_profile(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def joints(self, params_per_segment, tol: float = 1e-10, r_lo: int = 0, r_hi=None, cap: int = 1 << 22,
               out=None, packed: bool = False):
        """-j compute for start rows [r_lo, r_hi) (ggp_joints): (idx [k, 2] = (start, target) rows,
        val [k, 72] = mean[8], row-major cov[64]) in the reference's add order.
        packed=True (ggp_joints_packed): val [k, 44] = mean[8], then the covariance's upper triangle
        row by row -- the values the -j writer prints, 39% fewer bytes from the device.
        out=(idx, val): caller-owned int64 [cap, 2] and float64 [cap, 72 or 44] C-contiguous arrays to
        fill (cap = their length); the results are views of them, overwritten by the next call that
        gets the same buffers.  A caller streaming many start-row ranges (as the CLI does) reuses one
        pair instead of paging in fresh arrays on every call."""
        w = 44 if packed else 72
        p = np.ascontiguousarray(np.atleast_2d(params_per_segment), np.float64)
        r_hi = self.n_rows if r_hi is None else r_hi
        n = ctypes.c_int64()
        if out is None:
            idx = np.zeros((cap, 2), np.int64)
            val = np.zeros((cap, w))
        else:
            idx, val = out
            if (idx.dtype != np.int64 or val.dtype != np.float64 or idx.ndim != 2 or idx.shape[1] != 2
                    or val.ndim != 2 or val.shape[1] != w or not idx.flags.c_contiguous or not val.flags.c_contiguous):
                raise ValueError(f"out must be (int64 [cap, 2], float64 [cap, {w}]) C-contiguous arrays")
            cap = min(len(idx), len(val))
        fn = self._lib.ggp_joints_packed if packed else self._lib.ggp_joints
        self._check(fn(self._h, p.ctypes.data_as(N.c_double_p), p.shape[0], tol, r_lo, r_hi, cap,
                       idx.ctypes.data_as(N.c_int64_p), val.ctypes.data_as(N.c_double_p), ctypes.byref(n)))
        if n.value > cap:
            raise GGPError(f"{n.value} joints exceed cap {cap}: use a larger cap or a smaller row range")
        return idx[: n.value], val[: n.value]

    def enable_profile(self) -> None:
        n = ctypes.c_int32()
        self._check(self._lib.ggp_last_launch_profile(self._h, None, None, None, 0, ctypes.byref(n)))

    def disable_profile(self) -> None:
        """switch the launch events off again (ggp_last_launch_profile with cap < 0)"""
        n = ctypes.c_int32()
        self._check(self._lib.ggp_last_launch_profile(self._h, None, None, None, -1, ctypes.byref(n)))

    def launch_profile(self):
        cap = 4096
        ms = (ctypes.c_float * cap)()
        rows = (ctypes.c_int64 * cap)()
        kern = (ctypes.c_int32 * cap)()
        n = ctypes.c_int32()
        self._check(self._lib.ggp_last_launch_profile(self._h, ms, rows, kern, cap, ctypes.byref(n)))
        return list(ms[: n.value]), list(rows[: n.value]), [kernel_name(k) for k in kern[: n.value]]

    def info(self) -> dict:
        nl, mx = ctypes.c_int64(), ctypes.c_int64()
        k = ctypes.c_int32()
        self._check(self._lib.ggp_forest_info(self._h, ctypes.byref(nl), ctypes.byref(mx), ctypes.byref(k)))
        return {"levels": nl.value, "max_level_cells": mx.value, "kernel": k.value}

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.ggp_forest_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


# ---- reference-named entry points ---------------------------------------------------------
def total_likelihood(params_vec, forest: Forest) -> float:
    """+ll (likelihood.h:170-174).  Mutates the forest's carried root state."""
    return forest.total_likelihood(params_vec)


def total_likelihood_nlopt(params_vec, grad, forest: Forest) -> float:
    """-ll, the NLopt objective signature (likelihood.h:125-159); grad is ignored."""
    return -forest.total_likelihood(params_vec)


def total_likelihood_log_params(log_params_vec, grad, forest: Forest) -> float:
    """exp() of the parameters first (likelihood.h:161-167)."""
    return total_likelihood_nlopt([math.exp(v) for v in log_params_vec], grad, forest)
