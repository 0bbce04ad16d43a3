"""ctypes bindings of the two in-tree native libraries (include/ggp.h, include/ggp_host.h).

The device engine is the product path: there is no Python or CPU fallback.  If
lib/libggp.so is missing or cannot be loaded, ``engine()`` raises -- loudly -- rather
than silently computing something else.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_PKG, "lib")

GGP_OK, GGP_EINVAL, GGP_ENAN, GGP_EDEV, GGP_ENOMEM, GGP_ETIMEOUT = 0, 1, 2, 3, 4, 5
GGP_ALL_DEVICES = -1   # ggp_forest_desc.n_devices: every visible device
N_PARAMS = 11
STATE = 20
KERNELS = {"auto": 0, "lane": 1, "group": 2, "wave": 3, "pair": 4}

c_int64_p = ctypes.POINTER(ctypes.c_int64)
c_int32_p = ctypes.POINTER(ctypes.c_int32)
c_double_p = ctypes.POINTER(ctypes.c_double)
# int (*)(const double *x, double *value, void *data)   (ggp_objective_fn, include/ggp_host.h)
OBJECTIVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, c_double_p, c_double_p, ctypes.c_void_p)
AHEAD_NEED_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p)
AHEAD_TREE_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32), ctypes.c_int32,
                                 ctypes.c_void_p)


class ForestDesc(ctypes.Structure):
    """ggp_forest_desc (include/ggp.h)."""
    _fields_ = [
        ("n_cells", ctypes.c_int64), ("n_rows", ctypes.c_int64),
        ("row_offset", c_int64_p), ("parent", c_int32_p), ("daughter1", c_int32_p),
        ("daughter2", c_int32_p), ("segment", c_int32_p),
        ("time", c_double_p), ("log_length", c_double_p), ("fp", c_double_p),
        ("root_mean_xg", ctypes.c_double * 2), ("root_var_xg", ctypes.c_double * 2),
        ("leaf_mean_xg", ctypes.c_double * 2), ("leaf_var_xg", ctypes.c_double * 2),
        ("noise_scaled", ctypes.c_int32), ("division_binomial", ctypes.c_int32),
        ("fp_auto", ctypes.c_double), ("n_devices", ctypes.c_int32), ("kernel", ctypes.c_int32),
        ("devices", c_int32_p), ("max_shard_rows", ctypes.c_int64),
    ]


class ParamSetC(ctypes.Structure):
    """ggp_param_set (include/ggp_host.h)."""
    _fields_ = [
        ("name", (ctypes.c_char * 16) * N_PARAMS),
        ("kind", ctypes.c_int32 * N_PARAMS), ("set", ctypes.c_int32 * N_PARAMS),
        ("init", ctypes.c_double * N_PARAMS), ("step", ctypes.c_double * N_PARAMS),
        ("lower", ctypes.c_double * N_PARAMS), ("upper", ctypes.c_double * N_PARAMS),
    ]


# every symbol each header declares (tests check the exports against this list)
ENGINE_SYMBOLS = {
    "ggp_forest_create": (ctypes.c_int, [ctypes.POINTER(ForestDesc), ctypes.POINTER(ctypes.c_void_p)]),
    "ggp_forest_destroy": (None, [ctypes.c_void_p]),
    "ggp_total_loglik": (ctypes.c_int, [ctypes.c_void_p, c_double_p, c_double_p, c_int64_p, c_int64_p]),
    "ggp_total_loglik_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, c_double_p, c_double_p, c_int32_p]),
    "ggp_total_loglik_chain": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, c_double_p, c_double_p, c_int32_p,
                                              c_int64_p, c_int64_p]),
    "ggp_total_loglik_tree": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, c_double_p, c_int32_p, c_double_p,
                                             c_int32_p, c_int64_p, c_int64_p]),
    "ggp_keep_point_state": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "ggp_chain_fallbacks": (ctypes.c_int, [ctypes.c_void_p, c_int64_p]),
    "ggp_total_loglik_async": (ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    "ggp_loglik_result": (ctypes.c_int, [ctypes.c_void_p, c_double_p, c_int64_p, c_int64_p]),
    "ggp_predict": (ctypes.c_int, [ctypes.c_void_p, c_double_p, ctypes.c_int32, c_double_p,
                                   c_double_p, c_double_p]),
    "ggp_predict_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                           ctypes.POINTER(ctypes.c_float)]),
    "ggp_joints": (ctypes.c_int, [ctypes.c_void_p, c_double_p, ctypes.c_int32, ctypes.c_double, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_int64, c_int64_p, c_double_p, c_int64_p]),
    "ggp_joints_packed": (ctypes.c_int, [ctypes.c_void_p, c_double_p, ctypes.c_int32, ctypes.c_double,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, c_int64_p, c_double_p,
                                         c_int64_p]),
    "ggp_reset_state": (ctypes.c_int, [ctypes.c_void_p]),
    "ggp_get_state": (ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    "ggp_set_state": (ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    "ggp_last_launch_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                               c_int64_p, c_int32_p, ctypes.c_int32, c_int32_p]),
    "ggp_forest_info": (ctypes.c_int, [ctypes.c_void_p, c_int64_p, c_int64_p, c_int32_p]),
    "ggp_forest_shards": (ctypes.c_int, [ctypes.c_void_p, c_int32_p, c_int32_p, c_int64_p, c_int64_p,
                                         ctypes.c_int32]),
    "ggp_predict_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, c_double_p]),
    "ggp_debug_dawson": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, c_double_p, ctypes.c_int64, c_double_p]),
    "ggp_debug_tauint": (ctypes.c_int, [ctypes.c_int32, c_double_p, ctypes.c_int64, c_double_p]),
    "ggp_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "ggp_comm_attach": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_char_p]),
    "ggp_comm_nan_rank": (ctypes.c_int32, [ctypes.c_void_p]),
    "ggp_comm_size": (ctypes.c_int32, [ctypes.c_void_p]),
    "ggp_launch_clock": (ctypes.c_int, [ctypes.c_void_p, c_double_p, c_double_p]),
    "ggp_call_trace": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, c_double_p, ctypes.POINTER(ctypes.c_int32)]),
    "ggp_comm_local_nan": (ctypes.c_int32, [ctypes.c_void_p]),
    "ggp_device_count": (ctypes.c_int, [c_int32_p]),
    "ggp_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "ggp_version": (ctypes.c_char_p, []),
}

HOST_SYMBOLS = {
    "ggp_host_last_error": (ctypes.c_char_p, []),
    "ggp_csv_config_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "ggp_csv_config_free": (None, [ctypes.c_void_p]),
    "ggp_csv_config_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]),
    "ggp_param_file_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, ctypes.POINTER(ParamSetC)]),
    "ggp_dataset_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "ggp_dataset_free": (None, [ctypes.c_void_p]),
    "ggp_dataset_n_cells": (ctypes.c_int64, [ctypes.c_void_p]),
    "ggp_dataset_n_rows": (ctypes.c_int64, [ctypes.c_void_p]),
    "ggp_dataset_segments": (ctypes.c_int, [ctypes.c_void_p, c_int32_p, ctypes.c_int32, c_int32_p]),
    "ggp_dataset_is_binary": (ctypes.c_int, [ctypes.c_char_p]),
    "ggp_dataset_save": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "ggp_dataset_write_csv": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]),
    "ggp_dataset_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "ggp_dataset_create": (ctypes.c_int, [ctypes.c_int64, c_int64_p, c_double_p, c_double_p, c_double_p, c_int32_p,
                                          ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                          ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]),
    "ggp_forest_build": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_void_p)]),
    "ggp_host_forest_free": (None, [ctypes.c_void_p]),
    "ggp_host_forest_desc": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ForestDesc)]),
    "ggp_host_forest_cell_id": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_int64]),
    "ggp_host_forest_parent_id": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_int64]),
    "ggp_host_forest_n_roots": (ctypes.c_int64, [ctypes.c_void_p]),
    "ggp_synthetic_forest": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    "ggp_nldrmd_minimize": (ctypes.c_int, [ctypes.c_int32, OBJECTIVE_FN, ctypes.c_void_p, c_double_p, c_double_p,
                                           c_double_p, c_double_p, ctypes.c_double, ctypes.c_int64, c_double_p,
                                           c_int64_p]),
    "ggp_nldrmd_minimize_ahead": (ctypes.c_int, [ctypes.c_int32, OBJECTIVE_FN, AHEAD_NEED_FN, AHEAD_TREE_FN,
                                                 ctypes.c_void_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                                 ctypes.c_double, ctypes.c_int64, c_double_p, c_int64_p,
                                                 ctypes.c_int32, ctypes.c_int32]),
    "ggp_num_hessian": (ctypes.c_int, [ctypes.c_int32, OBJECTIVE_FN, ctypes.c_void_p, c_double_p, c_int32_p,
                                       ctypes.c_int32, ctypes.c_double, c_double_p]),
    "ggp_inverse_pplu": (ctypes.c_int, [ctypes.c_int32, c_double_p, c_double_p]),
}

_cache: dict = {}


def _load(name: str, table: dict):
    if name in _cache:
        return _cache[name]
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -m gfp_gaussian_process_amd.build_ext` "
            "(there is no CPU fallback for the likelihood engine)")
    lib = ctypes.CDLL(path)
    for sym, (res, args) in table.items():
        fn = getattr(lib, sym)
        fn.restype = res
        fn.argtypes = args
    _cache[name] = lib
    return lib


def elf_dynamic(path: str):
    """(DT_SONAME, [DT_NEEDED...]) of an ELF64 little-endian shared object, read from its dynamic
    section (memory-mapped: no full read of a large runtime library)"""
    import mmap
    import struct
    with open(path, "rb") as fh, mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ) as m:
        if m[:4] != b"\x7fELF" or m[4] != 2 or m[5] != 1:
            raise ValueError(f"{path}: not an ELF64 little-endian object")
        phoff, = struct.unpack_from("<Q", m, 0x20)
        phentsize, phnum = struct.unpack_from("<HH", m, 0x36)
        loads, dyn = [], None
        for i in range(phnum):
            p_type, _, p_offset, p_vaddr, _, p_filesz, _, _ = struct.unpack_from("<IIQQQQQQ", m, phoff + i * phentsize)
            if p_type == 1:
                loads.append((p_vaddr, p_offset, p_filesz))
            elif p_type == 2:
                dyn = (p_offset, p_filesz)
        if dyn is None:
            return None, []
        ents = [struct.unpack_from("<qQ", m, dyn[0] + 16 * k) for k in range(dyn[1] // 16)]
        strtab = next((v for t, v in ents if t == 5), None)
        if strtab is None:
            return None, []
        base = next((off + strtab - va for va, off, sz in loads if va <= strtab < va + sz), None)

        def cstr(o):
            end = m.find(b"\0", base + o)
            return m[base + o:end].decode()
        soname = next((cstr(v) for t, v in ents if t == 14), None)
        return soname, [cstr(v) for t, v in ents if t == 1]


def _one_hip_runtime() -> None:
    """One HIP runtime per process.  libggp.so needs libamdhip64.so.7; PyTorch-ROCm ships its own
    copy (same SONAME, another file) and its libraries ask for it by another name, so when the
    engine loads first the process would map two HIP runtimes, and torch's then sees no GPU
    (measured: "No HIP GPUs are available", tools/two_runtimes.py).  When torch is installed, its
    runtime is mapped first (RTLD_GLOBAL, without importing torch): the engine binds to it by
    SONAME and a later `import torch` finds the same file already loaded.  GGP_HIP_RUNTIME=rocm
    keeps /opt/rocm's (for processes that never import torch)."""
    if os.environ.get("GGP_HIP_RUNTIME", "") == "rocm":
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        hip = os.path.join(d, "lib", "libamdhip64.so")
        if not os.path.exists(hip):
            continue
        # only a runtime the engine would bind to by name: torch's SONAME must be the
        # libamdhip64 the engine library lists as NEEDED, else preloading would map a second runtime
        try:
            want = [n for n in elf_dynamic(os.path.join(LIB_DIR, engine_name()))[1] if n.startswith("libamdhip64")]
            have = elf_dynamic(hip)[0]
        except (OSError, ValueError):
            want, have = [], None
        if want and have == want[0]:
            ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)
        else:
            import warnings
            warnings.warn(f"torch's HIP runtime ({hip}, SONAME {have}) is not the {want[0] if want else 'libamdhip64'} "
                          "the engine needs: not preloaded; importing torch after the engine may map two HIP runtimes")
        return


def engine_name() -> str:
    """the engine library's file name: libggp.so, or GGP_ENGINE_LIB (A/B builds such as
    lib/libggp_exact.so, the GGP_EXACT arithmetic)"""
    return os.environ.get("GGP_ENGINE_LIB", "libggp.so")


EXACT_ENGINE = "libggp_exact.so"


def engine(name: str | None = None):
    """libggp.so (HIP, gfx950), or the engine library `name` (EXACT_ENGINE: the same C-ABI in the
    oracle's arithmetic)."""
    name = name or engine_name()
    if name not in _cache:
        _one_hip_runtime()
    return _load(name, ENGINE_SYMBOLS)


def host():
    """libggp_host.so (host ingest)."""
    return _load("libggp_host.so", HOST_SYMBOLS)
