"""CPU tests of the host-side ingest (libggp_host.so) and the C-ABI exports.

Topology must match the reference bit-exactly (BASELINE north star): the example's cell
ids, genealogy and init statistics are compared with an independent brute-force
restatement (tests/golden/example_topology.json, O(N^2) like build_cell_genealogy).
"""
import ctypes
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.usefixtures("built")


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_example_topology_bit_exact(example_paths):
    import gfp_gaussian_process_amd as g
    gold = json.load(open(os.path.join(GOLDEN, "example_topology.json")))
    hf = g.HostForest.from_csv(example_paths["csv"], example_paths["config"])
    assert hf.ids == gold["ids"]
    assert hf.parent_ids == gold["parent_ids"]
    for k in ("parent", "daughter1", "daughter2"):
        assert hf.a[k].tolist() == gold[k], k
    assert np.diff(hf.a["row_offset"]).tolist() == gold["rows"]
    for k in ("root_mean_xg", "root_var_xg", "leaf_mean_xg", "leaf_var_xg"):
        assert [float(v).hex() for v in hf.a[k]] == gold[k], k
    # the data columns themselves (exact sums as a checksum)
    ro = hf.a["row_offset"]
    for col, key in (("time", "time_sum"), ("log_length", "log_length_sum"), ("fp", "fp_sum")):
        tot = 0
        for c in range(hf.n_cells):
            cs = 0
            for v in hf.a[col][ro[c]:ro[c + 1]].tolist():
                cs = cs + v
            tot = tot + cs
        assert float(tot).hex() == gold[key], col
    assert hf.n_rows == 22065 and hf.n_cells == 77 and len(hf.roots) == 1


def test_parameter_file_kinds(example_paths, tmp_path):
    import gfp_gaussian_process_amd as g
    ps = g.ParameterSet.load(example_paths["params"])
    assert ps.kind[6] == "fixed" and ps.init[6] == 4.95e-04           # beta = 4.95E-04
    assert ps.kind[0] == "free" and ps.step[0] == 2.31e-04
    assert ps.lower[0] == 0.0 and ps.upper[0] == float("inf")          # Parameters.h:114-128
    p = _write(tmp_path, "p.txt", open(example_paths["params"]).read().replace(
        "gamma_lambda = 4.36E-02, 4.36E-03", "gamma_lambda = 4.36E-02, 1.0E-03, 2.0E-02, 8.0E-02"))
    ps = g.ParameterSet.load(p)
    assert ps.kind[1] == "bound" and (ps.lower[1], ps.upper[1]) == (2.0e-02, 8.0e-02)
    assert ps.bound() == [1]


def test_parameter_file_errors(tmp_path):
    import gfp_gaussian_process_amd as g
    bad = _write(tmp_path, "bad.txt", "mean_lambda = 1, 2, 3\n")
    with pytest.raises(g.GGPError, match="Invalide number of arguments"):
        g.ParameterSet.load(bad, check_complete=False)
    incomplete = _write(tmp_path, "inc.txt", "# only one\nmean_lambda = 1\n")
    with pytest.raises(g.GGPError, match="not found in parameter file"):
        g.ParameterSet.load(incomplete)
    nan = _write(tmp_path, "nan.txt", "mean_lambda = nan\n")
    with pytest.raises(g.GGPError, match="Nan"):
        g.ParameterSet.load(nan, check_complete=False)


def test_csv_config_parsing(example_paths, tmp_path):
    import gfp_gaussian_process_amd as g
    c = g.CSVConfig.load(example_paths["config"])
    assert c.get("time_col") == "time_min"          # trailing blanks trimmed
    assert c.get("cell_tags") == "lane,cell_id"
    assert c.get("parent_tags") == "lane,parent_id"
    d = g.CSVConfig.load(None)                      # CSVconfig.h:12-24 defaults
    assert (d.get("time_col"), d.get("length_col"), d.get("fp_col"), d.get("delm")) == ("time", "length", "gfp", ",")
    p = _write(tmp_path, "c.txt", "delm = ;\nrescale_time = 60\nlength_islog = true\nfp_auto = 12.5\n")
    c = g.CSVConfig.load(p)
    assert (c.get("delm"), float(c.get("rescale_time")), c.get("length_islog"), float(c.get("fp_auto"))) == (";", 60.0, "1", 12.5)


def test_read_data_semantics(tmp_path):
    """remove_last_decimal ids, new cell on id change, rescale_time, log(length), filter."""
    import gfp_gaussian_process_amd as g
    csv = _write(tmp_path, "in.csv", "\n".join([
        "cell,parent,time,length,gfp,keep",
        "1.0,0.0,0,2.0,100,1",       # id '1' (".0" stripped), parent '0'
        "1.0,0.0,60,2.2,110,true",
        "1.0,0.0,120,2.4,120,0",     # filtered
        "2.50,1.0,180,1.1,60,1",     # id '2.50' kept (last part not all zeros)
        "2.50,1.0,240,1.2,65,TRUE",
        "007.00,1,300,1.3,70,1",     # id '7', parent '1'
        "1.0,0.0,360,2.6,130,1",     # id '1' again, not consecutive -> a NEW cell
    ]) + "\n")
    cfg = _write(tmp_path, "cfg.txt", "time_col = time\ncell_tags = cell\nparent_tags = parent\nrescale_time = 60\nfilter_col = keep\n")
    hf = g.HostForest.from_csv(csv, cfg)
    assert hf.ids == ["1", "2.50", "7", "1"]
    assert hf.parent_ids == ["0", "1", "1", "0"]
    assert np.diff(hf.a["row_offset"]).tolist() == [2, 2, 1, 1]
    assert hf.a["time"].tolist() == [0.0, 1.0, 3.0, 4.0, 5.0, 6.0]
    assert hf.a["log_length"][0] == np.log(2.0)
    # parent = LAST matching cell (index 3); BOTH cells with id '1' list the children
    assert hf.a["parent"].tolist() == [-1, 3, 3, -1]
    assert hf.a["daughter1"].tolist() == [1, -1, -1, 1]
    assert hf.a["daughter2"].tolist() == [2, -1, -1, 2]


def test_third_daughter_is_an_error(tmp_path):
    import gfp_gaussian_process_amd as g
    rows = ["cell_id,parent_id,time,length,gfp", "1,0,0,2,100"]
    rows += [f"{k},1,{k},1,50" for k in (2, 3, 4)]
    csv = _write(tmp_path, "in.csv", "\n".join(rows) + "\n")
    with pytest.raises(g.GGPError, match="Both daughter pointers are set"):
        g.HostForest.from_csv(csv, None)


def test_missing_column_and_nan_rejected(tmp_path):
    import gfp_gaussian_process_amd as g
    csv = _write(tmp_path, "in.csv", "cell_id,parent_id,time,len,gfp\n1,0,0,2,100\n")
    with pytest.raises(g.GGPError, match="length_col"):
        g.HostForest.from_csv(csv, None)
    csv = _write(tmp_path, "in2.csv", "cell_id,parent_id,time,length,gfp\n1,0,0,nan,100\n")
    with pytest.raises(g.GGPError, match="Line no.2"):
        g.HostForest.from_csv(csv, None)


def test_segments(tmp_path):
    """get_segment_indices order + get_segment copies (new roots when a parent has no rows)."""
    import gfp_gaussian_process_amd as g
    csv = _write(tmp_path, "in.csv", "\n".join([
        "cell_id,parent_id,time,length,gfp,seg",
        "1,0,0,2,100,1", "1,0,1,2,100,1",
        "2,1,2,1,50,0", "2,1,3,1,50,0",
        "3,1,2,1,50,1", "3,1,3,1,50,0",
    ]) + "\n")
    cfg = _write(tmp_path, "cfg.txt", "time_col = time\nsegment_col = seg\n")
    ds = g.Dataset.read(csv, g.CSVConfig.load(cfg))
    assert ds.segment_indices() == [1, 0]            # order of first occurrence
    s0 = g.HostForest.build(ds, 0)
    assert s0.ids == ["2", "3"] and s0.a["parent"].tolist() == [-1, -1]   # parent 1 has no seg-0 rows
    s1 = g.HostForest.build(ds, 1)
    assert s1.ids == ["1", "3"] and s1.a["parent"].tolist() == [-1, 0]
    full = g.HostForest.build(ds, -1)
    assert full.a["segment"].tolist() == [1, 1, 0, 0, 1, 0]
    bad = _write(tmp_path, "bad.csv", "cell_id,parent_id,time,length,gfp,seg\n1,0,0,2,100,1\n1,0,1,2,100,2\n")
    with pytest.raises(g.GGPError, match="do not start at 0"):
        g.Dataset.read(bad, g.CSVConfig.load(cfg)).segment_indices()


def test_synthetic_forest_shape_and_determinism():
    import gfp_gaussian_process_amd as g
    a = g.HostForest.synthetic(100, 200)
    b = g.HostForest.synthetic(100, 200)
    assert a.n_cells == 300 and a.n_rows == 20000
    assert np.diff(a.a["row_offset"])[:3].tolist() == [100, 50, 50]
    for k in ("time", "log_length", "fp"):
        assert np.array_equal(a.a[k], b.a[k])
    # tree k of a shard starting at k0 is tree k0+k of the full forest
    s = g.HostForest.synthetic(10, 200, first_tree=40)
    assert np.array_equal(s.a["fp"], a.a["fp"][40 * 200:50 * 200])
    assert np.all(np.isfinite(a.a["fp"])) and np.all(a.a["fp"] > 0)
    # daughters start one minute after the mother's last row
    assert a.a["time"][100] == a.a["time"][99] + 1


def test_subset_trees_keeps_structure():
    import gfp_gaussian_process_amd as g
    f = g.HostForest.synthetic(6, 40, with_ids=True)
    s = f.subset_trees([3, 9])
    assert s.n_cells == 6 and s.a["parent"].tolist() == [-1, 0, 0, -1, 3, 3]
    assert s.ids == f.ids[3:6] + f.ids[9:12]
    assert np.array_equal(s.a["root_mean_xg"], f.a["root_mean_xg"])


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(ggp_[a-z0-9_]+)\s*\(", txt))


@pytest.mark.parametrize("lib,header", [("libggp.so", "ggp.h"), ("libggp_exact.so", "ggp.h"),
                                        ("libggp_host.so", "ggp_host.h")])
def test_library_exports_every_declared_symbol(lib, header):
    path = os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", lib)
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    declared = _declared(header)
    assert declared, header
    missing = declared - exported
    assert not missing, missing
    # and the python binding table covers exactly the header
    from gfp_gaussian_process_amd import _native as N
    table = N.HOST_SYMBOLS if lib == "libggp_host.so" else N.ENGINE_SYMBOLS
    assert set(table) == declared


def test_engine_library_loads_without_gpu():
    """dlopen + metadata calls only (no compute without a GPU)"""
    from gfp_gaussian_process_amd import _native as N
    lib = N.engine()
    assert lib.ggp_version().decode().startswith("ggp-mi355x")
    assert lib.ggp_strerror(N.GGP_ENAN).decode() == "Likelihood is Nan"


def test_forest_binary_roundtrip(tmp_path, example_paths):
    """HostForest.save / load: the SoA arrays, scalars and ids come back exactly, and the oracle
    gives the same likelihood on the reloaded forest"""
    import gfp_gaussian_process_amd as g
    from oracle import oracle as O
    hf = g.HostForest.from_csv(example_paths["csv"], example_paths["config"])
    path = str(tmp_path / "forest.npz")
    hf.save(path)
    back = g.HostForest.load(path)
    assert back.ids == hf.ids and back.parent_ids == hf.parent_ids
    assert set(back.a) == set(hf.a)
    for k, v in hf.a.items():
        assert np.array_equal(np.asarray(back.a[k]), np.asarray(v)), k
        assert np.asarray(back.a[k]).dtype == np.asarray(v).dtype, k
    P = g.ParameterSet.load(example_paths["params"]).get_init()
    assert O.OracleForest(back.a).total_likelihood(P)[0] == O.OracleForest(hf.a).total_likelihood(P)[0]
    syn = g.HostForest.synthetic(20, 30)
    syn.save(path)
    s2 = g.HostForest.load(path)
    assert s2.ids is None and np.array_equal(s2.a["time"], syn.a["time"])


def test_binary_dataset_roundtrip(tmp_path, example_paths):
    """the C++ binary dataset ("GGPD0001", ggp_dataset_save / load): the example read from CSV,
    saved and loaded, builds the bit-identical forest (topology, rows, init statistics) for the
    whole data set and per segment; a synthetic forest round-trips through from_forest; a
    truncated or foreign file is rejected"""
    import gfp_gaussian_process_amd as g
    ds = g.Dataset.read(example_paths["csv"], g.CSVConfig.load(example_paths["config"]))
    path = str(tmp_path / "example.ggpd")
    ds.save(path)
    back = g.Dataset.read(path)                        # Dataset.read detects the magic
    assert back.n_cells == ds.n_cells and back.n_rows == ds.n_rows
    assert back.segment_indices() == ds.segment_indices()
    a, b = g.HostForest.build(ds, -1), g.HostForest.build(back, -1)
    assert a.ids == b.ids and a.parent_ids == b.parent_ids
    for k, v in a.a.items():
        assert np.array_equal(np.asarray(b.a[k]), np.asarray(v)), k
    syn = g.HostForest.synthetic(30, 40, with_ids=True)
    p2 = str(tmp_path / "syn.ggpd")
    g.Dataset.from_forest(syn).save(p2)
    s2 = g.HostForest.build(g.Dataset.read(p2), -1)
    assert s2.ids == syn.ids and s2.a["parent"].tolist() == syn.a["parent"].tolist()
    for k in ("time", "log_length", "fp", "row_offset", "daughter1", "daughter2", "root_mean_xg", "root_var_xg",
              "leaf_mean_xg", "leaf_var_xg"):
        assert np.array_equal(np.asarray(s2.a[k]), np.asarray(syn.a[k])), k
    raw = open(p2, "rb").read()
    open(p2, "wb").write(raw[: len(raw) // 2])
    with pytest.raises(g.GGPError, match="truncated"):
        g.Dataset.load(p2)
    with pytest.raises(g.GGPError, match="GGPD0001"):
        g.Dataset.load(example_paths["params"])
    # a header whose counts exceed the file (valid offsets, 2^33 rows claimed) is refused before
    # anything is allocated from it (the columns alone would be 64 GB)
    import struct
    nr = 1 << 33
    open(p2, "wb").write(b"GGPD0001" + struct.pack("<qqd", 1, nr, 0.0) + struct.pack("<qq", 0, nr) + b"\0" * 64)
    with pytest.raises(g.GGPError, match="exceed"):
        g.Dataset.load(p2)


def test_dataset_csv_writer_roundtrip(tmp_path, example_paths):
    """ggp_dataset_write_csv (synthetic forests as the reference's input CSV): a
    synthetic forest and the example (with its segments) written as CSV + csv_config and read
    back by the reference-semantics reader build the bit-identical forest; ids read_data would
    renormalise are refused"""
    import gfp_gaussian_process_amd as g
    syn = g.HostForest.synthetic(40, 40, with_ids=True)
    csv, cfg = str(tmp_path / "syn.csv"), str(tmp_path / "syn_config.txt")
    g.Dataset.from_forest(syn).write_csv(csv, cfg)
    head = open(csv).readline().strip()
    assert head == ",cell_id,time_min,parent_id,log_length,gfp"
    back = g.HostForest.from_csv(csv, cfg)
    assert back.ids == syn.ids and back.parent_ids == syn.parent_ids
    for k in ("time", "log_length", "fp", "row_offset", "parent", "daughter1", "daughter2", "root_mean_xg",
              "root_var_xg", "leaf_mean_xg", "leaf_var_xg"):
        assert np.array_equal(np.asarray(back.a[k]), np.asarray(syn.a[k])), k
    ds = g.Dataset.read(example_paths["csv"], g.CSVConfig.load(example_paths["config"]))
    csv2, cfg2 = str(tmp_path / "ex.csv"), str(tmp_path / "ex_config.txt")
    ds.write_csv(csv2, cfg2)
    ds2 = g.Dataset.read(csv2, g.CSVConfig.load(cfg2))
    assert ds2.segment_indices() == ds.segment_indices()
    for seg in [-1] + ds.segment_indices()[:2]:
        a, b = g.HostForest.build(ds, seg), g.HostForest.build(ds2, seg)
        assert a.ids == b.ids
        for k, v in a.a.items():
            assert np.array_equal(np.asarray(b.a[k]), np.asarray(v)), (seg, k)
    bad = g.HostForest.synthetic(2, 40, with_ids=True)
    bad.ids = ["1.0"] + bad.ids[1:]
    with pytest.raises(g.GGPError, match="read back"):
        g.Dataset.from_forest(bad).write_csv(str(tmp_path / "bad.csv"), str(tmp_path / "bad_cfg.txt"))


def test_sparse_joints_converter_handcrafted(tmp_path):
    """joints_format.sparse_to_dense on a hand-made case: three rows, a duplicated (cell_id, time)
    column pair (a joint lands in both, Joint_vector::add), rows without joints, the last add
    winning, the dense header and blank blocks (correlation_tree.h:96-126)"""
    from gfp_gaussian_process_amd import joints_format as J
    pred = tmp_path / "p_prediction.csv"
    pred.write_text("no,name\n0,x\n\ncell_id,parent_id,time,log_length,fp,rest\n"
                    "1,0,0,0.5,9,z\n1,0,1,0.5,9,z\n2,1,5,0.6,8,z\n")
    v = lambda k: ",".join(str(k * 100 + i) for i in range(44))   # noqa: E731
    sp = tmp_path / "j_sparse.csv"
    sp.write_text("no,name\n0,x\n\nstart_row,column,h" + "," * 43 + "\n"
                  f"0,1,{v(1)}\n0,2,{v(2)}\n0,1,{v(3)}\n2,0,{v(4)}\n")
    out = tmp_path / "dense.csv"
    assert J.sparse_to_dense(str(sp), str(pred), str(out)) == 3
    blank = "," * 44
    want = ("no,name\n0,x\n\ncell_id,parent_id,time,1_0" + "," * 44 + "1_1" + "," * 44 + "2_5" + "," * 43 + "\n"
            + "1,0,0" + blank + "," + v(3) + "," + v(2) + "\n"
            + "1,0,1" + blank * 3 + "\n"
            + "2,1,5," + v(4) + blank * 2 + "\n")
    assert out.read_text() == want
    assert J.read_sparse(str(sp))[(0, 1)][0] == 300.0


_ONE_RUNTIME_CHILD = r'''
import sys
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native as N
N.engine()


def mapped(tag):
    return sorted({ln.split()[-1] for ln in open("/proc/self/maps") if tag in ln and "/" in ln})


after_engine = (mapped("libamdhip64"), mapped("libhsa-runtime64"))
import torch  # noqa: E402,F401
after_torch = (mapped("libamdhip64"), mapped("libhsa-runtime64"))
print(repr((after_engine, after_torch)))
'''


def test_one_hip_runtime_per_process_engine_first():
    """a process that loads the engine before torch maps exactly one libamdhip64 and one
    libhsa-runtime64, before and after `import torch` (the preload of torch's runtime is taken only
    when its SONAME is the one the engine needs: _native.elf_dynamic)"""
    import ast
    r = subprocess.run([sys.executable, "-c", f"ROOT={ROOT!r}\n" + _ONE_RUNTIME_CHILD], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    (hip_e, hsa_e), (hip_t, hsa_t) = ast.literal_eval(r.stdout.strip().splitlines()[-1])
    assert len(hip_e) == 1 and len(hsa_e) == 1, (hip_e, hsa_e)
    assert hip_t == hip_e and hsa_t == hsa_e, (hip_t, hsa_t)
