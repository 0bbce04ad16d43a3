"""Sharding inside the C-ABI (include/ggp.h "Sharding"): one handle over a
device list.  On the one-GPU box the list repeats ordinal 0 (logical shards, each a whole-tree
sub-forest with its own device buffers), which exercises exactly the code an 8-GPU node runs:
LPT over reduction blocks, per-shard launches from one host thread, block sums gathered and
summed on the host, global NaN ranks, row/cell scatter.

The bar is BITWISE: the total's shape (tree sums, block sums, a fixed pairwise tree over blocks)
depends on the tree count only, so any device list gives the same bits as one device -- for
the carried-state chain, NaN location, batch, -p rows, joints and the CLI's output files.
"""
import filecmp
import math
import os

import numpy as np
import pytest

from test_gpu_cli import INIT, _param_file, _run, _small_csv

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]

LISTS = [[0, 0], [0, 0, 0], [0] * 8]


def _forest(n_trees=300, rows=60):
    import gfp_gaussian_process_amd as g
    return g.HostForest.synthetic(n_trees, rows, with_ids=True)


@pytest.mark.parametrize("kernel", ["auto", "lane", "wave"])
def test_chain_bitwise_for_any_device_list(kernel):
    import gfp_gaussian_process_amd as g
    hf = _forest()
    one = g.Forest(hf, kernel=kernel)
    many = [g.Forest(hf, devices=d, kernel=kernel) for d in LISTS]
    chunked = g.Forest(hf, kernel=kernel, max_shard_rows=hf.n_rows // 7)
    assert [len(f.shards()) for f in many] == [2, 3, 8]
    assert len(chunked.shards()) >= 7
    assert sum(r for _, r, _ in chunked.shards()) == hf.n_rows
    P = list(INIT)
    for call in range(3):
        want = one.total_likelihood(P)
        for f in many + [chunked]:
            assert f.total_likelihood(P) == want, call
    st = one.state()
    for f in many + [chunked]:
        assert np.array_equal(f.state(), st)


def test_shards_balanced_by_rows():
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(1000, 200)
    f = g.Forest(hf, devices=[0] * 8)
    rows = [r for _, r, _ in f.shards()]
    assert sum(rows) == hf.n_rows and max(rows) - min(rows) <= 4 * 200   # blocks of 4 trees


def test_nan_location_for_any_device_list():
    import gfp_gaussian_process_amd as g
    hf = _forest(60, 40)
    P = list(INIT)
    P[2] = -1.0                                   # var_lambda < 0 (test_nan_reported_like_reference)
    got = []
    for d in ([0], [0, 0, 0], [0] * 5):
        with pytest.raises(g.LikelihoodIsNan) as e:
            g.Forest(hf, devices=d).total_likelihood(P)
        got.append((e.value.cell, e.value.row, e.value.cell_id))
    assert got[0][0] >= 0 and all(x == got[0] for x in got)


def test_nan_poisons_carried_state_until_reset():
    """after a NaN the carried state is unspecified (include/ggp.h "Errors"): the Forest refuses
    to evaluate until reset_state() or set_state()"""
    import gfp_gaussian_process_amd as g
    hf = _forest(20, 40)
    f, ref = g.Forest(hf), g.Forest(hf)
    bad = list(INIT)
    bad[2] = -1.0
    with pytest.raises(g.LikelihoodIsNan):
        f.total_likelihood(bad)
    with pytest.raises(g.GGPError, match="reset_state"):
        f.total_likelihood(INIT)
    f.reset_state()
    assert f.total_likelihood(INIT) == ref.total_likelihood(INIT)


def test_set_state_across_shards():
    import gfp_gaussian_process_amd as g
    hf = _forest(100, 40)
    a = g.Forest(hf)
    a.total_likelihood(INIT)
    ck = a.state()
    b = g.Forest(hf, devices=[0, 0, 0])
    b.set_state(ck)
    assert np.array_equal(b.state(), ck)
    for _ in range(2):
        assert b.total_likelihood(INIT) == a.total_likelihood(INIT)


def test_batch_bitwise_for_any_device_list():
    import gfp_gaussian_process_amd as g
    hf = _forest(120, 40)
    rng = np.random.default_rng(5)
    pts = np.stack([np.asarray(INIT) * (1 + 0.02 * rng.standard_normal(11)) for _ in range(7)])
    pts[3, 2] = -1.0
    a = g.Forest(hf, kernel="lane")
    want, wnan = a.total_likelihood_batch(pts)
    assert list(wnan) == [k == 3 for k in range(7)]
    for d in LISTS:
        got, gnan = g.Forest(hf, devices=d).total_likelihood_batch(pts)
        assert np.array_equal(gnan, wnan)
        assert np.array_equal(got[~wnan], want[~wnan])


@pytest.mark.parametrize("mode", ["devices", "chunks"])
def test_predict_bitwise_for_any_sharding(mode):
    """-p per shard (shards on one device share its forward/backward workspace, one after
    another): every output bitwise the one-shard smoother; ggp_predict_rows streams any range"""
    import gfp_gaussian_process_amd as g
    hf = _forest(200, 60)
    P = np.stack([np.asarray(INIT), np.asarray(INIT) * 1.01])
    hf.a["segment"] = (hf.a["time"] >= np.median(hf.a["time"])).astype(np.int32)
    want = g.Forest(hf).predict(P)
    f = g.Forest(hf, devices=[0, 0, 0]) if mode == "devices" else g.Forest(hf, max_shard_rows=hf.n_rows // 5)
    got = f.predict(P)
    for w, x in zip(want, got):
        assert np.array_equal(w, x)
    for lo, hi in ((0, hf.n_rows), (17, 1234), (hf.n_rows - 5, hf.n_rows), (100, 100)):
        assert np.array_equal(f.predict_rows(lo, hi), want[2][lo:hi])
    sm, cb = f.predict_profile()
    assert sm > 0 and cb > 0


def test_joints_bitwise_for_any_device_list():
    import gfp_gaussian_process_amd as g
    hf = _forest(30, 40)
    P = list(INIT)
    P[8] = 2.6e4                                  # the well-conditioned joints case (test_gpu_joints.py)
    one = g.Forest(hf)
    three = g.Forest(hf, devices=[0, 0, 0])
    for lo, hi in ((0, hf.n_rows), (33, 611)):
        iw, vw = one.joints(P, 1e-10, lo, hi)
        ig, vg = three.joints(P, 1e-10, lo, hi)
        assert len(iw) > 0
        assert np.array_equal(iw, ig) and np.array_equal(vw, vg)
        # the packed records (ggp_joints_packed) through the shard merge: means + upper triangle
        ip, vp = three.joints(P, 1e-10, lo, hi, packed=True)
        iu = np.triu_indices(8)
        want = np.concatenate([vw[:, :8], vw[:, 8:].reshape(-1, 8, 8)[:, iu[0], iu[1]]], axis=1)
        assert np.array_equal(ip, iw) and np.array_equal(vp, want)


def _cli_files(tmp_path, csv, cfg, pf, tag, extra):
    out = tmp_path / tag
    _run(["-i", csv, "-b", pf, "-c", cfg, "-o", str(out), *extra], tmp_path)
    return out


def test_cli_outputs_identical_for_any_device_list(tmp_path, example_paths):
    """-e / -s / -m / -p: the output files are byte-identical with the forest on one device, on
    three logical shards (-g 0,0,0) and in chunks (-chunk)"""
    csv = _small_csv(tmp_path / "forest.csv", n_trees=40, rows=40)
    cfg = example_paths["config"]
    pf = _param_file(tmp_path / "p.txt", {7: "3.35E-04, 3.35E-05", 8: "8.26E-01, 8.26E-02, 4.0E-01, 1.3E+00"})
    runs = {}
    for tag, extra in (("one", ["-g", "1"]), ("three", ["-g", "0,0,0"]), ("chunk", ["-g", "1", "-chunk", "300"])):
        out = _cli_files(tmp_path, csv, cfg, pf, tag, ["-e", "-s", "-m", "-t", "1e-3", "-p", *extra])
        runs[tag] = out
    names = sorted(n for n in os.listdir(runs["one"]) if not n.endswith(".log"))
    assert any(n.endswith("_prediction.csv") for n in names) and any("_scan_" in n for n in names)
    assert any(n.endswith("_iterations.csv") for n in names)
    for tag in ("three", "chunk"):
        assert sorted(n for n in os.listdir(runs[tag]) if not n.endswith(".log")) == names
        for n in names:
            assert filecmp.cmp(runs["one"] / n, runs[tag] / n, shallow=False), (tag, n)


def test_path_launch_bitwise_equal_to_level_launches(monkeypatch):
    """the path launch (one launch per evaluation, in-launch reduction) against
    level launches + k_reduce_blocks (GGP_WAVE_PATHS_MAX=0 at handle creation): the same bits
    for the chain, the carried state, the NaN location and batch points"""
    import gfp_gaussian_process_amd as g
    hf = _forest(200, 60)
    paths = g.Forest(hf, kernel="wave")
    monkeypatch.setenv("GGP_WAVE_PATHS_MAX", "0")
    levels = g.Forest(hf, kernel="wave")
    monkeypatch.delenv("GGP_WAVE_PATHS_MAX")
    P = list(INIT)
    for call in range(3):
        assert paths.total_likelihood(P) == levels.total_likelihood(P), call
    assert np.array_equal(paths.state(), levels.state())
    paths.enable_profile()
    levels.enable_profile()
    paths.total_likelihood(P)
    levels.total_likelihood(P)
    assert len(paths.launch_profile()[0]) == 1 and len(levels.launch_profile()[0]) >= 2
    bad = list(INIT)
    bad[2] = -1.0
    got = []
    for f in (paths, levels):
        with pytest.raises(g.LikelihoodIsNan) as e:
            f.total_likelihood(bad)
        got.append((e.value.cell, e.value.row))
    assert got[0] == got[1]


def _shards_of(lib, h):
    import ctypes
    n = ctypes.c_int32()
    assert lib.ggp_forest_shards(h, ctypes.byref(n), None, None, None, 0) == 0
    dv = (ctypes.c_int32 * max(1, n.value))()
    rows = (ctypes.c_int64 * max(1, n.value))()
    cells = (ctypes.c_int64 * max(1, n.value))()
    assert lib.ggp_forest_shards(h, ctypes.byref(n), dv, rows, cells, n.value) == 0
    return [(dv[k], rows[k], cells[k]) for k in range(n.value)]


def test_descriptor_device_sets():
    """The device-set values INTEGRATION.md's binding documents, through the raw C-ABI: a
    zero-filled descriptor's n_devices = 0 is device 0 only (one shard); GGP_ALL_DEVICES (-1) is
    one shard per visible device (ggp_device_count); n > 0 with devices = NULL is ordinals
    0..n-1.  Every form gives the same total (include/ggp.h "Sharding")."""
    import ctypes
    from gfp_gaussian_process_amd import _native as N
    lib = N.engine()
    hf = _forest(64, 40)
    nd = ctypes.c_int32()
    assert lib.ggp_device_count(ctypes.byref(nd)) == 0 and nd.value >= 1
    P = np.asarray(INIT, np.float64)
    cases = {"zero": (0, [(0, hf.n_rows, hf.n_cells)]),
             "all": (N.GGP_ALL_DEVICES, None),
             "one": (1, [(0, hf.n_rows, hf.n_cells)])}
    lls = {}
    for name, (n_dev, want) in cases.items():
        d = hf.desc()
        d.n_devices, d.devices = n_dev, None
        h = ctypes.c_void_p()
        rc = lib.ggp_forest_create(ctypes.byref(d), ctypes.byref(h))
        assert rc == 0, (name, rc)
        try:
            sh = _shards_of(lib, h)
            if want is not None:
                assert sh == want, (name, sh)
            else:   # every visible device once, the forest split by whole trees
                assert sorted(s[0] for s in sh) == list(range(nd.value)), sh
                assert sum(s[1] for s in sh) == hf.n_rows and sum(s[2] for s in sh) == hf.n_cells
            ll, nc, nr = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
            assert lib.ggp_total_loglik(h, P.ctypes.data_as(N.c_double_p), ctypes.byref(ll), ctypes.byref(nc),
                                        ctypes.byref(nr)) == 0
            lls[name] = ll.value
        finally:
            lib.ggp_forest_destroy(h)
    assert lls["zero"] == lls["all"] == lls["one"], lls
    # a descriptor naming a device that does not exist is refused, not silently remapped
    d = hf.desc()
    bad = np.asarray([nd.value], np.int32)
    d.n_devices, d.devices = 1, bad.ctypes.data_as(N.c_int32_p)
    h = ctypes.c_void_p()
    assert lib.ggp_forest_create(ctypes.byref(d), ctypes.byref(h)) != 0


def test_distinct_devices_bitwise():
    """the device list over DISTINCT ordinals [0..n-1] (and each twice) -- what `-g all` runs on a
    multi-GPU node: the chain, carried state, NaN location, batch points, -p rows and joints bitwise
    one device's.  Skipped on a one-GPU box (the repeated-ordinal lists above run the same code)."""
    import torch
    import gfp_gaussian_process_amd as g
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs two visible devices")
    hf = _forest(300, 60)
    lists = [list(range(n)), [k % n for k in range(2 * n)]]
    one = g.Forest(hf)
    many = [g.Forest(hf, devices=d) for d in lists]
    assert sorted({dv for dv, _, _ in many[0].shards()}) == list(range(n))
    for call in range(3):
        want = one.total_likelihood(INIT)
        for f in many:
            assert f.total_likelihood(INIT) == want, call
    for f in many:
        assert np.array_equal(f.state(), one.state())
    bad = list(INIT)
    bad[2] = -1.0
    got = []
    for d in [[0]] + lists:
        with pytest.raises(g.LikelihoodIsNan) as e:
            g.Forest(hf, devices=d).total_likelihood(bad)
        got.append((e.value.cell, e.value.row))
    assert all(x == got[0] for x in got)
    rng = np.random.default_rng(7)
    pts = np.stack([np.asarray(INIT) * (1 + 0.02 * rng.standard_normal(11)) for _ in range(5)])
    want, _ = g.Forest(hf, kernel="lane").total_likelihood_batch(pts)
    for d in lists:
        assert np.array_equal(g.Forest(hf, devices=d).total_likelihood_batch(pts)[0], want)
    pw = g.Forest(hf).predict(INIT)
    P8 = list(INIT)
    P8[8] = 2.6e4
    iw, vw = g.Forest(hf).joints(P8, 1e-10, 0, 500)
    for d in lists:
        f = g.Forest(hf, devices=d)
        for w, x in zip(pw, f.predict(INIT)):
            assert np.array_equal(w, x)
        ig, vg = f.joints(P8, 1e-10, 0, 500)
        assert np.array_equal(iw, ig) and np.array_equal(vw, vg)
