"""The CLI (lib/ggp, the reference's main.cpp surface) on the GPU against the CPU oracle:
-e, -s, -p and -m on the reference's example data set, -j on a small synthetic forest.

Tolerances: log-likelihood values 1e-9 relative (the north-star bar); -p values are printed
with 6 significant digits by the reference's writer, so they are compared after parsing at
1e-4 normalised by the standard deviations (the smoother's own tolerance is 1e-5, see
test_gpu_parity.py).  The -m trajectory is compared with the same Nelder-Mead restatement
driven by the oracle objective.
"""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("built")]
CLI = os.path.join(ROOT, "gfp_gaussian_process_amd", "lib", "ggp")
NAMES = ["mean_lambda", "gamma_lambda", "var_lambda", "mean_q", "gamma_q", "var_q", "beta",
         "var_x", "var_g", "var_dx", "var_dg"]
INIT = [2.31E-03, 4.36E-02, 9.75E-08, 9.03E+01, 1.60E-02, 1.94E+01, 4.95E-04, 3.35E-04, 8.26E-01,
        1.63E-04, 7.48E-01]


def _param_file(path, spec):
    """spec: {index: "init, step[, lower, upper]"}; every other parameter fixed at INIT"""
    with open(path, "w") as f:
        for i, n in enumerate(NAMES):
            f.write(f"{n} = {spec.get(i, repr(INIT[i]))}\n")
    return str(path)


def _run(args, cwd):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=600, cwd=cwd)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _ll_table(path):
    lines = open(path).read().split("log_likelihoods:\n")[1].strip().splitlines()[1:]
    return [[float(v) for v in ln.rstrip(",").split(",")] for ln in lines]


@pytest.fixture(scope="module")
def oracle_example(example_paths):
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.from_csv(example_paths["csv"], example_paths["config"], -1, "scaled", "binomial")
    return hf


def test_cli_evaluate_matches_oracle(tmp_path, example_paths, oracle_example):
    from oracle import oracle as O
    pf = _param_file(tmp_path / "p.txt", {})
    out = _run(["-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-e", "-o", str(tmp_path / "o")],
               tmp_path)
    ll = float(out.split("total log likelihood = ")[1].split()[0])
    ref = O.OracleForest(oracle_example.a).total_likelihood(INIT)[0]
    assert abs(ll - ref) / abs(ref) < 1e-9
    assert os.path.exists(tmp_path / "o" / "input_success.log")


def test_cli_scan_chain_matches_oracle(tmp_path, example_paths, oracle_example):
    """-s: one bound parameter, every sample on the carried state of the previous one"""
    from oracle import oracle as O
    pf = _param_file(tmp_path / "p.txt", {8: "8.26E-01, 2.0E-01, 4.0E-01, 1.3E+00"})
    _run(["-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-s", "-o", str(tmp_path / "o")],
         tmp_path)
    rows = _ll_table(tmp_path / "o" / "input_scan_var_g.csv")
    of = O.OracleForest(oracle_example.a)
    from gfp_gaussian_process_amd.optimize import arange
    samples = arange(0.4, 1.3, 0.2)
    assert len(rows) == len(samples)
    for k, (row, v) in enumerate(zip(rows, samples)):
        assert row[0] == k + 1 and row[9] == v
        p = list(INIT)
        p[8] = v
        ref = of.total_likelihood(p)[0]
        assert abs(row[-1] - ref) / abs(ref) < 1e-9, (k, row[-1], ref)


def test_cli_predict_matches_oracle(tmp_path, example_paths, oracle_example):
    from oracle import oracle as O
    pf = _param_file(tmp_path / "p.txt", {})
    _run(["-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-p", "-o", str(tmp_path / "o")],
         tmp_path)
    text = open(tmp_path / "o" / "input_f_b_prediction.csv").read()
    head, body = text.split("\ncell_id,parent_id,time,log_length,fp,")
    assert head.startswith("no,name,type,init,step,lower_bound,upper_bound,final\n0,mean_lambda,fixed,0.00231, , , ,")
    lines = body.strip().splitlines()[1:]
    hf = oracle_example
    assert len(lines) == hf.n_rows
    _, _, comb = O.OracleForest(hf.a).predict(INIT)
    got = np.array([[float(v) for v in ln.split(",")[5:]] for ln in lines])
    iu = np.triu_indices(4)
    ref_m = comb[:, :4]
    ref_c = comb[:, 4:].reshape(-1, 4, 4)
    sd = np.sqrt(np.abs(np.einsum("nii->ni", ref_c)))
    em = np.max(np.abs(got[:, :4] - ref_m) / (np.abs(ref_m) + sd))
    ec = np.max(np.abs(got[:, 4:] - ref_c[:, iu[0], iu[1]]) / (sd[:, iu[0]] * sd[:, iu[1]]))
    assert em < 1e-4 and ec < 1e-4, (em, ec)
    ids = [ln.split(",")[0] for ln in lines]
    assert ids[0] == hf.ids[0] and ids[-1] == hf.ids[-1]


def _g(x):
    """`std::ostream << double` under the default stream state: printf's "%.6g" """
    x = float(x)
    if x != x:
        return "-nan" if math.copysign(1.0, x) < 0 else "nan"
    return "%.6g" % x


def test_cli_prediction_text_is_the_rows_formatted(tmp_path, example_paths, oracle_example):
    """_prediction.csv byte for byte: every row's ids, time, log_length, fp and the 14 smoothed
    values of the same run's binary rows (-pbin, the exact doubles), formatted as the reference's
    write_predictions_to_file formats them (predictions.h:563-602); the writer's blocks are
    formatted on 7 threads and must come out in row order, the rows fetched from the device in
    spans of 5,000 (the next span copied while this one is formatted)"""
    pf = _param_file(tmp_path / "p.txt", {})
    env = dict(os.environ, GGP_IO_THREADS="7", GGP_PREDICT_SPAN="5000")
    for tag, extra in (("t", ["-p"]), ("b", ["-p", "-pbin"])):
        r = subprocess.run([CLI, "-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], *extra,
                            "-o", str(tmp_path / tag)], capture_output=True, text=True, timeout=600, cwd=tmp_path, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
    raw = open(tmp_path / "b" / "input_f_b_prediction.bin", "rb").read()
    assert raw[:8] == b"GGPP0001"
    n = int(np.frombuffer(raw[8:16], dtype=np.int64)[0])
    rows = np.frombuffer(raw[16:], dtype=np.float64).reshape(n, 14)
    hf = oracle_example
    a = hf.a
    cell = np.repeat(np.arange(hf.n_cells), np.diff(a["row_offset"]))
    body = open(tmp_path / "t" / "input_f_b_prediction.csv").read().split(
        "\ncell_id,parent_id,time,log_length,fp,mean_x,mean_g,mean_l,mean_q,cov_xx,cov_xg,cov_xl,cov_xq,"
        "cov_gg,cov_gl,cov_gq,cov_ll,cov_lq,cov_qq\n")[1]
    want = "".join(",".join([hf.ids[cell[r]], hf.parent_ids[cell[r]], _g(a["time"][r]), _g(a["log_length"][r]),
                             _g(a["fp"][r]), *[_g(v) for v in rows[r]]]) + "\n" for r in range(n))
    assert n == hf.n_rows and body == want


def test_cli_predict_binary_rows_fused_combine_identical(tmp_path, example_paths):
    """-p -pbin on the example with every smoother level on the lane kernels (GGP_SMOOTHER_LANE=1:
    the combine fused into the backward pass), with the separate combine (GGP_COMBINE_FUSED=0), and
    with the default schedule (lane-pair levels, the separate combine): the same binary rows"""
    pf = _param_file(tmp_path / "p.txt", {})
    files = []
    for tag, extra_env in (("fused", {"GGP_SMOOTHER_LANE": "1"}),
                           ("sep", {"GGP_SMOOTHER_LANE": "1", "GGP_COMBINE_FUSED": "0"}), ("auto", {})):
        env = dict(os.environ, **extra_env)
        r = subprocess.run([CLI, "-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-p", "-pbin",
                            "-o", str(tmp_path / tag)], capture_output=True, text=True, timeout=600, cwd=tmp_path,
                           env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        files.append(open(tmp_path / tag / "input_f_b_prediction.bin", "rb").read())
    assert files[0][:8] == b"GGPP0001" and len(files[0]) > 16
    assert files[0] == files[1] == files[2]


def test_cli_minimize_matches_oracle_trajectory(tmp_path, example_paths, oracle_example):
    """-m, log space, two free parameters: the GPU run's iteration log follows the same
    Nelder-Mead steps as the restatement driven by the oracle objective"""
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as Opt
    from oracle import oracle as O
    pf = _param_file(tmp_path / "p.txt", {7: "3.35E-04, 3.35E-05", 8: "8.26E-01, 8.26E-02"})
    _run(["-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-m", "-t", "1e-4",
          "-o", str(tmp_path / "o")], tmp_path)
    base = tmp_path / "o" / "input_f78_b"
    rows = _ll_table(str(base) + "_iterations.csv")
    of = O.OracleForest(oracle_example.a)
    seen = []

    def objective(p):
        v = of.total_likelihood(p)[0]
        seen.append((p.copy(), v))
        return v

    P = g.ParameterSet.load(pf)
    x, ll, rc = Opt.minimize_wrapper(objective, P, tolerance=1e-4, search_space="log")
    assert rc == Opt.FTOL_REACHED
    n = min(len(rows), len(seen), 25)
    assert n >= 10
    for k in range(n):
        assert np.allclose(rows[k][1:12], seen[k][0], rtol=1e-9), k
        assert abs(rows[k][12] - seen[k][1]) / abs(seen[k][1]) < 1e-9, k
    final = open(str(base) + "_final.csv").read()
    assert "errors^2:\nepsilon,var_x,var_g\n" in final and "n_data_points, 22065" in final
    assert "optimization_algorithm,LN_NELDERMEAD" in final
    fl = float(final.split("total_log_likelihoood,")[1].split()[0])
    assert abs(fl - ll) / abs(ll) < 1e-8
    pfile = open(str(base) + "_parameter_file.txt").read()
    assert pfile.startswith("# Generated parameter file")


def _small_csv(path, n_trees=2, rows=40):
    """a small synthetic forest in the example's column layout (lane 1, integer cell ids)"""
    import math
    import gfp_gaussian_process_amd as g
    hf = g.HostForest.synthetic(n_trees, rows)
    a = hf.a
    ro, par = a["row_offset"], a["parent"]
    with open(path, "w") as f:
        f.write(",cell_id,time_min,parent_id,lane,length,gfp\n")
        k = 0
        for c in range(hf.n_cells):
            pid = int(par[c]) + 11 if par[c] >= 0 else 7       # roots: parent 7 is not in the data
            for r in range(ro[c], ro[c + 1]):
                t, ln, fp = float(a["time"][r]), math.exp(float(a["log_length"][r])), float(a["fp"][r])
                f.write(f"{k},{c + 11},{t!r},{pid},1,{ln!r},{fp!r}\n")
                k += 1
    return str(path)


def test_cli_joints_dense_matrix(tmp_path, example_paths):
    """-j (implies -p): the reference's dense joint matrix (correlation_tree.h:96-126,
    588-648) against the engine's joints (ggp_joints, checked against the oracle in
    test_gpu_joints.py): column labels, one line per start row, 44 fields per column, the
    joint's 8 means and upper triangle where the walk reached the column, empty elsewhere.
    Values are printed with 6 significant digits (default stream precision)."""
    import gfp_gaussian_process_amd as g
    csv = _small_csv(tmp_path / "small.csv")
    pf = _param_file(tmp_path / "p.txt", {})
    out = tmp_path / "o"
    _run(["-i", csv, "-b", pf, "-c", example_paths["config"], "-j", "-o", str(out)], tmp_path)
    assert (out / "small_f_b_prediction.csv").exists()
    text = (out / "small_f_b_joints.csv").read_text()
    head, body = text.split("\ncell_id,parent_id,time,", 1)
    assert head.startswith("no,name,type,init,step,lower_bound,upper_bound,final\n0,mean_lambda,fixed,")
    lines = body.split("\n")
    assert lines[-1] == ""
    hdr, rows = lines[0].split(","), lines[1:-1]
    hf = g.HostForest.from_csv(csv, example_paths["config"])
    n = hf.n_rows
    cell = np.repeat(np.arange(hf.n_cells), np.diff(hf.a["row_offset"]))
    assert len(hdr) == 44 * n and len(rows) == n
    assert hdr[::44] == [f"{hf.ids[cell[r]]}_{hf.a['time'][r]:g}" for r in range(n)]
    assert all(x == "" for k, x in enumerate(hdr) if k % 44)
    ig, vg = g.Forest(hf).joints(INIT, 1e-10)
    want = {}
    for (s, t), v in zip(ig.tolist(), vg):
        want.setdefault(s, {})[t] = v
    assert len(want) > n // 2
    iu = np.triu_indices(8)
    for s, line in enumerate(rows):
        f = line.split(",")
        assert len(f) == 3 + 44 * n, s
        assert f[0] == hf.ids[cell[s]] and f[1] == hf.parent_ids[cell[s]]
        assert float(f[2]) == pytest.approx(hf.a["time"][s], rel=1e-5)
        got = {}
        for col in range(n):
            blk = f[3 + 44 * col: 3 + 44 * (col + 1)]
            if blk[0] == "":
                assert all(x == "" for x in blk), (s, col)
                continue
            got[col] = np.array([float(x) for x in blk])
        exp = want.get(s, {})
        assert set(got) == set(exp), s
        for col, v in got.items():
            ref = np.concatenate([exp[col][:8], exp[col][8:].reshape(8, 8)[iu]])
            # the same doubles (the engine is deterministic), printed as the reference's `<<`
            # prints them (printf "%.6g")
            assert f[3 + 44 * col: 3 + 44 * (col + 1)] == [_g(x) for x in ref], (s, col)


def _errors(path):
    block = open(path).read().split("errors^2:\n")[1].split("\n\n")[0].strip().splitlines()[1:]
    return np.array([[float(v) for v in ln.split(",")] for ln in block])


def test_cli_minimize_batched_hessian(tmp_path, example_paths):
    """-m -hb: the same optimiser trajectory; the error bars from one batched call per epsilon
    (points from the optimiser's final carried state, not chained).  The chained and unchained
    Hessians differ only through the carried root off-diagonals: compared at 10%."""
    pf = _param_file(tmp_path / "p.txt", {7: "3.35E-04, 3.35E-05", 8: "8.26E-01, 8.26E-02"})
    for tag, extra in (("a", []), ("b", ["-hb"])):
        _run(["-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-m", "-t", "1e-4",
              "-o", str(tmp_path / tag), *extra], tmp_path)
    ra = _ll_table(str(tmp_path / "a" / "input_f78_b") + "_iterations.csv")
    rb = _ll_table(str(tmp_path / "b" / "input_f78_b") + "_iterations.csv")
    assert ra == rb
    ea = _errors(str(tmp_path / "a" / "input_f78_b") + "_final.csv")
    eb = _errors(str(tmp_path / "b" / "input_f78_b") + "_final.csv")
    assert ea.shape == eb.shape == (3, 3)
    assert np.array_equal(ea[:, 0], eb[:, 0])
    assert np.all(eb[:, 1:] > 0)
    assert np.allclose(ea[:, 1:], eb[:, 1:], rtol=0.1), (ea, eb)


def test_cli_sparse_joints_rebuild_the_dense_file(tmp_path, example_paths):
    """-js writes one line per joint (_joints_sparse.csv, O(joints) instead of O(rows^2));
    joints_format.sparse_to_dense rebuilds the reference's dense _joints.csv from it and the
    _prediction.csv byte for byte -- so correlation_from_joint.py reads it unchanged"""
    from gfp_gaussian_process_amd import joints_format as J
    csv = _small_csv(tmp_path / "small.csv", n_trees=8, rows=40)
    pf = _param_file(tmp_path / "p.txt", {})
    for tag, flag in (("dense", "-j"), ("sparse", "-js")):
        _run(["-i", csv, "-b", pf, "-c", example_paths["config"], flag, "-o", str(tmp_path / tag)], tmp_path)
    dense = (tmp_path / "dense" / "small_f_b_joints.csv").read_bytes()
    sp = tmp_path / "sparse" / "small_f_b_joints_sparse.csv"
    assert sp.exists() and not (tmp_path / "sparse" / "small_f_b_joints.csv").exists()
    assert sp.stat().st_size < len(dense) / 2          # walks stay inside a tree (8 trees); dense: rows^2 fields
    out = tmp_path / "rebuilt.csv"
    J.sparse_to_dense(str(sp), str(tmp_path / "sparse" / "small_f_b_prediction.csv"), str(out))
    assert out.read_bytes() == dense


def test_cli_two_segments_matches_oracle(tmp_path, example_paths):
    """Two segments (segment_col) with two -b files through -e -m -s -p in one CLI run
    (main.cpp:402-443).  -e, -m and -s run per segment on get_segment copies (moma_input.h:
    580-620: a cell keeps its segment's rows; a parent without rows there leaves a new root),
    with _segment<i> file names (get_segment_file_number); -p runs the whole forest with each
    row's segment parameters, after -m has set the final values (run_minimization takes the
    parameter set by reference).  Checked against the oracle: -e and the -s samples (each on the
    carried state of the previous one) at 1e-9, the -m iteration log against the Nelder-Mead
    restatement driven by the oracle objective at 1e-9, and -p (6 significant digits printed)
    at 1e-4 of the standard deviations with the restatement's final parameters."""
    import glob
    import gfp_gaussian_process_amd as g
    from gfp_gaussian_process_amd import optimize as Opt
    from oracle import oracle as O
    hf0 = g.HostForest.synthetic(4, 60)   # per tree: a root (t 0-29) and two daughters (t 30-44)
    a = hf0.a
    ro, par = a["row_offset"], a["parent"]
    csv = tmp_path / "small.csv"
    with open(csv, "w") as f:
        f.write(",cell_id,time_min,parent_id,lane,length,gfp,seg\n")
        k = 0
        for c in range(hf0.n_cells):
            pid = int(par[c]) + 11 if par[c] >= 0 else 7
            for r in range(ro[c], ro[c + 1]):
                t = float(a["time"][r])
                seg = 1 if t >= 20.0 else 0        # roots split inside the cell, daughters all in 1
                f.write(f"{k},{c + 11},{t!r},{pid},1,{math.exp(float(a['log_length'][r]))!r},"
                        f"{float(a['fp'][r])!r},{seg}\n")
                k += 1
    cfg = tmp_path / "cfg.txt"
    cfg.write_text(open(example_paths["config"]).read() + "\nsegment_col = seg\n")
    bound = "6.0E-01, 1.0E-01, 4.0E-01, 1.3E+00"
    pf0 = _param_file(tmp_path / "p0.txt", {8: bound})
    pf1 = _param_file(tmp_path / "p1.txt", {0: repr(INIT[0] * 1.1), 8: bound})
    out = tmp_path / "o"
    stdout = _run(["-i", str(csv), "-b", f"{pf0} {pf1}", "-c", str(cfg), "-e", "-m", "-t", "1e-4", "-s", "-p",
                   "-o", str(out)], tmp_path)
    ds = g.Dataset.read(str(csv), g.CSVConfig.load(str(cfg)))
    assert ds.segment_indices() == [0, 1]
    segs = [g.HostForest.build(ds, s) for s in (0, 1)]
    assert segs[1].a["parent"].tolist().count(-1) == 4    # the split roots stay parents in segment 1
    assert segs[0].n_cells == 4 and segs[1].n_cells == 12
    finals = []
    for i, (pf, hs) in enumerate(zip((pf0, pf1), segs)):
        P = g.ParameterSet.load(pf)
        p_init = np.array(P.init)
        # -e: fresh copy, initial values
        ll = float(stdout.split(f"segment {i}: total log likelihood = ")[1].split()[0])
        ref = O.OracleForest(hs.a).total_likelihood(p_init)[0]
        assert abs(ll - ref) / abs(ref) < 1e-9, (i, ll, ref)
        # -m: the iteration log follows the restatement's steps on a fresh copy
        of = O.OracleForest(hs.a)
        seen = []

        def objective(p, of=of, seen=seen):
            v = of.total_likelihood(p)[0]
            seen.append((np.array(p), v))
            return v

        x, llmax, rc = Opt.minimize_wrapper(objective, P, tolerance=1e-4, search_space="log")
        finals.append(x)
        it = glob.glob(str(out / f"small_segment{i}_*_iterations.csv"))
        assert len(it) == 1, it
        rows = _ll_table(it[0])
        n = min(len(rows), len(seen))
        assert n >= 5 and len(rows) >= len(seen) - 1
        for k in range(n):
            assert np.allclose(rows[k][1:12], seen[k][0], rtol=1e-9), (i, k)
            assert abs(rows[k][12] - seen[k][1]) / abs(seen[k][1]) < 1e-9, (i, k)
        fin = open(it[0].replace("_iterations.csv", "_final.csv")).read()
        assert abs(float(fin.split("total_log_likelihoood,")[1].split()[0]) - llmax) / abs(llmax) < 1e-8
        assert f"n_data_points, {hs.n_rows}" in fin
        # -s: after -m (the scanned parameter replaces its final value), a fresh copy, chained
        rows = _ll_table(str(out / f"small_segment{i}_scan_var_g.csv"))
        samples = Opt.arange(0.4, 1.3, 0.1)
        assert len(rows) == len(samples)
        of = O.OracleForest(hs.a)
        for k, (row, v) in enumerate(zip(rows, samples)):
            p = x.copy()
            p[8] = v
            ref = of.total_likelihood(p)[0]
            assert row[9] == v and abs(row[-1] - ref) / abs(ref) < 1e-9, (i, k, row[-1], ref)
    # -p: the whole forest, row segment -> that segment's final parameters
    pred = glob.glob(str(out / "small*_prediction.csv"))
    assert len(pred) == 1, pred
    text = open(pred[0]).read()
    body = text.split("\ncell_id,parent_id,time,log_length,fp,")[1]
    lines = body.strip().splitlines()[1:]
    hf = g.HostForest.build(ds, -1)
    assert hf.a["segment"].tolist() == [1 if t >= 20.0 else 0 for t in hf.a["time"]]
    _, _, comb = O.OracleForest(hf.a).predict(np.stack(finals))
    got = np.array([[float(v) for v in ln.split(",")[5:]] for ln in lines])
    assert got.shape == (hf.n_rows, 14)
    iu = np.triu_indices(4)
    ref_m, ref_c = comb[:, :4], comb[:, 4:].reshape(-1, 4, 4)
    sd = np.sqrt(np.abs(np.einsum("nii->ni", ref_c)))
    em = np.max(np.abs(got[:, :4] - ref_m) / (np.abs(ref_m) + sd))
    ec = np.max(np.abs(got[:, 4:] - ref_c[:, iu[0], iu[1]]) / (sd[:, iu[0]] * sd[:, iu[1]]))
    assert em < 1e-4 and ec < 1e-4, (em, ec)


def test_cli_lookahead_and_chain_give_the_sequential_files(tmp_path, example_paths):
    """-m with the optimiser's lookahead (each reflected point and its three possible successors
    in one speculative launch) and the chained Hessian / scan calls: every output file byte for
    byte that of the call-by-call run (GGP_NM_LOOKAHEAD=0, GGP_CHAIN_FUSED=0) -- the same
    trajectory, iteration log, error bars (carried state included) and final values"""
    pf = _param_file(tmp_path / "p.txt", {0: "2.31E-03, 2.31E-04", 7: "3.35E-04, 3.35E-05", 8: "8.26E-01, 8.26E-02",
                                           6: "4.95E-04, 1.0E-04, 1.0E-04, 9.0E-04"})
    outs = {}
    for tag, env in (("seq", {"GGP_NM_LOOKAHEAD": "0", "GGP_CHAIN_FUSED": "0"}), ("fast", {})):
        e = dict(os.environ, **env)
        r = subprocess.run([CLI, "-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-m", "-s",
                            "-t", "1e-3", "-o", str(tmp_path / tag)], capture_output=True, text=True, timeout=600,
                           cwd=tmp_path, env=e)
        assert r.returncode == 0, r.stdout + r.stderr
        outs[tag] = {n: open(tmp_path / tag / n, "rb").read() for n in sorted(os.listdir(tmp_path / tag))
                     if n.endswith(".csv") or n.endswith(".txt")}
    assert sorted(outs["seq"]) == sorted(outs["fast"]) and len(outs["seq"]) >= 4, sorted(outs["seq"])
    for n in outs["seq"]:
        assert outs["seq"][n] == outs["fast"][n], n
    it = [n for n in outs["fast"] if n.endswith("_iterations.csv")]
    assert len(it) == 1 and len(_ll_table(str(tmp_path / "fast" / it[0]))) > 40, it


def test_cli_lookahead_nan_run_fails_like_the_sequential_one(tmp_path, example_paths):
    """-m in linear space with var_x free below zero: the run meets a NaN likelihood and quits
    (likelihood.h:71-93).  With the lookahead (a speculated call may be NaN without being made) the
    iteration log and the error log are byte for byte the call-by-call run's"""
    pf = _param_file(tmp_path / "p.txt", {7: "3.35E-04, 5.0E-04, -1.0E-03, 1.0E-03", 8: "8.26E-01, 8.26E-02"})
    outs = {}
    for tag, env in (("seq", {"GGP_NM_LOOKAHEAD": "0", "GGP_CHAIN_FUSED": "0"}), ("fast", {})):
        r = subprocess.run([CLI, "-i", example_paths["csv"], "-b", pf, "-c", example_paths["config"], "-m",
                            "-space", "linear", "-t", "1e-6", "-o", str(tmp_path / tag)], capture_output=True, text=True,
                           timeout=600, cwd=tmp_path, env=dict(os.environ, **env))
        assert r.returncode != 0 and "Likelihood is Nan" in r.stdout, r.stdout[-800:]
        outs[tag] = {n: open(tmp_path / tag / n, "rb").read().replace(str(tmp_path / tag).encode(), b"OUT")
                     for n in sorted(os.listdir(tmp_path / tag))}   # the logs name the output directory
    assert sorted(outs["seq"]) == sorted(outs["fast"])
    assert any(n.endswith("_error.log") for n in outs["seq"])
    for n in outs["seq"]:
        assert outs["seq"][n] == outs["fast"][n], n
