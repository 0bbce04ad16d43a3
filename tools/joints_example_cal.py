"""Calibration for tests/test_gpu_joints.py (example data set): per pair above the margin, the
GPU's normalised error against the oracle's own movement under +-1 ulp exp() noise (max over
3 seeds).  Prints quantiles; run on the GPU box."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gzip, shutil, tempfile
import gfp_gaussian_process_amd as g
from oracle import oracle as O
from test_gpu_joints import P, _norm_err, _ratio, MARGIN
d = tempfile.mkdtemp()
with gzip.open("tests/golden/example_input.csv.gz", "rb") as fi, open(d + "/in.csv", "wb") as fo:
    shutil.copyfileobj(fi, fo)
hf = g.HostForest.from_csv(d + "/in.csv", "tests/golden/example_csv_config.txt", -1, "scaled", "binomial")
fg, of = g.Forest(hf), O.OracleForest(hf.a)
ops = [O.OracleForest(hf.a, exp_ulp_noise=s) for s in (12345, 777, 4242)]
ro = hf.a["row_offset"]
last = int(ro[1]) - 1
for lo, hi in ((0, 40), (max(0, last - 20), last + 1)):
    ig, vg = fg.joints(P, 1e-10, lo, hi, cap=1 << 21)
    io, vo = of.joints(P, 1e-10, lo, hi, cap=1 << 21)
    kg = {tuple(k): n for n, k in enumerate(ig.tolist())}
    ko = {tuple(k): n for n, k in enumerate(io.tolist())}
    common = [k for k in sorted(set(kg) & set(ko)) if _ratio(vo[ko[k]]) > MARGIN * 1e-10]
    e = _norm_err(vg[[kg[k] for k in common]], vo[[ko[k] for k in common]])
    noise = np.zeros(len(common))
    seen = np.zeros(len(common), int)
    for op in ops:
        ip, vp = op.joints(P, 1e-10, lo, hi, cap=1 << 21)
        kp = {tuple(k): n for n, k in enumerate(ip.tolist())}
        has = [n for n, k in enumerate(common) if k in kp]
        en = _norm_err(vp[[kp[common[n]] for n in has]], vo[[ko[common[n]] for n in has]])
        noise[has] = np.maximum(noise[has], en)
        seen[has] += 1
    keep = seen == len(ops)
    print("pairs in every noisy run:", keep.sum(), "of", len(common))
    e, noise = e[keep], noise[keep]
    r = e / np.maximum(noise, 1e-12)
    print(f"[{lo},{hi}) pairs {len(common)} err q50 {np.median(e):.2e} q99 {np.quantile(e, .99):.2e} max {e.max():.2e}; "
          f"noise q50 {np.median(noise):.2e} max {noise.max():.2e}; err/noise q50 {np.median(r):.2f} q99 {np.quantile(r, .99):.2f} "
          f"max {r.max():.2f}; err where noise<1e-7: max {e[noise < 1e-7].max() if np.any(noise < 1e-7) else 0:.2e}")
