"""GPU vs oracle -j diagnosis: per (noise, division) combo, the smoother difference and the
worst joint pairs classified by (same cell / across a division, start at a last row)."""
import sys

import numpy as np

sys.path.insert(0, ".")
import gfp_gaussian_process_amd as g  # noqa: E402
from oracle import oracle as O  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
P_CONST = P[:8] + [2.6e4] + P[9:]   # constant noise needs var_g of the data scale (tests/test_gpu_joints.py)

for noise, div in ((1, 1), (0, 0), (1, 0), (0, 1)):
    hf = g.HostForest.synthetic(4, 40)
    hf.a["noise_scaled"] = noise
    hf.a["division_binomial"] = div
    fg, of = g.Forest(hf), O.OracleForest(hf.a)
    PP = P if noise else P_CONST
    pg = fg.predict(PP)
    po = of.predict(PP)
    for name, a, b in zip(("fwd", "bwd", "comb"), pg, po):
        sd = np.sqrt(np.abs(b[:, 4:].reshape(-1, 4, 4)[:, range(4), range(4)]))
        em = np.max(np.abs(a[:, :4] - b[:, :4]) / (np.abs(b[:, :4]) + sd))
        print(f"noise={noise} div={div} {name}: mean err {em:.2e}")
    ig, vg = fg.joints(PP, 1e-10)
    io, vo = of.joints(PP, 1e-10)
    ro = hf.a["row_offset"]
    cell = np.searchsorted(ro, np.arange(hf.n_rows), "right") - 1
    kg = {tuple(k): n for n, k in enumerate(ig.tolist())}
    ko = {tuple(k): n for n, k in enumerate(io.tolist())}
    common = sorted(set(kg) & set(ko))
    print(f"  pairs gpu {len(kg)} oracle {len(ko)} common {len(common)}")
    errs = []
    for k in common:
        a, b = vg[kg[k]], vo[ko[k]]
        sd = np.sqrt(np.abs(np.diag(b[8:].reshape(8, 8))))
        e = np.max(np.abs(a[:8] - b[:8]) / (np.abs(b[:8]) + sd))
        s, t = k
        last = s == ro[cell[s] + 1] - 1
        errs.append((e, s, t, int(cell[s]), int(cell[t]), bool(last)))
    errs.sort(reverse=True)
    bad = [x for x in errs if x[0] > 1e-6]
    print(f"  bad {len(bad)}: same-cell {sum(1 for x in bad if x[3] == x[4])} start-at-last {sum(1 for x in bad if x[5])}")
    for x in errs[:6]:
        print("   ", "err %.2e start %d target %d cells %d->%d last %s" % x)
        a, b = vg[kg[(x[1], x[2])]], vo[ko[(x[1], x[2])]]
        print("     gpu m", np.array2string(a[:8], precision=5), "\n     ora m", np.array2string(b[:8], precision=5))
