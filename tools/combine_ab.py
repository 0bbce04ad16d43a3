"""k_combine A/B (diagnostic): the -p combine with the oracle's operations (GGP_COMBINE_EXACT=1)
and in its fast form (=0: reciprocal pivots, reassociated mean), alternating, on a C5-shaped forest (500 rows per tree); the
combined rows of the two compared on a sample (means relative to |m| + sd, covariances to
sqrt(Cii Cjj), as tests/test_gpu_parity.py's smoother check).
  python tools/combine_ab.py [TREES]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]


def run(hf, exact, reps=3):
    os.environ["GGP_COMBINE_EXACT"] = str(exact)
    f = g.Forest(hf)
    f.predict(P, outputs=(False, False, False))
    cb = []
    for _ in range(reps):
        f.predict(P, outputs=(False, False, False))
        cb.append(f.predict_profile()[1])
    sample = np.concatenate([f.predict_rows(0, 50000), f.predict_rows(hf.n_rows - 50000, hf.n_rows)])
    f.close()
    return min(cb), sample


if __name__ == "__main__":
    trees = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
    hf = g.HostForest.synthetic(trees, 500)
    ref = None
    out = {"trees": trees, "rows": hf.n_rows, "combine_ms": {}}
    for rnd in range(2):
        for exact in (1, 0):
            ms, smp = run(hf, exact)
            key = "exact" if exact else "fast"
            out["combine_ms"].setdefault(key, []).append(round(ms, 4))
            if ref is None:
                ref = smp
            sd = np.sqrt(np.abs(np.einsum("nii->ni", ref[:, 4:].reshape(-1, 4, 4))))
            em = np.max(np.abs(smp[:, :4] - ref[:, :4]) / (np.abs(ref[:, :4]) + sd).clip(1e-300))
            ec = np.max(np.abs(smp[:, 4:].reshape(-1, 4, 4) - ref[:, 4:].reshape(-1, 4, 4))
                        / (sd[:, :, None] * sd[:, None, :]).clip(1e-300))
            out.setdefault("err_vs_exact", {})[key] = [float(em), float(ec)]
    print(json.dumps(out), flush=True)
