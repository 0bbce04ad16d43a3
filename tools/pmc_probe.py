"""One forest, one schedule, a few evaluations -- a target for rocprofv3 --pmc passes.

  python3 tools/pmc_probe.py TREES KERNEL CPW [EVALS]
KERNEL lane|group; CPW sets GGP_LANE_CPW / GGP_GROUP_CPW before the engine reads them.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
n, kernel, cpw = int(sys.argv[1]), sys.argv[2], sys.argv[3]
evals = int(sys.argv[4]) if len(sys.argv) > 4 else 3
os.environ["GGP_LANE_CPW" if kernel == "lane" else "GGP_GROUP_CPW"] = cpw
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
f = g.Forest(g.HostForest.synthetic(n, 200), kernel=kernel)
for _ in range(evals):
    v = f.total_likelihood(P)
print(n, kernel, cpw, v)
