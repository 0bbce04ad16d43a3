"""Diagnostic: the engine loaded BEFORE torch in one process.  Prints the HIP / HSA runtime
copies mapped after each step and whether both libraries still work."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def maps():
    return sorted({ln.split()[-1] for ln in open(f"/proc/{os.getpid()}/maps") if "libamdhip64" in ln or "hsa-runtime" in ln})


import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
f = g.Forest(g.HostForest.synthetic(8, 40))
print("engine first:", f.total_likelihood(P), maps(), flush=True)
import torch  # noqa: E402

x = torch.ones(4, device="cuda") * 2
print("torch after:", float(x.sum()), maps(), flush=True)
print("engine again:", f.total_likelihood(P), flush=True)
f.close()
print("ok", flush=True)
