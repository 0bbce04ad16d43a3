"""Generate tests/golden/tauint_quad.json: the integrals the reference's *tauint functions
define (mean_cov_model.h:9-67: int_{t0}^{t1} s^k exp(a s^2 + b s + c) ds, k = 0..3) by adaptive
quadrature (scipy.integrate.quad, epsrel 1e-13), so the GPU box checks the device tauints
without scipy or the oracle.  Cases: the reference's own test inputs (src/tests.h:112-117,
t1 < t0), generic ones, and propagator-like ones (a = Cll/2 ~ 5e-8, b ~ the B values of a step,
t in {0, dt, 2 dt}).  Run: python tests/golden/make_tauint_quad.py"""
import json
import math
import os

from scipy import integrate

CASES = [  # (a, b, c, t0, t1)
    (0.0111, 0.022, 0.01, 0.7, 0.2),       # src/tests.h:112-117: tauint(t1=0.2, t0=0.7)
    (0.0111, 0.022, 0.01, 0.2, 0.7),
    (0.3, -0.4, 0.5, 0.0, 1.0),
    (0.05, 0.8, -1.0, 1.0, 2.0),
    (4.875e-08, 2.8e-03, 0.74, 0.0, 1.0),  # propagator regime: a = var_lambda-scale / 2, dt = 1
    (4.875e-08, 2.8e-03, 0.74, 1.0, 2.0),
    (4.875e-08, -1.32e-02, 1.48, 0.0, 1.0),
    (2.0e-06, 5.0e-03, 1.5, 1.0, 2.0),
    (1.0e-3, 0.5, -0.3, 0.0, 0.25),
]


def main():
    out = {"note": "int_{t0}^{t1} s^k exp(a s^2 + b s + c) ds by scipy quad (epsrel 1e-13)", "cases": []}
    for a, b, c, t0, t1 in CASES:
        for k in range(4):
            v, err = integrate.quad(lambda s: s ** k * math.exp(a * s * s + b * s + c), t0, t1,
                                    epsabs=0, epsrel=1e-13, limit=400)
            out["cases"].append({"k": k, "a": a.hex(), "b": b.hex(), "c": c.hex(), "t0": t0.hex(),
                                 "t1": t1.hex(), "value": v.hex(), "err": err})
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tauint_quad.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
