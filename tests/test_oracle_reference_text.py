"""The oracle's propagator against the reference's own expression text, mechanically (verdict r4 6).

mean_cov_model.h's 4 tauint integrals, 4 means, 10 covariances and 16 cross-covariances are plain
double arithmetic; the reference cannot be compiled here (the file needs Eigen 3.3.7 for its `nm`
argument and its callers, and a stand-in header is not allowed), so this test reads the functions'
TEXT from /root/reference/src/mean_cov_model.h at run time, translates each C++ expression to a
Python expression token for token (same grouping and order; `exp`, `sqrt`, `pow` are the same glibc
calls through Python's math module; `pow(v, 2)` is v*v as gcc folds it; `Faddeeva::Dawson` is the
oracle's Dawson, so that the test isolates the expressions; `nm(i)` indexes a list) and evaluates it
with Python floats -- IEEE double, left to right, no fused multiply-add, as the reference's plain
x86-64 build evaluates it.  The oracle's C restatement must give the same bits for every output at
2,000 random states and parameter sets and at the reference test file's inputs.  A restatement typo
(a sign, a swapped b or c argument, a dropped term) shows up as differing bits here.

Build container only: skipped where /root/reference is absent (the GPU box).  Nothing of the
reference is stored in this repository; the translation is made in memory at each run."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

REF = "/root/reference/src/mean_cov_model.h"
pytestmark = [pytest.mark.skipif(not os.path.exists(REF), reason="needs the reference source text"),
              pytest.mark.usefixtures("built")]

_ARGS = "t bx bg bl bq Cxx Cxg Cxl Cxq Cgg Cgl Cgq Cll Clq Cqq ml gl sl2 mq gq sq2 b".split()


def _functions(text: str) -> dict:
    """{name: (params, body)} of every `double name(...) {...}` in the file"""
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = text.replace("\\\n", " ")
    out = {}
    for m in re.finditer(r"\bdouble\s+(\w+)\s*\(([^)]*)\)\s*\{", text):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        params = []
        for p in m.group(2).split(","):
            p = p.strip()
            name, _, default = p.partition("=")
            params.append((name.split()[-1], default.strip() or None))
        out[m.group(1)] = (params, text[m.end():i - 1])
    return out


def _expr(e: str) -> str:
    e = " ".join(e.split())
    # an integer / integer division would truncate in C++ and not in Python: none may occur
    assert not re.search(r"(?<![\w.])\d+\s*/\s*\d+(?![\w.eE])", e), e
    e = e.replace("Faddeeva::Dawson(", "DAW(")
    e = re.sub(r"\bnm\((\d)\)", r"nm[\1]", e)
    e = re.sub(r"\bpow\(", "POW(", e)
    e = re.sub(r"\bexp\(", "EXP(", e)
    e = re.sub(r"\bsqrt\(", "SQRT(", e)
    return e


def _translate(funcs: dict, dawson) -> dict:
    env = {"DAW": dawson, "EXP": math.exp, "SQRT": math.sqrt,
           "POW": lambda a, k: a * a if k == 2 else math.pow(a, k)}
    for name, (params, body) in funcs.items():
        sig = ", ".join(p if d is None else f"{p}={d}" for p, d in params)
        lines = []
        for st in body.split(";"):
            st = st.strip()
            if not st:
                continue
            m = re.match(r"double\s+(\w+)\s*=\s*(.*)$", st, flags=re.S)
            if m:
                lines.append(f"    {m.group(1)} = {_expr(m.group(2))}")
            elif st.startswith("return"):
                lines.append(f"    return {_expr(st[len('return'):])}")
            else:
                raise AssertionError(f"{name}: unexpected statement {st[:60]!r}")
        exec(f"def {name}({sig}):\n" + "\n".join(lines), env)
    return env


@pytest.fixture(scope="module")
def ref_model():
    from oracle import oracle as O
    funcs = _functions(open(REF).read())
    want = {"zerotauint", "onetauint", "twotauint", "treetauint", "mean_x", "mean_g", "mean_l", "mean_q",
            "cov_xx", "cov_xg", "cov_xl", "cov_xq", "cov_gg", "cov_gl", "cov_gq", "cov_ll", "cov_lq", "cov_qq"}
    want |= {f"cross_c{a}{b}" for a in "xglq" for b in "xglq"}
    assert want <= set(funcs), want - set(funcs)
    return _translate({k: funcs[k] for k in want}, O.dawson)


def _states(n, seed=2024):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        m = np.array([rng.uniform(0.3, 3.0), rng.uniform(1e3, 1e5), rng.uniform(1e-3, 5e-2), rng.uniform(10, 200)])
        d = np.array([10 ** rng.uniform(-6, -2), 10 ** rng.uniform(2, 7), 10 ** rng.uniform(-9, -6), 10 ** rng.uniform(0, 3)])
        R = np.eye(4)
        for i in range(4):
            for j in range(i + 1, 4):
                R[i, j] = R[j, i] = rng.uniform(-0.5, 0.5)
        C = R * np.sqrt(np.outer(d, d))
        t = float(rng.choice([1.0, 0.5, 2.0, rng.uniform(0.1, 5.0)]))
        base = np.array([2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04])
        p7 = base * 10 ** rng.uniform(-0.3, 0.3, 7)
        out.append((m, C, t, p7))
    return out


def _ref_mcm(R, m, C, t, p):
    a = dict(zip(_ARGS, [t, *m, C[0, 0], C[0, 1], C[0, 2], C[0, 3], C[1, 1], C[1, 2], C[1, 3], C[2, 2], C[2, 3],
                         C[3, 3], *p]))
    args = [a[k] for k in _ARGS]
    nm = [R["mean_x"](*args), R["mean_g"](*args), R["mean_l"](*args), R["mean_q"](*args)]
    nC = np.zeros((4, 4))
    names = {(0, 1): "xg", (0, 2): "xl", (0, 3): "xq", (1, 2): "gl", (1, 3): "gq", (2, 3): "lq",
             (0, 0): "xx", (1, 1): "gg", (2, 2): "ll", (3, 3): "qq"}
    for (i, j), s in names.items():
        f = R[f"cov_{s}"]
        v = f(*args, nm) if s in ("xg", "gg", "gl", "gq") else f(*args)
        nC[i, j] = nC[j, i] = v
    K = np.zeros((4, 4))
    for i, u in enumerate("xglq"):
        for j, w in enumerate("xglq"):
            f = R[f"cross_c{u}{w}"]
            K[i, j] = f(*args, nm) if u == "g" and w in "xglq" and f.__code__.co_argcount == 23 else f(*args)
    return np.array(nm), nC, K


def _same(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.array_equal(a.view(np.int64), b.view(np.int64)) or np.array_equal(a, b, equal_nan=True)


def test_tauint_bitwise_against_the_reference_text(ref_model):
    from oracle import oracle as O
    rng = np.random.default_rng(7)
    names = ["zerotauint", "onetauint", "twotauint", "treetauint"]
    n = 0
    for _ in range(2000):
        a = 10 ** rng.uniform(-9, -5)
        b = rng.uniform(-0.1, 0.1)
        c = rng.uniform(-3, 5)
        t1, t0 = (rng.uniform(0.1, 5), 0.0) if rng.random() < 0.7 else (rng.uniform(0.1, 5), rng.uniform(0.1, 5))
        for k in range(4):
            r = ref_model[names[k]](a, b, c, t1, t0)
            o = O.tauint(k, a, b, c, t1, t0)
            assert _same(r, o), (names[k], a, b, c, t1, t0, r, o)
            n += 1
    # the reference test file's reversed interval (tests.h:112-117: t1 = 0.2 < t0 = 0.7)
    for k in range(4):
        assert _same(ref_model[names[k]](0.5, 0.3, 0.1, 0.2, 0.7), O.tauint(k, 0.5, 0.3, 0.1, 0.2, 0.7))
    assert n == 8000


def test_mean_cov_model_and_cross_cov_bitwise_against_the_reference_text(ref_model):
    """mean_cov_model.h:211-274 (nm first, the covariances from it) and cross_cov_model
    (:380-432) at 2,000 random states / parameter sets and the reference test's
    mean_cov_model(cell, 1, 1, 2, 3, 4, 5, 6, 7) parameters (tests.h:190-221): every bit equal"""
    from oracle import oracle as O
    cases = _states(2000)
    rng = np.random.default_rng(5)
    m0, C0 = np.array([1.0, 2.0, 3.0, 4.0]), np.diag([0.1, 0.2, 0.3, 0.4])
    cases.append((m0, C0, 1.0, np.array([1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0])))
    diffs = 0
    for m, C, t, p in cases:
        nm, nC, K = _ref_mcm(ref_model, m, C, t, p)
        om, oC = O.mean_cov_model(m, C, t, p)
        oK = np.zeros(16)
        Cf = np.ascontiguousarray(C, np.float64).reshape(16)
        O.lib().ora_cross_cov_model(O._dp(np.ascontiguousarray(m)), O._dp(Cf), float(t), O._dp(np.ascontiguousarray(p)),
                                    O._dp(oK))
        ok = _same(nm, om) and _same(nC, oC) and _same(K, oK.reshape(4, 4))
        diffs += not ok
        assert ok, (m, C, t, p, nm - om, nC - oC, K - oK.reshape(4, 4))
    assert diffs == 0 and len(cases) == 2001
    del rng
