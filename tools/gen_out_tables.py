"""Generator (build-time tool, not shipped logic): the outputs of one propagation step
(ggp::outputs in csrc/ggp_prop.h, i.e. mean_cov_model.h:73-208) as a sparse trilinear form

    out_k = sum_e  kappa_e(params) * mono_e(state, t) * basis_e     (+ the -nm_i nm_j of a cov)

read symbolically from the C++ source itself (the expression text of ggp::outputs), expanded
with sympy.  Prints statistics; with --emit writes csrc/ggp_out_tables.inc.
"""
import argparse
import os
import re
import sys

import sympy as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gfp_gaussian_process_amd", "csrc", "ggp_prop.h")

STATE = "bx bg bl bq Cxx Cxg Cxl Cxq Cgg Cgl Cgq Cll Clq Cqq t".split()
# expansion variables: the OU means enter as deviations dl = bl - ml, dq = bq - mq, so the
# expanded polynomial does not cancel bq * I against mq * I (the reference computes (bq - mq) first)
EVARS = "bx bg dl dq Cxx Cxg Cxl Cxq Cgg Cgl Cgq Cll Clq Cqq t".split()
PARAMS = "ml gl sl2 mq gq sq2 k_xl k_xx k_ll k_qq gl2 gq2 gqq2".split()
ITASKS = ("O_2A O_1A O_1B O_2B O_1J O_2J O_1G O_2G O_3C O_4C O_3C2 O_3D2 O_4E O_4E2 O_4C2 O_4F2 "
          "Z_1A Z_2A Z_1B Z_2B Z_1J Z_2J Z_2I Z_5I Z_1G Z_2G Z_3C Z_4C Z_3E Z_4E Z_3E2 Z_3C2 Z_3D2 Z_4E2 "
          "Z_4C2 Z_4F2 Z_6H2 T_2A T_2B T_2J T_2G T_4C T_4C2 H_4C H_4C2").split()
# exp-derived scalars of the step (X slots and the reference's composite sub-expressions)
XBASIS = "r_ebt r_ebglt r_ebgqt r_ebt_gl r_ebglt_gl r_e2bt egl egq u_gl u_gl2 u_gq2 w_xx".split()
OUTS = "nm0 nm1 nm2 nm3 nxx nxg nxl nxq ngg ngl ngq nll nlq nqq".split()


def outputs_text():
    s = open(SRC).read()
    a = s.index("GGP_DEV void outputs(")
    a = s.index("double nm[4];", a)
    b = s.index("#undef DGL", a)
    return s[a:b]


def to_python(body):
    body = re.sub(r"//[^\n]*", "", body)
    body = re.sub(r"if constexpr \(\(PARTS & \d\) != 0\)", "", body)
    body = body.replace("{", " ").replace("}", " ")
    stmts = [x.strip() for x in body.split(";")]
    out = []
    for st in stmts:
        if not st or st.startswith("double nm[4]") or st.startswith("double nxg"):
            continue
        st = re.sub(r"\s+", " ", st)
        st = st.replace("const double ", "")
        st = re.sub(r"nm\[(\d)\]", r"nm\1", st)
        st = re.sub(r"I\[(\w+)\]", r"I_\1", st)
        st = st.replace("S.", "")
        # the reference's composite exp sub-expressions, kept as single values
        st = st.replace("(2 * gl * t - 3 + 4 * egl - (egl * egl))", "w_xx")
        st = st.replace("(1 - (egl * egl))", "u_gl2").replace("(1 - (egq * egq))", "u_gq2")
        st = st.replace("(1 - egl)", "u_gl")
        st = st.replace("/ e2bt", "* r_e2bt")
        out.append(st)
    return out


def symbols():
    env = {}
    for n in STATE + EVARS + PARAMS + XBASIS + ["nm0", "nm1", "nm2", "nm3"]:
        env[n] = sp.Symbol(n)
    for n in ITASKS:
        env["I_" + n] = sp.Symbol("I_" + n)
    for n in ("rgl", "rgq", "r_gl2", "r_gq2", "r_gqq2"):      # reciprocal operands of rdiv (unused)
        env[n] = None
    inv = {env["gl"]: 1 / env["gl"], env["gq"]: 1 / env["gq"], env["gl2"]: 1 / env["gl2"],
           env["gq2"]: 1 / env["gq2"], env["gqq2"]: 1 / env["gqq2"]}
    recip = {"ebt": "r_ebt", "ebglt": "r_ebglt", "ebgqt": "r_ebgqt", "ebt_gl": "r_ebt_gl", "ebglt_gl": "r_ebglt_gl"}
    for k, v in recip.items():
        env[k] = sp.Symbol("DEN_" + k)
        inv[env[k]] = env[v]

    def rdiv(x, d, r):
        return x * inv[d]
    env["rdiv"] = rdiv
    env["DGL"] = lambda x: x / env["gl"]
    env["DGQ"] = lambda x: x / env["gq"]
    return env


def outputs_symbolic():
    env = symbols()
    res = {}
    for st in to_python(outputs_text()):
        lhs, rhs = st.split("=", 1)
        lhs = lhs.strip()
        val = eval(rhs, {}, env)
        if not lhs.startswith("nm"):      # the covariances keep nm_i as values (phase 3)
            env[lhs] = val
        res[lhs] = val
    return env, {k: res[k] for k in OUTS}


def split_term(term, env):
    """term -> (kappa: sympy expr in params and numbers, mono: tuple of state names, basis: tuple)"""
    coeff, factors = term.as_coeff_mul()
    kappa = [coeff]
    mono, basis, nmv = [], [], []
    for f in factors:
        base, e = f.as_base_exp()
        name = str(base)
        if name in PARAMS:
            kappa.append(f)
        elif name in EVARS:
            assert e.is_Integer and e > 0, f
            mono += [name] * int(e)
        elif name in XBASIS or name.startswith("I_"):
            assert e.is_Integer and e > 0, f
            basis += [name] * int(e)
        elif name.startswith("nm"):
            nmv += [name] * int(e)
        else:
            raise ValueError(f"unclassified factor {f} in {term}")
    return sp.Mul(*kappa), tuple(sorted(mono)), tuple(sorted(basis)), tuple(sorted(nmv))


def analyse():
    env, outs = outputs_symbolic()
    table = {}
    for k in OUTS:
        e = sp.expand(outs[k].subs({env["bl"]: env["dl"] + env["ml"], env["bq"]: env["dq"] + env["mq"]}))
        terms = e.as_ordered_terms() if isinstance(e, sp.Add) else [e]
        rows = [split_term(t, env) for t in terms]
        table[k] = rows
    return table


VARS = ["one"] + EVARS                   # V[0] = 1.0 pads unused monomial slots
BASIS = (["one"] + ["I_" + n for n in ITASKS] + XBASIS
         + ["egl*egl", "egl*egq", "egl*u_gl", "egq*egq", "egq*u_gl", "u_gl*u_gl"])
L = 4                                     # terms per lane


def kappa_code(kap, env):
    """kappa = c * prod p^e over PARAMS"""
    c, fac = kap.as_coeff_mul()
    e = [0] * len(PARAMS)
    for f in fac:
        base, ex = f.as_base_exp()
        e[PARAMS.index(str(base))] += int(ex)
    return float(c), tuple(e)


def emit(table):
    """lanes in power-of-two aligned blocks, one block per output (largest first), so that a
    butterfly inside the block (DPP: xor 1, xor 2, half-mirror, mirror) sums the output"""
    env = symbols()
    kappas = []
    outs = []           # per output: (k, [terms], nm pair)
    for k, name in enumerate(OUTS):
        rows = [r for r in table[name] if not r[3]]
        nmrows = [r for r in table[name] if r[3]]
        assert len(nmrows) <= 1
        if nmrows:
            kap, mono, basis, nmv = nmrows[0]
            assert kap == -1 and not mono and not basis and len(nmv) == 2, nmrows
            nm = tuple(OUTS.index(v) for v in nmv)
        else:
            nm = (-1, -1)
        terms = []
        for kap, mono, basis, _ in rows:
            kc = kappa_code(kap, env)
            if kc not in kappas:
                kappas.append(kc)
            v = [VARS.index(x) for x in mono] + [0] * (3 - len(mono))
            bname = "*".join(basis) if basis else "one"
            terms.append((v[0], v[1], v[2], BASIS.index(bname), kappas.index(kc)))
        nl = -(-len(terms) // L)
        bs = 1
        while bs < nl:
            bs *= 2
        assert bs <= 16, (name, bs)
        outs.append((k, terms, nm, bs))
    order = sorted(outs, key=lambda o: -o[3])
    lane_terms = [[] for _ in range(64)]
    block = [1] * 64
    lead = [0] * len(OUTS)
    pos = 0
    for k, terms, nm, bs in order:
        assert pos % bs == 0
        lead[k] = pos
        for j in range(bs):
            block[pos + j] = bs
            lane_terms[pos + j] = terms[j * L:(j + 1) * L]
        pos += bs
    assert pos <= 64, pos
    nms = [o[2] for o in outs]
    assert len(BASIS) <= 64 and len(kappas) < 255
    out = []
    w = out.append
    w("// GENERATED by tools/gen_out_tables.py from ggp::outputs (ggp_prop.h) -- do not edit.")
    w("// The step outputs as  out_k = sum kappa(params) * V[v1] V[v2] V[v3] * Bv[basis]  over the")
    w("// terms of the lanes of output k's block (kOutLead[k], kOutBlock lanes, power-of-two aligned),")
    w("// minus out_nm_i * out_nm_j for a covariance.")
    w("// V  = " + " ".join(VARS))
    w("// Bv = " + " ".join(BASIS))
    w("// kappa params = " + " ".join(PARAMS))
    w(f"constexpr int kOutL = {L}, kOutLanes = {pos}, kOutN = {len(OUTS)}, kOutNV = {len(VARS)}, "
      f"kOutNB = {len(BASIS)}, kOutNK = {len(kappas)}, kOutNP = {len(PARAMS)};")
    w("struct OutTerm { unsigned char v1, v2, v3, basis, kap; };")
    w("constexpr OutTerm kOutTerm[64][kOutL] = {")
    for ln in range(64):
        chunk = lane_terms[ln]
        cells = [f"{{{a}, {b}, {c}, {d}, {e}}}" for a, b, c, d, e in chunk]
        cells += ["{0, 0, 0, 0, 255}"] * (L - len(chunk))     # kap 255: a zero term
        w("    {" + ", ".join(cells) + "},")
    w("};")
    w("constexpr unsigned char kOutBlock[64] = {" + ", ".join(str(x) for x in block) + "};")
    w("constexpr unsigned char kOutLead[kOutN] = {" + ", ".join(str(x) for x in lead) + "};")
    w("constexpr signed char kOutNm[kOutN][2] = {" + ", ".join(f"{{{a}, {b}}}" for a, b in nms) + "};")
    w("struct OutKappa { double c; signed char e[kOutNP]; };")
    w("constexpr OutKappa kOutKappa[kOutNK] = {")
    for c, e in kappas:
        w(f"    {{{c!r}, {{{', '.join(str(x) for x in e)}}}}},")
    w("};")
    path = os.path.join(ROOT, "gfp_gaussian_process_amd", "csrc", "ggp_out_tables.inc")
    open(path, "w").write("\n".join(out) + "\n")
    print("wrote", path, "lanes", pos, "kappas", len(kappas))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--emit", action="store_true")
    args = ap.parse_args()
    table = analyse()
    tot = 0
    monos, bases, kappas = set(), set(), set()
    for k, rows in table.items():
        nm = [r for r in rows if r[3]]
        print(f"{k}: {len(rows)} terms ({len(nm)} with nm)")
        tot += len(rows)
        for kap, mono, basis, nmv in rows:
            monos.add(mono)
            bases.add(basis)
            kappas.add(kap)
    print("total terms", tot, "distinct monomials", len(monos), "distinct bases", len(bases), "distinct kappas", len(kappas))
    print("max mono degree", max(len(m) for m in monos), "max basis degree", max(len(b) for b in bases))
    print("composite bases", sorted(b for b in bases if len(b) > 1))
    if args.emit:
        emit(table)


if __name__ == "__main__":
    main()
