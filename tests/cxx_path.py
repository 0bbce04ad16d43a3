"""Mechanical translation of the reference's C++ path functions into Python (test infrastructure).

Reads function TEXT from /root/reference/src at run time and turns each function body into a Python
function statement for statement: declarations, (chained / compound) assignments, the Eigen comma
initialiser, if / else, counted for loops, return and throw.  Expressions keep their tokens, grouping
and order (C++ and Python share the precedence and left-to-right associativity of + - * /); `a(i)` /
`a(i, j)` element access becomes `a[i]` / `a[i, j]`; `->` becomes `.`; glibc's log / exp / pow /
sqrt are the same calls through Python's math module (`pow(v, 2)` is v*v, as gcc folds it).  The
result is evaluated with Python floats: IEEE double, no fused multiply-add, as the reference's plain
x86-64 build (src/Makefile:2) evaluates it.  Nothing of the reference is stored in this repository.

Eigen 3.3.7 (absent from this image) is stood in for by `Mat`, a dense row-major matrix whose
operations are the ones these functions use, each with Eigen's documented arithmetic:
  * products: coefficient (i, j) = sum over k of a(i, k) * b(k, j).  Every product on the path has
    an inner dimension of at most 2, or one non-zero term per coefficient (the division maps'
    diagonal F), where the order of the sum cannot matter; any other product raises, so no
    summation order is ever assumed;
  * sums, differences, scalar multiples, negation, transpose, block: coefficient-wise;
  * the fixed-size 2x2 determinant m00*m11 - m10*m01 and inverse cofactor * (1/det)
    (Eigen/src/LU/InverseImpl.h compute_inverse_size2_helper);
  * the dynamic-size determinant through the unblocked partial-pivot LU (Eigen/src/LU/PartialPivLU.h:
    pivot on the first largest |a(i,k)|, divide the column by the pivot, rank-1 update; the sign
    times the product of the diagonal) -- likelihood.h:31 takes S as a dynamic MatrixXd;
  * a fixed-size type (Matrix2d, Vector4d) keeps its type across assignments (`S = ... + D`).
These Eigen restatements are the test's own (Eigen is not part of the reference text); they are the
only arithmetic here that is not read from the reference.
"""
from __future__ import annotations

import math
import re

SRC = "/root/reference/src"


class NanError(Exception):
    """std::domain_error("Likelihood is Nan") (likelihood.h:93)"""


class Ref:
    """a `double &` argument"""

    def __init__(self, v=0.0):
        self.v = v


class VecList(list):
    """a std::vector"""

    def size(self):
        return len(self)


FIXED = {"Matrix2d": (2, 2), "Matrix4d": (4, 4), "Vector4d": (4, 1), "Vector2d": (2, 1)}


class Mat:
    __slots__ = ("r", "c", "v", "fixed")

    def __init__(self, r, c, v=None, fixed=False):
        self.r, self.c = r, c
        self.v = list(v) if v is not None else [0.0] * (r * c)
        self.fixed = fixed

    # -- construction / Eigen static constructors --
    @staticmethod
    def typed(tname: str, m: "Mat | None" = None):
        if tname in FIXED:
            r, c = FIXED[tname]
            out = Mat(r, c, fixed=True)
            if m is not None:
                if (m.r * m.c) != r * c:
                    raise AssertionError(f"{tname} from {m.r}x{m.c}")
                out.v = list(m.v)
            return out
        if m is None:
            return Mat(0, 0)
        if tname.startswith("Vector") and m.c != 1 and m.r == 1:
            return Mat(m.c, 1, m.v)
        return Mat(m.r, m.c, m.v)

    def copy(self):
        return Mat(self.r, self.c, self.v, self.fixed)

    # -- element access: (i) linear (vectors, 1x1), (i, j) --
    def _k(self, k):
        if isinstance(k, tuple):
            i, j = k
            if not (0 <= i < self.r and 0 <= j < self.c):
                raise IndexError((i, j, self.r, self.c))
            return i * self.c + j
        if not 0 <= k < self.r * self.c:
            raise IndexError(k)
        return k

    def __getitem__(self, k):
        return self.v[self._k(k)]

    def __setitem__(self, k, val):
        self.v[self._k(k)] = float(val) if not isinstance(val, float) else val

    def size(self):
        return self.r * self.c

    def rows(self):
        return self.r

    def cols(self):
        return self.c

    # -- the comma initialiser: coefficients row by row, or one whole matrix of the same size --
    def comma(self, *vals):
        if len(vals) == 1 and isinstance(vals[0], Mat):
            if vals[0].r * vals[0].c != self.r * self.c:
                raise AssertionError("comma initialiser size")
            self.v = list(vals[0].v)
            return self
        if len(vals) != self.r * self.c:
            raise AssertionError(f"comma initialiser: {len(vals)} values for {self.r}x{self.c}")
        self.v = [float(x) for x in vals]
        return self

    # -- arithmetic --
    def __add__(self, o):
        if not isinstance(o, Mat) or (o.r, o.c) != (self.r, self.c):
            raise AssertionError("sum of different shapes")
        return Mat(self.r, self.c, [a + b for a, b in zip(self.v, o.v)])

    def __sub__(self, o):
        if not isinstance(o, Mat) or (o.r, o.c) != (self.r, self.c):
            raise AssertionError("difference of different shapes")
        return Mat(self.r, self.c, [a - b for a, b in zip(self.v, o.v)])

    def __neg__(self):
        return Mat(self.r, self.c, [-a for a in self.v])

    def __rmul__(self, s):
        if isinstance(s, Mat):
            return s.__mul__(self)
        s = float(s)
        return Mat(self.r, self.c, [s * a for a in self.v])

    def __mul__(self, o):
        if not isinstance(o, Mat):
            o = float(o)
            return Mat(self.r, self.c, [a * o for a in self.v])
        if self.c != o.r:
            raise AssertionError(f"product {self.r}x{self.c} * {o.r}x{o.c}")
        out = Mat(self.r, o.c)
        for i in range(self.r):
            for j in range(o.c):
                terms = [self.v[i * self.c + k] * o.v[k * o.c + j] for k in range(self.c)]
                if self.c > 2 and sum(1 for t in terms if t != 0.0) > 1:
                    raise AssertionError("a product whose value depends on Eigen's summation order")
                acc = terms[0]
                for t in terms[1:]:
                    acc = acc + t
                out.v[i * o.c + j] = acc
        return out

    def transpose(self):
        return Mat(self.c, self.r, [self.v[i * self.c + j] for j in range(self.c) for i in range(self.r)])

    def block(self, i0, j0, r, c):
        return Mat(r, c, [self.v[(i0 + i) * self.c + (j0 + j)] for i in range(r) for j in range(c)])

    def determinant(self):
        if (self.r, self.c) != (2, 2):
            raise AssertionError("determinant: 2x2 only")
        a00, a01, a10, a11 = self.v
        if self.fixed:
            return a00 * a11 - a10 * a01
        sign = 1.0                      # PartialPivLU, unblocked
        if abs(a10) > abs(a00):
            a00, a01, a10, a11 = a10, a11, a00, a01
            sign = -1.0
        if a00 != 0.0:
            a10 = a10 / a00
            a11 = a11 - a10 * a01
        return sign * (a00 * a11)

    def inverse(self):
        if not (self.fixed and (self.r, self.c) == (2, 2)):
            raise AssertionError("inverse: the fixed-size 2x2 closed form only")
        invdet = 1.0 / self.determinant()
        a00, a01, a10, a11 = self.v
        return Mat(2, 2, [a11 * invdet, -a01 * invdet, -a10 * invdet, a00 * invdet], fixed=True)


def eig(tname, fn, *args):
    """Eigen::<tname>::<fn>(args)"""
    if fn == "Identity":
        r, c = args
        m = Mat(r, c)
        for i in range(min(r, c)):
            m.v[i * c + i] = 1.0
        return m
    if fn == "Zero":
        r, c = (args[0], 1) if len(args) == 1 else args
        return Mat(r, c)
    raise AssertionError(f"Eigen::{tname}::{fn}")


def ctor(tname, *args):
    """a declaration with constructor arguments: sizes (dynamic) or coefficients (fixed vectors)"""
    if tname in FIXED:
        m = Mat.typed(tname)
        if args:
            m.comma(*args)
        return m
    if tname.startswith("Vector"):
        (n,) = args
        return Mat(n, 1)
    r, c = args
    return Mat(r, c)


def assign(old, new):
    """`lhs = rhs` for a whole Eigen object: the values copied INTO the target object (Eigen's
    assignment; a reference parameter's object is the caller's), a fixed-size target keeping its
    type and shape"""
    if isinstance(new, Mat):
        if not isinstance(old, Mat):
            return new.copy()
        if old.fixed and (new.r * new.c) != (old.r * old.c):
            raise AssertionError("fixed-size assignment of another shape")
        if not old.fixed:
            old.r, old.c = new.r, new.c
        old.v = list(new.v)
        return old
    return new


def as_type(tname, v):
    if tname in ("double",):
        return float(v)
    if tname in ("int", "size_t"):
        return int(v)
    if isinstance(v, Mat):
        return Mat.typed(tname, v)
    return v


# ------------------------------------------------------------------------------------------
# the translator
# ------------------------------------------------------------------------------------------
def strip_comments(text: str) -> str:
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return text.replace("\\\n", " ")


def functions(text: str) -> dict:
    """{name: (ret, params, body)} of every top-level function definition in the text"""
    text = strip_comments(text)
    out = {}
    pat = re.compile(r"(?m)^([A-Za-z_][\w:<>, *&]*?)\s+(\w+)\s*\(([^()]*)\)\s*\{")
    for m in pat.finditer(text):
        ret, name = m.group(1).strip(), m.group(2)
        if ret in ("else", "return") or name in ("if", "for", "while", "switch"):
            continue
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        params = []
        for p in _split_top(m.group(3), ","):
            p = " ".join(p.split())
            if not p:
                continue
            p, _, default = p.partition("=")
            p = p.strip()
            mm = re.match(r"(.*?)([&*]?)\s*(\w+)$", p)
            tname = mm.group(1).replace("const", "").strip().rstrip("&* ").strip()
            params.append((mm.group(3), tname, "&" in p, default.strip() or None))
        out.setdefault(name, (ret, params, text[m.end():i - 1]))
    return out


def _split_top(s: str, sep: str):
    """split at `sep` outside parentheses / braces / brackets"""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == sep and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur))
    return out


_CALLS = {"LOG", "EXP", "POW", "SQRT", "ISNAN", "DAW", "eig", "ctor", "assign", "as_type", "Ref", "VecList",
          "transpose", "inverse", "determinant", "block", "size", "rows", "cols", "is_root", "is_leaf",
          "comma", "copy", "range", "float", "int", "LOGV", "NanError"}


class Translator:
    def __init__(self, funcs: dict):
        self.funcs = funcs
        # `double &` parameters: passed as Ref, read and written as .v
        self.refs = {n: [p[2] and p[1] == "double" for p in f[1]] for n, f in funcs.items()}

    # -- expressions --
    def expr(self, e: str, refvars=()) -> str:
        e = " ".join(e.split())
        assert not re.search(r"(?<![\w.])\d+\s*/\s*\d+(?![\w.eE])", e), f"integer division in {e!r}"
        e = e.replace("->", ".")
        e = re.sub(r"(^|[(,]\s*)\*\s*(?=[A-Za-z_])", r"\1", e)   # *pointer as an argument: the object
        e = re.sub(r"\bstd::isnan\s*\(", "ISNAN(", e)
        e = re.sub(r"\bFaddeeva::Dawson\s*\(", "DAW(", e)
        e = re.sub(r"\bEigen::(\w+)::(\w+)\s*\(", r"eig('\1', '\2', ", e)
        e = re.sub(r"\b(?:std::)?log\s*\(", "LOG(", e)
        e = re.sub(r"\b(?:std::)?exp\s*\(", "EXP(", e)
        e = re.sub(r"\b(?:std::)?pow\s*\(", "POW(", e)
        e = re.sub(r"\b(?:std::)?sqrt\s*\(", "SQRT(", e)
        e = re.sub(r"\bM_PI\b", "PI", e)
        e = re.sub(r"\bnullptr\b", "None", e)
        e = re.sub(r"==\s*None\b", " is None", e)
        e = re.sub(r"!=\s*None\b", " is not None", e)
        e = e.replace("&&", " and ").replace("||", " or ")
        e = re.sub(r"!(?!=)", " not ", e)
        e = re.sub(r"\btrue\b", "True", e)
        e = re.sub(r"\bfalse\b", "False", e)
        e = self._index(e)
        e = self._ref_args(e, refvars)
        return e

    def _index(self, e: str) -> str:
        """`name(args)` where name is not a function: element access name[args]"""
        out, i = [], 0
        while i < len(e):
            m = re.match(r"[A-Za-z_][\w.]*", e[i:])
            if m and (i == 0 or not (e[i - 1].isalnum() or e[i - 1] in "_.'")):
                name = m.group(0)
                j = i + len(name)
                k = j
                while k < len(e) and e[k] == " ":
                    k += 1
                last = name.split(".")[-1]
                if k < len(e) and e[k] == "(" and last not in _CALLS and name not in self.funcs \
                        and name not in ("if", "not", "and", "or", "return"):
                    depth, q = 1, k + 1
                    while depth:
                        depth += {"(": 1, ")": -1}.get(e[q], 0)
                        q += 1
                    inner = self._index(e[k + 1:q - 1])
                    out.append(f"{name}[{inner}]")
                    i = q
                    continue
                out.append(name)
                i = j
                continue
            out.append(e[i])
            i += 1
        return "".join(out)

    def _ref_args(self, e: str, refvars) -> str:
        """a `double &` parameter: its value is name.v, except where it is passed on by reference"""
        for r in refvars:
            e = re.sub(rf"\b{r}\b(?!\.v)", f"{r}.v", e)
        for fname, flags in self.refs.items():
            if not any(flags):
                continue
            for m in list(re.finditer(rf"\b{fname}\(", e)):
                depth, q = 1, m.end()
                while depth:
                    depth += {"(": 1, ")": -1}.get(e[q], 0)
                    q += 1
                args = _split_top(e[m.end():q - 1], ",")
                for k, flag in enumerate(flags):
                    if flag and k < len(args):
                        args[k] = re.sub(r"\.v\s*$", "", args[k].strip())
                e = e[:m.end()] + ", ".join(a.strip() for a in args) + e[q - 1:]
        return e

    # -- statements --
    def block(self, text: str, ind: int, refvars) -> list:
        lines, i, text = [], 0, text.strip()
        while i < len(text):
            while i < len(text) and text[i] in " \n\t;":
                i += 1
            if i >= len(text):
                break
            rest = text[i:]
            m = re.match(r"(if|for)\s*\(", rest)
            if m:
                kw = m.group(1)
                q = i + m.end()
                depth = 1
                while depth:
                    depth += {"(": 1, ")": -1}.get(text[q], 0)
                    q += 1
                cond = text[i + m.end():q - 1]
                body, i = self._body(text, q)
                if kw == "if":
                    lines.append(" " * ind + f"if {self.expr(cond, refvars)}:")
                else:
                    lines.append(" " * ind + f"for {self._for(cond, refvars)}:")
                lines += self.block(body, ind + 4, refvars) or [" " * (ind + 4) + "pass"]
                while True:
                    mm = re.match(r"\s*else\s+if\s*\(", text[i:])
                    if mm:
                        q = i + mm.end()
                        depth = 1
                        while depth:
                            depth += {"(": 1, ")": -1}.get(text[q], 0)
                            q += 1
                        cond = text[i + mm.end():q - 1]
                        body, i = self._body(text, q)
                        lines.append(" " * ind + f"elif {self.expr(cond, refvars)}:")
                        lines += self.block(body, ind + 4, refvars) or [" " * (ind + 4) + "pass"]
                        continue
                    mm = re.match(r"\s*else\b", text[i:])
                    if mm:
                        body, i = self._body(text, i + mm.end())
                        lines.append(" " * ind + "else:")
                        lines += self.block(body, ind + 4, refvars) or [" " * (ind + 4) + "pass"]
                    break
                continue
            # a plain statement, up to ';' outside brackets
            depth, q = 0, i
            while q < len(text) and not (text[q] == ";" and depth == 0):
                depth += {"(": 1, "{": 1, "[": 1, ")": -1, "}": -1, "]": -1}.get(text[q], 0)
                q += 1
            st = text[i:q].strip()
            i = q + 1
            lines += [" " * ind + s for s in self.statement(st, refvars)]
        return lines

    def _body(self, text, q):
        """the statement block after an if / for / else header at q: (body, end)"""
        while text[q] in " \n\t":
            q += 1
        if text[q] == "{":
            depth, k = 1, q + 1
            while depth:
                depth += {"{": 1, "}": -1}.get(text[k], 0)
                k += 1
            return text[q + 1:k - 1], k
        depth, k = 0, q
        while not (text[k] == ";" and depth == 0):
            depth += {"(": 1, ")": -1}.get(text[k], 0)
            k += 1
        return text[q:k + 1], k + 1

    def _for(self, header, refvars):
        m = re.match(r"\s*(?:size_t|int)\s+(\w+)\s*=\s*(.+?);\s*(\w+)\s*<\s*(.+?);\s*(?:\+\+\s*(\w+)|(\w+)\s*\+\+)\s*$",
                     header)
        if not m or m.group(1) != m.group(3) or m.group(1) != (m.group(5) or m.group(6)):
            raise AssertionError(f"for header {header!r}")
        return f"{m.group(1)} in range({self.expr(m.group(2), refvars)}, {self.expr(m.group(4), refvars)})"

    def statement(self, st: str, refvars) -> list:
        st = " ".join(st.split())
        if not st:
            return []
        if st == "return":
            return ["return"]
        if st.startswith("return ") or st.startswith("return("):
            return [f"return {self.expr(st[6:], refvars)}"]
        if st.startswith("throw "):
            return [f"raise NanError({st[6:]!r})"]
        if re.match(r"(_file_\w+|std::cout)\s*<<", st):   # the log lines: their values, in order
            parts = [p for p in _split_stream(st)[1:] if not re.match(r"std::setprecision", p.strip())]
            return [f"LOGV({', '.join(self.expr(p, refvars) for p in parts)})"]
        if re.match(r"_file_\w+\.close\(\)$", st):
            return ["pass"]
        m = re.match(r"(?:const\s+)?(Eigen::\w+|double|int|size_t|bool|std::vector<.*>)\s+(\w+)\s*(.*)$", st)
        if m and not st.startswith("return"):
            tname = m.group(1).replace("Eigen::", "")
            name, rest = m.group(2), m.group(3).strip()
            if tname.startswith("std::vector"):
                if rest.startswith("{"):
                    return [f"{name} = VecList({rest.replace('{', '[').replace('}', ']')})"]
                if rest.startswith("("):
                    return [f"{name} = VecList([0.0] * ({self.expr(rest[1:-1], refvars)}))"]
                return [f"{name} = VecList()"]
            if not rest:
                if tname in ("double", "int", "size_t", "bool"):
                    return [f"{name} = None"]
                return [f"{name} = Mat.typed('{tname}')"]
            if rest.startswith("="):
                return [f"{name} = as_type('{tname}', {self.expr(rest[1:], refvars)})"]
            if rest.startswith("(") and rest.endswith(")"):
                return [f"{name} = ctor('{tname}', {self.expr(rest[1:-1], refvars)})"]
            raise AssertionError(f"declaration {st!r}")
        m = re.match(r"(.+?)\s*<<\s*(.+)$", st)
        if m and "=" not in st.split("<<")[0]:
            vals = _split_top(m.group(2), ",")
            return [f"{self.expr(m.group(1), refvars)}.comma({', '.join(self.expr(v, refvars) for v in vals)})"]
        m = re.match(r"(.+?)\s*([-+*/])=\s*(.+)$", st)
        if m and not re.search(r"[=!<>]$", m.group(1)):
            return [f"{self.expr(m.group(1), refvars)} {m.group(2)}= {self.expr(m.group(3), refvars)}"]
        parts = _split_assign(st)
        if len(parts) > 1:
            value = self.expr(parts[-1], refvars)
            targets = [self.expr(t, refvars) for t in parts[:-1]]
            if all(t.endswith("]") for t in targets):
                return [" = ".join(targets) + f" = {value}"]
            if len(targets) == 1:
                t = targets[0]
                return [f"{t} = assign({t}, {value})"]
            raise AssertionError(f"chained whole-object assignment {st!r}")
        return [self.expr(st, refvars)]

    def function(self, name: str) -> str:
        ret, params, body = self.funcs[name]
        refvars = [p for p, t, r, _ in params if r and t == "double"]
        def dflt(t, d):   # a double parameter's integer default is the double value
            return f"float({d})" if t == "double" else d
        lines = [f"def {name}({', '.join(p if d is None else f'{p}={dflt(t, d)}' for p, t, _, d in params)}):"]
        for p, tname, r, _ in params:   # Eigen arguments taken by value: a copy of the argument
            if not r and tname.startswith("Eigen::"):
                t = tname.replace("Eigen::", "")
                lines.append(f"    {p} = Mat.typed('{t}', {p}) if isinstance({p}, Mat) else {p}")
        lines += self.block(body, 4, refvars) or ["    pass"]
        return "\n".join(lines)


def _split_stream(st):
    out, depth, cur, i = [], 0, [], 0
    while i < len(st):
        ch = st[i]
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if depth == 0 and st.startswith("<<", i):
            out.append("".join(cur))
            cur = []
            i += 2
            continue
        cur.append(ch)
        i += 1
    out.append("".join(cur))
    return out


def _split_assign(st):
    """split `a = b = expr` at top-level single '=' signs"""
    out, depth, cur, i = [], 0, [], 0
    while i < len(st):
        ch = st[i]
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "=" and depth == 0 and (i + 1 >= len(st) or st[i + 1] != "=") and (i == 0 or st[i - 1] not in "=!<>+-*/"):
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
        i += 1
    out.append("".join(cur))
    return out


def load(names_by_file: dict, dawson, log_sink=None) -> dict:
    """translate the named functions of each reference file; returns the namespace"""
    funcs = {}
    for fname, names in names_by_file.items():
        fs = functions(open(f"{SRC}/{fname}").read())
        missing = set(names) - set(fs)
        if missing:
            raise AssertionError(f"{fname}: not found {sorted(missing)}")
        funcs.update({n: fs[n] for n in names})
    tr = Translator(funcs)
    sink = log_sink if log_sink is not None else []
    env = {"Mat": Mat, "eig": eig, "ctor": ctor, "assign": assign, "as_type": as_type, "VecList": VecList,
           "Ref": Ref, "NanError": NanError, "LOG": math.log, "EXP": math.exp, "SQRT": math.sqrt,
           "POW": lambda a, k: a * a if k == 2 else math.pow(a, k), "ISNAN": math.isnan, "DAW": dawson,
           "PI": math.pi, "LOGV": lambda *a: sink.append(a), "_save_ll": False, "_print_level": 0,
           "_iteration": 0}
    src = {}
    for n in funcs:
        src[n] = tr.function(n)
        exec(src[n], env)
    env["__sources__"] = src
    env["__log__"] = sink
    return env


class Cell:
    """MOMAdata's members the path reads (moma_input.h:21-75)"""

    def __init__(self, cell_id, time, log_length, fp, noise_model="scaled", cell_division_model="binomial",
                 fp_auto=0.0):
        self.cell_id = cell_id
        self.parent = self.daughter1 = self.daughter2 = None
        self.time = Mat(len(time), 1, time)
        self.log_length = Mat(len(log_length), 1, log_length)
        self.fp = Mat(len(fp), 1, fp)
        self.noise_model, self.cell_division_model, self.fp_auto = noise_model, cell_division_model, fp_auto
        self.mean_init_forward = Mat(4, 1)
        self.cov_init_forward = Mat(4, 4)
        self.mean_init_backward = Mat(4, 1)
        self.cov_init_backward = Mat(4, 4)
        self.mean = Mat(4, 1)
        self.cov = Mat(4, 4)

    def is_root(self):
        return self.parent is None

    def is_leaf(self):
        return self.daughter1 is None and self.daughter2 is None
