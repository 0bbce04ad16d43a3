"""Static instruction mix between s_memtime stamps of a kernel in a GGP_STAMPS assembly
listing (diagnostic): python tools/isa_segments.py file.s kernel_symbol_substring.
A -DGGP_MARKS listing puts ";@mark k" comments at the same points without stamps (the
shipped schedule, approximately: nothing pins instructions to the marks)."""
import sys
from collections import Counter

src, sym = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
inside, body = False, []
for ln in lines:
    if ln.startswith("_Z") and sym in ln.split(":")[0] and ":" in ln:
        inside = True
        continue
    if inside:
        if "s_endpgm" in ln:
            break
        body.append(ln.strip())
seg, segs = 0, {0: []}
for t in body:
    if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
        continue
    op = t.split()[0]
    if op == "s_memtime":
        seg += 1
        segs[seg] = []
        continue
    segs[seg].append(op)
for k, ops in segs.items():
    c = Counter(ops)
    f64 = sum(v for o, v in c.items() if "_f64" in o)
    valu = sum(v for o, v in c.items() if o.startswith("v_"))
    ds = sum(v for o, v in c.items() if o.startswith("ds_"))
    print(f"seg {k:2d}: {len(ops):5d} instr  valu {valu:4d} (f64 {f64:4d})  ds {ds:3d}  "
          f"waitcnt {c['s_waitcnt']:3d}  top: " + ", ".join(f"{o} {v}" for o, v in c.most_common(6)))
