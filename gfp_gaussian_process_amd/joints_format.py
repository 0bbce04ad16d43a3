"""-j output formats.

The reference writes one dense line per start row with 44 fields for EVERY row of the forest
(Joint_vector::write, correlation_tree.h:96-126): O(rows^2) text -- about 21 GB for the
example, infeasible at C5 (SURVEY finding 7).  The CLI's additive -js writes the sparse form
instead: after the same parameter tables, one line per (start row, column) that a joint lands
in, in the reference's add order:

    start_row,column,mean_0..mean_7,<36 upper-triangle covariances>

(the same iostream formatting as the dense file; a joint whose target (cell_id, time) occurs in
several columns appears once per column, as Joint_vector::add stores it in each).

sparse_to_dense rebuilds the reference's dense _joints.csv byte for byte from the sparse file and
the run's _prediction.csv (-j implies -p; that file lists every row's cell_id, parent_id and time
with the same formatting the dense header and rows use), so python_src/correlation_from_joint.py
(:505-544) reads it unchanged.  Streaming: one start row at a time.
"""
from __future__ import annotations

N_FIELDS = 44   # 8 means + 36 upper-triangle covariances


def _prediction_rows(prediction_path: str):
    """(cell_id, parent_id, time text) of every row, in input order"""
    rows, body = [], False
    with open(prediction_path) as f:
        for line in f:
            if body:
                p = line.rstrip("\n").split(",", 3)
                if len(p) >= 3:
                    rows.append((p[0], p[1], p[2]))
            elif line.startswith("cell_id,parent_id,time,"):
                body = True
    return rows


def sparse_to_dense(sparse_path: str, prediction_path: str, out_path: str) -> int:
    """write the dense _joints.csv; returns the number of rows"""
    rows = _prediction_rows(prediction_path)
    nr = len(rows)
    blank = "," * N_FIELDS
    with open(sparse_path) as fin, open(out_path, "w") as out:
        # the parameter tables, verbatim up to the sparse header
        for line in fin:
            if line.startswith("start_row,column,"):
                break
            out.write(line)
        out.write("cell_id,parent_id,time,")
        for r, (cid, _, t) in enumerate(rows):
            out.write(f"{cid}_{t}")
            out.write("," * (N_FIELDS - 1 if r == nr - 1 else N_FIELDS))
        out.write("\n")

        def emit(s: int, cols: dict):
            cid, pid, t = rows[s]
            parts = [f"{cid},{pid},{t}"]
            prev = 0
            for col in sorted(cols):
                parts.append(blank * (col - prev))
                parts.append("," + cols[col])
                prev = col + 1
            parts.append(blank * (nr - prev))
            out.write("".join(parts) + "\n")

        cur, cols = 0, {}
        for line in fin:
            s_txt, c_txt, vals = line.rstrip("\n").split(",", 2)
            s = int(s_txt)
            while cur < s:
                emit(cur, cols)
                cur, cols = cur + 1, {}
            cols[int(c_txt)] = vals          # the last add wins (Joint_vector::add)
        while cur < nr:
            emit(cur, cols)
            cur, cols = cur + 1, {}
    return nr


def read_sparse(sparse_path: str):
    """{(start_row, column): [44 floats]} of a sparse joints file"""
    out, body = {}, False
    with open(sparse_path) as f:
        for line in f:
            if body:
                p = line.rstrip("\n").split(",")
                out[(int(p[0]), int(p[1]))] = [float(v) for v in p[2:]]
            elif line.startswith("start_row,column,"):
                body = True
    return out
