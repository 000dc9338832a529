"""Shapes of the hoisted column programs of an EVM-shaped workload (CPU only): per level, how
many columns are calldata words (a CONCAT of ITE(SLT(i, size), byte_i, 0) bytes, optionally
under EXTRACT / BAND-with-constant, optionally after a variable prefix), keccak columns, and
the rest by root op.  Used to size the calldata-word column kernel (cw.hip).

    python tools/col_shapes.py c4 [n_tapes]
"""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])

from mythril_amd import synth_evm  # noqa: E402
from mythril_amd.tape import Op  # noqa: E402


def byte_item(nd, i):
    n = nd[i]
    if n["op"] != Op.ITE or n["width"] != 8:
        return None
    c, t, e = nd[n["a"]], nd[n["b"]], nd[n["c"]]
    if c["op"] != Op.SLT or t["op"] != Op.VAR or t["width"] != 8 or e["op"] != Op.CONST:
        return None
    k, s = nd[c["a"]], nd[c["b"]]
    if k["op"] != Op.CONST or s["op"] != Op.VAR:
        return None
    return ("byte", int(t["a"]), int(s["a"]))


def pieces(nd, i, out):
    n = nd[i]
    if n["op"] == Op.CONCAT:
        return pieces(nd, n["a"], out) and pieces(nd, n["b"], out)
    b = byte_item(nd, i)
    if b:
        out.append(b)
        return True
    if n["op"] == Op.VAR:
        out.append(("var", int(n["width"])))
        return True
    if n["op"] == Op.CONST:
        out.append(("const", int(n["width"])))
        return True
    return False


def classify(nd):
    r = len(nd) - 1
    n = nd[r]
    wrap = ""
    if n["op"] == Op.EXTRACT:
        wrap, r = "extract", int(n["a"])
    elif n["op"] == Op.BAND and nd[n["b"]]["op"] == Op.CONST:
        wrap, r = "band", int(n["a"])
    if nd[r]["op"] != Op.CONCAT and byte_item(nd, r) is None:
        return "root:" + Op(int(nd[len(nd) - 1]["op"])).name
    out = []
    if not pieces(nd, r, out) or not any(p[0] == "byte" for p in out):
        return "root:" + Op(int(nd[len(nd) - 1]["op"])).name
    kinds = "".join("b" if p[0] == "byte" else ("v" if p[0] == "var" else "c") for p in out)
    pre = kinds.rstrip("b")
    return f"cw[{wrap or '-'}] prefix={pre or '-'} bytes={kinds.count('b')}"


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else {"c3": 1000, "c4": 200, "c5": 256}[cfg]
    if cfg == "c4":
        import numpy as np
        from mythril_amd.evaluator import keccak256_host

        def hasher(a):
            return np.frombuffer(b"".join(keccak256_host([bytes(r) for r in a])), np.uint8).reshape(-1, 32)
        tb, _, _, _ = synth_evm.c4_workload(n, 256, seed=4, interpret_keccak=True, hoist=True, hasher_many=hasher)
    elif cfg == "c5":
        tb, _, _, _ = synth_evm.c3_workload(n, 256, seed=5, n_tx=5, checks_per_tx=(18, 24), n_args=5, hoist=True)
    else:
        tb, _, _, _ = synth_evm.c3_workload(n, 256, seed=3, hoist=True)
    cols = tb.columns
    progs = cols.programs
    per = collections.defaultdict(collections.Counter)
    nodes = collections.Counter()
    for k in range(cols.n):
        nd = progs.tape_nodes(k)
        shape = classify(nd)
        per[int(cols.level[k])][shape.split(" bytes")[0] if shape.startswith("cw") else shape] += 1
        nodes[shape.startswith("cw")] += len(nd)
    for lv in sorted(per):
        print(f"level {lv}: {sum(per[lv].values())} columns")
        for s, c in per[lv].most_common():
            print(f"   {c:5d}  {s}")
    print("nodes in calldata-word columns:", nodes[True], "other:", nodes[False])


if __name__ == "__main__":
    main()
