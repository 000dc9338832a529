"""How many hoisted tapes of an EVM-shaped workload are flat conjunctions once an atom may compare
a constant with a UNARY function of one variable (a chain of constant-operand ops) — sizing the
flat kernel's unary atoms (CPU only).

    python tools/flat_shapes.py c3|c5 [n_tapes]
"""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])

from mythril_amd import synth_evm  # noqa: E402
from mythril_amd.tape import Op  # noqa: E402

PRED = {Op.EQ, Op.ULT, Op.ULE, Op.SLT, Op.SLE}
UNARY_C = {Op.LSHR, Op.SHL, Op.ASHR, Op.BAND, Op.BOR, Op.BXOR, Op.UREM, Op.UDIV, Op.SMOD, Op.SREM, Op.SDIV,
           Op.ADD, Op.SUB, Op.MUL}


def unary_chain(nd, i, ops):
    """Node i as f(var) with f a chain of unary / constant-operand ops: the var, else None."""
    n = nd[i]
    op = Op(int(n["op"]))
    if op == Op.VAR and n["width"] > 0:
        return int(n["a"])
    if op in (Op.EXTRACT, Op.ZEXT, Op.SEXT, Op.BNOT, Op.NEG):
        ops.append((op.name, int(n["width"])))
        return unary_chain(nd, int(n["a"]), ops)
    if op in UNARY_C:
        a, b = nd[int(n["a"])], nd[int(n["b"])]
        if b["op"] == Op.CONST:
            ops.append((op.name, "c"))
            return unary_chain(nd, int(n["a"]), ops)
        if a["op"] == Op.CONST and op in (Op.ADD, Op.MUL, Op.BAND, Op.BOR, Op.BXOR, Op.SUB):
            ops.append((op.name, "c"))
            return unary_chain(nd, int(n["b"]), ops)
    return None


def atoms(nd, i, out):
    n = nd[i]
    op = Op(int(n["op"]))
    if op in (Op.AND, Op.OR):
        return atoms(nd, int(n["a"]), out) and atoms(nd, int(n["b"]), out)
    if op == Op.NOT:
        return atoms(nd, int(n["a"]), out)
    if op == Op.VAR and n["width"] == 0:
        out.append(("bool",))
        return True
    if op in PRED:
        a, b = int(n["a"]), int(n["b"])
        for x, y in ((a, b), (b, a)):
            if nd[y]["op"] == Op.CONST:
                ops = []
                v = unary_chain(nd, x, ops)
                if v is not None:
                    out.append(("cmp", tuple(o[0] for o in ops)))
                    return True
        return False
    if op in (Op.TRUE, Op.FALSE):
        return True
    return False


def main():
    cfg = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else (1000 if cfg == "c3" else 256)
    if cfg == "c3":
        tb = synth_evm.c3_workload(n, 64, hoist=True)[0]
    else:
        tb = synth_evm.c3_workload(n, 64, seed=5, n_tx=5, checks_per_tx=(18, 24), n_args=5, hoist=True)[0]
    flat, plain_flat, kinds, fail_ops = 0, 0, collections.Counter(), collections.Counter()
    for t in range(tb.n_tapes):
        nd = tb.tape_nodes(t)
        out = []
        if atoms(nd, len(nd) - 1, out):
            flat += 1
            if all(a[0] == "bool" or not a[1] for a in out):
                plain_flat += 1
            for a in out:
                if a[0] == "cmp":
                    kinds[a[1]] += 1
        else:
            fail_ops[Op(int(nd[-1]["op"])).name] += 1
    print(f"{cfg}: {tb.n_tapes} tapes, flat with unary atoms {flat}, flat as today {plain_flat}")
    print("atom chains:", kinds.most_common(20))
    print("non-flat roots:", fail_ops.most_common(8))


if __name__ == "__main__":
    main()


def distinct(cfg, n):
    """Distinct atoms (node structure hashed per tape-local subtree) and division constants."""
    import numpy as np
    if cfg == "c3":
        tb = synth_evm.c3_workload(n, 64, hoist=True)[0]
    else:
        tb = synth_evm.c3_workload(n, 64, seed=5, n_tx=5, checks_per_tx=(18, 24), n_args=5, hoist=True)[0]
    from mythril_amd.tape import from_words, limbs
    seen, divs = set(), collections.Counter()
    total = 0

    def key(nd, i):
        n_ = nd[i]
        op = int(n_["op"])
        if op == Op.CONST:
            w = int(n_["width"])
            return ("c", from_words(tb.consts[int(n_["a"]):int(n_["a"]) + limbs(w)]), w)
        if op == Op.VAR:
            return ("v", int(n_["a"]), int(n_["width"]))
        ch = []
        for f in ("a", "b"):
            j = int(n_[f])
            if op in (Op.EXTRACT, Op.ZEXT, Op.SEXT) and f == "b":
                ch.append(int(n_["b"]))
                continue
            if j < i:
                ch.append(key(nd, j))
        if op == Op.EXTRACT:
            ch.append(int(n_["c"]))
        return (op, int(n_["width"]), tuple(ch))

    for t in range(tb.n_tapes):
        nd = tb.tape_nodes(t)
        stack = [len(nd) - 1]
        while stack:
            i = stack.pop()
            op = Op(int(nd[i]["op"]))
            if op in (Op.AND, Op.OR):
                stack += [int(nd[i]["a"]), int(nd[i]["b"])]
            elif op == Op.NOT:
                stack.append(int(nd[i]["a"]))
            elif op in PRED:
                total += 1
                seen.add(key(nd, i))
                for j in (int(nd[i]["a"]), int(nd[i]["b"])):
                    while Op(int(nd[j]["op"])) not in (Op.VAR, Op.CONST):
                        o = Op(int(nd[j]["op"]))
                        if o in (Op.UREM, Op.SMOD, Op.UDIV, Op.SDIV, Op.SREM):
                            cb = nd[int(nd[j]["b"])]
                            divs[(o.name, from_words(tb.consts[int(cb["a"]):int(cb["a"]) + limbs(int(cb["width"]))]).bit_length())] += 1
                        j = int(nd[j]["a"])
    print(f"compare atoms {total}, distinct {len(seen)}; divisor bit lengths {sorted(divs.items())}")


if __name__ == "__main__" and len(sys.argv) > 3 and sys.argv[3] != "why":
    distinct(sys.argv[1], int(sys.argv[2]))


def why_not(cfg, n):
    """For tapes that are not flat: the kinds of the conjuncts that break it."""
    if cfg == "c3":
        tb = synth_evm.c3_workload(n, 64, hoist=True)[0]
    else:
        tb = synth_evm.c3_workload(n, 64, seed=5, n_tx=5, checks_per_tx=(18, 24), n_args=5, hoist=True)[0]
    bad = collections.Counter()
    per_tape = []
    for t in range(tb.n_tapes):
        nd = tb.tape_nodes(t)
        stack, nb = [len(nd) - 1], 0
        while stack:
            i = stack.pop()
            op = Op(int(nd[i]["op"]))
            if op == Op.AND:
                stack += [int(nd[i]["a"]), int(nd[i]["b"])]
                continue
            out = []
            if not atoms(nd, i, out):
                nb += 1
                sub = []
                j = i
                while len(sub) < 4:
                    o = Op(int(nd[j]["op"]))
                    sub.append(o.name)
                    if o in (Op.VAR, Op.CONST):
                        break
                    j = int(nd[j]["a"])
                a, b = int(nd[i]["a"]), int(nd[i]["b"])
                kid = (Op(int(nd[a]["op"])).name, Op(int(nd[b]["op"])).name) if op in PRED else ()
                bad[(op.name, kid)] += 1
        per_tape.append(nb)
    print("non-flat conjuncts:", bad.most_common(12))
    print("per tape non-flat conjuncts:", collections.Counter(per_tape).most_common(8))


if __name__ == "__main__" and len(sys.argv) > 3 and sys.argv[3] == "why":
    why_not(sys.argv[1], int(sys.argv[2]))
