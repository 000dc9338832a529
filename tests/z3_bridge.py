"""TEST INFRASTRUCTURE — re-expresses z3-free terms (mythril_amd.smt) and model records
(smt_model.Model) in the z3 stand-in (tests/fake_z3.py), so the workloads the drop-in tests and
bench legs already have (synth_evm's EVM-shaped paths, their fork children, their cached models)
can be replayed through the path a Mythril install takes: ``check_quick_sat`` on z3 ``BoolRef``
(model.py:101) over models read from ``z3.ModelRef`` (smt/model.py:13-18, ``Model.raw``).

Identity is preserved the way z3 preserves it: the stand-in hash-conses its ASTs, so a term
shared by two paths becomes ONE AST (what z3's AST table does for LASER's forked states).
Parity of the stand-in with real z3 is unpinned (tests/fake_z3.py)."""
from __future__ import annotations

from typing import Dict, Sequence

import fake_z3 as Z
from mythril_amd import smt as S

C = Z.C

_BV2 = {S.ADD: C.Z3_OP_BADD, S.SUB: C.Z3_OP_BSUB, S.MUL: C.Z3_OP_BMUL, S.UDIV: C.Z3_OP_BUDIV,
        S.UREM: C.Z3_OP_BUREM, S.SDIV: C.Z3_OP_BSDIV, S.SREM: C.Z3_OP_BSREM, S.SMOD: C.Z3_OP_BSMOD,
        S.BAND: C.Z3_OP_BAND, S.BOR: C.Z3_OP_BOR, S.BXOR: C.Z3_OP_BXOR, S.SHL: C.Z3_OP_BSHL,
        S.LSHR: C.Z3_OP_BLSHR, S.ASHR: C.Z3_OP_BASHR}
_PRED = {S.BVULT: C.Z3_OP_ULT, S.BVULE: C.Z3_OP_ULEQ, S.BVSLT: C.Z3_OP_SLT, S.BVSLE: C.Z3_OP_SLEQ,
         S.UMUL_NOOVFL: C.Z3_OP_BUMUL_NO_OVFL, S.SMUL_NOOVFL: C.Z3_OP_BSMUL_NO_OVFL,
         S.SMUL_NOUDFL: C.Z3_OP_BSMUL_NO_UDFL}


def _sort(t: S.Term):
    if t.sort == "bool":
        return Z.BoolSort()
    if t.sort == "bv":
        return Z.BitVecSort(t.width)
    rng = Z.BoolSort() if t.width == 0 else Z.BitVecSort(t.width)
    return Z.ArraySort(Z.BitVecSort(t.domain), rng)


class ToZ3:
    """Term -> stand-in AST, memoized per term (interned terms: one AST per distinct term)."""

    def __init__(self) -> None:
        self.memo: Dict[int, object] = {}
        self.keep: Dict[int, S.Term] = {}

    def __call__(self, root: S.Term):
        memo = self.memo
        for t in S.walk(root):
            if id(t) in memo:
                continue
            memo[id(t)] = self._one(t, [memo[id(a)] for a in t.args])
            self.keep[id(t)] = t
        return memo[id(root)]

    @staticmethod
    def _one(t: S.Term, a):
        k = t.kind
        if k == S.SYM:
            return Z.Bool(t.params[0]) if t.sort == "bool" else Z.BitVec(t.params[0], t.width)
        if k == S.VAL:
            return Z.BitVecVal(t.params[0], t.width)
        if k in (S.TRUE, S.FALSE):
            return Z.BoolVal(k == S.TRUE)
        if k == S.NOT:
            return Z.Not(a[0])
        if k == S.AND:
            return Z.And(*a)
        if k == S.OR:
            return Z.Or(*a)
        if k == S.XOR:
            return Z.bool_op(C.Z3_OP_XOR, *a)
        if k == S.IMPLIES:
            return Z.bool_op(C.Z3_OP_IMPLIES, *a)
        if k in (S.IFF, S.EQ):
            return Z.Eq(a[0], a[1])
        if k in (S.BITE, S.ITE):
            return Z.If(a[0], a[1], a[2])
        if k in _PRED:
            return Z.bool_op(_PRED[k], a[0], a[1])
        if k in _BV2:
            return Z.bv_op(_BV2[k], a[0], a[1])
        if k == S.NEG:
            return Z.bv_op(C.Z3_OP_BNEG, a[0])
        if k == S.BNOT:
            return Z.bv_op(C.Z3_OP_BNOT, a[0])
        if k == S.EXTRACT:
            return Z.Extract(t.params[0], t.params[1], a[0])
        if k == S.CONCAT:
            return Z.Concat(*a)
        if k == S.ZEXT:
            return Z.ZeroExt(t.params[0], a[0])
        if k == S.SEXT:
            return Z.SignExt(t.params[0], a[0])
        if k == S.ARRAY_SYM:
            s = _sort(t)
            return Z.Array(t.params[0], s.domain(), s.range())
        if k == S.CONST_ARRAY:
            return Z.K(Z.BitVecSort(t.domain), a[0])
        if k == S.STORE:
            return Z.Store(a[0], a[1], a[2])
        if k == S.SELECT:
            return Z.Select(a[0], a[1])
        if k == S.APP:
            name, dom = t.params
            rng = Z.BoolSort() if t.sort == "bool" else Z.BitVecSort(t.width)
            return Z.Function(name, *[Z.BitVecSort(w) for w in dom], rng)(*a)
        raise ValueError(f"no z3 form for term kind {k!r}")


def signature(roots: Sequence[S.Term]) -> Dict[str, tuple]:
    """name -> ("bv", w) | ("bool",) | ("array", dom, rng) | ("func", dom, rng) over the terms."""
    sig: Dict[str, tuple] = {}
    seen = set()
    for r in roots:
        for t in S.walk(r):
            if id(t) in seen:
                continue
            seen.add(id(t))
            if t.kind == S.SYM:
                sig[t.params[0]] = ("bool",) if t.sort == "bool" else ("bv", t.width)
            elif t.kind == S.ARRAY_SYM:
                sig[t.params[0]] = ("array", t.domain, t.width)
            elif t.kind == S.APP:
                sig[t.params[0]] = ("func", tuple(t.params[1]), t.width)
    return sig


def _lit(v, w):
    return Z.BoolVal(bool(v)) if w == 0 else Z.BitVecVal(int(v), w)


class Wrapped:
    """A mythril ``Model``: ``.raw`` = [ModelRef] (smt/model.py:13-18), hashed by identity."""

    def __init__(self, m):
        self.raw = [m]


def model_to_z3(rec, sig: Dict[str, tuple]) -> Wrapped:
    """The stand-in ``ModelRef`` holding ``rec``'s interpretations (arrays as ``as-array`` of a
    ``FuncInterp``, the form z3 returns them in), wrapped like a mythril ``Model``."""
    m = Z.ModelRef()
    for name, v in rec.assignment.items():
        s = sig.get(name)
        if s is None:
            continue
        if s[0] == "bool":
            m.set(Z.Bool(name).decl(), Z.BoolVal(bool(v)))
        else:
            m.set(Z.BitVec(name, s[1]).decl(), Z.BitVecVal(int(v), s[1]))
    for name, (entries, els) in rec.functions.items():
        s = sig.get(name)
        if s is None:
            continue
        if s[0] == "array":
            _, dom, rng = s
            rs = Z.BoolSort() if rng == 0 else Z.BitVecSort(rng)
            f = Z.FuncDeclRef(f"{name}!as", C.Z3_OP_UNINTERPRETED, (), (Z.BitVecSort(dom),), rs)
            ents = [Z.FuncEntry([Z.BitVecVal(k[0], dom)], _lit(v, rng)) for k, v in entries.items()]
            m.set(f, Z.FuncInterp(1, ents, _lit(els, rng)))
            m.set(Z.Array(name, Z.BitVecSort(dom), rs).decl(), Z.AsArray(f))
        else:
            _, dom, rng = s
            rs = Z.BoolSort() if rng == 0 else Z.BitVecSort(rng)
            f = Z.Function(name, *[Z.BitVecSort(w) for w in dom], rs)
            ents = [Z.FuncEntry([Z.BitVecVal(x, w) for x, w in zip(k, dom)], _lit(v, rng)) for k, v in entries.items()]
            m.set(f, Z.FuncInterp(len(dom), ents, _lit(els, rng)))
    return Wrapped(m)


def reference_replay(exprs, models, lz3):
    """The reference loop (support_utils.py:60-67: MRU first, bump on hit, per-expression memo)
    on the stand-in's own evaluator (``z3_quick_sat_loop`` over ``Model.raw``): the answers and
    the final MRU-first order.  ``models``: the cache's initial order, MRU first."""
    order = list(models)
    memo, out = {}, []
    for e in exprs:
        if e in memo:
            out.append(memo[e])
            continue
        hit = lz3.z3_quick_sat_loop(e, [m.raw[0] for m in order])
        ans = False if hit is False else next(m for m in order if m.raw[0] is hit)
        if ans is not False:
            order.remove(ans)
            order.insert(0, ans)
        memo[e] = ans
        out.append(ans)
    return out, order
