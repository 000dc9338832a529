"""TEST INFRASTRUCTURE — a direct evaluator of z3-free terms (mythril_amd.smt) under a model,
independent of the product lowering (lower.py), the tape format and the tape oracle.

It restates ``is_true(model.eval(expr, model_completion=True))`` (support_utils.py:64) on the term
DAG itself with Python big ints: SMT-LIB 2.6 FixedSizeBitVectors + z3 model completion (SURVEY
Appendix A): an absent constant is 0 / false, an absent function or array interpretation has no
entries and else value 0, UF / as-array lookups match argument tuples exactly, then fall back to
the else value.  The drop-in GPU tests compare the product against the reference's sequential
loop (tests/oracle_engine.py:ReferenceLoopCache) built on THIS evaluator, so a bug in lowering or
model serialization cannot hide behind a shared code path."""
from __future__ import annotations

from mythril_amd import smt as S


def _m(w):
    return (1 << w) - 1


def _s(v, w):
    return v - (1 << w) if v >> (w - 1) & 1 else v


def _udiv(a, b, w):
    return _m(w) if b == 0 else a // b


def _urem(a, b):
    return a if b == 0 else a % b


def _sdiv(a, b, w):
    sa, sb = _s(a, w), _s(b, w)
    if sb == 0:
        return 1 if sa < 0 else _m(w)
    q = abs(sa) // abs(sb)
    return (-q if (sa < 0) != (sb < 0) else q) & _m(w)


def _srem(a, b, w):
    sa, sb = _s(a, w), _s(b, w)
    if sb == 0:
        return a
    r = abs(sa) % abs(sb)
    return (-r if sa < 0 else r) & _m(w)


def _smod(a, b, w):
    sa, sb = _s(a, w), _s(b, w)
    if sb == 0:
        return a
    r = abs(sa) % abs(sb)
    if r == 0:
        return 0
    if sa < 0 and sb > 0:
        return (sb - r) & _m(w)
    if sa >= 0 and sb < 0:
        return (r + sb) & _m(w)
    if sa < 0 and sb < 0:
        return (-r) & _m(w)
    return r


def evaluate(expr: S.Term, model) -> object:
    """Value of ``expr`` under ``model`` (smt_model.Model) with completion: int for bit-vectors,
    bool for Bool, ("array", base, stores) for arrays."""
    asg, funcs = model.assignment, model.functions
    val = {}
    for t in S.walk(expr):
        k, w, a = t.kind, t.width, [val[id(x)] for x in t.args]
        if k == S.SYM:
            v = asg.get(t.params[0])
            r = (bool(v) if v is not None else False) if t.sort == "bool" else (int(v) & _m(w) if v is not None else 0)
        elif k == S.VAL:
            r = t.params[0]
        elif k == S.TRUE:
            r = True
        elif k == S.FALSE:
            r = False
        elif k == S.NOT:
            r = not a[0]
        elif k == S.AND:
            r = all(a)
        elif k == S.OR:
            r = any(a)
        elif k == S.XOR:
            r = a[0] != a[1]
        elif k == S.IMPLIES:
            r = (not a[0]) or a[1]
        elif k == S.IFF:
            r = a[0] == a[1]
        elif k == S.BITE or k == S.ITE:
            r = a[1] if a[0] else a[2]
        elif k == S.EQ:
            r = a[0] == a[1]
        elif k == S.BVULT:
            r = a[0] < a[1]
        elif k == S.BVULE:
            r = a[0] <= a[1]
        elif k == S.BVSLT:
            r = _s(a[0], t.args[0].width) < _s(a[1], t.args[0].width)
        elif k == S.BVSLE:
            r = _s(a[0], t.args[0].width) <= _s(a[1], t.args[0].width)
        elif k == S.UMUL_NOOVFL:
            r = a[0] * a[1] <= _m(t.args[0].width)
        elif k == S.SMUL_NOOVFL:
            aw = t.args[0].width
            r = _s(a[0], aw) * _s(a[1], aw) <= (1 << (aw - 1)) - 1
        elif k == S.SMUL_NOUDFL:
            aw = t.args[0].width
            r = _s(a[0], aw) * _s(a[1], aw) >= -(1 << (aw - 1))
        elif k == S.ADD:
            r = (a[0] + a[1]) & _m(w)
        elif k == S.SUB:
            r = (a[0] - a[1]) & _m(w)
        elif k == S.MUL:
            r = (a[0] * a[1]) & _m(w)
        elif k == S.NEG:
            r = (-a[0]) & _m(w)
        elif k == S.UDIV:
            r = _udiv(a[0], a[1], w)
        elif k == S.UREM:
            r = _urem(a[0], a[1])
        elif k == S.SDIV:
            r = _sdiv(a[0], a[1], w)
        elif k == S.SREM:
            r = _srem(a[0], a[1], w)
        elif k == S.SMOD:
            r = _smod(a[0], a[1], w)
        elif k == S.BAND:
            r = a[0] & a[1]
        elif k == S.BOR:
            r = a[0] | a[1]
        elif k == S.BXOR:
            r = a[0] ^ a[1]
        elif k == S.BNOT:
            r = ~a[0] & _m(w)
        elif k == S.SHL:
            r = 0 if a[1] >= w else (a[0] << a[1]) & _m(w)
        elif k == S.LSHR:
            r = 0 if a[1] >= w else a[0] >> a[1]
        elif k == S.ASHR:
            r = (_s(a[0], w) >> min(a[1], w)) & _m(w)
        elif k == S.EXTRACT:
            hi, lo = t.params
            r = (a[0] >> lo) & _m(hi - lo + 1)
        elif k == S.CONCAT:
            r = (a[0] << t.args[1].width) | a[1]
        elif k == S.ZEXT:
            r = a[0]
        elif k == S.SEXT:
            r = _s(a[0], t.args[0].width) & _m(w)
        elif k == S.ARRAY_SYM:
            interp = funcs.get(t.params[0])
            r = ("array", ("table", interp), ())
        elif k == S.CONST_ARRAY:
            r = ("array", ("const", a[0]), ())
        elif k == S.STORE:
            base, stores = a[0][1], a[0][2]
            r = ("array", base, stores + ((a[1], a[2]),))
        elif k == S.SELECT:
            base, stores = a[0][1], a[0][2]
            r = None
            for key, v in reversed(stores):    # the outermost store wins
                if key == a[1]:
                    r = v
                    break
            if r is None:
                if base[0] == "const":
                    r = base[1]
                else:
                    r = _lookup(base[1], (a[1],), t.sort)
        elif k == S.APP:
            r = _lookup(funcs.get(t.params[0]), tuple(a), t.sort)
        else:
            raise ValueError(f"term kind {k!r}")
        val[id(t)] = r
    return val[id(expr)]


def _lookup(interp, args, sort):
    if interp is None:
        return False if sort == "bool" else 0
    table, els = interp
    if args in table:
        v = table[args]
    else:
        v = els
    return bool(v) if sort == "bool" else int(v)


def is_true(expr: S.Term, model) -> bool:
    return evaluate(expr, model) is True
