"""z3 host side of the lowering pass (imported only where ``z3-solver`` exists).

Reference call site: ``model_cache.check_quick_sat(simplify(And(*constraints)).raw)``
(``mythril/support/model.py:101``) hands a z3 ``BoolRef`` to quick-sat, which evaluates it under
each cached ``Model`` (``support_utils.py:62-64``).  This module

* walks that ``BoolRef`` DAG by ``decl().kind()`` into the tape IR, sharing
  sub-terms by ``get_id()``; every kind not listed raises :class:`LoweringError` (fail closed);
* reads a ``mythril.laser.smt.Model`` / ``z3.ModelRef`` WITHOUT completion into the
  :class:`~mythril_amd.smt_model.Model` record (constants; ``FuncInterp`` entries + else value;
  arrays given as ``as-array``, ``K`` or ``Store`` chains over ``K``);
* keeps the reference's own loop (:func:`z3_quick_sat_loop`) for tapes the evaluator rejects, and
  a ``Z3Backend`` that is ``solver_worker`` (model.py:28-65).

z3 is absent from this container and from the GPU box, so this module is exercised only on a
z3 host; its verdicts are checked there against ``z3_quick_sat_loop``.
"""
from __future__ import annotations

from copy import deepcopy
from typing import Dict, List, Sequence, Tuple

import numpy as np
import z3  # noqa: F401  (ImportError here means: no z3 host)
from z3 import z3consts as C

from .exceptions import LoweringError, note_fail_closed
from .lower import SymbolTable, serialize_models
from .smt_model import Model
from .tape import Tape, TapeBatch

_BIN = {C.Z3_OP_BADD: "add", C.Z3_OP_BSUB: "sub", C.Z3_OP_BMUL: "mul",
        C.Z3_OP_BUDIV: "udiv", C.Z3_OP_BUDIV_I: "udiv", C.Z3_OP_BUREM: "urem", C.Z3_OP_BUREM_I: "urem",
        C.Z3_OP_BSDIV: "sdiv", C.Z3_OP_BSDIV_I: "sdiv", C.Z3_OP_BSREM: "srem", C.Z3_OP_BSREM_I: "srem",
        C.Z3_OP_BSMOD: "smod", C.Z3_OP_BSMOD_I: "smod", C.Z3_OP_BAND: "band", C.Z3_OP_BOR: "bor",
        C.Z3_OP_BXOR: "bxor", C.Z3_OP_BSHL: "shl", C.Z3_OP_BLSHR: "lshr", C.Z3_OP_BASHR: "ashr"}
_NARY_BV = {C.Z3_OP_BADD: "add", C.Z3_OP_BMUL: "mul", C.Z3_OP_BAND: "band", C.Z3_OP_BOR: "bor", C.Z3_OP_BXOR: "bxor"}
_PRED = {C.Z3_OP_ULT: ("ult", False), C.Z3_OP_ULEQ: ("ule", False), C.Z3_OP_UGT: ("ult", True),
         C.Z3_OP_UGEQ: ("ule", True), C.Z3_OP_SLT: ("slt", False), C.Z3_OP_SLEQ: ("sle", False),
         C.Z3_OP_SGT: ("slt", True), C.Z3_OP_SGEQ: ("sle", True),
         C.Z3_OP_BUMUL_NO_OVFL: ("umul_noovfl", False), C.Z3_OP_BSMUL_NO_OVFL: ("smul_noovfl", False),
         C.Z3_OP_BSMUL_NO_UDFL: ("smul_noudfl", False)}


def _width(e) -> int:
    s = e.sort()
    k = s.kind()
    if k == z3.Z3_BOOL_SORT:
        return 0
    if k == z3.Z3_BV_SORT:
        return s.size()
    if k == z3.Z3_ARRAY_SORT:
        r = s.range()
        return 0 if r.kind() == z3.Z3_BOOL_SORT else r.size()
    raise LoweringError(f"sort {s} not supported")


def lower_z3_term(root, syms: SymbolTable) -> Tape:
    """Iterative post-order walk of a z3 BoolRef DAG into one tape."""
    tp = Tape()
    done: Dict[int, int] = {}
    stack = [(root, False)]
    while stack:
        e, ready = stack.pop()
        eid = e.get_id()
        if eid in done:
            continue
        if not ready:
            stack.append((e, True))
            for ch in reversed(e.children()):
                if ch.get_id() not in done:
                    stack.append((ch, False))
            continue
        done[eid] = _lower_node(e, [done[c.get_id()] for c in e.children()], tp, syms)
    return tp.finish(done[root.get_id()])


def _lower_node(e, a: List[int], tp: Tape, syms: SymbolTable) -> int:
    if z3.is_quantifier(e) or z3.is_var(e):
        raise LoweringError("quantifiers / bound variables")
    d = e.decl()
    k = d.kind()
    w = _width(e)
    if k == C.Z3_OP_TRUE:
        return tp.true()
    if k == C.Z3_OP_FALSE:
        return tp.false()
    if k == C.Z3_OP_BNUM:
        return tp.const(e.as_long(), w)
    if k == C.Z3_OP_UNINTERPRETED:
        name = d.name()
        if e.num_args() == 0:
            if e.sort().kind() == z3.Z3_ARRAY_SORT:
                dom = e.sort().domain()
                if dom.kind() != z3.Z3_BV_SORT:
                    raise LoweringError("array domain")
                return tp.array_var(syms.func(name, (dom.size(),), w), w)
            return tp.var(syms.var(name, w), w)
        args = [e.arg(i) for i in range(e.num_args())]
        return tp.uf(syms.func(name, tuple(_width(x) for x in args), w), w, *a)
    if k == C.Z3_OP_AND:
        return tp.and_(*a)
    if k == C.Z3_OP_OR:
        return tp.or_(*a)
    if k == C.Z3_OP_NOT:
        return tp.not_(a[0])
    if k == C.Z3_OP_XOR:
        return tp.xor(a[0], a[1])
    if k == C.Z3_OP_IMPLIES:
        return tp.implies(a[0], a[1])
    if k in (C.Z3_OP_IFF, C.Z3_OP_EQ):
        if e.arg(0).sort().kind() == z3.Z3_ARRAY_SORT:
            raise LoweringError("array equality")
        return tp.eq(a[0], a[1])
    if k == C.Z3_OP_DISTINCT:
        terms = [tp.distinct(a[i], a[j]) for i in range(len(a)) for j in range(i + 1, len(a))]
        return tp.and_(*terms)
    if k == C.Z3_OP_ITE:
        if e.sort().kind() == z3.Z3_ARRAY_SORT:
            raise LoweringError("array-valued ite")
        return tp.ite(a[0], a[1], a[2])
    if k in _PRED:
        name, swap = _PRED[k]
        x, y = (a[1], a[0]) if swap else (a[0], a[1])
        return getattr(tp, name)(x, y)
    if k in _NARY_BV and len(a) > 2:
        acc = a[0]
        for x in a[1:]:
            acc = getattr(tp, _NARY_BV[k])(acc, x)
        return acc
    if k in _BIN:
        return getattr(tp, _BIN[k])(a[0], a[1])
    if k == C.Z3_OP_BNEG:
        return tp.neg(a[0])
    if k == C.Z3_OP_BNOT:
        return tp.bnot(a[0])
    if k == C.Z3_OP_BNAND:
        return tp.bnot(tp.band(a[0], a[1]))
    if k == C.Z3_OP_BNOR:
        return tp.bnot(tp.bor(a[0], a[1]))
    if k == C.Z3_OP_BXNOR:
        return tp.bnot(tp.bxor(a[0], a[1]))
    if k == C.Z3_OP_CONCAT:
        return tp.concat(*a)
    if k == C.Z3_OP_EXTRACT:
        hi, lo = d.params()
        return tp.extract(hi, lo, a[0])
    if k == C.Z3_OP_ZERO_EXT:
        return tp.zext(d.params()[0], a[0])
    if k == C.Z3_OP_SIGN_EXT:
        return tp.sext(d.params()[0], a[0])
    if k == C.Z3_OP_REPEAT:
        return tp.concat(*([a[0]] * d.params()[0]))
    if k == C.Z3_OP_SELECT:
        return tp.select(a[0], a[1])
    if k == C.Z3_OP_STORE:
        return tp.store(a[0], a[1], a[2])
    if k == C.Z3_OP_CONST_ARRAY:
        return tp.const_array(a[0])
    raise LoweringError(f"z3 kind {k} ({d.name()}) not in the tape vocabulary")


# ---------------------------------------------------------------------------- models
def _raw_models(model) -> list:
    return list(getattr(model, "raw", [model]))


def _value(v) -> int:
    if z3.is_true(v):
        return 1
    if z3.is_false(v):
        return 0
    if z3.is_bv_value(v):
        return v.as_long()
    raise LoweringError(f"model value {v} is not a literal")


def _func_interp(fi) -> Tuple[Dict[tuple, int], int]:
    entries: Dict[tuple, int] = {}
    for i in range(fi.num_entries()):
        ent = fi.entry(i)
        key = tuple(_value(ent.arg_value(j)) for j in range(fi.arity()))
        entries.setdefault(key, _value(ent.value()))  # first entry wins, as in z3's lookup
    return entries, _value(fi.else_value())


def _array_interp(m, v) -> Tuple[Dict[tuple, int], int]:
    """An array value: ``as-array f`` (read f's FuncInterp), or ``Store`` chain over ``K``."""
    if z3.is_as_array(v):
        return _func_interp(m.get_interp(z3.get_as_array_func(v)))
    stores = []
    while z3.is_store(v):
        stores.append((_value(v.arg(1)), _value(v.arg(2))))
        v = v.arg(0)
    if z3.is_K(v):
        entries: Dict[tuple, int] = {}
        for key, val in stores:  # outermost store wins
            entries.setdefault((key,), val)
        return entries, _value(v.arg(0))
    raise LoweringError(f"array interpretation {v} not supported")


def model_record(model) -> Model:
    """Read a mythril ``Model`` (its single ``z3.ModelRef``, solver.py:88-97) without completion."""
    raws = _raw_models(model)
    assignment, functions = {}, {}
    for m in raws:
        for d in m.decls():
            name = d.name()
            if d.arity() == 0:
                v = m.get_interp(d)
                if d.range().kind() == z3.Z3_ARRAY_SORT:
                    functions[name] = _array_interp(m, v)
                else:
                    assignment[name] = _value(v)
            else:
                functions[name] = _func_interp(m.get_interp(d))
    return Model(assignment, functions)


def lower_batch_z3(exprs: Sequence, models: Sequence):
    syms = SymbolTable()
    tapes, ok = [], np.ones(len(exprs), bool)
    for i, e in enumerate(exprs):
        try:
            tapes.append(lower_z3_term(e, syms))
        except (LoweringError, TypeError) as err:
            note_fail_closed(err)
            ok[i] = False
            t = Tape()
            tapes.append(t.finish(t.false()))
    recs = []
    for m in models:
        try:
            recs.append(model_record(m))
        except LoweringError:
            ok[:] = False  # a model we cannot read: route the whole batch to the z3 loop
            recs.append(Model())
    return TapeBatch(tapes), serialize_models(recs, syms), ok


def z3_quick_sat_loop(expr, order):
    """The reference's loop (support_utils.py:62-66) for conjunctions the evaluator rejects."""
    for model in order:
        if z3.is_true(deepcopy(model).eval(expr, model_completion=True)):
            return model
    return False


class Z3Backend:
    """``solver_worker`` (model.py:28-65) on z3 ``Optimize``."""

    def solve(self, constraints, minimize, maximize, timeout_ms):
        s = z3.Optimize()
        s.set("timeout", int(timeout_ms))
        for c in constraints:
            s.add(getattr(c, "raw", c))
        for e in minimize:
            s.minimize(getattr(e, "raw", e))
        for e in maximize:
            s.maximize(getattr(e, "raw", e))
        r = s.check()
        if r == z3.sat:
            try:
                from mythril.laser.smt.model import Model as MModel  # the caller's wrapper type
                return "sat", lambda: MModel([s.model()])
            except ImportError:
                return "sat", s.model
        return ("unknown" if r == z3.unknown else "unsat"), None
