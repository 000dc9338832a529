"""z3 host side of the lowering pass (imported only where ``z3-solver`` exists).

Reference call site: ``model_cache.check_quick_sat(simplify(And(*constraints)).raw)``
(``mythril/support/model.py:101``) hands a z3 ``BoolRef`` to quick-sat, which evaluates it under
each cached ``Model`` (``support_utils.py:62-64``).  This module

* translates that ``BoolRef`` DAG by ``decl().kind()`` into interned
  :mod:`mythril_amd.smt` terms (:class:`Z3Terms`, memoized by ``get_id()``), so a z3 query takes
  the same incremental path as a z3-free one: the engine's persistent hash-consed DAG, resident
  model rows and per-conjunct verdict rows (support.py ``VerdictEngine``); every kind not listed
  raises :class:`LoweringError` (fail closed);
* reads a ``mythril.laser.smt.Model`` / ``z3.ModelRef`` WITHOUT completion into the
  :class:`~mythril_amd.smt_model.Model` record (constants; ``FuncInterp`` entries + else value;
  arrays given as ``as-array``, ``K`` or ``Store`` chains over ``K``);
* keeps the reference's own loop (:func:`z3_quick_sat_loop`) for tapes the evaluator rejects, and
  a ``Z3Backend`` that is ``solver_worker`` (model.py:28-65).

z3 is absent from this container and from the GPU box: the tests drive this module through a
stand-in of the z3py surface it uses (tests/fake_z3.py); on a z3 host its verdicts are checked
against ``z3_quick_sat_loop``.  Parity with real z3 is unpinned.
"""
from __future__ import annotations

from copy import deepcopy
from typing import Dict, List, Sequence, Tuple

import numpy as np
import z3  # noqa: F401  (ImportError here means: no z3 host)
from z3 import z3consts as C

from . import smt as S
from .exceptions import LoweringError, note_fail_closed
from .lower import lower_batch, serialize_models
from .smt_model import Model
from .tape import BOOL

_BIN = {C.Z3_OP_BSUB: S.SUB, C.Z3_OP_BUDIV: S.UDIV, C.Z3_OP_BUDIV_I: S.UDIV, C.Z3_OP_BUREM: S.UREM,
        C.Z3_OP_BUREM_I: S.UREM, C.Z3_OP_BSDIV: S.SDIV, C.Z3_OP_BSDIV_I: S.SDIV, C.Z3_OP_BSREM: S.SREM,
        C.Z3_OP_BSREM_I: S.SREM, C.Z3_OP_BSMOD: S.SMOD, C.Z3_OP_BSMOD_I: S.SMOD, C.Z3_OP_BSHL: S.SHL,
        C.Z3_OP_BLSHR: S.LSHR, C.Z3_OP_BASHR: S.ASHR}
_NARY_BV = {C.Z3_OP_BADD: S.ADD, C.Z3_OP_BMUL: S.MUL, C.Z3_OP_BAND: S.BAND, C.Z3_OP_BOR: S.BOR, C.Z3_OP_BXOR: S.BXOR}
_NOT_OF = {C.Z3_OP_BNAND: S.BAND, C.Z3_OP_BNOR: S.BOR, C.Z3_OP_BXNOR: S.BXOR}
_PRED = {C.Z3_OP_ULT: (S.BVULT, False), C.Z3_OP_ULEQ: (S.BVULE, False), C.Z3_OP_UGT: (S.BVULT, True),
         C.Z3_OP_UGEQ: (S.BVULE, True), C.Z3_OP_SLT: (S.BVSLT, False), C.Z3_OP_SLEQ: (S.BVSLE, False),
         C.Z3_OP_SGT: (S.BVSLT, True), C.Z3_OP_SGEQ: (S.BVSLE, True),
         C.Z3_OP_BUMUL_NO_OVFL: (S.UMUL_NOOVFL, False), C.Z3_OP_BSMUL_NO_OVFL: (S.SMUL_NOOVFL, False),
         C.Z3_OP_BSMUL_NO_UDFL: (S.SMUL_NOUDFL, False)}


def _width(e) -> int:
    s = e.sort()
    k = s.kind()
    if k == z3.Z3_BOOL_SORT:
        return BOOL
    if k == z3.Z3_BV_SORT:
        return s.size()
    if k == z3.Z3_ARRAY_SORT:
        r = s.range()
        return BOOL if r.kind() == z3.Z3_BOOL_SORT else r.size()
    raise LoweringError(f"sort {s} not supported")


def _fold(kind: str, args: List[S.Term]) -> S.Term:
    acc = args[0]
    for x in args[1:]:
        acc = S.Term(kind, "bv", acc.width, (acc, x))
    return acc


class Z3Terms:
    """z3 ASTs -> interned :mod:`mythril_amd.smt` terms, memoized by ``get_id()``.

    z3 hash-conses its ASTs, so the conjuncts a forked state shares with its parent (svm.py:351-358)
    and the keccak axioms riding on every query (constraints.py:127-128) are the same z3 ASTs from
    call to call; each is translated once, and — the terms being interned — always to the same
    term object, which the engine's persistent DAG (``IncrementalLowering``) and per-conjunct
    verdict rows (``ConjunctRows``) key on.  The ASTs are held while memoized (their ids stay
    valid); past ``MAX_MEMO`` entries the memo starts over.  A kind outside the vocabulary raises
    :class:`LoweringError` (fail closed), remembered per AST."""

    MAX_MEMO = 1 << 20

    def __init__(self) -> None:
        self.reset()

    def reset(self) -> None:
        self._memo: Dict[int, Tuple[object, object]] = {}   # get_id() -> (AST, Term or LoweringError)
        self.translated = 0   # ASTs translated (not memo hits): the new nodes of the stream

    def term(self, root) -> S.Term:
        memo = self._memo
        if len(memo) > self.MAX_MEMO:
            self.reset()
            memo = self._memo
        hit = memo.get(root.get_id())
        if hit is None:
            stack = [root]
            while stack:
                e = stack[-1]
                eid = e.get_id()
                if eid in memo:
                    stack.pop()
                    continue
                if z3.is_quantifier(e) or z3.is_var(e):
                    memo[eid] = (e, LoweringError("quantifiers / bound variables"))
                    stack.pop()
                    continue
                kids = e.children()
                pending = False
                for ch in reversed(kids):
                    if ch.get_id() not in memo:
                        stack.append(ch)
                        pending = True
                if pending:
                    continue
                stack.pop()
                args = []
                err = None
                for ch in kids:
                    t = memo[ch.get_id()][1]
                    if isinstance(t, LoweringError):
                        err = t
                        break
                    args.append(t)
                if err is None:
                    try:
                        r = _translate(e, args)
                    except (LoweringError, TypeError) as x:
                        r = x if isinstance(x, LoweringError) else LoweringError(str(x))
                else:
                    r = err
                memo[eid] = (e, r)
                self.translated += 1
            hit = memo[root.get_id()]
        if isinstance(hit[1], LoweringError):
            raise hit[1]
        return hit[1]


def _translate(e, a: List[S.Term]) -> S.Term:
    """One z3 node (kind by ``decl().kind()``) over its translated children."""
    d = e.decl()
    k = d.kind()
    w = _width(e)
    if k == C.Z3_OP_TRUE:
        return S.BoolVal(True)
    if k == C.Z3_OP_FALSE:
        return S.BoolVal(False)
    if k == C.Z3_OP_BNUM:
        return S.BitVecVal(e.as_long(), w)
    if k == C.Z3_OP_UNINTERPRETED:
        name = d.name()
        if e.num_args() == 0:
            if e.sort().kind() == z3.Z3_ARRAY_SORT:
                dom = e.sort().domain()
                if dom.kind() != z3.Z3_BV_SORT:
                    raise LoweringError("array domain")
                return S.Array(name, dom.size(), w)
            return S.BoolSym(name) if w == BOOL else S.BitVecSym(name, w)
        dom = tuple(x.width for x in a)
        if any(x.sort != "bv" for x in a):
            raise LoweringError(f"function {name}: non-bit-vector argument")
        if not 1 <= len(a) <= 2:
            raise LoweringError(f"function {name}: arity {len(a)} not supported")
        return S.Term(S.APP, "bool" if w == BOOL else "bv", w, tuple(a), (name, dom))
    if k == C.Z3_OP_AND:
        return S.And(*a)
    if k == C.Z3_OP_OR:
        return S.Or(*a)
    if k == C.Z3_OP_NOT:
        return S.Not(a[0])
    if k == C.Z3_OP_XOR:
        return S.Xor(a[0], a[1])
    if k == C.Z3_OP_IMPLIES:
        return S.Implies(a[0], a[1])
    if k in (C.Z3_OP_IFF, C.Z3_OP_EQ):
        x, y = a
        if x.sort == "bool":
            return S.Term(S.IFF, "bool", BOOL, (x, y))
        return S.Term(S.EQ, "bool", BOOL, (x, y))   # (array equality: the lowering fails closed)
    if k == C.Z3_OP_DISTINCT:
        return S.And(*[S.Not(S.Term(S.IFF if a[i].sort == "bool" else S.EQ, "bool", BOOL, (a[i], a[j])))
                       for i in range(len(a)) for j in range(i + 1, len(a))])
    if k == C.Z3_OP_ITE:
        return S.If(a[0], a[1], a[2])
    if k in _PRED:
        kind, swap = _PRED[k]
        x, y = (a[1], a[0]) if swap else (a[0], a[1])
        return S.Term(kind, "bool", BOOL, (x, y))
    if k in _NARY_BV:
        return _fold(_NARY_BV[k], a)
    if k in _BIN:
        return S.Term(_BIN[k], "bv", w, (a[0], a[1]))
    if k == C.Z3_OP_BNEG:
        return S.Term(S.NEG, "bv", w, (a[0],))
    if k == C.Z3_OP_BNOT:
        return S.Term(S.BNOT, "bv", w, (a[0],))
    if k in _NOT_OF:
        return S.Term(S.BNOT, "bv", w, (S.Term(_NOT_OF[k], "bv", w, (a[0], a[1])),))
    if k == C.Z3_OP_CONCAT:
        return S.Concat(*a)
    if k == C.Z3_OP_EXTRACT:
        hi, lo = d.params()
        return S.Extract(hi, lo, a[0])
    if k == C.Z3_OP_ZERO_EXT:
        return S.ZeroExt(d.params()[0], a[0])
    if k == C.Z3_OP_SIGN_EXT:
        return S.SignExt(d.params()[0], a[0])
    if k == C.Z3_OP_REPEAT:
        return S.Concat(*([a[0]] * d.params()[0]))
    if k == C.Z3_OP_SELECT:
        return S.Select(a[0], a[1])
    if k == C.Z3_OP_STORE:
        return S.Store(a[0], a[1], a[2])
    if k == C.Z3_OP_CONST_ARRAY:
        dom = e.sort().domain()
        if dom.kind() != z3.Z3_BV_SORT:
            raise LoweringError("array domain")
        return S.Term(S.CONST_ARRAY, "array", w, (a[0],), (), dom.size())
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


def lower_batch_z3(exprs: Sequence, models: Sequence, terms: "Z3Terms" = None, hoist: bool = False):
    """Whole-batch form (no state across calls): ``(TapeBatch, ModelBatch, supported mask)``.
    The engine's drop-in path does not use it — it keeps a :class:`Z3Terms` and the persistent
    DAG instead (support.py ``VerdictEngine``)."""
    terms = terms or Z3Terms()
    ok = np.ones(len(exprs), bool)
    roots = []
    for i, e in enumerate(exprs):
        try:
            roots.append(terms.term(e))
        except LoweringError as err:
            note_fail_closed(err)
            ok[i] = False
            roots.append(S.BoolVal(False))
    tb, syms, ok2 = lower_batch(roots, hoist=hoist)
    ok &= np.asarray(ok2, bool)
    recs = []
    for m in models:
        try:
            recs.append(model_record(m))
        except LoweringError:
            ok[:] = False  # a model we cannot read: route the whole batch to the z3 loop
            recs.append(Model())
    return tb, serialize_models(recs, syms), ok


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
