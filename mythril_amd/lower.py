"""Lowering pass: constraint terms -> tape IR, candidate models -> SoA model batch.

This is the build's counterpart of the step ``model_cache.check_quick_sat(simplify(And(*constraints)).raw)``
(reference ``mythril/support/model.py:101``): the conjunction handed to quick-sat is flattened
into a postfix tape (include/mq.h) and the candidate models into the ``mq_model_batch`` layout.
It lowers the z3-free terms of :mod:`mythril_amd.smt`; :mod:`mythril_amd.lower_z3` walks real
z3 ASTs into the same :class:`SymbolTable` and tape.

Fail closed: anything outside the vocabulary (array-valued ``ite``, array equality, functions of
arity > 2, widths > 65535) raises :class:`LoweringError`; the query then keeps the reference's
z3 evaluation path.

``z3.simplify`` preserves equivalence over all interpretations and completion makes evaluation
total, so lowering the raw conjunction or its simplified form yields the same verdict on every
model ("Equivalence lets the lowering choose its input").
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import smt as S
from .exceptions import LoweringError
from .models import FuncSpec, ModelBatch
from .smt_model import Model
from .tape import BOOL, NONE, ColumnSet, Tape, TapeBatch, limbs, to_words

MAX_WIDTH = 0xFFFF


class SymbolTable:
    """Free constants -> model variable indices; UFs and symbolic arrays -> model function ids.

    A constant is identified by (name, width) — z3 declarations with equal names but different
    sorts are different declarations.  A symbolic array ``Array(name, dom, rng)`` is read through
    the model's interpretation of ``name`` (its ``as-array`` function, arity 1)."""

    def __init__(self, derive_constant_lookups: bool = True, interpret_keccak: bool = False) -> None:
        self.vars: Dict[Tuple[str, int], int] = {}
        self.var_widths: List[int] = []
        self.funcs: Dict[str, int] = {}
        self.func_specs: List[FuncSpec] = []
        self.func_names: List[str] = []
        self.derive = derive_constant_lookups
        # lower keccak256_<n>(x) to in-kernel keccak-f[1600] instead of the model's UF table:
        # exact only for keccak-consistent candidate sets (C4), never for z3 models in general
        self.interpret_keccak = interpret_keccak
        self.derived: Dict[int, Tuple[str, Tuple[int, ...]]] = {}  # var index -> (function, const args)
        self.hoisted_vars = set()   # variables computed on the device from column programs

    def derived_var(self, fname: str, args: Tuple[int, ...], width: int) -> int:
        """A model-only quantity: the interpretation of function/array ``fname`` at CONSTANT
        arguments (``select(<tx>_calldata, 4)``, ``keccak256_256(c)``).  Its value is fixed per
        model, so it is looked up once per model at serialization (entries, then else value —
        the same rule the kernel applies) and stored as an SoA column like any constant."""
        key = ("@" + fname + ":" + ",".join(str(a) for a in args), width)
        i = self.vars.get(key)
        if i is None:
            i = self.var(key[0], width)
            self.derived[i] = (fname, tuple(args))
        return i

    def var(self, name: str, width: int) -> int:
        key = (name, width)
        i = self.vars.get(key)
        if i is None:
            i = len(self.var_widths)
            self.vars[key] = i
            self.var_widths.append(width)
        return i

    def func(self, name: str, arg_widths: Sequence[int], result_width: int) -> int:
        i = self.funcs.get(name)
        spec = FuncSpec(len(arg_widths), result_width, tuple(arg_widths))
        if i is None:
            if not 1 <= len(arg_widths) <= 2:
                raise LoweringError(f"function {name}: arity {len(arg_widths)} not supported")
            i = len(self.func_specs)
            self.funcs[name] = i
            self.func_specs.append(spec)
            self.func_names.append(name)
        elif self.func_specs[i] != spec:
            raise LoweringError(f"function {name} used with two signatures")
        return i


def _w(t: S.Term) -> int:
    if t.width > MAX_WIDTH:
        raise LoweringError(f"width {t.width} exceeds the tape format")
    return t.width


def lower_term(root: S.Term, syms: SymbolTable, hoisted: Optional[Dict[int, int]] = None,
               value_root: bool = False) -> Tape:
    """Lower one Bool term (the quick-sat conjunction) to a tape; iterative over the DAG.
    ``hoisted``: id(term) -> variable index of terms replaced by derived columns."""
    if root.sort != "bool" and not value_root:
        raise LoweringError("quick-sat root must be Bool")
    hoisted = hoisted or {}
    tp = Tape()
    node: Dict[int, int] = {}

    def arr_node(arr: S.Term, r: int) -> int:
        if r >= 0:
            return r
        r = tp.array_var(syms.func(arr.params[0], (arr.domain,), arr.width), arr.width)
        node[id(arr)] = r
        return r

    for t in _walk_cut(root, hoisted):
        k = t.kind
        if id(t) in hoisted and t is not root:
            node[id(t)] = tp.var(hoisted[id(t)], _w(t))
            continue
        a = [node[id(x)] for x in t.args]
        if k == S.SYM:
            r = tp.var(syms.var(t.params[0], _w(t)), _w(t))
        elif k == S.VAL:
            r = tp.const(t.params[0], _w(t))
        elif k == S.TRUE:
            r = tp.true()
        elif k == S.FALSE:
            r = tp.false()
        elif k == S.NOT:
            r = tp.not_(a[0])
        elif k == S.AND:
            r = tp.and_(*a)
        elif k == S.OR:
            r = tp.or_(*a)
        elif k == S.XOR:
            r = tp.xor(a[0], a[1])
        elif k == S.IMPLIES:
            r = tp.implies(a[0], a[1])
        elif k == S.IFF:
            r = tp.iff(a[0], a[1])
        elif k == S.BITE:
            r = tp.bite(a[0], a[1], a[2])
        elif k == S.EQ:
            if t.args[0].sort == "array":
                raise LoweringError("array equality")
            r = tp.eq(a[0], a[1])
        elif k == S.BVULT:
            r = tp.ult(a[0], a[1])
        elif k == S.BVULE:
            r = tp.ule(a[0], a[1])
        elif k == S.BVSLT:
            r = tp.slt(a[0], a[1])
        elif k == S.BVSLE:
            r = tp.sle(a[0], a[1])
        elif k == S.UMUL_NOOVFL:
            r = tp.umul_noovfl(a[0], a[1])
        elif k == S.SMUL_NOOVFL:
            r = tp.smul_noovfl(a[0], a[1])
        elif k == S.SMUL_NOUDFL:
            r = tp.smul_noudfl(a[0], a[1])
        elif k in _BIN:
            r = getattr(tp, _BIN[k])(a[0], a[1])
        elif k == S.NEG:
            r = tp.neg(a[0])
        elif k == S.BNOT:
            r = tp.bnot(a[0])
        elif k == S.EXTRACT:
            r = tp.extract(t.params[0], t.params[1], a[0])
        elif k == S.CONCAT:
            _w(t)
            r = tp.concat(a[0], a[1])
        elif k == S.ZEXT:
            r = tp.zext(t.params[0], a[0])
        elif k == S.SEXT:
            r = tp.sext(t.params[0], a[0])
        elif k == S.ITE:
            r = tp.ite(a[0], a[1], a[2])
        elif k == S.ARRAY_SYM:
            r = -1  # materialised at its first table use (a symbol only read at constant indices
            #         never enters the model's function tables)
        elif k == S.CONST_ARRAY:
            r = tp.const_array(a[0])
        elif k == S.STORE:
            r = tp.store(arr_node(t.args[0], a[0]), a[1], a[2])
        elif k == S.SELECT:
            arr, idx = t.args
            if syms.derive and arr.kind == S.ARRAY_SYM and idx.kind == S.VAL:
                r = tp.var(syms.derived_var(arr.params[0], (idx.params[0],), _w(t)), _w(t))
            else:
                r = tp.select(arr_node(arr, a[0]), a[1])
        elif k == S.KECCAK:
            r = tp.keccak(a[0])
        elif k == S.APP and syms.interpret_keccak and _is_keccak_uf(t.params[0]):
            r = tp.keccak(a[0])
        elif k == S.APP:
            name, dom = t.params
            fid = syms.func(name, dom, t.width)
            if syms.derive and all(x.kind == S.VAL for x in t.args):
                r = tp.var(syms.derived_var(name, tuple(x.params[0] for x in t.args), _w(t)), _w(t))
            else:
                r = tp.uf(fid, t.width, *a)
        else:
            raise LoweringError(f"term kind {k!r} not in the tape vocabulary")
        node[id(t)] = r
    return tp.finish(node[id(root)], value_root=value_root)


def _walk_cut(root: S.Term, cut: Dict[int, int]) -> List[S.Term]:
    """Postfix order of the DAG under ``root`` that does not descend into ``cut`` terms."""
    order: List[S.Term] = []
    seen = set()
    stack = [(root, False)]
    while stack:
        t, done = stack.pop()
        if done:
            order.append(t)
            continue
        if id(t) in seen:
            continue
        seen.add(id(t))
        stack.append((t, True))
        if id(t) in cut and t is not root:
            continue
        for a in reversed(t.args):
            if id(a) not in seen:
                stack.append((a, False))
    return order


_LEAVES = frozenset({S.SYM, S.VAL, S.TRUE, S.FALSE, S.ARRAY_SYM})


def shared_subterms(roots: Sequence[S.Term], min_nodes: int = 8, min_tapes: int = 2) -> List[S.Term]:
    """Maximal sub-terms (BV/Bool sorted, >= ``min_nodes`` tree nodes) that occur in at least
    ``min_tapes`` of the roots — candidates for batch-level hoisting into model columns."""
    count: Dict[int, int] = {}
    terms: Dict[int, S.Term] = {}
    for r in roots:
        for t in S.walk(r):
            if t.kind in _LEAVES or t.sort == "array" or t is r:
                continue
            count[id(t)] = count.get(id(t), 0) + 1
            terms[id(t)] = t
    size: Dict[int, int] = {}

    def tree_size(t: S.Term) -> int:   # capped tree size (cheap, memoised)
        s = size.get(id(t))
        if s is None:
            s = 1 + sum(0 if a.kind in _LEAVES else tree_size(a) for a in t.args)
            s = min(s, 1 << 20)
            size[id(t)] = s
        return s

    eligible = {i for i, c in count.items() if c >= min_tapes and terms[i].width <= 2048}
    chosen: Dict[int, S.Term] = {}
    for r in roots:   # top-down: the first eligible term on every path is maximal for that root
        stack = list(r.args)
        seen = set()
        while stack:
            t = stack.pop()
            if id(t) in seen or t.kind in _LEAVES:
                continue
            seen.add(id(t))
            if id(t) in eligible:
                for w in S.walk(t):   # iterative: sizes of deep chains without recursion limits
                    if w.kind not in _LEAVES:
                        tree_size(w)
                if tree_size(t) >= min_nodes:
                    chosen[id(t)] = t
                    continue
            stack.extend(t.args)
    return list(chosen.values())


def _is_keccak_uf(name: str) -> bool:
    """``keccak256_<n>`` (keccak_function_manager.py:77), not its inverse ``keccak256_<n>-1``."""
    return name.startswith("keccak256_") and name[10:].isdigit()


_BIN = {S.ADD: "add", S.SUB: "sub", S.MUL: "mul", S.UDIV: "udiv", S.UREM: "urem", S.SDIV: "sdiv",
        S.SREM: "srem", S.SMOD: "smod", S.BAND: "band", S.BOR: "bor", S.BXOR: "bxor",
        S.SHL: "shl", S.LSHR: "lshr", S.ASHR: "ashr"}


def lower_batch(roots: Sequence[S.Term], syms: Optional[SymbolTable] = None, hoist: bool = False,
                hoist_min_nodes: int = 8):
    """Lower N conjunctions over one shared symbol table.  Returns ``(TapeBatch | None, syms,
    supported_mask)``: a root that fails to lower is replaced by a FALSE placeholder tape and
    flagged unsupported (the caller routes it to z3).

    ``hoist``: sub-terms shared by several roots are evaluated once per model into derived
    columns (``TapeBatch.columns``, variables named ``@h<k>``) instead of once per (tape, model).
    Verdicts are unchanged: a sub-term's value depends only on the model."""
    syms = syms or SymbolTable()
    hoisted: Dict[int, int] = {}
    col_terms: List[S.Term] = []
    if hoist and len(roots) > 1:
        col_terms = shared_subterms(roots, hoist_min_nodes)
        for k, t in enumerate(col_terms):
            hoisted[id(t)] = syms.var(f"@h{k}", t.width)
            syms.hoisted_vars.add(hoisted[id(t)])
    tapes, ok = [], np.ones(len(roots), bool)
    for i, r in enumerate(roots):
        try:
            tapes.append(lower_term(r, syms, hoisted))
        except (LoweringError, TypeError):
            ok[i] = False
            t = Tape()
            tapes.append(t.finish(t.false()))
    tb = TapeBatch(tapes) if tapes else None
    if tb is not None and col_terms:
        progs, levels = [], []
        lvl: Dict[int, int] = {}
        for t in col_terms:   # column programs; a column may read columns nested inside it
            inner = [h for h in _walk_cut(t, hoisted) if id(h) in hoisted and h is not t]
            lvl[id(t)] = 0
            progs.append(lower_term(t, syms, hoisted, value_root=True))
        # levels: longest chain of nested columns (terms are acyclic)
        changed = True
        while changed:
            changed = False
            for t in col_terms:
                inner = [h for h in _walk_cut(t, hoisted) if id(h) in hoisted and h is not t]
                want = 1 + max((lvl[id(h)] for h in inner), default=-1)
                if want > lvl[id(t)]:
                    lvl[id(t)] = want
                    changed = True
        levels = [lvl[id(t)] for t in col_terms]
        tb.columns = ColumnSet(TapeBatch(progs), [hoisted[id(t)] for t in col_terms], levels)
    return tb, syms, ok


def serialize_models(models: Sequence[Model], syms: SymbolTable, index_base: int = 0) -> ModelBatch:
    """Candidate models (global order, index 0 = MRU) -> ``mq_model_batch`` (SoA u32 limbs +
    per-function CSR tables), WITHOUT completion: an absent constant stays 0 / false and an
    absent function has no entries and else 0."""
    M = len(models)
    widths = syms.var_widths
    off = np.zeros(len(widths) + 1, np.int64)
    off[1:] = np.cumsum([limbs(w) for w in widths])
    words = np.zeros((int(off[-1]), M), np.uint32)
    names = [None] * len(widths)
    for (name, w), i in syms.vars.items():
        names[i] = (name, w)
    for m, mod in enumerate(models):
        asg = mod.assignment
        for i, (name, w) in enumerate(names):
            if i in syms.derived:
                fname, fargs = syms.derived[i]
                interp = mod.functions.get(fname)
                v = 0 if interp is None else interp[0].get(fargs, interp[1])
            else:
                v = asg.get(name)
            if v is None:
                continue
            v = int(v) & ((1 << max(w, 1)) - 1)
            words[off[i]:off[i + 1], m] = to_words(v, w)
    fmodels = []
    for mod in models:
        fm = {}
        for f, name in enumerate(syms.func_names):
            interp = mod.functions.get(name)
            if interp is not None:
                fm[f] = interp
        fmodels.append({"funcs": fm})
    if not syms.func_specs:
        return ModelBatch(widths, words, index_base=index_base)
    fb = ModelBatch.from_python(widths or [], fmodels, syms.func_specs, index_base)
    return ModelBatch(widths, words, syms.func_specs, fb.entry_ptr, fb.entry_words, fb.entry_base,
                      fb.else_words, fb.else_base, index_base)
