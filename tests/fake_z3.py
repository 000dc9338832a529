"""A test-only stand-in for the part of the z3py API that ``mythril_amd.lower_z3`` uses
(SURVEY Appendix F), so the z3 side of the lowering pass executes on hosts without z3.

It is NOT z3: terms are hash-consed Python objects carrying a decl kind, params, children and
a sort; ``ModelRef.eval(e, model_completion=True)`` evaluates them with SMT-LIB 2.6
FixedSizeBitVector semantics and z3's completion rules as SURVEY Appendix A states them (an
absent constant is 0 / false, an absent function or array is the constant 0, a ``FuncInterp``
answers its first matching entry, else its else value).  Parity of this stand-in with real z3 is
UNPINNED: it exercises every branch of the lowering and model reader and cross-checks them
against an evaluator written independently of the tape IR, nothing more.

Install with :func:`install` (``sys.modules['z3']``), remove with :func:`uninstall`.
"""
from __future__ import annotations

import itertools
import sys
import types
from typing import Dict, List, Optional, Tuple

# ----------------------------------------------------------------------------- constants
Z3_BOOL_SORT, Z3_BV_SORT, Z3_ARRAY_SORT, Z3_INT_SORT = 1, 4, 5, 2

_KIND_NAMES = """TRUE FALSE EQ DISTINCT ITE AND OR IFF XOR NOT IMPLIES
BNUM BNEG BADD BSUB BMUL BSDIV BUDIV BSREM BUREM BSMOD BSDIV_I BUDIV_I BSREM_I BUREM_I BSMOD_I
BSDIV0 BUDIV0 ULEQ SLEQ UGEQ SGEQ ULT SLT UGT SGT BAND BOR BNOT BXOR BNAND BNOR BXNOR
CONCAT SIGN_EXT ZERO_EXT EXTRACT REPEAT BCOMP BSHL BLSHR BASHR ROTATE_LEFT
BUMUL_NO_OVFL BSMUL_NO_OVFL BSMUL_NO_UDFL STORE SELECT CONST_ARRAY AS_ARRAY UNINTERPRETED""".split()
z3consts = types.ModuleType("z3.z3consts")
for _i, _n in enumerate(_KIND_NAMES):
    setattr(z3consts, "Z3_OP_" + _n, 0x100 + _i)
C = z3consts


# ----------------------------------------------------------------------------- sorts / decls
class SortRef:
    def __init__(self, kind: int, size: int = 0, dom: "SortRef" = None, rng: "SortRef" = None):
        self._k, self._size, self._dom, self._rng = kind, size, dom, rng

    def kind(self):
        return self._k

    def size(self):
        return self._size

    def domain(self):
        return self._dom

    def range(self):
        return self._rng

    def key(self):
        return (self._k, self._size, self._dom.key() if self._dom else None, self._rng.key() if self._rng else None)

    def __eq__(self, o):
        return isinstance(o, SortRef) and self.key() == o.key()

    def __hash__(self):
        return hash(self.key())


def BoolSort():
    return SortRef(Z3_BOOL_SORT)


def BitVecSort(w):
    return SortRef(Z3_BV_SORT, w)


def ArraySort(dom, rng):
    return SortRef(Z3_ARRAY_SORT, 0, dom, rng)


def IntSort():
    return SortRef(Z3_INT_SORT)


class FuncDeclRef:
    def __init__(self, name: str, kind: int, params=(), dom=(), rng: SortRef = None):
        self._name, self._kind, self._params, self._dom, self._rng = name, kind, list(params), tuple(dom), rng

    def name(self):
        return self._name

    def kind(self):
        return self._kind

    def params(self):
        return list(self._params)

    def arity(self):
        return len(self._dom)

    def domain(self, i):
        return self._dom[i]

    def range(self):
        return self._rng

    def key(self):
        return (self._name, self._kind, tuple(self._params), tuple(s.key() for s in self._dom), self._rng.key())

    def __eq__(self, o):
        return isinstance(o, FuncDeclRef) and self.key() == o.key()

    def __hash__(self):
        return hash(self.key())

    def __call__(self, *args):
        return _mk(C.Z3_OP_UNINTERPRETED, self._rng, args, name=self._name, dom=self._dom)


# ----------------------------------------------------------------------------- terms
_intern: Dict[tuple, "ExprRef"] = {}
_ids = itertools.count(1)


class ExprRef:
    __slots__ = ("_decl", "_args", "_sort", "_val", "_id", "__weakref__")

    def get_id(self):
        return self._id

    def decl(self):
        return self._decl

    def children(self):
        return list(self._args)

    def num_args(self):
        return len(self._args)

    def arg(self, i):
        return self._args[i]

    def sort(self):
        return self._sort

    def size(self):
        return self._sort.size()

    def as_long(self):
        assert self._decl.kind() == C.Z3_OP_BNUM
        return self._val

    def __repr__(self):
        d = self._decl
        if d.kind() == C.Z3_OP_BNUM:
            return f"#x{self._val:x}[{self._sort.size()}]"
        if not self._args:
            return d.name()
        return f"({d.name()} {' '.join(map(repr, self._args))})"


def _mk(kind, sort, args=(), name=None, params=(), val=None, dom=None):
    name = name or kind_name(kind)
    args = tuple(args)
    key = (kind, name, tuple(params), tuple(a._id for a in args), sort.key(), val)
    e = _intern.get(key)
    if e is None:
        e = ExprRef()
        e._decl = FuncDeclRef(name, kind, params, dom if dom is not None else tuple(a._sort for a in args), sort)
        e._args, e._sort, e._val, e._id = args, sort, val, next(_ids)
        _intern[key] = e
    return e


def kind_name(kind):
    for n in _KIND_NAMES:
        if getattr(C, "Z3_OP_" + n) == kind:
            return n.lower()
    return f"k{kind}"


class QuantifierRef(ExprRef):
    """A universally quantified formula (never produced by Mythril; the lowering must reject it)."""


def ForAll(body):
    q = QuantifierRef()
    q._decl = FuncDeclRef("forall", -1, (), (), BoolSort())
    q._args, q._sort, q._val, q._id = (body,), BoolSort(), None, next(_ids)
    return q


def is_quantifier(e):
    return isinstance(e, QuantifierRef)


def is_var(e):
    return False


# constructors (z3py names)
def BitVec(name, w):
    return _mk(C.Z3_OP_UNINTERPRETED, BitVecSort(w), name=name)


def BitVecVal(v, w):
    return _mk(C.Z3_OP_BNUM, BitVecSort(w), val=v & ((1 << w) - 1))


def Bool(name):
    return _mk(C.Z3_OP_UNINTERPRETED, BoolSort(), name=name)


def BoolVal(b):
    return _mk(C.Z3_OP_TRUE if b else C.Z3_OP_FALSE, BoolSort(), name="true" if b else "false")


def Int(name):
    return _mk(C.Z3_OP_UNINTERPRETED, IntSort(), name=name)


def Array(name, dom, rng):
    return _mk(C.Z3_OP_UNINTERPRETED, ArraySort(dom, rng), name=name)


def Function(name, *sorts):
    return FuncDeclRef(name, C.Z3_OP_UNINTERPRETED, (), sorts[:-1], sorts[-1])


def K(dom, v):
    return _mk(C.Z3_OP_CONST_ARRAY, ArraySort(dom, v.sort()), (v,))


def Store(a, k, v):
    return _mk(C.Z3_OP_STORE, a.sort(), (a, k, v))


def Select(a, k):
    return _mk(C.Z3_OP_SELECT, a.sort().range(), (a, k))


def If(c, a, b):
    return _mk(C.Z3_OP_ITE, a.sort(), (c, a, b))


def Concat(*a):
    return _mk(C.Z3_OP_CONCAT, BitVecSort(sum(x.size() for x in a)), a)


def Extract(hi, lo, a):
    return _mk(C.Z3_OP_EXTRACT, BitVecSort(hi - lo + 1), (a,), params=(hi, lo))


def ZeroExt(k, a):
    return _mk(C.Z3_OP_ZERO_EXT, BitVecSort(a.size() + k), (a,), params=(k,))


def SignExt(k, a):
    return _mk(C.Z3_OP_SIGN_EXT, BitVecSort(a.size() + k), (a,), params=(k,))


def RepeatBitVec(k, a):
    return _mk(C.Z3_OP_REPEAT, BitVecSort(a.size() * k), (a,), params=(k,))


def bool_op(kind, *a):
    return _mk(kind, BoolSort(), a)


def bv_op(kind, *a):
    return _mk(kind, a[0].sort(), a)


def And(*a):
    return bool_op(C.Z3_OP_AND, *a)


def Or(*a):
    return bool_op(C.Z3_OP_OR, *a)


def Not(a):
    return bool_op(C.Z3_OP_NOT, a)


def Eq(a, b):
    return bool_op(C.Z3_OP_IFF if a.sort().kind() == Z3_BOOL_SORT else C.Z3_OP_EQ, a, b)


# ----------------------------------------------------------------------------- predicates
def is_true(e):
    return isinstance(e, ExprRef) and e.decl().kind() == C.Z3_OP_TRUE


def is_false(e):
    return isinstance(e, ExprRef) and e.decl().kind() == C.Z3_OP_FALSE


def is_bv_value(e):
    return isinstance(e, ExprRef) and e.decl().kind() == C.Z3_OP_BNUM


def is_as_array(e):
    return isinstance(e, ExprRef) and e.decl().kind() == C.Z3_OP_AS_ARRAY


def get_as_array_func(e):
    return e.decl().params()[0]


def is_store(e):
    return isinstance(e, ExprRef) and e.decl().kind() == C.Z3_OP_STORE


def is_K(e):
    return isinstance(e, ExprRef) and e.decl().kind() == C.Z3_OP_CONST_ARRAY


def AsArray(f: FuncDeclRef):
    return _mk(C.Z3_OP_AS_ARRAY, ArraySort(f.domain(0), f.range()), (), name="as-array", params=(f,))


# ----------------------------------------------------------------------------- models
class FuncEntry:
    def __init__(self, args, value):
        self._args, self._value = args, value

    def num_args(self):
        return len(self._args)

    def arg_value(self, j):
        return self._args[j]

    def value(self):
        return self._value


class FuncInterp:
    def __init__(self, arity, entries, else_value):
        self._arity, self._entries, self._else = arity, list(entries), else_value

    def arity(self):
        return self._arity

    def num_entries(self):
        return len(self._entries)

    def entry(self, i):
        return self._entries[i]

    def else_value(self):
        return self._else


class ModelRef:
    """Constants -> literal terms, functions -> FuncInterp, array constants -> AsArray / K /
    Store terms (the three forms of SURVEY Appendix F)."""

    def __init__(self):
        self._interp: Dict[FuncDeclRef, object] = {}

    def set(self, decl: FuncDeclRef, value) -> None:
        self._interp[decl] = value

    def decls(self):
        return list(self._interp)

    def get_interp(self, d):
        return self._interp.get(d)

    def __getitem__(self, d):
        return self._interp.get(d)

    def eval(self, e, model_completion=False):
        assert model_completion
        v = _Eval(self).ev(e)
        if e.sort().kind() == Z3_BOOL_SORT:
            return BoolVal(bool(v))
        return BitVecVal(v, e.size())


def _lit(v):
    if is_true(v):
        return 1
    if is_false(v):
        return 0
    return v.as_long()


def _s(x, w):
    return x - (1 << w) if x >> (w - 1) & 1 else x


class _Arr:
    """An array value: a lookup table plus a default."""

    def __init__(self, table, default):
        self.table, self.default = table, default

    def get(self, k):
        return self.table.get(k, self.default)


class _Eval:
    """SMT-LIB bit-vector semantics + completion, written against the
    stand-in's term objects only (independent of the tape IR and of the oracle)."""

    def __init__(self, m: ModelRef):
        self.m = m
        self.memo: Dict[int, object] = {}

    def func_table(self, decl: FuncDeclRef):
        fi = self.m.get_interp(decl)
        if fi is None:
            return _Arr({}, 0)
        tab = {}
        for i in range(fi.num_entries()):
            en = fi.entry(i)
            tab.setdefault(tuple(_lit(en.arg_value(j)) for j in range(fi.arity())), _lit(en.value()))
        return _Arr(tab, _lit(fi.else_value()))

    def array_value(self, v) -> _Arr:
        if is_as_array(v):
            t = self.func_table(get_as_array_func(v))
            return _Arr({k[0]: x for k, x in t.table.items()}, t.default)
        return self.ev(v)

    def ev(self, e):
        r = self.memo.get(e.get_id())
        if r is None:
            r = self._ev(e)
            self.memo[e.get_id()] = r
        return r

    def _ev(self, e):
        d = e.decl()
        k = d.kind()
        a = e.children()
        srt = e.sort()
        w = srt.size() if srt.kind() == Z3_BV_SORT else 0
        M = (1 << w) - 1 if w else 1
        if k == C.Z3_OP_TRUE:
            return 1
        if k == C.Z3_OP_FALSE:
            return 0
        if k == C.Z3_OP_BNUM:
            return e.as_long()
        if k == C.Z3_OP_UNINTERPRETED:
            if not a:
                v = self.m.get_interp(d)
                if srt.kind() == Z3_ARRAY_SORT:
                    return _Arr({}, 0) if v is None else self.array_value(v)
                return 0 if v is None else _lit(v)
            t = self.func_table(d)
            return t.table.get(tuple(self.ev(x) for x in a), t.default)
        if k == C.Z3_OP_CONST_ARRAY:
            return _Arr({}, self.ev(a[0]))
        if k == C.Z3_OP_STORE:
            base = self.ev(a[0])
            tab = dict(base.table)
            tab[self.ev(a[1])] = self.ev(a[2])
            return _Arr(tab, base.default)
        if k == C.Z3_OP_SELECT:
            return self.ev(a[0]).get(self.ev(a[1]))
        v = [self.ev(x) for x in a]
        aw = a[0].sort().size() if a and a[0].sort().kind() == Z3_BV_SORT else 0
        if k == C.Z3_OP_AND:
            return int(all(v))
        if k == C.Z3_OP_OR:
            return int(any(v))
        if k == C.Z3_OP_NOT:
            return 1 - v[0]
        if k == C.Z3_OP_XOR:
            return v[0] ^ v[1]
        if k == C.Z3_OP_IMPLIES:
            return int((not v[0]) or v[1])
        if k in (C.Z3_OP_EQ, C.Z3_OP_IFF):
            return int(v[0] == v[1])
        if k == C.Z3_OP_DISTINCT:
            return int(len(set(v)) == len(v))
        if k == C.Z3_OP_ITE:
            return v[1] if v[0] else v[2]
        if k == C.Z3_OP_ULT:
            return int(v[0] < v[1])
        if k == C.Z3_OP_ULEQ:
            return int(v[0] <= v[1])
        if k == C.Z3_OP_UGT:
            return int(v[0] > v[1])
        if k == C.Z3_OP_UGEQ:
            return int(v[0] >= v[1])
        if k == C.Z3_OP_SLT:
            return int(_s(v[0], aw) < _s(v[1], aw))
        if k == C.Z3_OP_SLEQ:
            return int(_s(v[0], aw) <= _s(v[1], aw))
        if k == C.Z3_OP_SGT:
            return int(_s(v[0], aw) > _s(v[1], aw))
        if k == C.Z3_OP_SGEQ:
            return int(_s(v[0], aw) >= _s(v[1], aw))
        if k == C.Z3_OP_BUMUL_NO_OVFL:
            return int(v[0] * v[1] <= (1 << aw) - 1)
        if k == C.Z3_OP_BSMUL_NO_OVFL:
            return int(_s(v[0], aw) * _s(v[1], aw) < (1 << (aw - 1)))
        if k == C.Z3_OP_BSMUL_NO_UDFL:
            return int(_s(v[0], aw) * _s(v[1], aw) >= -(1 << (aw - 1)))
        if k == C.Z3_OP_BADD:
            return sum(v) & M
        if k == C.Z3_OP_BMUL:
            r = 1
            for x in v:
                r = r * x & M
            return r
        if k == C.Z3_OP_BAND:
            r = M
            for x in v:
                r &= x
            return r
        if k == C.Z3_OP_BOR:
            r = 0
            for x in v:
                r |= x
            return r
        if k == C.Z3_OP_BXOR:
            r = 0
            for x in v:
                r ^= x
            return r
        if k == C.Z3_OP_BSUB:
            return (v[0] - v[1]) & M
        if k == C.Z3_OP_BNEG:
            return -v[0] & M
        if k == C.Z3_OP_BNOT:
            return ~v[0] & M
        if k == C.Z3_OP_BNAND:
            return ~(v[0] & v[1]) & M
        if k == C.Z3_OP_BNOR:
            return ~(v[0] | v[1]) & M
        if k == C.Z3_OP_BXNOR:
            return ~(v[0] ^ v[1]) & M
        if k in (C.Z3_OP_BUDIV, C.Z3_OP_BUDIV_I):
            return M if v[1] == 0 else v[0] // v[1]
        if k in (C.Z3_OP_BUREM, C.Z3_OP_BUREM_I):
            return v[0] if v[1] == 0 else v[0] % v[1]
        if k in (C.Z3_OP_BSDIV, C.Z3_OP_BSDIV_I):
            x, y = _s(v[0], w), _s(v[1], w)
            if y == 0:
                return 1 if x < 0 else M
            q = abs(x) // abs(y)
            return (-q if (x < 0) != (y < 0) else q) & M
        if k in (C.Z3_OP_BSREM, C.Z3_OP_BSREM_I):
            x, y = _s(v[0], w), _s(v[1], w)
            if y == 0:
                return v[0]
            r = abs(x) % abs(y)
            return (-r if x < 0 else r) & M
        if k in (C.Z3_OP_BSMOD, C.Z3_OP_BSMOD_I):
            x, y = _s(v[0], w), _s(v[1], w)
            return v[0] if y == 0 else (x % y) & M       # Python's % takes the divisor's sign
        if k == C.Z3_OP_BSHL:
            return 0 if v[1] >= w else (v[0] << v[1]) & M
        if k == C.Z3_OP_BLSHR:
            return 0 if v[1] >= w else v[0] >> v[1]
        if k == C.Z3_OP_BASHR:
            return (_s(v[0], w) >> min(v[1], w)) & M
        if k == C.Z3_OP_CONCAT:
            r = 0
            for x, t in zip(v, a):
                r = (r << t.size()) | x
            return r
        if k == C.Z3_OP_EXTRACT:
            hi, lo = d.params()
            return (v[0] >> lo) & ((1 << (hi - lo + 1)) - 1)
        if k == C.Z3_OP_ZERO_EXT:
            return v[0]
        if k == C.Z3_OP_SIGN_EXT:
            return _s(v[0], aw) & M
        if k == C.Z3_OP_REPEAT:
            r = 0
            for _ in range(d.params()[0]):
                r = (r << aw) | v[0]
            return r
        raise NotImplementedError(kind_name(k))


# ----------------------------------------------------------------------------- solver
sat, unsat, unknown = "sat", "unsat", "unknown"


class Optimize:
    """Decides satisfiability by trying the candidate models it was seeded with
    (``Optimize.candidates``, a class attribute the test sets); ``unknown`` when none fits and
    ``Optimize.exhaustive`` is False, else ``unsat``.  Records timeout and objectives."""
    candidates: List[ModelRef] = []
    exhaustive = False
    last: Optional["Optimize"] = None

    def __init__(self):
        self.assertions, self.objectives, self.params = [], [], {}
        self._model = None
        Optimize.last = self

    def set(self, k, v):
        self.params[k] = v

    def add(self, c):
        self.assertions.append(c)

    def minimize(self, e):
        self.objectives.append(("min", e))

    def maximize(self, e):
        self.objectives.append(("max", e))

    def check(self):
        for m in self.candidates:
            if all(is_true(m.eval(c, model_completion=True)) for c in self.assertions):
                self._model = m
                return sat
        return unsat if self.exhaustive else unknown

    def model(self):
        return self._model


# ----------------------------------------------------------------------------- install
def install():
    mod = sys.modules[__name__]
    saved = {k: sys.modules.get(k) for k in ("z3", "z3.z3consts", "mythril_amd.lower_z3")}
    sys.modules["z3"] = mod
    sys.modules["z3.z3consts"] = z3consts
    sys.modules.pop("mythril_amd.lower_z3", None)
    return saved


def uninstall(saved):
    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v
