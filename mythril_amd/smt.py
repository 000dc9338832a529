"""z3-free symbolic terms with the constructor vocabulary of the reference's SMT layer.

The reference builds path constraints through thin wrappers over z3
(``mythril/laser/smt/{bitvec,bitvec_helper,bool,array,function}.py``, ``symbol_factory``
``mythril/laser/smt/__init__.py:83-154``).  This module restates that vocabulary — with the
same operator meanings — as hash-consed Python terms, so that the quick-sat path can be
driven, tested and benchmarked where z3 is absent (this container and the GPU box).  On a
z3 host the adapter lowers real z3 ASTs instead (:mod:`mythril_amd.lower_z3`); both lowerings
produce the same tape IR.

Operator meanings follow the reference exactly:
  * ``a / b`` is **bvsdiv** (``bitvec.py:96-103``); ``UDiv``/``URem``/``SRem`` are helpers;
  * ``< > <= >=`` are **signed** (``bitvec.py:138-180``); ``ULT/UGT`` are unsigned and
    ``ULE``/``UGE`` are built as ``Or(ULT, ==)`` / ``Or(UGT, ==)`` (``bitvec_helper.py:85-112``);
  * ``==``/``!=`` between bit-vectors of different widths zero-pad the narrower operand
    (``bitvec.py:16-22``);
  * ``<<`` is bvshl and ``>>`` is **bvashr** (``bitvec.py:218-246``); ``LShR`` is logical;
  * Bool ``==`` is iff; ``And``/``Or`` are n-ary (``bool.py:98-125``).

Terms are interned: structurally equal terms are the same object, so ``is``/``id`` identify
them, hashing is O(1), and a DAG shares sub-terms exactly like z3's AST table.
"""
from __future__ import annotations

import weakref
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

from .tape import BOOL

# term kinds (not tape opcodes: the lowering maps these onto include/mq.h opcodes)
SYM = "sym"            # free constant: params = (name,)
VAL = "val"            # BV literal: params = (value,)
TRUE, FALSE = "true", "false"
NOT, AND, OR, XOR, IMPLIES, IFF, BITE = "not", "and", "or", "xor", "=>", "iff", "bite"
EQ, BVULT, BVULE, BVSLT, BVSLE = "=", "bvult", "bvule", "bvslt", "bvsle"
UMUL_NOOVFL, SMUL_NOOVFL, SMUL_NOUDFL = "bvumul_noovfl", "bvsmul_noovfl", "bvsmul_noudfl"
ADD, SUB, MUL, NEG = "bvadd", "bvsub", "bvmul", "bvneg"
UDIV, UREM, SDIV, SREM, SMOD = "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"
BAND, BOR, BXOR, BNOT = "bvand", "bvor", "bvxor", "bvnot"
SHL, LSHR, ASHR = "bvshl", "bvlshr", "bvashr"
EXTRACT, CONCAT, ZEXT, SEXT, ITE = "extract", "concat", "zero_extend", "sign_extend", "ite"
SELECT, STORE, CONST_ARRAY, ARRAY_SYM, APP = "select", "store", "K", "array", "app"
KECCAK = "keccak256"   # interpreted keccak (not a reference constructor: see Keccak256)

_INTERN: "weakref.WeakValueDictionary[tuple, Term]" = weakref.WeakValueDictionary()


class Term:
    """One interned node.  ``sort`` is "bool", "bv" or "array"; ``width`` is the BV width
    (0 for Bool; the range width for arrays, with ``domain`` the index width)."""

    __slots__ = ("kind", "sort", "width", "args", "params", "domain", "__weakref__")

    def __new__(cls, kind: str, sort: str, width: int, args: Tuple["Term", ...] = (),
                params: tuple = (), domain: int = 0):
        key = (kind, sort, width, tuple(id(a) for a in args), params, domain)
        t = _INTERN.get(key)
        if t is not None and t.args == args:
            return t
        t = object.__new__(cls)
        t.kind, t.sort, t.width, t.args, t.params, t.domain = kind, sort, width, args, params, domain
        _INTERN[key] = t
        return t

    # identity semantics: interning makes structural equality object identity
    def __hash__(self) -> int:
        return id(self)

    def __repr__(self) -> str:
        if self.kind == SYM:
            return str(self.params[0])
        if self.kind == VAL:
            return f"{self.params[0]:#x}[{self.width}]"
        if self.kind in (TRUE, FALSE):
            return self.kind
        inner = " ".join([repr(p) for p in self.params] + [repr(a) for a in self.args])
        return f"({self.kind} {inner})"

    def __bool__(self) -> bool:
        """Like z3's ``BoolRef.__bool__``: literal true/false, or structural identity of the two
        sides of an equality (what lets ``lru_cache`` compare keys, support_utils.py:60)."""
        if self.kind == TRUE:
            return True
        if self.kind == FALSE:
            return False
        if self.kind in (EQ, IFF) and len(self.args) == 2:
            return self.args[0] is self.args[1]
        raise TypeError(f"symbolic term {self!r} has no truth value")

    # ------------------------------------------------------------ BV operators (bitvec.py)
    def size(self) -> int:
        return self.width

    @property
    def symbolic(self) -> bool:
        return self.kind != VAL

    @property
    def value(self) -> Optional[int]:
        if self.kind == VAL:
            return self.params[0]
        if self.kind == TRUE:
            return True
        if self.kind == FALSE:
            return False
        return None

    def _other(self, o) -> "Term":
        if isinstance(o, Term):
            return o
        if isinstance(o, bool) and self.sort == "bool":
            return BoolVal(o)
        return BitVecVal(int(o), self.width)

    def __add__(self, o): return _bin(ADD, self, self._other(o))
    def __radd__(self, o): return _bin(ADD, self._other(o), self)
    def __sub__(self, o): return _bin(SUB, self, self._other(o))
    def __rsub__(self, o): return _bin(SUB, self._other(o), self)
    def __mul__(self, o): return _bin(MUL, self, self._other(o))
    def __rmul__(self, o): return _bin(MUL, self._other(o), self)
    def __truediv__(self, o): return _bin(SDIV, self, self._other(o))
    def __and__(self, o): return _bin(BAND, self, self._other(o))
    def __or__(self, o): return _bin(BOR, self, self._other(o))
    def __xor__(self, o): return _bin(BXOR, self, self._other(o))
    def __lshift__(self, o): return _bin(SHL, self, self._other(o))
    def __rshift__(self, o): return _bin(ASHR, self, self._other(o))
    def __neg__(self): return Term(NEG, "bv", _bv(self), (self,))
    def __invert__(self): return Term(BNOT, "bv", _bv(self), (self,))
    def __lt__(self, o): return _pred(BVSLT, self, self._other(o))
    def __gt__(self, o): return _pred(BVSLT, self._other(o), self)
    def __le__(self, o): return _pred(BVSLE, self, self._other(o))
    def __ge__(self, o): return _pred(BVSLE, self._other(o), self)

    def __eq__(self, o):  # type: ignore[override]
        o = self._other(o)
        if self.sort == "bool":
            _bool(o)
            return Term(IFF, "bool", BOOL, (self, o))
        a, b = _pad(self, o)
        return Term(EQ, "bool", BOOL, (a, b))

    def __ne__(self, o):  # type: ignore[override]
        return Not(self.__eq__(o))

    # ------------------------------------------------------------ arrays (array.py:20-30)
    def __getitem__(self, idx) -> "Term":
        if self.sort != "array":
            raise TypeError("select on a non-array")
        if not isinstance(idx, Term):
            idx = BitVecVal(int(idx), self.domain)
        return Term(SELECT, "bool" if self.width == BOOL else "bv", self.width, (self, idx))


def _bv(t: Term) -> int:
    if t.sort != "bv":
        raise TypeError(f"expected a bit-vector, got {t.sort}")
    return t.width


def _bool(*ts: Term) -> None:
    for t in ts:
        if t.sort != "bool":
            raise TypeError(f"expected Bool, got {t.sort}")


def _same(a: Term, b: Term) -> int:
    w = _bv(a)
    if _bv(b) != w:
        raise TypeError(f"width mismatch {w} vs {b.width}")
    return w


def _bin(kind: str, a: Term, b: Term) -> Term:
    return Term(kind, "bv", _same(a, b), (a, b))


def _pred(kind: str, a: Term, b: Term) -> Term:
    _same(a, b)
    return Term(kind, "bool", BOOL, (a, b))


def _pad(a: Term, b: Term) -> Tuple[Term, Term]:
    """``_padded_operation`` (bitvec.py:16-22): zero-extend the narrower side by Concat(0, x);
    the wider operand goes first, as in the reference."""
    if _bv(a) == _bv(b):
        return a, b
    if a.width < b.width:
        a, b = b, a
    return a, Concat(BitVecVal(0, a.width - b.width), b)


# ---------------------------------------------------------------- symbol_factory
def BitVecSym(name: str, size: int) -> Term:
    return Term(SYM, "bv", int(size), (), (str(name),))


def BitVecVal(value: int, size: int) -> Term:
    size = int(size)
    return Term(VAL, "bv", size, (), (int(value) & ((1 << size) - 1),))


def BoolSym(name: str) -> Term:
    return Term(SYM, "bool", BOOL, (), (str(name),))


def BoolVal(value: bool) -> Term:
    return Term(TRUE if value else FALSE, "bool", BOOL)


class _SymbolFactory:
    """Mirror of ``symbol_factory`` (mythril/laser/smt/__init__.py:83-154)."""
    Bool = staticmethod(BoolVal)
    BoolSym = staticmethod(BoolSym)
    BitVecVal = staticmethod(BitVecVal)
    BitVecSym = staticmethod(BitVecSym)


symbol_factory = _SymbolFactory()


def _as_bool(x) -> Term:
    return x if isinstance(x, Term) else BoolVal(bool(x))


# ---------------------------------------------------------------- bool.py
def And(*args) -> Term:
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = tuple(args[0])
    ts = tuple(_as_bool(a) for a in args)
    _bool(*ts)
    if not ts:
        return BoolVal(True)
    return Term(AND, "bool", BOOL, ts)


def Or(*args) -> Term:
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = tuple(args[0])
    ts = tuple(_as_bool(a) for a in args)
    _bool(*ts)
    if not ts:
        return BoolVal(False)
    return Term(OR, "bool", BOOL, ts)


def Not(a) -> Term:
    a = _as_bool(a)
    _bool(a)
    return Term(NOT, "bool", BOOL, (a,))


def Xor(a, b) -> Term:
    a, b = _as_bool(a), _as_bool(b)
    _bool(a, b)
    return Term(XOR, "bool", BOOL, (a, b))


def Implies(a, b) -> Term:
    a, b = _as_bool(a), _as_bool(b)
    _bool(a, b)
    return Term(IMPLIES, "bool", BOOL, (a, b))


def is_true(a: Term) -> bool:
    return a.kind == TRUE


def is_false(a: Term) -> bool:
    return a.kind == FALSE


# ---------------------------------------------------------------- bitvec_helper.py
def If(c, a, b) -> Term:
    """bitvec_helper.py:44-72: ints are lifted to the width of the BV operand (default 256)."""
    c = _as_bool(c)
    _bool(c)
    if isinstance(a, Term) and a.sort == "bool":
        b = _as_bool(b)
        _bool(b)
        return Term(BITE, "bool", BOOL, (c, a, b))
    w = 256
    if isinstance(a, Term):
        w = a.width
    if isinstance(b, Term):
        w = b.width
    a = a if isinstance(a, Term) else BitVecVal(int(a), w)
    b = b if isinstance(b, Term) else BitVecVal(int(b), w)
    if a.sort == "array" or b.sort == "array":
        # an array-valued If (the state-merge plugin: If(cond, state1.balances, state2.balances),
        # merge_states.py:27-29): the lowering pushes every select through it
        if a.sort != b.sort or a.width != b.width or a.domain != b.domain:
            raise TypeError("If over arrays of different sorts")
        return Term(ITE, "array", a.width, (c, a, b), (), a.domain)
    return Term(ITE, "bv", _same(a, b), (c, a, b))


def ULT(a: Term, b: Term) -> Term: return _pred(BVULT, a, b)
def UGT(a: Term, b: Term) -> Term: return _pred(BVULT, b, a)
def ULE(a: Term, b: Term) -> Term: return Or(ULT(a, b), a == b)   # bitvec_helper.py:105-112
def UGE(a: Term, b: Term) -> Term: return Or(UGT(a, b), a == b)   # bitvec_helper.py:85-92
def UDiv(a: Term, b: Term) -> Term: return _bin(UDIV, a, b)
def URem(a: Term, b: Term) -> Term: return _bin(UREM, a, b)
def SRem(a: Term, b: Term) -> Term: return _bin(SREM, a, b)
def SMod(a: Term, b: Term) -> Term: return _bin(SMOD, a, b)
def LShR(a: Term, b: Term) -> Term: return _bin(LSHR, a, b)


def Concat(*args) -> Term:
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = tuple(args[0])
    acc = args[0]
    _bv(acc)
    for x in args[1:]:
        if acc.kind == VAL and x.kind == VAL:   # concrete: folded, as z3's simplify does
            acc = BitVecVal((acc.params[0] << x.width) | x.params[0], acc.width + x.width)
        else:
            acc = Term(CONCAT, "bv", acc.width + _bv(x), (acc, x))
    return acc


def Extract(high: int, low: int, bv: Term) -> Term:
    w = _bv(bv)
    if not 0 <= low <= high < w:
        raise TypeError(f"Extract({high},{low}) out of range for width {w}")
    if bv.kind == VAL:
        return BitVecVal(bv.params[0] >> low, high - low + 1)
    return Term(EXTRACT, "bv", high - low + 1, (bv,), (int(high), int(low)))


def ZeroExt(k: int, bv: Term) -> Term:
    return bv if k == 0 else Term(ZEXT, "bv", _bv(bv) + int(k), (bv,), (int(k),))


def SignExt(k: int, bv: Term) -> Term:
    return bv if k == 0 else Term(SEXT, "bv", _bv(bv) + int(k), (bv,), (int(k),))


def Sum(*args: Term) -> Term:
    acc = args[0]
    for x in args[1:]:
        acc = acc + x
    return acc


def _lift256(x) -> Term:
    return x if isinstance(x, Term) else BitVecVal(int(x), 256)


def BVAddNoOverflow(a, b, signed: bool) -> Term:
    """z3 ``Z3_mk_bvadd_no_overflow`` as the z3 API builds it (bitvec_helper.py:200-212)."""
    a, b = _lift256(a), _lift256(b)
    w = _same(a, b)
    if signed:
        zero = BitVecVal(0, w)
        return Implies(And(_pred(BVSLT, zero, a), _pred(BVSLT, zero, b)), _pred(BVSLT, zero, a + b))
    s = ZeroExt(1, a) + ZeroExt(1, b)
    return Extract(w, w, s) == BitVecVal(0, 1)


def BVMulNoOverflow(a, b, signed: bool) -> Term:
    """bitvec_helper.py:215-228 -> ``bvumul_noovfl`` / ``bvsmul_noovfl``."""
    a, b = _lift256(a), _lift256(b)
    return _pred(SMUL_NOOVFL if signed else UMUL_NOOVFL, a, b)


def BVSubNoUnderflow(a, b, signed: bool) -> Term:
    """bitvec_helper.py:231-246; unsigned form is ``bvule(b, a)``."""
    a, b = _lift256(a), _lift256(b)
    w = _same(a, b)
    if signed:
        zero = BitVecVal(0, w)
        return Implies(And(_pred(BVSLT, a, zero), _pred(BVSLT, zero, b)), _pred(BVSLT, a - b, zero))
    return _pred(BVULE, b, a)


# ---------------------------------------------------------------- array.py / function.py
def Array(name: str, domain: int, value_range: int) -> Term:
    """A symbolic array constant (array.py:45-57): read through the model's interpretation."""
    return Term(ARRAY_SYM, "array", int(value_range), (), (str(name),), int(domain))


def K(domain: int, value_range: int, value: int) -> Term:
    """Constant array (array.py:60-73)."""
    return Term(CONST_ARRAY, "array", int(value_range), (BitVecVal(value, value_range),), (), int(domain))


def Store(arr: Term, idx, val) -> Term:
    if arr.sort != "array":
        raise TypeError("store on non-array")
    idx = idx if isinstance(idx, Term) else BitVecVal(int(idx), arr.domain)
    val = val if isinstance(val, Term) else BitVecVal(int(val), arr.width)
    if idx.width != arr.domain or val.width != arr.width:
        raise TypeError("store sort mismatch")
    return Term(STORE, "array", arr.width, (arr, idx, val), (), arr.domain)


def Select(arr: Term, idx) -> Term:
    return arr[idx]


class Function:
    """Uninterpreted function (function.py:7-29): ``keccak256_<n>``, ``keccak256_<n>-1``, ``Power``."""

    def __init__(self, name: str, domain: Sequence[int], value_range: int):
        self.name = str(name)
        self.domain = tuple(int(d) for d in domain)
        self.range = int(value_range)

    def __call__(self, *items) -> Term:
        if len(items) != len(self.domain):
            raise TypeError(f"{self.name} expects {len(self.domain)} arguments")
        args = tuple(x if isinstance(x, Term) else BitVecVal(int(x), w) for x, w in zip(items, self.domain))
        for x, w in zip(args, self.domain):
            if _bv(x) != w:
                raise TypeError(f"{self.name}: argument width {x.width} != {w}")
        return Term(APP, "bv", self.range, args, (self.name, self.domain))


def Keccak256(data: Term) -> Term:
    """INTERPRETED keccak256 of the big-endian bytes of ``data`` (256-bit result).  Not z3's
    semantics — Mythril models hashes as the UF ``keccak256_<n>`` — and only equal to it on
    keccak-consistent models.  Concrete inputs are what ``find_concrete_keccak``
    hashes (keccak_function_manager.py:56-69)."""
    w = _bv(data)
    if w % 8:
        raise TypeError("keccak input width must be a multiple of 8")
    return Term(KECCAK, "bv", 256, (data,))


def walk(root: Term) -> List[Term]:
    """Postfix order of the DAG under ``root`` (each node once; iterative: tapes can be 10^4 deep)."""
    order: List[Term] = []
    seen = set()
    stack: List[Tuple[Term, bool]] = [(root, False)]
    while stack:
        t, done = stack.pop()
        if done:
            order.append(t)
            continue
        if id(t) in seen:
            continue
        seen.add(id(t))
        stack.append((t, True))
        for a in reversed(t.args):
            if id(a) not in seen:
                stack.append((a, False))
    return order


def symbols(root: Term) -> Dict[str, Term]:
    """Free constants, symbolic arrays and UF applications' function names under ``root``."""
    out: Dict[str, Term] = {}
    for t in walk(root):
        if t.kind in (SYM, ARRAY_SYM):
            out[t.params[0]] = t
    return out
