"""Constraint tapes: the z3-independent IR evaluated by the MI355X kernels.

A tape is the lowering of ONE quick-sat query, i.e. of the z3 term
``simplify(And(*constraints)).raw`` that ``get_model`` hands to
``ModelCache.check_quick_sat`` (reference ``mythril/support/model.py:101``,
``mythril/support/support_utils.py:60-67``).  It is a topologically ordered DAG
(postfix order, operands before users, hash-consed like z3's own AST table —
SURVEY §8 a5) whose last node is the Bool root.

The node vocabulary mirrors the term constructors of the reference's SMT layer
(``mythril/laser/smt/bitvec.py:63-246``, ``bitvec_helper.py``, ``bool.py:98-134``,
``array.py:20-73``, ``function.py:7-29``).  Opcode numbers and the
packed layouts are the C-ABI of ``include/mq.h``.
"""
from __future__ import annotations

import enum
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

NONE = 0xFFFFFFFF
BOOL = 0  # width 0 == Bool sort


class Op(enum.IntEnum):
    CONST = 1
    VAR = 2
    TRUE = 3
    FALSE = 4
    NOT = 10
    AND = 11
    OR = 12
    XOR = 13
    IMPLIES = 14
    IFF = 15
    BITE = 16
    EQ = 20
    ULT = 21
    ULE = 22
    SLT = 23
    SLE = 24
    UMUL_NOOVFL = 25
    SMUL_NOOVFL = 26
    SMUL_NOUDFL = 27
    ADD = 30
    SUB = 31
    MUL = 32
    NEG = 33
    UDIV = 34
    UREM = 35
    SDIV = 36
    SREM = 37
    SMOD = 38
    BAND = 40
    BOR = 41
    BXOR = 42
    BNOT = 43
    SHL = 44
    LSHR = 45
    ASHR = 46
    EXTRACT = 50
    CONCAT = 51
    ZEXT = 52
    SEXT = 53
    ITE = 54
    SELECT = 60
    STORE = 61
    CONST_ARRAY = 62
    ARRAY_VAR = 63
    UF = 64
    UF_CHUNK = 65
    UF_WIDE = 66
    KECCAK = 70


ARRAY_OPS = frozenset({Op.STORE, Op.CONST_ARRAY, Op.ARRAY_VAR})
BOOL_RESULT_OPS = frozenset({
    Op.TRUE, Op.FALSE, Op.NOT, Op.AND, Op.OR, Op.XOR, Op.IMPLIES, Op.IFF, Op.BITE,
    Op.EQ, Op.ULT, Op.ULE, Op.SLT, Op.SLE, Op.UMUL_NOOVFL, Op.SMUL_NOOVFL, Op.SMUL_NOUDFL})

NODE_DTYPE = np.dtype([("op", "<u2"), ("width", "<u2"), ("a", "<u4"), ("b", "<u4"), ("c", "<u4")])
FUNC_DTYPE = np.dtype([("arity", "<u2"), ("result_width", "<u2"), ("arg_width", "<u2", (2,))])


def limbs(width: int) -> int:
    """Number of little-endian u32 limbs that hold a value of ``width`` bits (Bool -> 1)."""
    return 1 if width == 0 else (width + 31) // 32


def to_words(value: int, width: int) -> List[int]:
    n = limbs(width)
    value &= (1 << max(width, 1)) - 1
    return [(value >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def from_words(words: Sequence[int]) -> int:
    v = 0
    for i, w in enumerate(words):
        v |= int(w) << (32 * i)
    return v


class SortError(TypeError):
    pass


class Tape:
    """Hash-consing builder for one constraint DAG.

    Node handles are plain ``int`` indices.  Every constructor checks sorts the way
    z3 does for the corresponding ``Z3_mk_*`` call and raises :class:`SortError`.
    """

    def __init__(self) -> None:
        self.nodes: List[Tuple[int, int, int, int, int]] = []
        self.kind: List[str] = []          # "bool" | "bv" | "array"
        self.consts: List[int] = []        # local const pool (u32 words)
        self._memo: Dict[Tuple[int, int, int, int, int], int] = {}
        self._const_memo: Dict[Tuple[int, int], int] = {}

    # ------------------------------------------------------------ internals
    def _add(self, op: Op, width: int, a: int = 0, b: int = 0, c: int = 0, kind: str = "bv") -> int:
        key = (op.value if isinstance(op, Op) else op, width, a, b, c)
        hit = self._memo.get(key)
        if hit is not None:
            return hit
        idx = len(self.nodes)
        self.nodes.append(key)
        self.kind.append(kind)
        self._memo[key] = idx
        return idx

    def width(self, n: int) -> int:
        return self.nodes[n][1]

    def _bv(self, *ns: int) -> int:
        w = None
        for n in ns:
            if self.kind[n] != "bv":
                raise SortError(f"node {n} is {self.kind[n]}, expected bit-vector")
            if w is None:
                w = self.width(n)
            elif self.width(n) != w:
                raise SortError(f"width mismatch {w} vs {self.width(n)}")
        return w

    def _bool(self, *ns: int) -> None:
        for n in ns:
            if self.kind[n] != "bool":
                raise SortError(f"node {n} is {self.kind[n]}, expected Bool")

    def __len__(self) -> int:
        return len(self.nodes)

    @property
    def root(self) -> int:
        return len(self.nodes) - 1

    def finish(self, root: int, value_root: bool = False) -> "Tape":
        """Make ``root`` the last node (the evaluated root) — re-emits the live DAG in postfix order.
        ``value_root``: a BV/Bool root whose VALUE is the result (column programs of hoisting)."""
        if value_root:
            if self.kind[root] == "array":
                raise SortError("a column program's root cannot be an array")
        else:
            self._bool(root)
        if root == len(self.nodes) - 1 and not getattr(self, "has_dead", False):
            return self
        out = Tape()
        remap: Dict[int, int] = {}
        order: List[int] = []
        seen = set()
        stack = [(root, False)]
        while stack:
            n, done = stack.pop()
            if done:
                order.append(n)
                continue
            if n in seen:
                continue
            seen.add(n)
            stack.append((n, True))
            for ch in reversed(self.children(n)):
                if ch not in seen:
                    stack.append((ch, False))
        for n in order:
            op, w, a, b, c = self.nodes[n]
            op = Op(op)
            args = [a, b, c]
            for i in self.operand_slots(op):
                if args[i] != NONE:
                    args[i] = remap[args[i]]
            if op == Op.CONST:
                words = self.consts[a:a + limbs(w)]
                remap[n] = out.const(from_words(words), w)
                continue
            remap[n] = out._add(op, w, args[0], args[1], args[2], self.kind[n])
        return out

    @staticmethod
    def operand_slots(op: Op) -> Tuple[int, ...]:
        """Which of (a, b, c) are node references for ``op``."""
        if op in (Op.CONST, Op.VAR, Op.TRUE, Op.FALSE, Op.ARRAY_VAR):
            return ()
        if op in (Op.NOT, Op.NEG, Op.BNOT, Op.EXTRACT, Op.ZEXT, Op.SEXT, Op.CONST_ARRAY, Op.KECCAK):
            return (0,)
        if op in (Op.BITE, Op.ITE, Op.STORE):
            return (0, 1, 2)
        if op in (Op.UF, Op.UF_CHUNK):
            return (1, 2)
        if op == Op.UF_WIDE:
            return (1,)
        return (0, 1)

    def children(self, n: int) -> List[int]:
        op, w, a, b, c = self.nodes[n]
        args = (a, b, c)
        return [args[i] for i in self.operand_slots(Op(op)) if args[i] != NONE]

    # ------------------------------------------------------------ leaves
    def const(self, value: int, width: int) -> int:
        if width <= 0:
            raise SortError("BV constants need width >= 1 (use true()/false())")
        value &= (1 << width) - 1
        key = (value, width)
        off = self._const_memo.get(key)
        if off is None:
            off = len(self.consts)
            self.consts.extend(to_words(value, width))
            self._const_memo[key] = off
        return self._add(Op.CONST, width, off)

    def var(self, index: int, width: int) -> int:
        return self._add(Op.VAR, width, index, kind="bool" if width == BOOL else "bv")

    def true(self) -> int:
        return self._add(Op.TRUE, BOOL, kind="bool")

    def false(self) -> int:
        return self._add(Op.FALSE, BOOL, kind="bool")

    # ------------------------------------------------------------ Bool
    def not_(self, a: int) -> int:
        self._bool(a)
        return self._add(Op.NOT, BOOL, a, kind="bool")

    def _bool2(self, op: Op, a: int, b: int) -> int:
        self._bool(a, b)
        return self._add(op, BOOL, a, b, kind="bool")

    def and_(self, *args: int) -> int:
        if not args:
            return self.true()
        acc = args[0]
        self._bool(acc)
        for x in args[1:]:
            acc = self._bool2(Op.AND, acc, x)
        return acc

    def or_(self, *args: int) -> int:
        if not args:
            return self.false()
        acc = args[0]
        self._bool(acc)
        for x in args[1:]:
            acc = self._bool2(Op.OR, acc, x)
        return acc

    def xor(self, a: int, b: int) -> int:
        return self._bool2(Op.XOR, a, b)

    def implies(self, a: int, b: int) -> int:
        return self._bool2(Op.IMPLIES, a, b)

    def iff(self, a: int, b: int) -> int:
        return self._bool2(Op.IFF, a, b)

    def bite(self, c: int, a: int, b: int) -> int:
        self._bool(c, a, b)
        return self._add(Op.BITE, BOOL, c, a, b, kind="bool")

    # ------------------------------------------------------------ predicates
    def _pred(self, op: Op, a: int, b: int) -> int:
        self._bv(a, b)
        return self._add(op, BOOL, a, b, kind="bool")

    def eq(self, a: int, b: int) -> int:
        if self.kind[a] == "bool":
            return self.iff(a, b)
        return self._pred(Op.EQ, a, b)

    def distinct(self, a: int, b: int) -> int:
        return self.not_(self.eq(a, b))

    def ult(self, a: int, b: int) -> int:
        return self._pred(Op.ULT, a, b)

    def ule(self, a: int, b: int) -> int:
        return self._pred(Op.ULE, a, b)

    def ugt(self, a: int, b: int) -> int:
        return self._pred(Op.ULT, b, a)

    def uge(self, a: int, b: int) -> int:
        return self._pred(Op.ULE, b, a)

    def slt(self, a: int, b: int) -> int:
        return self._pred(Op.SLT, a, b)

    def sle(self, a: int, b: int) -> int:
        return self._pred(Op.SLE, a, b)

    def sgt(self, a: int, b: int) -> int:
        return self._pred(Op.SLT, b, a)

    def sge(self, a: int, b: int) -> int:
        return self._pred(Op.SLE, b, a)

    def umul_noovfl(self, a: int, b: int) -> int:
        return self._pred(Op.UMUL_NOOVFL, a, b)

    def smul_noovfl(self, a: int, b: int) -> int:
        return self._pred(Op.SMUL_NOOVFL, a, b)

    def smul_noudfl(self, a: int, b: int) -> int:
        return self._pred(Op.SMUL_NOUDFL, a, b)

    # ------------------------------------------------------------ BV
    def _bin(self, op: Op, a: int, b: int) -> int:
        w = self._bv(a, b)
        return self._add(op, w, a, b)

    def add(self, a, b): return self._bin(Op.ADD, a, b)
    def sub(self, a, b): return self._bin(Op.SUB, a, b)
    def mul(self, a, b): return self._bin(Op.MUL, a, b)
    def udiv(self, a, b): return self._bin(Op.UDIV, a, b)
    def urem(self, a, b): return self._bin(Op.UREM, a, b)
    def sdiv(self, a, b): return self._bin(Op.SDIV, a, b)
    def srem(self, a, b): return self._bin(Op.SREM, a, b)
    def smod(self, a, b): return self._bin(Op.SMOD, a, b)
    def band(self, a, b): return self._bin(Op.BAND, a, b)
    def bor(self, a, b): return self._bin(Op.BOR, a, b)
    def bxor(self, a, b): return self._bin(Op.BXOR, a, b)
    def shl(self, a, b): return self._bin(Op.SHL, a, b)
    def lshr(self, a, b): return self._bin(Op.LSHR, a, b)
    def ashr(self, a, b): return self._bin(Op.ASHR, a, b)

    def neg(self, a: int) -> int:
        return self._add(Op.NEG, self._bv(a), a)

    def bnot(self, a: int) -> int:
        return self._add(Op.BNOT, self._bv(a), a)

    def extract(self, hi: int, lo: int, a: int) -> int:
        w = self._bv(a)
        if not (0 <= lo <= hi < w):
            raise SortError(f"extract({hi},{lo}) out of range for width {w}")
        return self._add(Op.EXTRACT, hi - lo + 1, a, hi, lo)

    def concat(self, *args: int) -> int:
        acc = args[0]
        self._bv(acc)
        for x in args[1:]:
            self._bv(x)
            acc = self._add(Op.CONCAT, self.width(acc) + self.width(x), acc, x)
        return acc

    def zext(self, k: int, a: int) -> int:
        w = self._bv(a)
        return a if k == 0 else self._add(Op.ZEXT, w + k, a, k)

    def sext(self, k: int, a: int) -> int:
        w = self._bv(a)
        return a if k == 0 else self._add(Op.SEXT, w + k, a, k)

    def ite(self, c: int, a: int, b: int) -> int:
        self._bool(c)
        if self.kind[a] == "bool":
            return self.bite(c, a, b)
        w = self._bv(a, b)
        return self._add(Op.ITE, w, c, a, b)

    def keccak(self, a: int) -> int:
        w = self._bv(a)
        if w % 8:
            raise SortError("keccak input width must be a multiple of 8")
        return self._add(Op.KECCAK, 256, a)

    # ------------------------------------------------------------ arrays / UF
    def array_var(self, func: int, range_width: int) -> int:
        return self._add(Op.ARRAY_VAR, range_width, func, kind="array")

    def const_array(self, value: int) -> int:
        return self._add(Op.CONST_ARRAY, self.width(value), value, kind="array")

    def store(self, arr: int, idx: int, val: int) -> int:
        if self.kind[arr] != "array":
            raise SortError("store on non-array")
        return self._add(Op.STORE, self.width(arr), arr, idx, val, kind="array")

    def select(self, arr: int, idx: int) -> int:
        if self.kind[arr] != "array":
            raise SortError("select on non-array")
        w = self.width(arr)
        return self._add(Op.SELECT, w, arr, idx, kind="bool" if w == BOOL else "bv")

    def uf(self, func: int, result_width: int, *args: int) -> int:
        if not 1 <= len(args) <= 2:
            raise SortError("UF arity must be 1 or 2")
        b = args[0]
        c = args[1] if len(args) > 1 else NONE
        return self._add(Op.UF, result_width, func, b, c, kind="bool" if result_width == BOOL else "bv")

    def uf_wide(self, func: int, result_width: int, chunks: Sequence[int]) -> int:
        """Arity-1 lookup of a key given as 256-bit chunks, lowest first (mq.h MQ_OP_UF_CHUNK /
        MQ_OP_UF_WIDE): a key wider than any value may be."""
        prev = NONE
        for ch in chunks:
            if self.kind[ch] != "bv" or self.width(ch) > 256:
                raise SortError("UF key chunks are BV values of at most 256 bits")
            prev = self._add(Op.UF_CHUNK, 64, func, ch, prev)
        if prev == NONE:
            raise SortError("UF key without chunks")
        return self._add(Op.UF_WIDE, result_width, func, prev, NONE, kind="bool" if result_width == BOOL else "bv")

    # ------------------------------------------------------------ packing
    def packed(self) -> Tuple[np.ndarray, np.ndarray]:
        nodes = np.array(self.nodes, dtype=np.uint64).reshape(-1, 5) if self.nodes else np.zeros((0, 5), np.uint64)
        arr = np.zeros(len(self.nodes), dtype=NODE_DTYPE)
        if len(self.nodes):
            arr["op"] = nodes[:, 0]
            arr["width"] = nodes[:, 1]
            arr["a"] = nodes[:, 2]
            arr["b"] = nodes[:, 3]
            arr["c"] = nodes[:, 4]
        return arr, np.asarray(self.consts, dtype=np.uint32)


class TapeBatch:
    """N tapes packed into the ``mq_tape_batch`` layout (include/mq.h)."""

    def __init__(self, tapes: Sequence[Tape]):
        node_chunks, const_chunks = [], []
        offsets = [0]
        cbase = 0
        for t in tapes:
            if len(t) == 0:
                raise ValueError("empty tape")
            arr, consts = t.packed()
            arr = arr.copy()
            is_const = arr["op"] == Op.CONST
            arr["a"][is_const] += np.uint32(cbase)
            node_chunks.append(arr)
            const_chunks.append(consts)
            cbase += len(consts)
            offsets.append(offsets[-1] + len(arr))
        self.n_tapes = len(tapes)
        self.nodes = np.concatenate(node_chunks) if node_chunks else np.zeros(0, NODE_DTYPE)
        self.consts = np.concatenate(const_chunks).astype(np.uint32) if const_chunks else np.zeros(0, np.uint32)
        if self.consts.size == 0:
            self.consts = np.zeros(1, np.uint32)
        self.offsets = np.asarray(offsets, dtype=np.int64)
        self.columns = None  # Optional[ColumnSet]: model-level sub-terms hoisted out of the batch

    @classmethod
    def from_arrays(cls, nodes: np.ndarray, offsets: np.ndarray, consts: np.ndarray) -> "TapeBatch":
        self = cls.__new__(cls)
        self.nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.consts = np.ascontiguousarray(consts, dtype=np.uint32)
        if self.consts.size == 0:
            self.consts = np.zeros(1, np.uint32)
        self.n_tapes = len(self.offsets) - 1
        self.columns = None
        return self

    def tape_nodes(self, t: int) -> np.ndarray:
        return self.nodes[self.offsets[t]:self.offsets[t + 1]]

    def sizes(self) -> np.ndarray:
        return np.diff(self.offsets)

    def subset(self, idx: Sequence[int]) -> "TapeBatch":
        chunks = [self.tape_nodes(int(t)) for t in idx]
        offs = np.zeros(len(chunks) + 1, np.int64)
        offs[1:] = np.cumsum([len(c) for c in chunks])
        nodes = np.concatenate(chunks) if chunks else np.zeros(0, NODE_DTYPE)
        return TapeBatch.from_arrays(nodes, offs, self.consts)


class ColumnSet:
    """Sub-terms shared by several tapes of a batch, hoisted into derived model columns.

    A shared sub-term depends only on the model, so it is evaluated once per model (column program
    ``programs`` tape k, BV/Bool root) and written into model variable ``var_index[k]``; the tapes
    of the batch read it as a variable.  ``level[k]``: columns of level j only read columns of
    levels < j (one launch per level)."""

    def __init__(self, programs: "TapeBatch", var_index: Sequence[int], level: Sequence[int]):
        self.programs = programs
        self.var_index = np.asarray(var_index, dtype=np.int32)
        self.level = np.asarray(level, dtype=np.int32)

    @property
    def n(self) -> int:
        return int(self.var_index.size)
