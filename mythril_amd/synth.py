"""Seeded synthetic workloads, all RNG = numpy PCG64 with committed seeds.

* ``c2_workload``  — config C2: N tapes of ~64 DAG nodes over {ADD, MUL, AND, EQ, ULT}
  with a Bool-AND root over 4 comparisons, V = 8 free 256-bit vars, M i.i.d. uniform
  256-bit models; 10 % of the tapes have ONE planted satisfying model at a uniformly random
  index (they contain an EQ so no other model satisfies them w.p. 1-2^-256·M), the other
  90 % are unsatisfiable against every model (no early exit: the worst case).
* ``fuzz_tape``    — random well-sorted tapes over the whole op vocabulary and mixed widths
  (parity tests).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from .models import FuncSpec, ModelBatch
from .tape import BOOL, Op, Tape, TapeBatch, limbs

M256 = (1 << 256) - 1


def random_words(rng: np.random.Generator, n_rows: int, n_models: int) -> np.ndarray:
    return rng.integers(0, 1 << 32, size=(n_rows, n_models), dtype=np.uint64).astype(np.uint32)


def _model_value(words: np.ndarray, v: int, m: int, nl: int = 8) -> int:
    col = words[v * nl:(v + 1) * nl, m]
    return sum(int(x) << (32 * i) for i, x in enumerate(col))


# ---------------------------------------------------------------- C2
class _C2Expr:
    """Random expression tree over {ADD, MUL, AND} returned as (tape node, python value fn)."""

    def __init__(self, rng: np.random.Generator, tape: Tape, n_vars: int, vals: Sequence[int]):
        self.rng, self.t, self.n_vars, self.vals = rng, tape, n_vars, vals

    def leaf(self) -> Tuple[int, int]:
        if self.rng.random() < 0.7:
            v = int(self.rng.integers(self.n_vars))
            return self.t.var(v, 256), self.vals[v]
        c = int.from_bytes(self.rng.bytes(32), "little")
        return self.t.const(c, 256), c

    def tree(self, n_ops: int) -> Tuple[int, int]:
        if n_ops == 0:
            return self.leaf()
        left = int(self.rng.integers(0, n_ops))
        a, va = self.tree(left)
        b, vb = self.tree(n_ops - 1 - left)
        op = self.rng.choice(3, p=[0.4, 0.25, 0.35])
        if op == 0:
            return self.t.add(a, b), (va + vb) & M256
        if op == 1:
            return self.t.mul(a, b), (va * vb) & M256
        return self.t.band(a, b), va & vb


def c2_tape(rng: np.random.Generator, planted_vals: Optional[Sequence[int]], n_vars: int = 8,
            n_cmp: int = 4, ops_per_side: int = 5) -> Tape:
    t = Tape()
    vals = planted_vals if planted_vals is not None else [0] * n_vars
    gen = _C2Expr(rng, t, n_vars, vals)
    cmps = []
    for i in range(n_cmp):
        a, va = gen.tree(ops_per_side)
        b, vb = gen.tree(ops_per_side - 2)
        kind = "eq" if i == 0 else ("eq" if rng.random() < 0.3 else "ult")
        if kind == "eq":
            # EQ(a, b + c): planted -> c = a(p) - b(p); else c uniform (unsat w.p. ~1)
            if planted_vals is not None:
                c = (va - vb) & M256
            else:
                c = int.from_bytes(rng.bytes(32), "little")
            cmps.append(t.eq(a, t.add(b, t.const(c, 256))))
        else:
            if planted_vals is not None and not va < vb:
                a, b = b, a
            cmps.append(t.ult(a, b))
    return t.finish(t.and_(*cmps))


def c2_workload(n_tapes: int = 10_000, n_models: int = 100_000, seed: int = 2,
                planted_frac: float = 0.1, n_vars: int = 8) -> Tuple[TapeBatch, ModelBatch, np.ndarray]:
    """Returns (tapes, models, expected_first_hit) — expected is exact for planted tapes and -1
    for the rest (holds w.p. 1 - O(M·2^-256)); tests confirm it with the oracle at small M."""
    rng = np.random.Generator(np.random.PCG64(seed))
    words = random_words(rng, 8 * n_vars, n_models)
    tapes: List[Tape] = []
    expected = np.full(n_tapes, -1, np.int32)
    planted = rng.random(n_tapes) < planted_frac
    for i in range(n_tapes):
        if planted[i]:
            p = int(rng.integers(n_models))
            vals = [_model_value(words, v, p) for v in range(n_vars)]
            tapes.append(c2_tape(rng, vals, n_vars))
            expected[i] = p
        else:
            tapes.append(c2_tape(rng, None, n_vars))
    models = ModelBatch([256] * n_vars, words)
    return TapeBatch(tapes), models, expected


# ---------------------------------------------------------------- fuzz (parity)
_BV_BIN = [Op.ADD, Op.SUB, Op.MUL, Op.UDIV, Op.UREM, Op.SDIV, Op.SREM, Op.SMOD,
           Op.BAND, Op.BOR, Op.BXOR, Op.SHL, Op.LSHR, Op.ASHR]
_PRED = [Op.EQ, Op.ULT, Op.ULE, Op.SLT, Op.SLE, Op.UMUL_NOOVFL, Op.SMUL_NOOVFL, Op.SMUL_NOUDFL]
# multiplication / division / the multiplication-overflow predicates stop at 512 bits (mq.h)
_MULDIV = frozenset({Op.MUL, Op.UDIV, Op.UREM, Op.SDIV, Op.SREM, Op.SMOD,
                     Op.UMUL_NOOVFL, Op.SMUL_NOOVFL, Op.SMUL_NOUDFL})
FUZZ_WIDTHS = (1, 8, 32, 64, 160, 256, 512, 544, 768, 1088, 2048)


def interesting_value(rng: np.random.Generator, w: int) -> int:
    m = (1 << w) - 1
    r = rng.random()
    if r < 0.15:
        return int(rng.choice([0, 1, 2, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, w, w - 1, w + 1])) & m if w > 1 else int(rng.integers(2))
    if r < 0.3:
        return int(rng.integers(0, 64)) & m
    nbytes = (w + 7) // 8
    return int.from_bytes(rng.bytes(nbytes), "little") & m


def fuzz_models(rng: np.random.Generator, var_widths: Sequence[int], n_models: int,
                funcs: Sequence[FuncSpec] = (), entries_per_model: int = 3,
                key_pool: Optional[dict] = None) -> ModelBatch:
    models = []
    for m in range(n_models):
        d = {"vars": {}, "funcs": {}}
        for v, w in enumerate(var_widths):
            if rng.random() < 0.9:
                d["vars"][v] = interesting_value(rng, w) if w else int(rng.integers(2))
        for f, spec in enumerate(funcs):
            if rng.random() < 0.1:
                continue  # function absent from this model -> completion default
            table = {}
            for _ in range(int(rng.integers(0, entries_per_model + 1))):
                pool = (key_pool or {}).get(f)
                if pool and rng.random() < 0.6:
                    args = pool[int(rng.integers(len(pool)))]
                else:
                    args = tuple(interesting_value(rng, aw) for aw in spec.arg_widths)
                table[args] = interesting_value(rng, spec.result_width) if spec.result_width else int(rng.integers(2))
            els = interesting_value(rng, spec.result_width) if spec.result_width else int(rng.integers(2))
            d["funcs"][f] = (table, els)
        models.append(d)
    return ModelBatch.from_python(var_widths, models, funcs)


class _Fuzz:
    def __init__(self, rng, tape: Tape, var_widths, funcs, max_width: int, ops=None, widths=None):
        self.rng, self.t, self.vw, self.funcs, self.maxw = rng, tape, var_widths, funcs, max_width
        self.ops = set(ops) if ops is not None else None
        self.widths = widths
        self.pool = {}  # width -> list of bv nodes

    def allowed(self, op):
        return self.ops is None or op in self.ops

    def bv_leaf(self, w: int) -> int:
        cands = [v for v, vw in enumerate(self.vw) if vw == w]
        if cands and self.rng.random() < 0.6:
            return self.t.var(int(self.rng.choice(cands)), w)
        return self.t.const(interesting_value(self.rng, w), w)

    def bv(self, w: int, depth: int) -> int:
        rng, t = self.rng, self.t
        if depth <= 0 or rng.random() < 0.2:
            return self.bv_leaf(w)
        r = rng.random()
        if r < 0.45:
            op = _BV_BIN[int(rng.integers(len(_BV_BIN)))]
            if not self.allowed(op):
                return self.bv_leaf(w)
            if w > 512 and op in _MULDIV:
                op = Op.BXOR
            a = self.bv(w, depth - 1)
            if op in (Op.SHL, Op.LSHR, Op.ASHR) and rng.random() < 0.6:
                b = t.const(int(rng.integers(0, w + 3)) & ((1 << w) - 1), w)
            else:
                b = self.bv(w, depth - 1)
            return t._bin(op, a, b)
        if r < 0.55 and self.allowed(Op.NEG):
            x = self.bv(w, depth - 1)
            return t.neg(x) if rng.random() < 0.5 else (t.bnot(x) if self.allowed(Op.BNOT) else x)
        if self.widths is not None and r >= 0.65:
            return self.bv_leaf(w)
        if r < 0.65 and self.allowed(Op.ITE):
            return t.ite(self.boolean(depth - 1), self.bv(w, depth - 1), self.bv(w, depth - 1))
        if r < 0.75 and self.allowed(Op.EXTRACT):
            src_w = min(self.maxw, w + int(rng.integers(0, 64)))
            lo = int(rng.integers(0, src_w - w + 1))
            return t.extract(lo + w - 1, lo, self.bv(src_w, depth - 1))
        if r < 0.83 and w >= 2 and self.allowed(Op.CONCAT):
            hw = int(rng.integers(1, w))
            return t.concat(self.bv(hw, depth - 1), self.bv(w - hw, depth - 1))
        if r < 0.90 and w >= 2 and self.allowed(Op.ZEXT):
            k = int(rng.integers(1, w))
            x = self.bv(w - k, depth - 1)
            return t.zext(k, x) if rng.random() < 0.5 else t.sext(k, x)
        if r < 0.96 and self.funcs and self.allowed(Op.UF):
            cands = [f for f, s in enumerate(self.funcs) if s.result_width == w]
            if cands:
                f = int(rng.choice(cands))
                spec = self.funcs[f]
                if spec.arity == 1 and rng.random() < 0.5 and self.allowed(Op.SELECT):
                    arr = t.array_var(f, w)
                    for _ in range(int(rng.integers(0, 3))):
                        arr = t.store(arr, self.bv(spec.arg_widths[0], depth - 2), self.bv(w, depth - 2))
                    return t.select(arr, self.bv(spec.arg_widths[0], depth - 1))
                args = [self.bv(aw, depth - 1) for aw in spec.arg_widths]
                return t.uf(f, w, *args)
        if self.allowed(Op.SELECT) and self.allowed(Op.CONST_ARRAY) and rng.random() < 0.5:
            kw = int(rng.choice([8, 32, 256])) if self.maxw >= 256 else 8
            arr = t.const_array(self.bv(w, depth - 2))
            for _ in range(int(rng.integers(1, 3))):
                arr = t.store(arr, self.bv(kw, depth - 2), self.bv(w, depth - 2))
            return t.select(arr, self.bv(kw, depth - 1))
        return self.bv_leaf(w)

    def boolean(self, depth: int) -> int:
        rng, t = self.rng, self.t
        if depth <= 0:
            return t.true() if rng.random() < 0.5 else t.false()
        r = rng.random()
        if r < 0.55:
            op = _PRED[int(rng.integers(len(_PRED)))]
            if not self.allowed(op):
                op = Op.EQ
            w = int(rng.choice(self.widths or [w for w in FUZZ_WIDTHS if w <= self.maxw]))
            if w > 512 and op in _MULDIV:
                op = Op.EQ
            a = self.bv(w, depth - 1)
            b = self.bv(w, depth - 1) if rng.random() < 0.7 else a
            if op == Op.EQ and rng.random() < 0.3:
                b = a  # force some true EQs
            return t._pred(op, a, b)
        if r < 0.75:
            return t.and_(self.boolean(depth - 1), self.boolean(depth - 1))
        if r < 0.85:
            return t.or_(self.boolean(depth - 1), self.boolean(depth - 1))
        if r < 0.90:
            return t.not_(self.boolean(depth - 1))
        if r < 0.93:
            return t.xor(self.boolean(depth - 1), self.boolean(depth - 1))
        if r < 0.95:
            return t.implies(self.boolean(depth - 1), self.boolean(depth - 1))
        if r < 0.97:
            return t.iff(self.boolean(depth - 1), self.boolean(depth - 1))
        bvars = [v for v, w in enumerate(self.vw) if w == BOOL]
        if bvars and rng.random() < 0.5:
            return t.var(int(rng.choice(bvars)), BOOL)
        return t.bite(self.boolean(depth - 1), self.boolean(depth - 1), self.boolean(depth - 1))


def fuzz_tape(rng: np.random.Generator, var_widths: Sequence[int], funcs: Sequence[FuncSpec] = (),
              depth: int = 4, max_width: int = 256, ops=None, widths=None) -> Tape:
    t = Tape()
    fz = _Fuzz(rng, t, var_widths, funcs, max_width, ops, widths)
    root = fz.boolean(depth)
    return t.finish(root)


# the op set of the gfx950 assembly interpreter (full-width 256-bit arithmetic, Bool logic)
ASM_OPS = frozenset({Op.ADD, Op.SUB, Op.MUL, Op.NEG, Op.BNOT, Op.BAND, Op.BOR, Op.BXOR, Op.ITE,
                     Op.EQ, Op.ULT, Op.ULE, Op.SLT, Op.SLE})


def fuzz_workload(seed: int, n_tapes: int, n_models: int, max_width: int = 256, depth: int = 4,
                  with_funcs: bool = True, ops=None, asm_only: bool = False):
    rng = np.random.Generator(np.random.PCG64(seed))
    if asm_only:
        var_widths = [256] * 8
        tapes = [fuzz_tape(rng, var_widths, (), depth, 256, ASM_OPS, widths=[256]) for _ in range(n_tapes)]
        return TapeBatch(tapes), fuzz_models(rng, var_widths, n_models)
    widths = [w for w in FUZZ_WIDTHS if w <= max_width]
    var_widths = [int(rng.choice(widths)) for _ in range(10)] + [256, 256, BOOL, 8]
    funcs: List[FuncSpec] = []
    if with_funcs:
        funcs = [FuncSpec(1, 256, (256,)), FuncSpec(1, 8, (256,)), FuncSpec(2, 256, (256, 256))]
        if max_width >= 512:
            funcs.append(FuncSpec(1, 256, (512,)))
        if max_width >= 1088:   # keccak256_1088 and its inverse (a 1088-bit result)
            funcs += [FuncSpec(1, 256, (1088,)), FuncSpec(1, 1088, (256,))]
    tapes = [fuzz_tape(rng, var_widths, funcs, depth, max_width, ops) for _ in range(n_tapes)]
    models = fuzz_models(rng, var_widths, n_models, funcs)
    return TapeBatch(tapes), models


# ---------------------------------------------------------------- constant-operand fuzz (asm parity)
CONST_OPS = (Op.UDIV, Op.UREM, Op.SDIV, Op.SREM, Op.SMOD, Op.SHL, Op.LSHR, Op.ASHR)


def _const_operand(rng: np.random.Generator, op: Op, w: int) -> int:
    m = (1 << w) - 1
    r = rng.random()
    if op in (Op.SHL, Op.LSHR, Op.ASHR):
        return int(rng.choice([0, 1, 7, 8, 31, 32, 33, 63, 64, 100, 128, 224, 255, w - 1, w, w + 5])) & m if r < 0.9 \
            else int(rng.integers(0, 1 << 16)) & m
    if r < 0.25:
        return (1 << int(rng.integers(0, w))) & m                          # powers of two
    if r < 0.6:
        v = int(rng.integers(1, 1 << min(w, 32)))                          # fits 32 bits
        return v if rng.random() < 0.5 or w < 2 else (-v) & m              # negative for the signed ops
    if r < 0.7:
        return int(rng.choice([1, 3, 10, 0xFFFFFFFF, (1 << 31) + 1, m]))  & m
    return interesting_value(rng, w)                                       # wide (C++ fallback)


def const_op_workload(seed: int, n_tapes: int, n_models: int):
    """Tapes dominated by shifts / divisions by constants, extract / concat / sign extension and
    array lookups at widths 8..256 over a mix of preloaded (var < 8) and other variables: the
    assembly interpreters' translated forms (gen_qsa.py), checked against the oracle."""
    rng = np.random.Generator(np.random.PCG64(seed))
    widths = (8, 32, 64, 160, 256)
    var_widths = [256, 256, 64, 8, 256, 160, 32, 256] + [int(rng.choice(widths)) for _ in range(8)] + [BOOL, 256]
    funcs = [FuncSpec(1, 256, (256,)), FuncSpec(1, 32, (160,)), FuncSpec(1, BOOL, (256,))]
    tapes = []
    for i in range(n_tapes):
        t = Tape()
        lo_vars = i % 3 == 0          # a third of the tapes read only variables 0..7
        nv = 8 if lo_vars else len(var_widths) - 1

        def var(w):
            c = [v for v in range(nv) if var_widths[v] == w]
            return t.var(int(rng.choice(c)), w) if c else t.const(interesting_value(rng, w), w)

        w = int(rng.choice(widths))
        x = var(w)
        k = int(rng.integers(1, 4))
        for _ in range(k):
            op = CONST_OPS[int(rng.integers(len(CONST_OPS)))]
            if w != 256 and op in (Op.SDIV, Op.SREM, Op.SMOD, Op.ASHR) and rng.random() < 0.7:
                op = Op.UREM
            c = t.const(_const_operand(rng, op, w), w)
            x = t._bin(op, x, c)
            if rng.random() < 0.3:
                x = t.add(x, var(w))
        r = rng.random()
        if r < 0.2 and w >= 16:
            hi = int(rng.integers(7, w))
            lo = int(rng.integers(0, hi - 6))
            x = t.extract(hi, lo, x)
            w = hi - lo + 1
        elif r < 0.35 and w <= 128:
            x = t.concat(var(8), x) if rng.random() < 0.5 else t.concat(x, t.const(int(rng.integers(0, 256)), 8))
            w = w + 8
        elif r < 0.5 and w <= 160:
            x = t.sext(256 - w, x)
            w = 256
        if not lo_vars and rng.random() < 0.3 and w == 256:
            f = int(rng.integers(0, 3))
            app = t.uf(f, funcs[f].result_width, x if f != 1 else t.extract(159, 0, x))
            root = app if funcs[f].result_width == BOOL else t.ult(app, t.uf(0, 256, var(256)) if f == 0 else var(32))
        else:
            y = var(w)
            cmp = [t.ult, t.ule, t.slt, t.eq][int(rng.integers(4))]
            root = t.or_(cmp(x, y), t.eq(x, t.const(interesting_value(rng, w), w)))
        tapes.append(t.finish(root))
    return TapeBatch(tapes), fuzz_models(rng, var_widths, n_models, funcs)


# ---------------------------------------------------------------- flat conjunctions (fc.hip parity)
FLAT_WIDTHS = (1, 8, 31, 32, 33, 64, 160, 255, 256)


def flat_workload(seed: int, n_tapes: int, n_models: int, n_bool: int = 6, planted_frac: float = 0.5,
                  max_items: int = 12, or_frac: float = 0.0):
    """Tapes that are ANDs of Bool variables (negated or not) and comparisons of one variable with
    a constant -- every predicate (EQ / distinct / unsigned and signed orders), the constant on
    either side, NOT over a compare, widths that end inside a limb -- the shape the flat-
    conjunction kernel (fc.hip) takes.  About ``planted_frac`` of the tapes are built to hold on a
    random model (items chosen true there, constants at or next to its values).  With
    ``or_frac``, that share of the tapes are instead an OR of the items, NOT of their AND, or an
    OR of a NOT(AND) with the rest (the kernel's negated conjunctions, by De Morgan).  Returns
    (tapes, models)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    bv_widths = [int(w) for w in rng.choice(FLAT_WIDTHS, 6)] + [256, 8]
    var_widths = [BOOL] * n_bool + bv_widths
    mb = fuzz_models(rng, var_widths, n_models)
    preds = ("eq", "distinct", "ult", "ule", "ugt", "uge", "slt", "sle", "sgt", "sge")

    def holds(p, x, c, w):
        sx = x - (1 << w) if x >> (w - 1) else x
        sc = c - (1 << w) if c >> (w - 1) else c
        return {"eq": x == c, "distinct": x != c, "ult": x < c, "ule": x <= c, "ugt": x > c, "uge": x >= c,
                "slt": sx < sc, "sle": sx <= sc, "sgt": sx > sc, "sge": sx >= sc}[p]

    tapes = []
    for _ in range(n_tapes):
        t = Tape()
        target = int(rng.integers(n_models)) if rng.random() < planted_frac else None
        items = []
        for _ in range(int(rng.integers(1, max_items + 1))):
            if rng.random() < 0.4:
                v = int(rng.integers(n_bool))
                b = t.var(v, BOOL)
                val = mb.var_value(v, target) if target is not None else int(rng.integers(2))
                items.append(b if val or target is None and rng.random() < 0.5 else t.not_(b))
                continue
            v = n_bool + int(rng.integers(len(bv_widths)))
            w = var_widths[v]
            m = (1 << w) - 1
            if target is not None:
                x = mb.var_value(v, target)
                c = (x + int(rng.integers(-1, 2))) & m if rng.random() < 0.7 else interesting_value(rng, w)
            else:
                c = interesting_value(rng, w)
            p = str(rng.choice(preds))
            left = rng.random() < 0.3           # the constant on the left: c OP x
            negate = rng.random() < 0.2
            if target is not None:
                xv = mb.var_value(v, target)
                ok = holds(p, c, xv, w) if left else holds(p, xv, c, w)
                if ok == negate:                 # make the item true on the target
                    negate = not negate
            a, b = (t.const(c, w), t.var(v, w)) if left else (t.var(v, w), t.const(c, w))
            node = getattr(t, p)(a, b)
            items.append(t.not_(node) if negate else node)
        if rng.random() < 0.1:
            items.append(t.true())
        if len(items) >= 2 and rng.random() < or_frac:
            k, half = int(rng.integers(3)), len(items) // 2
            if k == 0:
                root = t.or_(*items)
            elif k == 1:
                root = t.not_(t.and_(*items))
            else:
                root = t.or_(t.not_(t.and_(*items[:half])), *items[half:])
            tapes.append(t.finish(root))
            continue
        tapes.append(t.finish(t.and_(*items)))
    return TapeBatch(tapes), mb
