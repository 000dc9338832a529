"""ORACLE (test infrastructure only — never imported by the product path).

Executable specification, in Python big ints, of the reference's quick-sat hot path:

* ``first_hit``  restates ``ModelCache.check_quick_sat``
  (``mythril/support/support_utils.py:60-67``): walk the candidates in order
  (index 0 = MRU = ``reversed(self.model_cache.lru_cache.keys())``, line 62) and return
  the first whose evaluation is literally ``true`` (``is_true``, line 64).
* ``eval_tape``  restates z3 ``model.eval(expr, model_completion=True)``
  (called at support_utils.py:64 via ``mythril/laser/smt/model.py:45-58``) on the tape
  lowering of ``simplify(And(*constraints)).raw`` (``mythril/support/model.py:101``):
  SMT-LIB 2.6 FixedSizeBitVectors + z3 model completion, SURVEY.md Appendix A.
  z3 (``z3-solver >=4.8.8.0,<=4.12.5.0``, requirements.txt:36) is not installed, so
  this is a restatement of its published semantics; parity of the restatement is pinned
  by the reference's own vectors in tests/golden (EIP-145 shift vectors, VMTests
  arithmetic/bitwise/sha3 KATs) and is otherwise spec-derived ("parity unpinned" for
  model-completion and UF/array behaviour, which no reference test covers).
"""
from __future__ import annotations

import os
import sys
from typing import List, Sequence

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from keccak_ref import keccak256  # noqa: E402
from mythril_amd.tape import NONE, Op, TapeBatch, from_words, limbs  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402


def _mask(w: int) -> int:
    return (1 << w) - 1


def _signed(x: int, w: int) -> int:
    return x - (1 << w) if x >> (w - 1) & 1 else x


def bv_udiv(a: int, b: int, w: int) -> int:
    return _mask(w) if b == 0 else a // b


def bv_urem(a: int, b: int, w: int) -> int:
    return a if b == 0 else a % b


def bv_sdiv(a: int, b: int, w: int) -> int:
    m = _mask(w)
    sa, sb = a >> (w - 1) & 1, b >> (w - 1) & 1
    na = (-a) & m if sa else a
    nb = (-b) & m if sb else b
    q = bv_udiv(na, nb, w)
    return (-q) & m if sa ^ sb else q


def bv_srem(a: int, b: int, w: int) -> int:
    m = _mask(w)
    sa, sb = a >> (w - 1) & 1, b >> (w - 1) & 1
    na = (-a) & m if sa else a
    nb = (-b) & m if sb else b
    r = bv_urem(na, nb, w)
    return (-r) & m if sa else r


def bv_smod(a: int, b: int, w: int) -> int:
    m = _mask(w)
    sa, sb = a >> (w - 1) & 1, b >> (w - 1) & 1
    na = (-a) & m if sa else a
    nb = (-b) & m if sb else b
    u = bv_urem(na, nb, w)
    if u == 0:
        return u
    if not sa and not sb:
        return u
    if sa and not sb:
        return ((-u) + b) & m
    if not sa and sb:
        return (u + b) & m
    return (-u) & m


def bv_shl(a: int, b: int, w: int) -> int:
    return 0 if b >= w else (a << b) & _mask(w)


def bv_lshr(a: int, b: int, w: int) -> int:
    return 0 if b >= w else a >> b


def bv_ashr(a: int, b: int, w: int) -> int:
    s = _signed(a, w)
    if b >= w:
        return _mask(w) if s < 0 else 0
    return (s >> b) & _mask(w)


class _Arr:
    """Array value: ("K", v) | ("F", func) | ("S", base, key, val)."""
    __slots__ = ("kind", "a", "b", "c")

    def __init__(self, kind, a=None, b=None, c=None):
        self.kind, self.a, self.b, self.c = kind, a, b, c


def _func_lookup(models: ModelBatch, f: int, m: int, args) -> int:
    table, els = models.func_table(f, m)
    return table.get(tuple(args), els)


def _entries(models: ModelBatch, f: int, m: int):
    """The model's table of arity-1 function f in entry order: [(key, value)] (duplicates kept)."""
    spec = models.funcs[f]
    lo, hi = int(models.entry_ptr[f, m]), int(models.entry_ptr[f, m + 1])
    base, nk, nv = int(models.entry_base[f]), limbs(spec.arg_widths[0]), limbs(spec.result_width)
    out = []
    for e in range(lo, hi):
        w0 = base + e * spec.stride
        out.append((from_words(models.entry_words[w0:w0 + nk]), from_words(models.entry_words[w0 + nk:w0 + nk + nv])))
    return out


def _select(models: ModelBatch, m: int, arr: _Arr, idx: int) -> int:
    # select(store(A,k,v), i) = i==k ? v : select(A, i); select(K(d), i) = d;
    # select(as-array f, i) = f's FuncInterp entry or else (SURVEY Appendix A "Arrays").
    while arr.kind == "S":
        if arr.b == idx:
            return arr.c
        arr = arr.a
    if arr.kind == "K":
        return arr.a
    return _func_lookup(models, arr.a, m, (idx,))


def eval_nodes(nodes, consts, models: ModelBatch, m: int) -> list:
    """Evaluate every node of one tape under model m; returns the per-node values."""
    vals: List[object] = []
    for nd in nodes:
        op = Op(int(nd["op"]))
        w = int(nd["width"])
        a, b, c = int(nd["a"]), int(nd["b"]), int(nd["c"])
        V = vals
        if op == Op.CONST:
            r = from_words(consts[a:a + limbs(w)]) & _mask(w)
        elif op == Op.VAR:
            r = models.var_value(a, m) if a < models.n_vars else 0
            r &= _mask(max(w, 1))
        elif op == Op.TRUE:
            r = 1
        elif op == Op.FALSE:
            r = 0
        elif op == Op.NOT:
            r = 1 - V[a]
        elif op == Op.AND:
            r = V[a] & V[b]
        elif op == Op.OR:
            r = V[a] | V[b]
        elif op == Op.XOR:
            r = V[a] ^ V[b]
        elif op == Op.IMPLIES:
            r = (1 - V[a]) | V[b]
        elif op == Op.IFF:
            r = int(V[a] == V[b])
        elif op == Op.BITE:
            r = V[b] if V[a] else V[c]
        elif op in (Op.EQ, Op.ULT, Op.ULE, Op.SLT, Op.SLE, Op.UMUL_NOOVFL, Op.SMUL_NOOVFL, Op.SMUL_NOUDFL):
            x, y = V[a], V[b]
            aw = int(nodes[a]["width"])
            if op == Op.EQ:
                r = int(x == y)
            elif op == Op.ULT:
                r = int(x < y)
            elif op == Op.ULE:
                r = int(x <= y)
            elif op == Op.SLT:
                r = int(_signed(x, aw) < _signed(y, aw))
            elif op == Op.SLE:
                r = int(_signed(x, aw) <= _signed(y, aw))
            elif op == Op.UMUL_NOOVFL:
                r = int(x * y < (1 << aw))
            elif op == Op.SMUL_NOOVFL:
                r = int(_signed(x, aw) * _signed(y, aw) <= (1 << (aw - 1)) - 1)
            else:
                r = int(_signed(x, aw) * _signed(y, aw) >= -(1 << (aw - 1)))
        elif op == Op.ADD:
            r = (V[a] + V[b]) & _mask(w)
        elif op == Op.SUB:
            r = (V[a] - V[b]) & _mask(w)
        elif op == Op.MUL:
            r = (V[a] * V[b]) & _mask(w)
        elif op == Op.NEG:
            r = (-V[a]) & _mask(w)
        elif op == Op.UDIV:
            r = bv_udiv(V[a], V[b], w)
        elif op == Op.UREM:
            r = bv_urem(V[a], V[b], w)
        elif op == Op.SDIV:
            r = bv_sdiv(V[a], V[b], w)
        elif op == Op.SREM:
            r = bv_srem(V[a], V[b], w)
        elif op == Op.SMOD:
            r = bv_smod(V[a], V[b], w)
        elif op == Op.BAND:
            r = V[a] & V[b]
        elif op == Op.BOR:
            r = V[a] | V[b]
        elif op == Op.BXOR:
            r = V[a] ^ V[b]
        elif op == Op.BNOT:
            r = (~V[a]) & _mask(w)
        elif op == Op.SHL:
            r = bv_shl(V[a], V[b], w)
        elif op == Op.LSHR:
            r = bv_lshr(V[a], V[b], w)
        elif op == Op.ASHR:
            r = bv_ashr(V[a], V[b], w)
        elif op == Op.EXTRACT:
            r = (V[a] >> c) & _mask(b - c + 1)
        elif op == Op.CONCAT:
            r = (V[a] << int(nodes[b]["width"])) | V[b]
        elif op == Op.ZEXT:
            r = V[a]
        elif op == Op.SEXT:
            r = _signed(V[a], w - b) & _mask(w)
        elif op == Op.ITE:
            r = V[b] if V[a] else V[c]
        elif op == Op.ARRAY_VAR:
            r = _Arr("F", a)
        elif op == Op.CONST_ARRAY:
            r = _Arr("K", V[a])
        elif op == Op.STORE:
            r = _Arr("S", V[a], V[b], V[c])
        elif op == Op.SELECT:
            r = _select(models, m, V[a], V[b])
        elif op == Op.UF:
            args = [V[b]] if c == NONE else [V[b], V[c]]
            r = _func_lookup(models, a, m, args)
        elif op == Op.UF_CHUNK:
            # wide-key lookup, key chunk k (mq.h): the ordered entries of the model's table whose
            # key bits [256k, 256k + 256) equal the chunk, within the previous chunk's set
            k, q = 0, c
            while q != NONE:
                k, q = k + 1, int(nodes[q]["c"])
            ents = _entries(models, a, m)
            if len(ents) > 64:
                raise ValueError("unsupported: more than 64 entries under a wide-key lookup")
            prev = set(range(len(ents))) if c == NONE else V[c]
            r = {e for e in prev if (ents[e][0] >> (256 * k)) & _mask(256) == V[b]}
        elif op == Op.UF_WIDE:
            ents = _entries(models, a, m)
            r = ents[min(V[b])][1] if V[b] else models.func_table(a, m)[1]
        elif op == Op.KECCAK:
            aw = int(nodes[a]["width"])
            r = int.from_bytes(keccak256(V[a].to_bytes(aw // 8, "big")), "big")
        else:  # pragma: no cover
            raise ValueError(f"unknown op {op}")
        vals.append(r)
    return vals


def eval_tape(batch: TapeBatch, t: int, models: ModelBatch, m: int) -> bool:
    """is_true(model_m.eval(tape_t, model_completion=True))  (support_utils.py:64)."""
    nodes = batch.tape_nodes(t)
    return eval_nodes(nodes, batch.consts, models, m)[-1] == 1


def first_hit(batch: TapeBatch, models: ModelBatch) -> List[int]:
    """check_quick_sat for every tape: first satisfying GLOBAL candidate index or -1."""
    out = []
    for t in range(batch.n_tapes):
        hit = -1
        for m in range(models.n_models):
            if eval_tape(batch, t, models, m):
                hit = models.index_base + m
                break
        out.append(hit)
    return out


def verdicts(batch: TapeBatch, models: ModelBatch) -> List[List[bool]]:
    return [[eval_tape(batch, t, models, m) for m in range(models.n_models)] for t in range(batch.n_tapes)]
