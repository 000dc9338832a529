"""Candidate-model generator: candidates BEYOND the 100-entry LRU.

The reference tries only the models z3 returned earlier (``ModelCache``, support_utils.py:56-67,
filled at model.py:125), at most 100 of them, so every path the cached models miss costs a z3
``Optimize.check`` (model.py:104-130).  A fork (svm.py:351-358) usually differs from a path the
cache already satisfies in one or a few branch conditions — a selector, ``require(x == c)``,
``x < c`` — so mutating a cached model's inputs towards the constants those conditions compare
against often yields a satisfying assignment without a solver call.  That is what this module
generates, for the GPU to evaluate in bulk (M up to 10^5 per launch):

* **directed** candidates: for a conjunction, each cached model with ALL the conjunct's
  invertible branch conditions patched to a satisfying value (polarity from ``Not``);
* **single mutations**: one condition patched to ``c``, ``c - 1`` or ``c + 1``;
* **boundary** values of single variables (0, 1, 2^w - 1, 2^(w-1), 2^(w-1) - 1) and
  **random fills**.

A branch condition is *invertible* when it compares a constant with an expression that maps
bits of model inputs one to one: variables, calldata bytes at constant offsets (derived
variables), ``Extract``, ``Concat``, ``ZeroExt`` and the calldata-byte shape ``If(i < size,
byte, 0)`` (calldata.py:234-246).  Patching a derived variable (the interpretation of
``<tx>_calldata`` at a constant index) also adds that entry to the candidate's table, so every
candidate is a consistent model: evaluating it is exactly ``model.eval(expr, model_completion=
True)`` of the model :meth:`CandidateSet.materialize` returns.

Generated candidates sit strictly AFTER the LRU models in global candidate order (index >= the
LRU size), so an LRU hit is never pre-empted and the reference's first-hit / bump semantics are
untouched.  They are only used behind ``Args.quick_sat_candidates`` and only for verdict
callers (``Constraints.is_possible``), never for callers that read model contents
(arbitrary_jump.py:29-32, instructions.py:1742-1746).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .models import ModelBatch
from .smt_model import Model, as_record
from .tape import limbs, to_words

_EQ, _ULT, _ULE, _SLT, _SLE = 20, 21, 22, 23, 24
_PREDS = (_EQ, _ULT, _ULE, _SLT, _SLE)

# a bit map: tuple of segments from the low bit up: (var, var_lo_bit, n_bits) or (-1, const, n_bits);
# a floor (var, minimum) says a mapped calldata byte is only read when that size variable exceeds
# its offset (If(i < size, byte, 0), calldata.py:234-246).  A patch is a tuple of assignments
# (var, lo, n_bits, bits), floors written as (var, -1, 0, minimum).
Segment = Tuple[int, int, int]


class _BitMaps:
    """Which DAG nodes are one-to-one maps of model-input bits (memoised per node)."""

    def __init__(self, nodes: np.ndarray, consts: np.ndarray, opaque=frozenset()):
        self.opaque = opaque   # variables that are not free model inputs (never patched)
        self.op = nodes["op"].astype(np.int64)
        self.w = nodes["width"].astype(np.int64)
        self.a = nodes["a"].astype(np.int64)
        self.b = nodes["b"].astype(np.int64)
        self.c = nodes["c"].astype(np.int64)
        self.consts = consts
        self.memo: Dict[int, Optional[Tuple[Segment, ...]]] = {}
        self.cvals: Dict[int, int] = {}
        self.floors: Dict[int, Tuple[Tuple[int, int], ...]] = {}

    def const_value(self, n: int) -> Optional[int]:
        if self.op[n] != 1:
            return None
        v = self.cvals.get(n)
        if v is not None:
            return v
        nl = limbs(int(self.w[n]))
        off = int(self.a[n])
        v = 0
        for i in range(nl):
            v |= int(self.consts[off + i]) << (32 * i)
        v &= (1 << int(self.w[n])) - 1
        self.cvals[n] = v
        return v

    def map(self, n: int) -> Optional[Tuple[Segment, ...]]:
        if n in self.memo:
            return self.memo[n]
        op, w = int(self.op[n]), int(self.w[n])
        r: Optional[Tuple[Segment, ...]] = None
        fl: Tuple[Tuple[int, int], ...] = ()
        if op == 2 and w > 0 and int(self.a[n]) not in self.opaque:   # VAR
            r = ((int(self.a[n]), 0, w),)
        elif op == 1:                                          # CONST
            r = ((-1, self.const_value(n), w),)
        elif op == 50:                                         # EXTRACT(x, hi, lo)
            x = self.map(int(self.a[n]))
            if x is not None:
                r, fl = _slice(x, int(self.c[n]), w), self.floors[int(self.a[n])]
        elif op == 51:                                         # CONCAT(hi, lo)
            hi, lo = self.map(int(self.a[n])), self.map(int(self.b[n]))
            if hi is not None and lo is not None:
                r = lo + hi
                fl = self.floors[int(self.a[n])] + self.floors[int(self.b[n])]
        elif op == 52:                                         # ZEXT(x, k)
            x = self.map(int(self.a[n]))
            if x is not None:
                r, fl = x + ((-1, 0, w - int(self.w[int(self.a[n])])),), self.floors[int(self.a[n])]
        elif op == 54:                                         # ITE(c, x, 0): calldata byte shape
            x = self.map(int(self.b[n]))
            e = self.const_value(int(self.c[n]))
            if x is not None and e == 0:
                r = x
                fl = self.floors[int(self.b[n])]
                c = int(self.a[n])                              # i < size (signed, calldata.py:243)
                if int(self.op[c]) in (_SLT, _ULT) and int(self.op[int(self.b[c])]) == 2:
                    i = self.const_value(int(self.a[c]))
                    if i is not None and i < (1 << 31):
                        fl = fl + ((int(self.a[int(self.b[c])]), i + 1),)
        self.memo[n] = r
        self.floors[n] = tuple(sorted(set(fl)))
        return r


def _slice(segs: Tuple[Segment, ...], lo: int, n: int) -> Tuple[Segment, ...]:
    out, pos = [], 0
    for v, s, k in segs:
        a, b = max(lo, pos), min(lo + n, pos + k)
        if a < b:
            if v < 0:
                out.append((-1, (s >> (a - pos)) & ((1 << (b - a)) - 1), b - a))
            else:
                out.append((v, s + a - pos, b - a))
        pos += k
    return tuple(out)


def _patch_for(segs: Tuple[Segment, ...], value: int) -> Optional[Tuple[Tuple[int, int, int, int], ...]]:
    """Variable bit assignments (var, lo, n_bits, bits) that make the mapped expression equal
    ``value``; None if a constant segment disagrees."""
    out, pos = [], 0
    for v, s, k in segs:
        bits = (value >> pos) & ((1 << k) - 1)
        if v < 0:
            if bits != s:
                return None
        else:
            out.append((v, s, k, bits))
        pos += k
    return tuple(out)


def _wanted(op: int, const_left: bool, c: int, w: int, positive: Optional[bool]) -> List[int]:
    """Values of the mapped side that satisfy (positive) / falsify (negative) the predicate."""
    m = (1 << w) - 1
    if positive is None:
        return sorted({c, (c - 1) & m, (c + 1) & m})
    if op == _EQ:
        return [c] if positive else [(c + 1) & m, (c - 1) & m]
    strict = op in (_ULT, _SLT)
    # X < c / X <= c  (const on the right) or c < X / c <= X (const on the left)
    if not const_left:
        lo_side = (c - 1) & m if strict else c
        return [lo_side, 0] if positive else [c if strict else (c + 1) & m]
    hi_side = (c + 1) & m if strict else c
    return [hi_side, m >> (1 if op in (_SLT, _SLE) else 0)] if positive else [c if strict else (c - 1) & m]


def _candidate_rows(lru: ModelBatch, src: np.ndarray, starts: np.ndarray, sizes: np.ndarray,
                    blocks: List[Tuple[Tuple, np.ndarray]], syms, off: np.ndarray, K: int) -> np.ndarray:
    """The whole batch's variable rows [rows, n_lru + K]: the LRU's, then each generated
    candidate's base LRU row with its block's patch applied — value assignments in patch order
    (the last assignment of a bit wins), then the size floors.  The host extension's loop
    (csrc/lowerwalk.cpp candidate_rows, writing the candidates' columns in place); the numpy form
    below where it is not built (the tests compare the two)."""
    from .lower import _walker
    n_lru = lru.n_models
    walker = _walker()
    if walker is not None and n_lru and K and os.environ.get("MQ_PY_CANDIDATES") != "1":
        words = np.empty((int(off[-1]), n_lru + K), np.uint32)
        words[:, :n_lru] = lru.var_words
        gen = words[:, n_lru:]
        widths = syms.var_widths
        walker.candidate_rows(gen, np.ascontiguousarray(lru.var_words, np.uint32), np.ascontiguousarray(src, np.int64),
                              np.ascontiguousarray(starts, np.int64), [p for p, _ in blocks],
                              np.ascontiguousarray(off[:-1], np.int64),
                              np.asarray([limbs(w) for w in widths], np.int64))
        return words
    gen = lru.var_words[:, src].copy() if n_lru else np.zeros((int(off[-1]), K), np.uint32)
    # each block's patch over its candidate range.  Per (limb row, block) the composed update
    # (mask, bits) of the block's value assignments, in patch order (the last assignment of a
    # bit wins); the limb updates of a patch element are computed once (elements recur in many
    # blocks: the random mixes reuse the directed singles).  Then ONE vectorised update per
    # row over every block that patches it, and the size floors (applied after the values of
    # their block) per variable
    widths = syms.var_widths
    cache: Dict[Tuple, List[Tuple[int, int, int]]] = {}
    row_ops: Dict[int, Dict[int, List[int]]] = {}
    floor_ops: Dict[int, Dict[int, int]] = {}
    for j, (patch, _) in enumerate(blocks):
        for el in patch:
            v, lo, n, bits = el
            if lo < 0:   # size >= minimum (values < 2^32 in their low limb)
                fj = floor_ops.setdefault(v, {})
                fj[j] = max(fj.get(j, 0), bits)
                continue
            ups = cache.get(el)
            if ups is None:
                ups = []
                o = int(off[v])
                for i in range(lo // 32, (lo + n - 1) // 32 + 1):
                    blo = 32 * i
                    a, b2 = max(lo, blo), min(lo + n, blo + 32)
                    mask = ((1 << (b2 - a)) - 1) << (a - blo)
                    ups.append((o + i, mask, ((bits >> (a - lo)) << (a - blo)) & mask))
                cache[el] = ups
            for row, mask, val in ups:
                d = row_ops.get(row)
                if d is None:
                    d = row_ops[row] = {}
                c = d.get(j)
                if c is None:
                    d[j] = [mask, val]
                else:
                    c[1] = (c[1] & ~mask) | val
                    c[0] |= mask
    nb = int(sizes.max()) if len(sizes) else 0
    ar = np.arange(nb, dtype=np.int64)

    def cols_of(js: np.ndarray):
        """(block columns [k, nb] of the full-size blocks among js, their positions in js, the others)."""
        full = sizes[js] == nb
        return starts[js[full]][:, None] + ar[None, :], np.flatnonzero(full), np.flatnonzero(~full)

    for row, d in row_ops.items():
        js = np.fromiter(d.keys(), np.int64, len(d))
        mv = np.asarray(list(d.values()), np.uint64).astype(np.uint32).reshape(-1, 2)
        keep, val = ~mv[:, 0], mv[:, 1]
        cols, fi, pi = cols_of(js)
        if len(fi):
            gen[row, cols] = (gen[row, cols] & keep[fi][:, None]) | val[fi][:, None]
        for k in pi:   # (a partial block: the budget's last random block)
            sl = slice(int(starts[js[k]]), int(starts[js[k] + 1]))
            gen[row, sl] = (gen[row, sl] & keep[k]) | val[k]
    for v, fj in floor_ops.items():
        r0, nl = int(off[v]), limbs(widths[v])
        js = np.fromiter(fj.keys(), np.int64, len(fj))
        mins = np.fromiter(fj.values(), np.int64, len(fj)).astype(np.uint32)
        cols, fi, pi = cols_of(js)
        groups = [(cols, mins[fi][:, None])] + [(np.arange(int(starts[js[k]]), int(starts[js[k] + 1]))[None, :],
                                                 mins[k:k + 1][:, None]) for k in pi]
        for cc, mn in groups:
            if not cc.size:
                continue
            x = gen[r0, cc]
            small = ~gen[r0 + 1:r0 + nl][:, cc].any(axis=0) if nl > 1 else np.ones(x.shape, bool)
            gen[r0, cc] = np.where(small & (x < mn), mn, x)
    return np.concatenate([lru.var_words, gen], axis=1)


class CandidateSet:
    """The LRU models followed by the generated candidates, serialized (``batch``), plus what is
    needed to turn a generated candidate back into a model (:meth:`materialize`).  Candidates
    come in blocks: one patch applied to a range of base models."""

    def __init__(self, batch: ModelBatch, n_lru: int, base: np.ndarray, block_of: np.ndarray,
                 block_patches: List[Tuple], syms, lru_models):
        self.batch = batch
        self.n_lru = n_lru
        self.base = base                  # [K] LRU index each candidate derives from (-1: none)
        self.block_of = block_of          # [K] its block
        self.block_patches = block_patches   # per block: tuple of (var, lo, n_bits, bits)
        self.syms = syms
        self.lru_models = list(lru_models)

    @property
    def n_generated(self) -> int:
        return self.batch.n_models - self.n_lru

    def patch(self, k: int) -> Tuple:
        return self.block_patches[int(self.block_of[k])]

    def materialize(self, index: int) -> Model:
        """Global candidate ``index`` (>= n_lru) as a model: the base model with the patched
        variables assigned and the patched derived variables entered in their tables."""
        k = index - self.n_lru
        b = int(self.base[k])
        rec = as_record(self.lru_models[b]) if b >= 0 else Model()
        asg = dict(rec.assignment)
        funcs = {name: (dict(e), els) for name, (e, els) in rec.functions.items()}
        names = {i: key for key, i in self.syms.vars.items()}
        vals: Dict[int, int] = {}
        for v, lo, n, bits in sorted(self.patch(k), key=lambda p: p[1] < 0):   # floors last
            if v not in vals:
                name, w = names[v]
                if v in self.syms.derived:
                    fname, fargs = self.syms.derived[v]
                    interp = funcs.get(fname)
                    vals[v] = 0 if interp is None else int(interp[0].get(fargs, interp[1]))
                else:
                    vals[v] = int(asg.get(name, 0) or 0)
            if lo < 0:
                if vals[v] < (1 << 32) and vals[v] < bits:
                    vals[v] = bits
                continue
            vals[v] = (vals[v] & ~(((1 << n) - 1) << lo)) | (bits << lo)
        for v, val in vals.items():
            name, w = names[v]
            if v in self.syms.derived:
                fname, fargs = self.syms.derived[v]
                e, els = funcs.get(fname, ({}, 0))
                e = dict(e)
                e[tuple(fargs)] = val
                funcs[fname] = (e, els)
            else:
                asg[name] = val
        return Model(asg, funcs)


class CandidateGenerator:
    """Generates up to ``max_candidates`` candidates for a batch of conjunctions (seeded)."""

    def __init__(self, max_candidates: int = 100_000, seed: int = 0, random_frac: float = 0.05, per_query: int = 16,
                 fill: bool = False):
        self.max_candidates = int(max_candidates)
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.random_frac = random_frac
        self.per_query = int(per_query)   # patches per query (each over every base model)
        self.fill = fill                  # fill max_candidates with random mixes (throughput runs)

    # ------------------------------------------------------------ targets
    def _targets(self, db, syms):
        """Per query: list of (patch-option lists) of its invertible branch conditions."""
        # a derived variable of a value slice (lower.py _wide_eq) shares its bits with the other
        # slices of the same function value: patching one alone would split them
        from .lower import SLICE
        opaque = frozenset(v for v, (f, _) in syms.derived.items() if SLICE in f)
        bm = _BitMaps(db.nodes, db.consts, opaque)
        op, a, b = bm.op, bm.a, bm.b
        per_query = []
        for q in range(db.n_tapes):
            roots = db.roots[db.root_offsets[q]:db.root_offsets[q + 1]]
            opts = []
            for r in roots:
                r = int(r)
                positive: Optional[bool] = True
                if op[r] == 10:                        # NOT(pred): the branch not taken
                    r, positive = int(a[r]), False
                # a conjunct that is itself an OR / deeper: look one level for a predicate
                if op[r] not in _PREDS:
                    continue
                x, y = int(a[r]), int(b[r])
                cx, cy = bm.const_value(x), bm.const_value(y)
                if cx is not None and cy is None:
                    segs, c, const_left, fl = bm.map(y), cx, True, None
                elif cy is not None and cx is None:
                    segs, c, const_left, fl = bm.map(x), cy, False, None
                else:
                    continue
                if segs is None or all(v < 0 for v, _, _ in segs):
                    continue
                floors = bm.floors[y if const_left else x]
                w = int(bm.w[x])
                o = []
                for val in _wanted(int(op[r]), const_left, c, w, positive):
                    p = _patch_for(segs, val)
                    if p is not None:
                        o.append(p + tuple((v, -1, 0, mn) for v, mn in floors))
                if o:
                    opts.append(o)
            per_query.append(opts)
        return per_query

    # ------------------------------------------------------------ generation
    def generate(self, db, syms, lru_batch: ModelBatch, lru_models: Sequence) -> CandidateSet:
        """``lru_batch`` (the serialized LRU, MRU first, index_base 0) followed by generated
        candidates; their model rows are patched copies of LRU rows (random fills: fresh).

        Blocks of one patch over every base model, in order: per query all its invertible
        conditions patched at once (two rounds of options), then single conditions newest first,
        at most ``per_query`` patches per query; random multi-condition mixes and boundary /
        random values of plain variables add ``random_frac`` of that.  The budget adapts to the
        batch: ``per_query`` x bases per query, capped by ``max_candidates``."""
        rng = self.rng
        n_lru = lru_batch.n_models
        per_query = self._targets(db, syms)
        base_ids = np.arange(n_lru, dtype=np.int64) if n_lru else np.full(1, -1, np.int64)
        nb = len(base_ids)
        n_q = sum(1 for o in per_query if o)
        budget = max(0, self.max_candidates - n_lru)
        if not self.fill:
            budget = min(budget, self.per_query * nb * max(n_q, 1))
        blocks: List[Tuple[Tuple, np.ndarray]] = []
        total = [0]
        seen = set()

        def add(patch: Tuple, bases: np.ndarray = base_ids, dedupe: bool = True) -> bool:
            if total[0] + len(bases) > budget:
                return False
            if dedupe:
                if patch in seen:
                    return True
                seen.add(patch)
            blocks.append((patch, bases))
            total[0] += len(bases)
            return True

        used = [0] * len(per_query)
        for rnd in range(2):
            for q, opts in enumerate(per_query):
                if not opts:
                    continue
                patch = tuple(p for o in opts for p in (o[0] if rnd == 0 else o[int(rng.integers(len(o)))]))
                if add(patch):
                    used[q] += 1
        depth = max((len(o) for o in per_query), default=0)
        for back in range(1, depth + 1):
            for q, opts in enumerate(per_query):
                if back > len(opts):
                    continue
                for p in opts[-back]:
                    if used[q] >= self.per_query:
                        break
                    if add(p):
                        used[q] += 1
        singles = [p for opts in per_query for o in opts for p in o]
        plain = [v for v, w in enumerate(syms.var_widths) if w > 0 and v not in syms.derived
                 and v not in syms.hoisted_vars]
        # (each random patch over every base model, like the directed ones)
        n_rand = budget - total[0] if self.fill else int(total[0] * self.random_frac)
        for _ in range(-(-n_rand // nb)):
            bases = base_ids if total[0] + nb <= budget else base_ids[:budget - total[0]]
            if not len(bases):
                break
            if singles and rng.random() < 0.7:
                k = int(rng.integers(1, 4))
                patch = tuple(q for i in rng.integers(0, len(singles), k) for q in singles[int(i)])
            elif plain:
                v = plain[int(rng.integers(len(plain)))]
                w = syms.var_widths[v]
                val = int(rng.choice([0, 1, (1 << w) - 1, 1 << (w - 1), (1 << (w - 1)) - 1,
                                      int.from_bytes(rng.bytes((w + 7) // 8), "little")])) & ((1 << w) - 1)
                patch = ((v, 0, w, val),)
            else:
                break
            if not add(patch, bases, dedupe=False):
                break
        return self._serialize(lru_batch, blocks, syms, lru_models)

    # ------------------------------------------------------------ serialization
    def _serialize(self, lru: ModelBatch, blocks: List[Tuple[Tuple, np.ndarray]], syms, lru_models) -> CandidateSet:
        n_lru = lru.n_models
        sizes = np.asarray([len(b) for _, b in blocks], np.int64)
        K = int(sizes.sum())
        base = np.concatenate([b for _, b in blocks]) if blocks else np.zeros(0, np.int64)
        block_of = np.repeat(np.arange(len(blocks), dtype=np.int64), sizes)
        starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        off = lru.var_word_offsets()
        src = np.where(base >= 0, base, 0)
        words = _candidate_rows(lru, src, starts, sizes, blocks, syms, off, K)
        M = n_lru + K
        if not lru.funcs:
            return CandidateSet(ModelBatch(lru.var_widths, words), n_lru, base, block_of,
                                [p for p, _ in blocks], syms, lru_models)
        # function tables: the base model's entries, preceded by an entry for every derived variable
        # of that function the candidate's patch changed (so table and derived column agree; first
        # match wins)
        F = len(lru.funcs)
        func_index = {name: f for f, name in enumerate(syms.func_names)}
        dfunc = {v: func_index[fn] for v, (fn, _) in syms.derived.items() if fn in func_index}
        # per function: (block, position among the block's changed derived vars of it, var) triples
        per_f: Dict[int, Tuple[List[int], List[int], List[int]]] = {}
        for j, (patch, _) in enumerate(blocks):
            vs = {el[0] for el in patch if el[0] in dfunc and el[1] >= 0}
            if not vs:
                continue
            pos: Dict[int, int] = {}
            for v in sorted(vs):
                f = dfunc[v]
                t = per_f.setdefault(f, ([], [], []))
                t[0].append(j)
                t[1].append(pos.get(f, 0))
                t[2].append(v)
                pos[f] = pos.get(f, 0) + 1
        eptr = np.zeros((F, M + 1), np.int64)
        ew_chunks, el_chunks = [], []
        ebase = np.zeros(F, np.int64)
        elb = np.zeros(F, np.int64)
        wpos = epos = 0
        for f, spec in enumerate(lru.funcs):
            s = spec.stride
            base_ptr = lru.entry_ptr[f]
            base_cnt = np.diff(base_ptr)                                   # [n_lru]
            cnt_gen = base_cnt[src] if n_lru else np.zeros(K, np.int64)
            trip = per_f.get(f)
            if trip is not None:
                tj, ti, tv = (np.asarray(x, np.int64) for x in trip)
                add_cnt = np.repeat(np.bincount(tj, minlength=len(blocks)), sizes)
            else:
                add_cnt = np.zeros(K, np.int64)
            counts = np.concatenate([base_cnt, cnt_gen + add_cnt])
            eptr[f, 1:] = np.cumsum(counts)
            ent = lru.entry_words[int(lru.entry_base[f]):int(lru.entry_base[f]) + int(base_ptr[-1]) * s].reshape(-1, s)
            out = np.zeros((int(eptr[f, -1]), s), np.uint32)
            out[:int(base_ptr[-1])] = ent
            gstarts = eptr[f, n_lru:n_lru + K]
            if trip is not None:
                # the changed derived vars' entries (key = their constant arguments, value = the
                # candidate's patched column), one row per (triple, candidate of its block)
                lens = sizes[tj]
                rep = np.repeat(np.arange(len(tj)), lens)
                within = np.arange(int(lens.sum())) - np.repeat(np.cumsum(lens) - lens, lens)
                cols = starts[tj][rep] + within
                rows = gstarts[cols] + ti[rep]
                uv, vinv = np.unique(tv, return_inverse=True)
                keys = np.asarray([[w for aw, av in zip(spec.arg_widths, syms.derived[int(v)][1])
                                    for w in to_words(int(av), aw)] for v in uv], np.uint32)
                klen = keys.shape[1]
                nl = limbs(syms.var_widths[int(uv[0])])
                out[rows, :klen] = keys[vinv[rep]]
                vrow = off[uv][vinv[rep]]
                out[rows, klen:klen + nl] = words[vrow[:, None] + np.arange(nl)[None, :], (n_lru + cols)[:, None]]
            if n_lru and K:
                gstart = gstarts + add_cnt
                rep = cnt_gen
                tot = int(rep.sum())
                if tot:
                    cand = np.repeat(np.arange(K), rep)
                    within = np.arange(tot) - np.repeat(np.cumsum(rep) - rep, rep)
                    dst = gstart[cand] + within
                    srcrow = base_ptr[src[cand]] + within
                    out[dst] = ent[srcrow]
            ebase[f] = wpos
            ew_chunks.append(out.reshape(-1))
            wpos += out.size
            nr = limbs(spec.result_width)
            lel = lru.else_words[int(lru.else_base[f]):int(lru.else_base[f]) + n_lru * nr].reshape(-1, nr) \
                if n_lru else np.zeros((0, nr), np.uint32)
            gel = lel[src] if n_lru else np.zeros((K, nr), np.uint32)
            elb[f] = epos
            el = np.concatenate([lel, gel]).reshape(-1)
            el_chunks.append(el)
            epos += el.size
        mb = ModelBatch(lru.var_widths, words, lru.funcs, eptr, np.concatenate(ew_chunks), ebase,
                        np.concatenate(el_chunks), elb, 0)
        return CandidateSet(mb, n_lru, base, block_of, [p for p, _ in blocks], syms, lru_models)
