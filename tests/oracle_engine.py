"""Test-only helpers: an oracle-backed verdict engine (so the host-side quick-sat logic can be
checked on CPU) and a literal restatement of the reference's sequential loop to compare against.

Never used by the product: ``mythril_amd.support`` defaults to the GPU ``VerdictEngine``."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

import cref
import pyoracle
from mythril_amd.lower import lower_batch, lower_term, serialize_models, SymbolTable
from mythril_amd.tape import TapeBatch


class OracleEngine:
    """Same contract as ``mythril_amd.support.VerdictEngine.rows`` — evaluated by oracle/cref.c."""

    def __init__(self):
        self.launches = 0
        self.pairs = 0

    def rows(self, exprs, models):
        if not models:
            return [np.zeros(0, bool) for _ in exprs]
        tb, syms, ok = lower_batch(exprs)
        mb = serialize_models(models, syms)
        v = cref.verdicts(tb, mb)
        self.launches += 1
        self.pairs += tb.n_tapes * mb.n_models
        return [v[i].copy() if ok[i] else None for i in range(len(exprs))]


def eval_under(expr, model) -> bool:
    """is_true(model.eval(expr, model_completion=True)) by the Python oracle (one model)."""
    syms = SymbolTable()
    tb = TapeBatch([lower_term(expr, syms)])
    mb = serialize_models([model], syms)
    return pyoracle.eval_tape(tb, 0, mb, 0)


class ReferenceLoopCache:
    """support_utils.py:34-67 verbatim in behaviour: LRU of 100, MRU-first loop, bump on hit,
    per-expression memo (functools.lru_cache(2**10) semantics for these small tests: unbounded)."""

    def __init__(self):
        self.lru = OrderedDict()
        self.memo = {}

    def put(self, model, value):
        if model in self.lru:
            del self.lru[model]
        elif len(self.lru) >= 100:
            self.lru.popitem(last=False)
        self.lru[model] = value

    def get(self, model):
        if model not in self.lru:
            return -1
        self.lru.move_to_end(model)
        return self.lru[model]

    def check_quick_sat(self, expr):
        if expr in self.memo:
            return self.memo[expr]
        res = False
        for model in reversed(list(self.lru.keys())):
            if eval_under(expr, model):
                self.put(model, self.get(model) + 1)
                res = model
                break
        self.memo[expr] = res
        return res


def apply_columns(tb, mb):
    """Oracle evaluation of a hoisted batch's column programs (tape.py ColumnSet), level by level,
    written into the model variables they define (the device does this in qs_column_kernel)."""
    from mythril_amd.models import ModelBatch
    from mythril_amd.tape import to_words
    cols = tb.columns
    words = mb.var_words.copy()
    out = ModelBatch(mb.var_widths, words, mb.funcs, mb.entry_ptr, mb.entry_words, mb.entry_base,
                     mb.else_words, mb.else_base, mb.index_base)
    off = out.var_word_offsets()
    for lvl in sorted(set(int(x) for x in cols.level)):
        for k in np.flatnonzero(cols.level == lvl):
            v = int(cols.var_index[k])
            w = int(mb.var_widths[v])
            nodes = cols.programs.tape_nodes(int(k))
            for m in range(mb.n_models):
                val = pyoracle.eval_nodes(nodes, cols.programs.consts, out, m)[-1]
                out.var_words[off[v]:off[v + 1], m] = to_words(int(val), w)
    return out
