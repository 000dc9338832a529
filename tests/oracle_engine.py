"""Test-only helpers: an oracle-backed verdict engine (so the host-side quick-sat logic can be
checked on CPU) and a literal restatement of the reference's sequential loop to compare against.

Never used by the product: ``mythril_amd.support`` defaults to the GPU ``VerdictEngine``."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

import cref
import pyoracle
import term_eval
from mythril_amd.lower import lower_batch, lower_term, serialize_models, SymbolTable
from mythril_amd.support import VerdictEngine
from mythril_amd.tape import TapeBatch


class OracleEngine(VerdictEngine):
    """The product ``VerdictEngine`` — batching, incremental DAG lowering, model serialization —
    with only the device evaluation swapped for oracle/cref.c, so the host-side quick-sat logic
    runs on CPU exactly as in the product (tests only)."""

    hoist_min_models = 1 << 30   # the oracle evaluates unhoisted tapes

    def __init__(self):
        super().__init__(evaluator=None)

    def _first_hit(self, tb, mb):
        import time
        if hasattr(tb, "root_offsets"):
            tb = tb.to_tapes()
        t = time.perf_counter()
        return cref.first_hit(tb, mb)[0], t, t

    def _compile(self, tb):
        return tb   # the oracle evaluates the batch itself

    def _evaluate(self, tb, mb, upload=True):
        if hasattr(tb, "root_offsets"):   # DagBatch -> self-contained tapes
            tb = tb.to_tapes()
        fh, _ = cref.first_hit(tb, mb)
        return cref.verdicts(tb, mb), fh


def eval_under(expr, model) -> bool:
    """is_true(model.eval(expr, model_completion=True)) by the Python oracle (one model)."""
    syms = SymbolTable()
    tb = TapeBatch([lower_term(expr, syms)])
    mb = serialize_models([model], syms)
    return pyoracle.eval_tape(tb, 0, mb, 0)


class ReferenceLoopCache:
    """Checked per model by tests/term_eval.py (direct term evaluation, independent of the
    product lowering).  support_utils.py:34-67 verbatim in behaviour: LRU of 100, MRU-first loop, bump on hit,
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
            if term_eval.is_true(expr, model):
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
