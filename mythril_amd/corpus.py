"""Harvest / replay corpus of quick-sat queries.

The reference can dump the queries that reach z3 (``--solver-log``, ``mythril/support/model.py:51-62``)
but not the ones quick-sat answers.  :class:`Recorder` is the missing hook: attached to a
:class:`~mythril_amd.support.ModelCache`, it stores every ``check_quick_sat`` evaluation as one
record — the lowered conjunction (one tape), the candidate models in the order they were tried
(MRU first, serialized without completion) and the answer (index of the first hit in that order,
-1 none, -2 unsupported).  On a z3 + solc host this turns ``myth analyze X.sol -t 3`` into the C1
corpus; here it records the synthetic and test workloads.

Record format: one ``.npz`` per query (numpy arrays only, loadable with ``allow_pickle=False``):
tape ``nodes`` (structured mq_node array), ``offsets``, ``consts``; models ``var_widths``,
``var_words``, ``func_arr``, ``entry_ptr``, ``entry_words``, ``entry_base``, ``else_words``,
``else_base``; ``answer`` (int32) and ``seq`` (int64).
"""
from __future__ import annotations

import glob
import os
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .models import FuncSpec, ModelBatch
from .tape import FUNC_DTYPE, NODE_DTYPE, TapeBatch


def save_record(path: str, tb: TapeBatch, mb: ModelBatch, answer: int, seq: int = 0) -> None:
    np.savez(path, nodes=np.asarray(tb.nodes, NODE_DTYPE), offsets=tb.offsets, consts=tb.consts,
             var_widths=mb.var_widths, var_words=mb.var_words, func_arr=mb.func_arr[:len(mb.funcs)],
             entry_ptr=mb.entry_ptr, entry_words=mb.entry_words, entry_base=mb.entry_base,
             else_words=mb.else_words, else_base=mb.else_base,
             answer=np.int32(answer), seq=np.int64(seq))


def load_record(path: str) -> Tuple[TapeBatch, ModelBatch, int]:
    with np.load(path, allow_pickle=False) as z:
        tb = TapeBatch.from_arrays(z["nodes"], z["offsets"], z["consts"])
        funcs = [FuncSpec(int(f["arity"]), int(f["result_width"]), tuple(int(w) for w in f["arg_width"][:int(f["arity"])]))
                 for f in z["func_arr"]]
        mb = ModelBatch(z["var_widths"], z["var_words"], funcs, z["entry_ptr"], z["entry_words"], z["entry_base"],
                        z["else_words"], z["else_base"])
        return tb, mb, int(z["answer"])


def records(directory: str) -> List[str]:
    return sorted(glob.glob(os.path.join(directory, "q*.npz")))


class Recorder:
    """Attach with ``model_cache.recorder = Recorder(dir)`` (or :func:`mythril_amd.support.enable_dump`)."""

    def __init__(self, directory: str):
        self.directory = directory
        os.makedirs(directory, exist_ok=True)
        self.seq = len(records(directory))

    def record(self, expr, order: Sequence, answer: int) -> Optional[str]:
        from .smt import Term
        from .smt_model import as_record
        try:
            if isinstance(expr, Term):
                from .lower import lower_batch, serialize_models
                tb, syms, ok = lower_batch([expr])
                mb = serialize_models([as_record(m) for m in order], syms)
            else:
                from .lower_z3 import lower_batch_z3
                tb, mb, ok = lower_batch_z3([expr], order)
            if not ok[0]:
                answer = -2
        except Exception:
            return None   # a query the lowering cannot express is not part of the corpus
        if mb.n_models == 0:
            return None
        path = os.path.join(self.directory, f"q{self.seq:08d}.npz")
        save_record(path, tb, mb, answer, self.seq)
        self.seq += 1
        return path


def replay(directory: str, first_hit) -> Iterator[Tuple[str, int, int]]:
    """Re-evaluate every record with ``first_hit(tb, mb) -> int`` (the GPU evaluator in the product,
    the oracle in tests); yields ``(path, recorded, replayed)``."""
    for path in records(directory):
        tb, mb, ans = load_record(path)
        yield path, ans, int(first_hit(tb, mb))
