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
``else_base``; ``answer`` (int32: the evaluator's first hit), ``ref_answer`` (int32: the
reference loop's own first hit, ``z3_quick_sat_loop`` = support_utils.py:62-66 run by z3 on the
same query and order, recorded where z3 is importable; -3 = not recorded) and ``seq`` (int64).
A corpus harvested on a z3 host is therefore a parity fixture: :func:`replay` checks the
evaluator against z3's answer, not against itself.
"""
from __future__ import annotations

import glob
import os
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .models import FuncSpec, ModelBatch
from .tape import FUNC_DTYPE, NODE_DTYPE, TapeBatch


NOT_RECORDED = -3


def save_record(path: str, tb: TapeBatch, mb: ModelBatch, answer: int, seq: int = 0,
                ref_answer: int = NOT_RECORDED) -> None:
    np.savez(path, nodes=np.asarray(tb.nodes, NODE_DTYPE), offsets=tb.offsets, consts=tb.consts,
             var_widths=mb.var_widths, var_words=mb.var_words, func_arr=mb.func_arr[:len(mb.funcs)],
             entry_ptr=mb.entry_ptr, entry_words=mb.entry_words, entry_base=mb.entry_base,
             else_words=mb.else_words, else_base=mb.else_base,
             answer=np.int32(answer), ref_answer=np.int32(ref_answer), seq=np.int64(seq))


def load_record(path: str, reference: bool = False) -> Tuple[TapeBatch, ModelBatch, int]:
    """``(tape, models, answer)``; ``reference=True``: the reference loop's answer when it was
    recorded (a z3 host), else the evaluator's."""
    with np.load(path, allow_pickle=False) as z:
        tb = TapeBatch.from_arrays(z["nodes"], z["offsets"], z["consts"])
        funcs = [FuncSpec(int(f["arity"]), int(f["result_width"]), tuple(int(w) for w in f["arg_width"][:int(f["arity"])]))
                 for f in z["func_arr"]]
        mb = ModelBatch(z["var_widths"], z["var_words"], funcs, z["entry_ptr"], z["entry_words"], z["entry_base"],
                        z["else_words"], z["else_base"])
        ans = int(z["answer"])
        if reference and "ref_answer" in z.files and int(z["ref_answer"]) != NOT_RECORDED:
            ans = int(z["ref_answer"])
        return tb, mb, ans


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
        ref = NOT_RECORDED
        if not isinstance(expr, Term):
            # z3 host: the reference's own loop on the same query and order is the fixture answer
            from .lower_z3 import z3_quick_sat_loop
            hit = z3_quick_sat_loop(expr, list(order))
            ref = -1 if hit is False else next(i for i, m in enumerate(order) if m is hit)
        path = os.path.join(self.directory, f"q{self.seq:08d}.npz")
        save_record(path, tb, mb, answer, self.seq, ref)
        self.seq += 1
        return path


def replay(directory: str, first_hit) -> Iterator[Tuple[str, int, int]]:
    """Re-evaluate every record with ``first_hit(tb, mb) -> int`` (the GPU evaluator in the product,
    the oracle in tests); yields ``(path, recorded, replayed)`` where ``recorded`` is the reference
    loop's answer when the corpus was harvested on a z3 host, else the evaluator's own."""
    for path in records(directory):
        tb, mb, ans = load_record(path, reference=True)
        yield path, ans, int(first_hit(tb, mb))
