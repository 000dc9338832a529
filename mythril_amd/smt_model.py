"""Candidate models in a z3-independent form — the counterpart of ``Model``
(reference ``mythril/laser/smt/model.py:6-59``) for the z3-free term layer
(:mod:`mythril_amd.smt`).

A model holds interpretations WITHOUT completion, exactly what ``z3.ModelRef`` stores and what
``check_quick_sat`` deep-copies before evaluating with completion (``support_utils.py:63``):

* ``assignment[name]``  — value of a free BV / Bool constant (absent: 0 / false under completion);
* ``functions[name]``   — ``(entries, else_value)`` of an uninterpreted function
  (``keccak256_<n>``, ``keccak256_<n>-1``, ``Power``) or of a symbolic array read through its
  ``as-array`` interpretation (``balance``, ``<tx>_calldata``, ``Storage<addr>``); ``entries``
  maps argument tuples to values (absent function: no entries, else 0).

``ModelRecord`` is the serialisation contract shared with :mod:`mythril_amd.lower_z3`, which reads
a real ``z3.ModelRef`` into the same two dictionaries ("Reading a model").
Models are compared by identity (the reference's LRU keys are ``Model`` objects without
``__eq__``/``__hash__``, support_utils.py:34-53).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Mapping, Optional, Tuple, Union

FuncInterp = Tuple[Dict[Tuple[int, ...], int], int]


class Model:
    """A candidate model (one internal interpretation, as quick-sat models always hold:
    ``solver.py:88-97``)."""

    __slots__ = ("assignment", "functions", "__weakref__")

    def __init__(self, assignment: Optional[Mapping[str, Union[int, bool]]] = None,
                 functions: Optional[Mapping[str, FuncInterp]] = None):
        self.assignment: Dict[str, Union[int, bool]] = dict(assignment or {})
        self.functions: Dict[str, FuncInterp] = {}
        for name, (entries, els) in (functions or {}).items():
            norm = {}
            for k, v in dict(entries).items():
                norm[k if isinstance(k, tuple) else (k,)] = v
            self.functions[name] = (norm, els)

    def decls(self) -> List[str]:
        """Names interpreted by this model (``Model.decls``, smt/model.py:20-25)."""
        return list(self.assignment) + list(self.functions)

    def __getitem__(self, item: str):
        """Interpretation of a constant or function, None if absent (smt/model.py:27-43)."""
        if item in self.assignment:
            return self.assignment[item]
        return self.functions.get(item)

    def record(self) -> "Model":
        return self

    def __repr__(self) -> str:
        return f"Model({self.assignment!r}, {self.functions!r})"


def as_record(model) -> Model:
    """The z3-independent record of a candidate: our own ``Model`` as is, a wrapped z3 model
    through :func:`mythril_amd.lower_z3.model_record` (imported lazily: z3 only exists there)."""
    if isinstance(model, Model):
        return model
    from .lower_z3 import model_record  # z3 host only
    return model_record(model)


def merge_names(models: Iterable[Model]) -> Tuple[List[str], List[str]]:
    vs, fs = {}, {}
    for m in models:
        for k in m.assignment:
            vs[k] = None
        for k in m.functions:
            fs[k] = None
    return list(vs), list(fs)
