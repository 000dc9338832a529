"""Helpers to load the committed golden fixtures (tests/golden/*.json) as tapes."""
from __future__ import annotations

import json
import os

import numpy as np

from mythril_amd.tape import NODE_DTYPE, Op, Tape, TapeBatch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def fixture_tape(entry) -> Tape:
    """The entry's tape (its nodes and consts; finish() picks the root)."""
    t = Tape()
    for row in entry["nodes"]:
        op, w, a, b, c = row
        t.nodes.append((op, w, a, b, c))
        t.kind.append("bool" if w == 0 and op not in (Op.STORE, Op.CONST_ARRAY, Op.ARRAY_VAR) else "bv")
    t.consts = list(entry["consts"])
    return t


def check_tape(entry, expected: int, negate: bool = False) -> Tape:
    """Tape whose root is EQ(value_node, expected) (or expected ^ 1 when negate)."""
    t = fixture_tape(entry)
    v = entry["value_node"]
    w = t.width(v)
    c = t.const(expected ^ (1 if negate else 0), w)
    root = t.eq(v, c)
    return t.finish(root)


def constraint_tape(entry) -> Tape:
    """The entry's EXP constraint tape (the product lowering of the conjunction of
    ``c == Power(b, e)``, tests/golden/make_golden.py), Power = model function 0."""
    t = fixture_tape(entry["constraint"])
    return t.finish(len(t.nodes) - 1)


def power_models(entries) -> "ModelBatch":
    """Two models over one 8-bit variable and the 2-argument ``Power`` table (function 0): model
    0 holds every (b, e) -> pow(b, e, 2^256) entry the entries list, model 1 none (z3's
    completion: else 0)."""
    from mythril_amd.models import FuncSpec, ModelBatch
    table = {}
    for e in entries:
        for b, x, r in e.get("power", ()):
            table[(int(b, 16), int(x, 16))] = int(r, 16)
    return ModelBatch.from_python([8], [{"funcs": {0: (table, 0)}}, {}], [FuncSpec(2, 256, (256, 256))])
