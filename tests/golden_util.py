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
