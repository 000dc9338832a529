"""Conjunct splitting of small drop-in batches (support.py split_conjuncts): a conjunction split
into groups of its conjuncts, evaluated per group and AND-ed, gives the verdict rows of the
whole conjunction.  Checked with the oracle (cref) on the CPU; the GPU path runs it in
test_support_gpu / bench.py's dropin leg."""
import numpy as np
import pytest

import cref
from mythril_amd import support as sp
from mythril_amd.lower import IncrementalLowering
from mythril_amd.synth_evm import dropin_workload


@pytest.mark.parametrize("groups", [2, 5, 64])
def test_split_and_merge_equals_whole(groups):
    exprs, recs, planted = dropin_workload(6, 24, seed=11, query_seed=2)
    inc = IncrementalLowering()
    db, ok = inc.lower(exprs)
    mb = inc.serialize(recs)
    whole = cref.verdicts(db.to_tapes(), mb)
    split, starts = sp.split_conjuncts(db, groups)
    assert starts is not None and split.n_tapes > db.n_tapes
    assert split.n_tapes <= db.n_tapes * groups
    # every original conjunct lands in exactly one group, in order
    assert np.array_equal(split.roots, db.roots)
    assert set(db.root_offsets.tolist()) <= set(split.root_offsets.tolist())
    parts = cref.verdicts(split.to_tapes(), mb)
    merged = np.logical_and.reduceat(parts, starts, axis=0)
    assert np.array_equal(merged, whole)
    # the planted models satisfy their query
    for q, p in enumerate(planted):
        if p >= 0:
            assert merged[q, p]


def test_split_noop_cases():
    exprs, recs, _ = dropin_workload(2, 4, seed=3)
    db, _ = IncrementalLowering().lower(exprs)
    assert sp.split_conjuncts(db, 1)[1] is None
    assert sp.split_conjuncts(db, 0)[1] is None
