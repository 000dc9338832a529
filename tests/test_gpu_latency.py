"""GPU parity of the drop-in path's latency mode: a single EVM-shaped conjunction split into its
conjuncts (support.py split_conjuncts) and evaluated with MQ_OPT_LATENCY_WAVES (the G kernel with
one tape per wave) gives the oracle's verdicts, the same as the throughput launch."""
import numpy as np
import pytest

import cref
from mythril_amd import support as sp
from mythril_amd.lower import IncrementalLowering
from mythril_amd.synth_evm import dropin_workload

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m", [(1, 16), (1, 100), (3, 64)])
def test_latency_mode_split_matches_oracle(evaluator, n, m):
    exprs, recs, planted = dropin_workload(n, m, seed=5, query_seed=3)
    inc = IncrementalLowering()
    db, ok = inc.lower(exprs)
    mb = inc.serialize(recs)
    whole_ref = cref.verdicts(db.to_tapes(), mb)
    split, starts = sp.split_conjuncts(db, 64)
    tb = split.to_tapes()
    ref = cref.verdicts(tb, mb)
    evaluator.upload_models(mb)
    out = {}
    for waves in (0, 1 << 20):
        evaluator.set_option(evaluator.OPT_LATENCY_WAVES, waves)
        try:
            ct = evaluator.compile(split)
            v, fh = evaluator.verdicts(ct)
            out[waves] = (v, ct.asm_split()[2])
            ct.free()
        finally:
            evaluator.set_option(evaluator.OPT_LATENCY_WAVES, 0)
        assert (v == ref).all()
        assert np.array_equal(np.logical_and.reduceat(v, starts, axis=0), whole_ref)
    if evaluator.asm_ready:                  # the EVM-shaped conjuncts (variable divisions too) run on P / G
        assert out[0][1] is True and out[1 << 20][1] is True


def test_verdict_engine_small_batch_answers(evaluator):
    """check_quick_sat_batch through the VerdictEngine (split + latency mode) returns the reference
    loop's answers (support_utils.py:60-67) on the oracle's verdicts."""
    exprs, recs, planted = dropin_workload(2, 40, seed=9, query_seed=4)
    eng = sp.VerdictEngine(evaluator)
    cache = sp.ModelCache(eng)
    for r in reversed(recs):
        cache.put(r, 1)
    answers = cache.check_quick_sat_batch(exprs)
    inc = IncrementalLowering()
    db, _ = inc.lower(exprs)
    v = cref.verdicts(db.to_tapes(), inc.serialize(recs))
    order = list(range(len(recs)))
    for q, a in enumerate(answers):
        hit = next((i for i in order if v[q, i]), None)
        if hit is None:
            assert a is False
        else:
            assert a is recs[hit]
            order.remove(hit)
            order.insert(0, hit)
