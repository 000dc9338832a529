"""Generated candidates on the GPU: M reaches 10^5 in the drop-in path,
and every "sat" answer on a generated candidate is re-checked by the oracle — the candidate's
tape verdict by oracle/cref.c on the same serialized batch, the first-hit property on the
candidates before it, and the materialized model by direct term evaluation."""
import numpy as np
import pytest

import cref
import term_eval
from mythril_amd import support as sp
from mythril_amd.candidates import CandidateGenerator
from mythril_amd.synth_evm import fork_workload

pytestmark = pytest.mark.gpu


def test_candidates_reach_1e5_and_every_hit_rechecks(evaluator):
    exprs, recs, parents = fork_workload(48, 100, seed=11)
    eng = sp.VerdictEngine(evaluator)
    fh, cs = eng.candidate_first_hits(exprs, recs, CandidateGenerator(100_000, seed=3, fill=True))
    assert cs.batch.n_models == 100_000 and cs.n_lru == 100
    tb = eng.incremental.lower(exprs)[0].to_tapes()
    lru = fh < cs.n_lru
    assert not (lru & (fh >= 0)).any()        # forks: no cached model satisfies them
    gen = np.flatnonzero(fh >= cs.n_lru)
    assert len(gen) > 0
    for q in gen:
        h = int(fh[q])
        assert cref.eval_tape(tb, int(q), cs.batch, h) == 1
        assert term_eval.is_true(exprs[q], cs.materialize(h))
    for q in gen[:4]:                         # first-hit property on the candidates before it
        sub = cs.batch.shard(0, int(fh[q]))
        assert cref.first_hit(tb.subset([int(q)]), sub)[0][0] == -1
    for q in np.flatnonzero(fh == -1)[:6]:    # misses: no candidate satisfies (oracle, all 10^5)
        assert cref.first_hit(tb.subset([int(q)]), cs.batch)[0][0] == -1


def test_is_possible_batch_with_candidates_on_gpu():
    exprs, recs, _ = fork_workload(16, 60, seed=12)
    sp.reset_caches()
    sp.args.quick_sat_candidates = True
    try:
        for m in reversed(recs):
            sp.model_cache.put(m, 1)
        sp.set_solver_backend(sp.NoSolver())
        got = sp.is_possible_batch([sp.Constraints(list(e.args)) for e in exprs])
        # a candidate answer enters the LRU (model.py:125), so a later fork may hit it in quick-sat
        assert sum(got) == sp.counters["candidate_answers"] + sp.counters["quick_sat_answers"]
        assert sp.counters["candidate_answers"] > 0
        assert len(sp.model_cache.model_cache.lru_cache) == min(100, 60 + sp.counters["candidate_answers"])
    finally:
        sp.args.quick_sat_candidates = False
        sp.set_solver_backend(None)
        sp.reset_caches()
