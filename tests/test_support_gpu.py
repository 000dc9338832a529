"""The drop-in boundary on the GPU: ModelCache / get_model / is_possible_batch backed by the HIP
evaluator (no oracle in the product path), compared with the reference's sequential loop
(support_utils.py:60-67) restated in tests/oracle_engine.py."""
import random

import pytest

from oracle_engine import ReferenceLoopCache
from mythril_amd import smt as S
from mythril_amd import support as sp
from mythril_amd.smt_model import Model

pytestmark = pytest.mark.gpu

x = S.BitVecSym("x", 256)
y = S.BitVecSym("y", 256)
cd = S.Array("1_calldata", 256, 8)
bal = S.Array("balance", 256, 256)
kec = S.Function("keccak256_512", [512], 256)


def _expr(rng):
    v = rng.randrange(6)
    c = S.BitVecVal(v, 256)
    ops = [lambda: x == v, lambda: S.ULT(x, c), lambda: S.UGT(y, c), lambda: S.And(x == v, y == (v + 1) % 6),
           lambda: S.Or(x == v, y == v), lambda: (x * y + c) == x,
           lambda: S.If(S.ULT(c, S.BitVecVal(3, 256)), cd[x], S.BitVecVal(0, 8)) == v,
           lambda: S.UGE(bal[y], c), lambda: kec(S.Concat(x, y)) == v,
           lambda: S.Extract(7, 0, S.UDiv(x + c, y)) == v, lambda: S.URem(x, y) == c,
           lambda: (S.LShR(x, c) ^ (y << c)) == c]
    return ops[rng.randrange(len(ops))]()


def _model(rng):
    return Model({"x": rng.randrange(6), "y": rng.randrange(6)},
                 {"1_calldata": ({(rng.randrange(6),): rng.randrange(6)}, rng.randrange(3)),
                  "balance": ({(rng.randrange(6),): rng.randrange(8)}, rng.randrange(4)),
                  "keccak256_512": ({((rng.randrange(6) << 256) | rng.randrange(6),): rng.randrange(6)}, 0)})


@pytest.mark.parametrize("seed", range(3))
def test_gpu_model_cache_matches_reference_loop(seed):
    rng = random.Random(seed)
    eng = sp.VerdictEngine()
    gpu, ref = sp.ModelCache(eng), ReferenceLoopCache()
    pool = [_model(rng) for _ in range(140)]
    for m in pool[:80]:
        gpu.put(m, 1)
        ref.put(m, 1)
    nxt = 80
    for _ in range(3):
        exprs = [_expr(rng) for _ in range(40)]
        gpu.prefetch(exprs)
        for e in exprs:
            if rng.random() < 0.15 and nxt < len(pool):
                gpu.put(pool[nxt], 1)
                ref.put(pool[nxt], 1)
                nxt += 1
            assert gpu.check_quick_sat(e) is ref.check_quick_sat(e)
        assert list(gpu.model_cache.lru_cache) == list(ref.lru)
    assert gpu.stats["unsupported"] == 0
    assert eng.launches < 3 * 40


def test_gpu_get_model_quick_sat_answers():
    sp.reset_caches()
    try:
        m = Model({"x": 4, "y": 1})
        sp.model_cache.put(m, 1)
        assert sp.get_model(sp.Constraints([x == 4, S.ULT(y, x)])) is m
        assert sp.counters["quick_sat_answers"] == 1 and sp.counters["solver_calls"] == 0
        assert sp.is_possible_batch([sp.Constraints([x == 4]), sp.Constraints([y == 1, x == 4])]) == [True, True]
    finally:
        sp.reset_caches()


def test_gpu_fork_children_reuse_parent_conjuncts():
    """LASER's fork stream (svm.py:351-358) on EVM-shaped paths: the parents are checked, then
    their JUMPI successors (parent + cond / parent + Not(cond)).  The children evaluate only the
    new branch conjuncts on the device (the parents' conjunct rows are cached per model), and every
    answer and the final LRU order equal the reference loop's (term_eval, independent of the
    lowering)."""
    from mythril_amd.synth_evm import dropin_workload, fork_children
    parents, recs, _ = dropin_workload(12, 60, seed=21)
    kids = fork_children(parents, seed=5)
    eng = sp.VerdictEngine()
    gpu, ref = sp.ModelCache(eng), ReferenceLoopCache()
    for r in reversed(recs):
        gpu.put(r, 1)
        ref.put(r, 1)
    got = gpu.check_quick_sat_batch(parents)
    before = dict(eng.stats)
    got += gpu.check_quick_sat_batch(kids)
    want = [ref.check_quick_sat(e) for e in parents + kids]
    assert all((a is False and b is False) or a is b for a, b in zip(got, want))
    assert list(gpu.model_cache.lru_cache) == list(ref.lru)
    new = eng.stats["conjuncts_evaluated"] - before["conjuncts_evaluated"]
    assert 0 < new <= len(kids), new                  # one new branch conjunct per child at most
    assert eng.stats["conjuncts_cached"] - before["conjuncts_cached"] > 10 * len(parents)
    assert sum(a is not False for a in got) > 0
