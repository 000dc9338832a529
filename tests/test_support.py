"""Host-side drop-in boundary (mythril_amd.support) on CPU: the reference semantics of
LRUCache / ModelCache.check_quick_sat / get_model / Constraints.is_possible
(support_utils.py:34-67, model.py:68-130, constraints.py:28-55), with the verdict engine
replaced by the oracle (tests only — the product engine is the GPU)."""
import random

import numpy as np
import pytest

import keccak_ref
from oracle_engine import OracleEngine, ReferenceLoopCache, eval_under
from mythril_amd import smt as S
from mythril_amd import support as sp
from mythril_amd.exceptions import SolverTimeOutException, UnsatError
from mythril_amd.function_managers import ExponentFunctionManager, KeccakFunctionManager
from mythril_amd.smt_model import Model


@pytest.fixture
def cache():
    return sp.ModelCache(OracleEngine())


@pytest.fixture
def fresh(monkeypatch):
    """Fresh process-global caches with the oracle engine and a scripted solver."""
    sp.reset_caches()
    sp.model_cache = sp.ModelCache(OracleEngine())
    yield
    sp.reset_caches()
    sp.set_solver_backend(None)


x = S.BitVecSym("x", 256)
y = S.BitVecSym("y", 256)


def test_lru_cache_semantics():
    c = sp.LRUCache(3)
    for k in "abc":
        c.put(k, 1)
    assert c.get("a") == 1 and list(c.lru_cache) == ["b", "c", "a"]
    assert c.get("zz") == -1
    c.put("d", 1)                      # evicts LRU "b"
    assert list(c.lru_cache) == ["c", "a", "d"]
    c.put("c", 5)                      # existing key: moved to MRU, nothing evicted
    assert list(c.lru_cache) == ["a", "d", "c"] and c.lru_cache["c"] == 5


def test_first_hit_is_mru_first_and_bumps(cache):
    m1, m2, m3 = Model({"x": 5}), Model({"x": 7}), Model({"x": 5})
    for m in (m1, m2, m3):
        cache.put(m, 1)
    expr = S.And(x == 5)
    assert cache.check_quick_sat(expr) is m3           # MRU first
    assert cache.model_cache.lru_cache[m3] == 2
    e2 = S.ULT(x, S.BitVecVal(6, 256))
    assert cache.check_quick_sat(e2) is m3
    assert list(cache.model_cache.lru_cache) == [m1, m2, m3]
    assert cache.check_quick_sat(S.And(x == 7)) is m2  # bump m2 to MRU
    assert list(cache.model_cache.lru_cache) == [m1, m3, m2]


def test_memoized_false_and_memoized_hit(cache):
    expr = S.And(x == 9)
    cache.put(Model({"x": 1}), 1)
    assert cache.check_quick_sat(expr) is False
    m9 = Model({"x": 9})
    cache.put(m9, 1)
    assert cache.check_quick_sat(expr) is False         # memoized False (lru_cache, support_utils.py:60)
    e2 = S.And(x == 1)
    m1 = cache.check_quick_sat(e2)
    cache.put(m9, 1)
    before = list(cache.model_cache.lru_cache)
    assert cache.check_quick_sat(e2) is m1              # memo hit: same model, no bump
    assert list(cache.model_cache.lru_cache) == before


def test_model_completion_defaults(cache):
    m = Model({})                                       # nothing assigned: x -> 0, b -> false
    cache.put(m, 1)
    assert cache.check_quick_sat(S.And(x == 0)) is m
    assert cache.check_quick_sat(S.Not(S.BoolSym("b"))) is m
    arr = S.Array("balance", 256, 256)
    assert cache.check_quick_sat(arr[x] == 0) is m      # absent array -> K(0)
    f = S.Function("keccak256_512", [512], 256)
    assert cache.check_quick_sat(f(S.BitVecSym("k", 512)) == 0) is m


def test_uf_and_array_tables(cache):
    f = S.Function("keccak256_512", [512], 256)
    k = S.BitVecSym("k", 512)
    m = Model({"k": 3}, {"keccak256_512": ({(3,): 0xABC}, 7), "balance": ({(5,): 100}, 1)})
    cache.put(m, 1)
    bal = S.Array("balance", 256, 256)
    assert cache.check_quick_sat(f(k) == 0xABC) is m
    assert cache.check_quick_sat(S.And(bal[S.BitVecVal(5, 256)] == 100, bal[x] == 1)) is m
    assert cache.check_quick_sat(S.Store(bal, x, S.BitVecVal(42, 256))[S.BitVecVal(0, 256)] == 42) is m
    assert cache.check_quick_sat(S.And(f(k) == 7)) is False


def test_unsupported_fails_closed(cache):
    """A conjunction outside the tape vocabulary (here a ternary UF) gets no quick answer
    without z3 (it goes to the solver, like any miss) and is counted as unsupported."""
    cache.put(Model({"x": 1}), 1)
    g = S.Function("g", [256, 256, 256], 256)
    assert cache.check_quick_sat(S.And(g(x, x, x) == 0, x == 1)) is False
    assert cache.stats["unsupported"] == 1
    assert cache.check_quick_sat(x == 1) is not False


def _random_expr(rng):
    v = rng.randrange(6)
    ops = [lambda: x == v, lambda: S.ULT(x, S.BitVecVal(v, 256)), lambda: S.UGT(y, S.BitVecVal(v, 256)),
           lambda: S.And(x == v, y == (v + 1) % 6), lambda: S.Or(x == v, y == v), lambda: (x + y) == v]
    return ops[rng.randrange(len(ops))]()


@pytest.mark.parametrize("seed", range(4))
def test_batched_prefetch_is_sequentially_exact(seed):
    """Queries answered through prefetch (one launch) + lazy evaluation of models inserted
    mid-batch give exactly the sequential loop's answers and final LRU order."""
    rng = random.Random(seed)
    eng = OracleEngine()
    gpu, ref = sp.ModelCache(eng), ReferenceLoopCache()
    pool = [Model({"x": rng.randrange(6), "y": rng.randrange(6)}) for _ in range(130)]
    for m in pool[:60]:
        gpu.put(m, 1)
        ref.put(m, 1)
    nxt = 60
    for rnd in range(3):
        exprs = [_random_expr(rng) for _ in range(25)]
        gpu.prefetch(exprs)
        for e in exprs:
            if rng.random() < 0.2 and nxt < len(pool):      # a z3 fallback inserting a new model
                gpu.put(pool[nxt], 1)
                ref.put(pool[nxt], 1)
                nxt += 1
            assert gpu.check_quick_sat(e) is ref.check_quick_sat(e)
        assert list(gpu.model_cache.lru_cache) == list(ref.lru)
        assert list(gpu.model_cache.lru_cache.values()) == list(ref.lru.values())
    assert eng.launches < 3 * 25  # batching actually batches


class ScriptedSolver(sp.SolverBackend):
    def __init__(self, answers):
        self.answers = answers
        self.calls = 0

    def solve(self, constraints, minimize, maximize, timeout_ms):
        self.calls += 1
        r = self.answers(constraints)
        if isinstance(r, Model):
            asg, fns = r.assignment, r.functions
            return "sat", lambda: Model(asg, fns)
        return r, None


def test_get_model_gating_and_fallback(fresh):
    solver = ScriptedSolver(lambda cs: Model({"x": 3}))
    sp.set_solver_backend(solver)
    c = sp.Constraints([x == 3])
    m = sp.get_model(c)
    assert solver.calls == 1 and m.assignment == {"x": 3}
    cached = list(sp.model_cache.model_cache.lru_cache)
    assert len(cached) == 1 and cached[0] is not m              # model.py:125-126 calls s.model() twice
    c2 = sp.Constraints([S.ULT(x, S.BitVecVal(10, 256))])
    assert sp.get_model(c2) is cached[0] and solver.calls == 1  # quick-sat hit: no solver call
    assert sp.get_model(c2) is cached[0]                         # lru_cache(2**23) memo
    sp.get_model(c2, minimize=(x,))                              # minimize bypasses quick-sat
    assert solver.calls == 2
    with pytest.raises(UnsatError):
        sp.get_model((x == 1, False))                            # Python False -> UnsatError
    sp.set_solver_backend(ScriptedSolver(lambda cs: "unsat"))
    with pytest.raises(UnsatError) as ei:
        sp.get_model(sp.Constraints([x == 77]))
    assert not isinstance(ei.value, SolverTimeOutException)
    sp.set_solver_backend(ScriptedSolver(lambda cs: "unknown"))
    with pytest.raises(SolverTimeOutException):
        sp.get_model(sp.Constraints([x == 78]))


def test_timeout_budget(fresh):
    sp.time_handler.start_execution(0)
    try:
        with pytest.raises(SolverTimeOutException):
            sp.get_model(sp.Constraints([x == 1]))
    finally:
        sp.time_handler._start_time = None


def test_is_possible_semantics(fresh):
    sp.set_solver_backend(ScriptedSolver(lambda cs: "unknown"))
    c = sp.Constraints([x == 5])
    assert c.is_possible() is False                  # default timeout: timeout prunes
    assert c.is_possible(solver_timeout=100) is True  # custom timeout: timeout keeps
    sp.set_solver_backend(ScriptedSolver(lambda cs: "unsat"))
    assert sp.Constraints([x == 6]).is_possible() is False
    assert sp.Constraints([x == 6]).get_model() is None


def test_is_possible_batch_matches_sequential(fresh):
    rng = random.Random(5)

    def answers(cs):
        # a tiny exact "solver": search x, y in [0, 6) with the oracle
        expr = S.And(*cs)
        for xv in range(6):
            for yv in range(6):
                m = Model({"x": xv, "y": yv})
                if eval_under(expr, m):
                    return m
        return "unsat"

    states = [sp.Constraints([_random_expr(rng), _random_expr(rng)]) for _ in range(30)]
    sp.set_solver_backend(ScriptedSolver(answers))
    batch = sp.is_possible_batch(states)
    order_batch = [(dict(m.assignment), v) for m, v in sp.model_cache.model_cache.lru_cache.items()]
    sp.reset_caches()
    sp.model_cache = sp.ModelCache(OracleEngine())
    sp.set_solver_backend(ScriptedSolver(answers))
    seq = [c.is_possible() for c in states]
    order_seq = [(dict(m.assignment), v) for m, v in sp.model_cache.model_cache.lru_cache.items()]
    assert batch == seq and order_batch == order_seq
    assert any(seq) and not all(seq)


def test_keccak_manager_shapes():
    km = KeccakFunctionManager(hasher=keccak_ref.keccak256)
    assert km.get_empty_keccak_hash().value == int.from_bytes(keccak_ref.keccak256(b""), "big")
    c = km.create_keccak(S.BitVecVal(0, 256))
    assert c.value == 0x290DECD9548B62A8D60345A988386FC84BA6BC95484008F6362F93160EF3E563
    k = S.BitVecSym("k", 512)
    h = km.create_keccak(k)
    assert h.kind == S.APP and h.params[0] == "keccak256_512"
    cond = km.create_conditions()
    names = {t.params[0] for t in S.walk(cond) if t.kind == S.APP}
    assert names == {"keccak256_512", "keccak256_512-1", "keccak256_256", "keccak256_256-1"}
    lo, hi = km.interval(512)
    v = (lo + 63) // 64 * 64
    assert lo <= v < hi
    # a model whose table maps k to an in-interval multiple of 64 and inverts it satisfies the axioms
    good = Model({"k": 11}, {"keccak256_512": ({(11,): v}, 0), "keccak256_512-1": ({(v,): 11}, 0),
                             "keccak256_256": ({(0,): c.value}, 0), "keccak256_256-1": ({(c.value,): 0}, 0)})
    assert eval_under(cond, good)
    bad = Model({"k": 11}, {"keccak256_512": ({(11,): v + 1}, 0), "keccak256_512-1": ({(v + 1,): 11}, 0),
                            "keccak256_256": ({(0,): c.value}, 0), "keccak256_256-1": ({(c.value,): 0}, 0)})
    assert not eval_under(cond, bad)


def test_exponent_manager():
    em = ExponentFunctionManager()
    v, c = em.create_condition(S.BitVecVal(3, 256), S.BitVecVal(5, 256))
    assert v.value == 243 and eval_under(c, Model({}, {"Power": ({(3, 5): 243}, 0)}))
    e = S.BitVecSym("e", 256)
    p, cond = em.create_condition(S.BitVecVal(256, 256), e)
    table = {(256, i): pow(256, i, 2 ** 256) for i in range(32)}
    table[(256, 33)] = 256
    assert eval_under(cond, Model({"e": 33}, {"Power": (dict(table), 0)}))
    assert not eval_under(cond, Model({"e": 33}, {"Power": ({(256, 33): 256}, 0)}))  # axioms missing


def test_prefetch_skips_memoized_and_leaves_nothing_pending(cache):
    """a conjunction already answered by the check_quick_sat memo must not stay in
    the pending set (it would ride along in every later launch)."""
    m = Model({"x": 4})
    cache.put(m, 1)
    e1 = S.And(x == 4)
    assert cache.check_quick_sat(e1) is m
    cache.prefetch([e1])
    assert e1 not in cache._pending and e1 not in cache._rows
    e2 = S.ULT(x, S.BitVecVal(9, 256))
    cache.prefetch([e2])            # prefetched but never asked (answered elsewhere)
    cache.discard([e2])
    assert not cache._pending and not cache._rows


def test_is_possible_batch_discards_rows_answered_by_get_model_memo(fresh):
    sp.set_solver_backend(ScriptedSolver(lambda cs: Model({"x": 2})))
    c = sp.Constraints([x == 2])
    assert c.is_possible()                        # solver call, model cached, get_model memoized
    assert sp.is_possible_batch([c, c]) == [True, True]
    assert not sp.model_cache._pending and not sp.model_cache._rows


def test_check_quick_sat_memo_is_bounded_lru(cache):
    cache.put(Model({"x": 1}), 1)
    cache.MEMO_SIZE = 4
    exprs = [S.And(x == v) for v in range(6)]
    for e in exprs:
        cache.check_quick_sat(e)
    assert list(cache._memo) == exprs[2:]
    cache.check_quick_sat(exprs[2])              # a memo hit moves to MRU
    assert list(cache._memo)[-1] is exprs[2]


def test_keccak_manager_reset_keeps_index_counter():
    """kfm.py:48-54: reset() does not rewind _index_counter."""
    km = KeccakFunctionManager(hasher=keccak_ref.keccak256)
    lo0, _ = km.interval(512)
    km.reset()
    lo1, _ = km.interval(512)
    assert lo1 != lo0


def test_generated_candidates_answer_fork_verdicts(fresh):
    """Args.quick_sat_candidates: forks the LRU misses (fork_workload: a cached path + one new
    branch condition) are answered by generated candidates without the solver; every answer is
    a model that satisfies the query under direct term evaluation."""
    import term_eval
    from mythril_amd.synth_evm import fork_workload
    exprs, recs, parents = fork_workload(24, 40, seed=9)
    solver = ScriptedSolver(lambda cs: "unknown")
    sp.set_solver_backend(solver)
    for m in reversed(recs):
        sp.model_cache.put(m, 1)
    sp.args.quick_sat_candidates, budget = True, sp.args.quick_sat_candidate_budget
    sp.args.quick_sat_candidate_budget = 6000
    try:
        states = [sp.Constraints(list(e.args)) for e in exprs]
        got = sp.is_possible_batch(states)
    finally:
        sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget = False, budget
    # a candidate answer enters the LRU, so a later fork may hit it in quick-sat instead
    assert sp.counters["candidate_answers"] > 0
    assert sp.counters["candidate_answers"] + sp.counters["quick_sat_answers"] == sum(got)
    assert solver.calls == len(states) - sum(got)
    # each answered state: get_model (memoized) returns a model that satisfies the full query
    for st, e, ok in zip(states, exprs, got):
        if ok:
            a = sp.get_model(st, solver_timeout=None, verdict_only=True)   # is_possible's call form
            assert term_eval.is_true(e, a)


def test_candidate_answers_enter_the_lru_like_solver_answers(fresh):
    """INTEGRATION.md "Generated candidates": a candidate answer is cached in the LRU where z3's
    sat model would be (model.py:125) and answers a later state through quick-sat; a candidate
    miss is solved under the plain get_model key (a later Constraints.get_model() does not call
    the solver again)."""
    import term_eval
    from mythril_amd.synth_evm import fork_workload
    exprs, recs, _ = fork_workload(6, 20, seed=9)
    solved = Model({"sender_1": 1})
    solver = ScriptedSolver(lambda cs: solved)
    sp.set_solver_backend(solver)
    for m in reversed(recs):
        sp.model_cache.put(m, 1)
    sp.args.quick_sat_candidates, budget = True, sp.args.quick_sat_candidate_budget
    sp.args.quick_sat_candidate_budget = 6000
    try:
        states = [sp.Constraints(list(e.args)) for e in exprs]
        answered = []
        for st, e in zip(states, exprs):
            n_lru = len(sp.model_cache.model_cache.lru_cache)
            before = sp.counters["candidate_answers"]
            assert st.is_possible()
            if sp.counters["candidate_answers"] > before:
                # the candidate is now the MRU entry, and it satisfies the state
                mru = next(reversed(sp.model_cache.model_cache.lru_cache))
                assert len(sp.model_cache.model_cache.lru_cache) == min(n_lru + 1, 100)
                assert term_eval.is_true(e, mru)
                answered.append((st, e, mru))
        assert answered, "no fork was answered by a generated candidate"
        # the same state again, read by a model-content caller: quick-sat returns the candidate
        st, e, mru = answered[0]
        sp.get_model.cache_clear()
        sp.model_cache._memo.clear()
        assert sp.get_model(st) is mru
        # a state no candidate satisfies: the solver runs once, under the plain key
        contra = sp.Constraints(list(exprs[0].args) + [S.Not(exprs[0].args[0])])
        calls = solver.calls
        assert contra.is_possible()
        assert solver.calls == calls + 1
        assert contra.get_model() is not None and solver.calls == calls + 1
    finally:
        sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget = False, budget


def test_candidates_off_by_default(fresh):
    from mythril_amd.synth_evm import fork_workload
    exprs, recs, _ = fork_workload(4, 10, seed=10)
    sp.set_solver_backend(ScriptedSolver(lambda cs: "unknown"))
    for m in reversed(recs):
        sp.model_cache.put(m, 1)
    assert sp.is_possible_batch([sp.Constraints(list(e.args)) for e in exprs]) == [False] * 4
    assert sp.counters["candidate_answers"] == 0


class CountingOracleEngine(OracleEngine):
    """OracleEngine that records what reaches the device hook (tapes, uploads)."""

    def __init__(self):
        super().__init__()
        self.uploads = 0
        self.tapes = []

    def _evaluate(self, tb, mb, upload=True):
        self.uploads += int(upload)
        self.tapes.append(tb.n_tapes)
        self.upload_seq_fake = self.uploads
        return super()._evaluate(tb, mb, upload)


def test_child_paths_reuse_cached_conjunct_rows():
    """A stream of forked paths (each query = a previous path + new conjuncts, svm.py:351-358):
    only conjuncts never seen under the current models reach the device, one tape each, and the
    answers equal the reference loop's (term_eval, independent of the lowering)."""
    from mythril_amd.synth_evm import dropin_workload
    exprs, recs, _ = dropin_workload(6, 20, seed=11)
    eng = CountingOracleEngine()
    cache, ref = sp.ModelCache(eng), ReferenceLoopCache()
    for r in reversed(recs):
        cache.put(r, 1)
        ref.put(r, 1)
    rng = random.Random(3)
    stream = list(exprs)
    for e in exprs:   # children: the parent's conjuncts plus one or two new ones
        extra = [S.ULT(S.BitVecVal(rng.randrange(1 << 20), 256), S.BitVecVal(rng.randrange(1 << 20), 256))
                 for _ in range(rng.randrange(1, 3))]
        stream.append(S.And(*(list(e.args) + extra)))
    got = cache.check_quick_sat_batch(stream[:6])
    n_first = sum(eng.tapes)
    got += cache.check_quick_sat_batch(stream[6:])
    want = [ref.check_quick_sat(e) for e in stream]
    assert all((a is False and b is False) or a is b for a, b in zip(got, want))
    st = eng.stats
    assert st["conjuncts_cached"] > 0
    # the children added at most 2 new conjuncts each (plus nothing else)
    assert sum(eng.tapes) - n_first <= 2 * 6
    assert list(cache.model_cache.lru_cache.keys()) == list(ref.lru.keys())


def test_conjunct_rows_follow_new_models():
    """A model inserted between two batches (a solver answer, model.py:125) is evaluated for the
    cached conjuncts too; a query over it is answered exactly."""
    x, y = S.BitVecSym("x", 256), S.BitVecSym("y", 256)
    c1, c2 = S.ULT(x, S.BitVecVal(10, 256)), x + y == S.BitVecVal(7, 256)
    m_old = Model({"x": 100, "y": 0})
    m_new = Model({"x": 3, "y": 4})
    eng = CountingOracleEngine()
    assert eng.rows([S.And(c1, c2)], [m_old])[0].tolist() == [False]
    rows = eng.rows([S.And(c1, c2), c1], [m_new, m_old])
    assert rows[0].tolist() == [True, False] and rows[1].tolist() == [True, False]
    n = len(eng.tapes)
    rows = eng.rows([S.And(c2, c1)], [m_old, m_new])   # same conjuncts, same models: no launch
    assert rows[0].tolist() == [False, True] and len(eng.tapes) == n
    assert eng.stats["conjuncts_cached"] >= 2


def test_resident_models_are_not_reuploaded():
    """The device batch is the candidate set in slot order: a new order of the same models (an
    LRU bump) and repeated calls upload nothing new; a new model does."""
    x = S.BitVecSym("x", 256)
    ms = [Model({"x": i}) for i in range(5)]

    class FakeEv:
        upload_seq = 1

    eng = CountingOracleEngine()
    eng._ev = FakeEv()
    eng.conj_tapes = 0   # whole-query path: every call reaches the device hook
    q = [S.ULT(x, S.BitVecVal(3, 256))]
    eng.rows(q, ms)
    eng.rows([S.ULT(x, S.BitVecVal(4, 256))], list(reversed(ms)))
    assert eng.uploads == 1
    r = eng.rows([S.ULT(x, S.BitVecVal(2, 256))], ms[2:] + ms[:2])
    assert r[0].tolist() == [False, False, False, True, True]
    assert eng.uploads == 1
    eng.rows(q, ms + [Model({"x": 0})])
    assert eng.uploads == 2


def test_fork_stream_witnesses_and_both_candidate_arms(fresh):
    """bench.py's "z3 calls avoided" stream (synth_evm.fork_stream_workload): every successor's
    known witness satisfies it (checked by the independent term evaluator), the solver stand-in
    returns it and get_model caches it like z3's model (model.py:124-126) — in BOTH arms — and
    generated candidates then avoid more solver calls than quick-sat alone, with every state
    still possible."""
    import term_eval
    from mythril_amd.synth_evm import fork_stream_workload
    states, wits, recs = fork_stream_workload(24, 60, seed=21)
    assert all(term_eval.is_true(S.And(*st), w) for st, w in zip(states, wits))
    res = {}
    for cand in (False, True):
        sp.reset_caches()
        sp.model_cache = sp.ModelCache(OracleEngine())
        solver = sp.WitnessSolver(states, wits)
        sp.set_solver_backend(solver)
        saved = sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget
        sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget = cand, 20000
        try:
            for m in reversed(recs):
                sp.model_cache.put(m, 1)
            alive = sp.is_possible_batch([sp.Constraints(st) for st in states])
        finally:
            sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget = saved
        assert all(alive)
        assert solver.calls == sp.counters["solver_calls"]
        # every solver answer entered the LRU (it holds at most 100 models)
        lru = list(sp.model_cache.model_cache.lru_cache.keys())
        assert len(lru) == min(100, len(recs) + solver.calls + sp.counters["candidate_answers"])
        res[cand] = dict(sp.counters)
    assert res[True]["solver_calls"] < res[False]["solver_calls"]
    assert res[True]["get_model_calls"] == res[False]["get_model_calls"] == len(states)


def test_model_slots_survive_solver_model_churn():
    """A long run's solver answers churn through the 100-entry LRU; batches then name only the
    few models not evaluated yet.  The engine's model slots (and with them the cached conjunct
    verdicts) start over only past ~4x the LRU's capacity, not every ~260 models."""
    eng = OracleEngine()
    cache = sp.ModelCache(eng)
    for i in range(100):
        cache.put(Model({"x": i}), 1)
    cache.check_quick_sat(x == 5)
    epoch = eng.incremental.slot_epoch
    n = 100
    for b in range(6):                  # prefetched batches; a solver model arrives before each
        exprs = [x == 10_000 + 50 * b + k for k in range(50)]
        cache.prefetch(exprs)
        for e in exprs:
            cache.put(Model({"x": n}), 1)   # (the pending rows need this one model only)
            n += 1
            assert cache.check_quick_sat(e) is False
    assert n == 400 and eng.incremental.slot_epoch == epoch


def test_solver_worker_is_reused_and_replaced_after_a_failure(fresh):
    """The solver runs on one persistent worker thread (model.py:104-113 starts a ThreadPool(1)
    per call); a call that raises discards it, and the next call gets a new one -- answers and
    exceptions as the reference's."""
    import threading
    seen = []

    class Recording(sp.SolverBackend):
        def __init__(self, fail=False):
            self.fail = fail

        def solve(self, constraints, minimize, maximize, timeout_ms):
            seen.append(threading.get_ident())
            if self.fail:
                raise RuntimeError("solver crashed")
            return "unsat", None

    sp.set_solver_backend(Recording())
    for v in (90, 91, 92):
        with pytest.raises(UnsatError):
            sp.get_model(sp.Constraints([x == v]))
    assert len(set(seen)) == 1 and seen[0] != threading.get_ident()
    pool = sp._solver_pool
    sp.set_solver_backend(Recording(fail=True))
    with pytest.raises(SolverTimeOutException):       # an exception is "unknown" (model.py:111-113)
        sp.get_model(sp.Constraints([x == 93]))
    assert sp._solver_pool is None                     # discarded, as terminate() does
    sp.set_solver_backend(Recording())
    with pytest.raises(UnsatError):
        sp.get_model(sp.Constraints([x == 94]))
    assert sp._solver_pool is not None and sp._solver_pool is not pool   # a new worker


def test_conjunct_row_numbering_and_query_reduction():
    """ConjunctRows.rows_for numbers new conjunct nodes in order of first appearance (duplicates
    share a row, the table grows past its first capacity), and the drop-in rows of a batch with an
    empty conjunction (And() of nothing: true), a failing query and repeated conjuncts equal the
    reference loop's per-model verdicts."""
    rows = sp.ConjunctRows()
    r = rows.rows_for(np.array([7, 3, 7, 2000, 3], np.int64), 4)
    assert r.tolist() == [0, 1, 0, 2, 1] and rows.n_rows == 3
    r2 = rows.rows_for(np.array([5000, 2000, 9], np.int64), 300)
    assert r2.tolist() == [3, 2, 4] and rows.R.shape[1] >= 300 and len(rows.row_of) > 5000
    x, y = S.BitVecSym("x", 256), S.BitVecSym("y", 256)
    g = S.Function("g3", [8, 8, 8], 8)
    v = S.BitVecSym("v", 8)
    ms = [Model({"x": i, "y": 7 - i, "v": i}) for i in range(8)]
    c1, c2 = S.ULT(x, S.BitVecVal(5, 256)), S.UGT(y, S.BitVecVal(2, 256))
    qs = [S.And(c1, c2), S.And(), S.And(c1, g(v, v, v) == 0), S.And(c2, c1, c2), S.And(c1)]
    eng = OracleEngine()
    got = eng.rows(qs, ms)
    assert got[2] is None
    for q, row in zip(qs, got):
        if row is None:
            continue
        assert row.tolist() == [eval_under(q, m) for m in ms]
