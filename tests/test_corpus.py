"""Harvest hook + corpus format (mythril_amd.corpus): every evaluated
check_quick_sat query is recorded (tape, candidate order, answer) and replays to the same answer."""
import random

import numpy as np

import cref
from oracle_engine import OracleEngine
from mythril_amd import smt as S
from mythril_amd import support as sp
from mythril_amd.corpus import Recorder, load_record, records, replay
from mythril_amd.smt_model import Model

x = S.BitVecSym("x", 256)
y = S.BitVecSym("y", 256)
bal = S.Array("balance", 256, 256)


def _expr(rng):
    v = rng.randrange(6)
    c = S.BitVecVal(v, 256)
    return rng.choice([x == v, S.ULT(x, c), S.And(x == v, y == (v + 1) % 6), (x + y) == v,
                       S.UGE(bal[y], c), S.Or(x == v, bal[x] == c)])


def _oracle_first_hit(tb, mb):
    fh, _ = cref.first_hit(tb, mb)
    return fh[0]


def test_recorded_queries_replay_to_the_same_answer(tmp_path):
    rng = random.Random(3)
    cache = sp.ModelCache(OracleEngine())
    cache.recorder = Recorder(str(tmp_path))
    for _ in range(40):
        cache.put(Model({"x": rng.randrange(6), "y": rng.randrange(6)}, {"balance": ({(rng.randrange(6),): rng.randrange(6)}, rng.randrange(3))}), 1)
    answers = []
    for _ in range(30):
        e = _expr(rng)
        r = cache.check_quick_sat(e)
        answers.append(r)
    files = records(str(tmp_path))
    assert len(files) == cache.stats["queries"] > 0
    hits = 0
    for path, recorded, replayed in replay(str(tmp_path), _oracle_first_hit):
        assert recorded == replayed, path
        hits += recorded >= 0
    assert hits == cache.stats["hits"]
    tb, mb, ans = load_record(files[0])
    assert tb.n_tapes == 1 and mb.n_models == 40


def test_enable_dump_on_the_global_cache(tmp_path):
    sp.reset_caches()
    sp.model_cache = sp.ModelCache(OracleEngine())
    try:
        sp.enable_dump(str(tmp_path))
        sp.model_cache.put(Model({"x": 2}), 1)
        assert sp.get_model(sp.Constraints([x == 2])) is not None
        assert len(records(str(tmp_path))) == 1
        sp.enable_dump(None)
        assert sp.model_cache.recorder is None
    finally:
        sp.reset_caches()


def test_records_mark_the_reference_answer_not_recorded_without_z3(tmp_path):
    """Without z3 (z3-free terms) the reference loop's answer is not recorded (-3) and replay
    falls back to the evaluator's own answer; on a z3 host ref_answer holds z3's first hit."""
    from mythril_amd.corpus import NOT_RECORDED
    cache = sp.ModelCache(OracleEngine())
    cache.recorder = Recorder(str(tmp_path))
    cache.put(Model({"x": 1}), 1)
    cache.check_quick_sat(S.And(x == 1))
    (path,) = records(str(tmp_path))
    with np.load(path, allow_pickle=False) as z:
        assert int(z["ref_answer"]) == NOT_RECORDED and int(z["answer"]) == 0
    assert load_record(path, reference=True)[2] == 0
