"""UF keys wider than any value (keccak256_<n> of a SHA3 input longer than 256 bytes,
instructions.py:1018-1055 / keccak_function_manager.py:56-64): lowered as 256-bit chunk lookups
(mq.h MQ_OP_UF_CHUNK / MQ_OP_UF_WIDE) instead of one 4096-bit key, so a single long SHA3 input no
longer makes every later conjunction of the path unsupported.  CPU: the lowering's shape, the
oracle's verdicts against the independent term evaluator, the > 64-entry rule, and the drop-in
engine (oracle-backed) answering such states without an unsupported count."""
import random

import numpy as np
import pytest

import cref
import keccak_ref
import pyoracle
import term_eval
from oracle_engine import OracleEngine, ReferenceLoopCache
from mythril_amd import smt as S
from mythril_amd import support as sp
from mythril_amd.function_managers import KeccakFunctionManager
from mythril_amd.lower import WIDE_KEY_BITS, lower_batch, serialize_models
from mythril_amd.smt_model import Model
from mythril_amd.tape import Op

F4096 = S.Function("keccak256_4096", [4096], 256)
INV4096 = S.Function("keccak256_4096-1", [256], 4096)
F2560 = S.Function("keccak256_2560", [2560], 256)


def _wide_cases(rng):
    """Expressions over two 4096-bit messages (sixteen 256-bit words; the second straddles its
    words with byte pieces) and a 2560-bit one, and models whose tables hold some of them."""
    w = [S.BitVecSym(f"w{i}", 256) for i in range(16)]
    b = [S.BitVecSym(f"b{i}", 8) for i in range(8)]
    m1 = S.Concat(*w)
    m2 = S.Concat(*b[:4], *w[1:15], S.BitVecSym("t448", 448), *b[4:])     # 32+3584+448+32
    assert m2.size() == 4096
    m3 = S.Concat(*w[:10])
    c = S.BitVecVal(rng.getrandbits(4096), 4096)
    y = S.BitVecSym("y", 256)
    exprs = [
        F4096(m1) == y,
        S.ULT(F4096(m2), y),
        INV4096(F4096(m1)) == m1,                    # the manager's injectivity axiom
        F4096(m1) == F4096(m2),
        F4096(c) == y,                               # constant wide key
        F2560(m3) == y,
        S.Not(F4096(m2) == S.BitVecVal(0, 256)),
        S.And(F4096(m1) == y, S.ULT(w[0], w[1])),
    ]
    models = []
    for _ in range(60):
        vals = {f"w{i}": rng.choice([0, 1, rng.getrandbits(256)]) for i in range(16)}
        vals.update({f"b{i}": rng.getrandbits(8) for i in range(8)})
        vals["t448"] = rng.getrandbits(448)
        vals["y"] = rng.choice([0, 5, rng.getrandbits(256)])
        k1 = term_eval.evaluate(m1, Model(vals))
        k2 = term_eval.evaluate(m2, Model(vals))
        k3 = term_eval.evaluate(m3, Model(vals))
        f, inv = {}, {}
        for k in (k1, k2, c.params[0], rng.getrandbits(4096)):
            if rng.random() < 0.6:
                f[(k,)] = rng.choice([vals["y"], 0, rng.getrandbits(256)])
        for (k,), h in f.items():
            if rng.random() < 0.7:
                inv[(h,)] = k if rng.random() < 0.8 else rng.getrandbits(4096)
        f3 = {(k3,): vals["y"]} if rng.random() < 0.5 else {}
        models.append(Model(vals, {"keccak256_4096": (f, rng.choice([0, vals["y"]])),
                                   "keccak256_4096-1": (inv, 0),
                                   "keccak256_2560": (f3, 0)}))
    return exprs, models


@pytest.mark.parametrize("seed", range(3))
def test_wide_key_lookups_lower_to_chunks_and_match_term_evaluation(seed):
    rng = random.Random(seed)
    exprs, models = _wide_cases(rng)
    tb, syms, ok = lower_batch(exprs)
    assert ok.all()
    for t in range(tb.n_tapes):
        nodes = tb.tape_nodes(t)
        assert int(nodes["width"].max()) <= WIDE_KEY_BITS, t        # no 4096-bit value left
    ops = set(int(o) for t in range(tb.n_tapes) for o in tb.tape_nodes(t)["op"])
    assert int(Op.UF_CHUNK) in ops and int(Op.UF_WIDE) in ops
    mb = serialize_models(models, syms)
    v = cref.verdicts(tb, mb)
    want = np.array([[term_eval.is_true(e, m) for m in models] for e in exprs])
    assert (v == want).all(), np.argwhere(v != want)[:5]
    assert 0 < want.mean() < 1
    fh, _ = cref.first_hit(tb, mb)
    assert (fh != -2).all()
    # the Python oracle agrees on a few models
    for t in range(tb.n_tapes):
        for m in range(0, len(models), 15):
            assert pyoracle.eval_tape(tb, t, mb, m) == bool(want[t, m])


def test_wide_key_compiles_inside_the_evaluator_limits():
    from mythril_amd.evaluator import compile_info
    rng = random.Random(5)
    exprs, _ = _wide_cases(rng)
    tb, _, ok = lower_batch(exprs)
    for t in range(tb.n_tapes):
        ci = compile_info(tb, t)
        assert ci.supported, (t, ci.why)


def test_more_than_64_entries_under_a_wide_lookup_is_unsupported_for_those_tapes_only():
    """The chunk sets are 64-bit entry masks: a batch whose models hold more than 64 entries of a
    wide-key function answers -2 for the tapes that look it up (every device, the oracle) and
    normally for the rest."""
    rng = random.Random(9)
    exprs, models = _wide_cases(rng)
    x = S.BitVecSym("w0", 256)
    exprs = exprs + [x == 1]
    big = dict(models[3].functions["keccak256_4096"][0])
    while len(big) <= 64:
        big[(rng.getrandbits(4096),)] = rng.getrandbits(256)
    models[3] = Model(models[3].assignment, {**models[3].functions, "keccak256_4096": (big, 0)})
    tb, syms, ok = lower_batch(exprs)
    mb = serialize_models(models, syms)
    fh, _ = cref.first_hit(tb, mb)
    uses = [any(int(o) == Op.UF_CHUNK and int(a) == syms.func_names.index("keccak256_4096")
                for o, a in zip(tb.tape_nodes(t)["op"], tb.tape_nodes(t)["a"])) for t in range(tb.n_tapes)]
    assert any(uses) and not all(uses)
    for t in range(tb.n_tapes):
        assert (fh[t] == -2) == uses[t], t
    with pytest.raises(ValueError):
        pyoracle.eval_tape(tb, uses.index(True), mb, 3)


def test_one_long_sha3_input_does_not_make_later_queries_unsupported():
    """Drop-in: a path that hashed a 512-byte message carries the manager's axioms for
    keccak256_4096 in every later state; those states are answered (hits and misses equal to
    the reference loop's) with no unsupported count."""
    sp.reset_caches()
    km = KeccakFunctionManager(hasher=keccak_ref.keccak256)
    w = [S.BitVecSym(f"w{i}", 256) for i in range(16)]
    msg = S.Concat(*w)
    h = km.create_keccak(msg)
    h2 = km.create_keccak(S.Concat(w[0], S.BitVecVal(3, 256)))
    cond = km.create_conditions()
    lo, hi = km.interval(4096)
    lo, lo2 = (lo + 63) // 64 * 64, (km.interval(512)[0] + 63) // 64 * 64   # multiples of 64 inside
    rng = random.Random(2)
    models = []
    for i in range(12):
        vals = {f"w{j}": rng.getrandbits(256) for j in range(16)}
        key = term_eval.evaluate(msg, Model(vals))
        key2 = (vals["w0"] << 256) | 3
        v = (lo + 64 * rng.randrange(1, 1000)) if i % 3 else lo + 1     # every third breaks urem 64
        v2 = lo2 + 64 * rng.randrange(1, 1000)
        models.append(Model(vals, {"keccak256_4096": ({(key,): v}, 0), "keccak256_4096-1": ({(v,): key}, 0),
                                   "keccak256_512": ({(key2,): v2}, 0), "keccak256_512-1": ({(v2,): key2}, 0)}))
    cache = sp.ModelCache(OracleEngine())
    ref = ReferenceLoopCache()
    for m in models:
        cache.put(m, 1)
        ref.put(m, 1)
    queries = [S.And(cond, S.ULT(w[1], w[2])), S.And(cond, w[3] == 7), S.And(cond, S.UGT(h, h2)),
               S.And(cond, S.ULT(w[5], w[4]), S.ULT(w[6], w[5]))]
    for q in queries:
        got, exp = cache.check_quick_sat(q), ref.check_quick_sat(q)
        assert got is exp
    assert cache.stats["unsupported"] == 0
    assert any(cache.check_quick_sat(q) is not False for q in queries)
    sp.reset_caches()
