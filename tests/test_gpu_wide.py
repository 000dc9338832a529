"""GPU parity for values wider than 512 bits: keccak inputs longer than 64 bytes
and everything that touches them — Concat / Extract / EQ / ITE at 544..2048 bits, UF keys and
inverse-UF results of those widths, multi-block interpreted keccak — bit-exact against the oracle
(oracle/cref.c holds values up to 2048 bits)."""
import numpy as np
import pytest

import cref
import keccak_ref
from mythril_amd.models import ModelBatch
from mythril_amd.synth import fuzz_workload
from mythril_amd.tape import Tape, TapeBatch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_wide_fuzz_verdicts_match_oracle(evaluator, seed):
    tb, mb = fuzz_workload(200 + seed, 60, 100, max_width=2048, depth=4)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    assert ct.split()[2] > 0            # the wide kinds actually ran
    v_gpu, fh_gpu = evaluator.verdicts(ct)
    v_ref = cref.verdicts(tb, mb)
    mism = np.argwhere(v_gpu != v_ref)
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (fh_gpu == fh_ref).all()
    assert (evaluator.first_hit(ct) == fh_ref).all()


def test_c4_wide_keccak_inputs_match_oracle(evaluator):
    """WalletLibrary-shaped paths: keccak256_544 / _768 / _1088 of calldata Concats, the manager's
    axioms over all three sizes (inv(f(x)) == x at n bits), inverse results Extract'ed."""
    from mythril_amd.synth_evm import c4_wide_workload
    tb, mb, exp, _ = c4_wide_workload(40, 3000, seed=44, hasher=keccak_ref.keccak256)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    fh = evaluator.first_hit(ct)
    ref, _ = cref.first_hit(tb, mb)
    assert (ref[exp >= 0] <= exp[exp >= 0]).all() and (ref[exp >= 0] >= 0).all()
    assert (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    v, _ = evaluator.verdicts(ct)
    assert (v == cref.verdicts(tb, mb)).all()


def test_c4_wide_hoisted_columns(evaluator):
    """The same batch with batch-level hoisting: the shared axiom conjunct (all wide values)
    becomes a once-per-model column program on the wide kernels; verdicts are unchanged."""
    from mythril_amd.synth_evm import c4_wide_workload
    tb0, mb0, _, _ = c4_wide_workload(24, 1500, seed=45, hasher=keccak_ref.keccak256)
    ref, _ = cref.first_hit(tb0, mb0)
    tb, mb, _, _ = c4_wide_workload(24, 1500, seed=45, hasher=keccak_ref.keccak256, hoist=True)
    assert tb.columns is not None and tb.columns.n > 0
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    assert (evaluator.first_hit(ct) == ref).all()


def test_keccak_op_wide_widths(evaluator):
    """Interpreted keccak of 65..256-byte arguments: one block up to 135 bytes, two blocks from
    136 bytes on (the pad byte then opens the second block)."""
    rng = np.random.default_rng(12)
    widths = [8 * k for k in (65, 68, 96, 127, 128, 135, 136, 137, 200, 255, 256)]
    M = 70
    mb = ModelBatch(widths, np.vstack([rng.integers(0, 1 << 32, ((w + 31) // 32, M), dtype=np.uint64).astype(np.uint32)
                                       for w in widths]))
    tapes = []
    for v, w in enumerate(widths):
        t = Tape()
        k = t.keccak(t.var(v, w))
        val = sum(int(mb.var_words[int(mb.var_word_offsets()[v]) + i, 0]) << (32 * i) for i in range((w + 31) // 32))
        val &= (1 << w) - 1
        dig = int.from_bytes(keccak_ref.keccak256(val.to_bytes(w // 8, "big")), "big")
        tapes.append(t.finish(t.eq(k, t.const(dig, 256))))
    tb = TapeBatch(tapes)
    evaluator.upload_models(mb)
    v_gpu, fh = evaluator.verdicts(tb)
    assert (fh != -2).all()
    assert v_gpu[:, 0].all()
    assert (v_gpu == cref.verdicts(tb, mb)).all()


@pytest.mark.parametrize("seed", range(2))
def test_keccak_columns_match_unhoisted_oracle(evaluator, monkeypatch, seed):
    """Interpreted keccak of Concat(variables, constants) at 256..2048 bits, shared by several
    conjunctions: hoisted into keccak columns computed by the dedicated keccak-f[1600] kernel
    (mq_tapes_column_keccak), then read by the tapes.  Verdicts equal the oracle's on the
    UNhoisted lowering and the interpreter path's (MQ_NO_KECCAK_COLUMNS=1)."""
    from mythril_amd import smt as S
    from mythril_amd.lower import SymbolTable, lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    rng = np.random.default_rng(70 + seed)
    words = [S.BitVecSym(f"w{i}", 256) for i in range(6)]
    sel = S.BitVecSym("sel", 32)
    msgs = [S.Concat(words[0], S.BitVecVal(1, 256)),                                   # mapping slot (512)
            S.Concat(sel, words[1], S.BitVecVal(7, 256)),                              # 544
            S.Concat(words[2], words[3], S.BitVecVal(2, 256)),                         # 768
            S.Concat(words[4], S.BitVecVal(3, 256), words[5], words[0], S.BitVecVal(9, 32)),   # 1056
            S.Concat(*(words + [S.BitVecVal(5, 256), words[1]])),                      # 2048 (two blocks)
            words[3]]                                                                  # 256
    hs = [S.Keccak256(m) for m in msgs]
    roots = []
    for i in range(40):
        h = hs[int(rng.integers(len(hs)))]
        g = hs[int(rng.integers(len(hs)))]
        c = int(rng.integers(0, 1 << 32))
        hi = 7 if i % 2 else 15   # a byte (a hit among 600 models is likely) or 16 bits (unlikely)
        roots.append(S.And(S.ULT(S.BitVecVal(c, 256), h),
                           S.Extract(hi, 0, g) == S.BitVecVal(int(rng.integers(0, 1 << (hi + 1))), hi + 1)))
    models = [Model({**{f"w{i}": int.from_bytes(rng.bytes(32), "little") for i in range(6)},
                     "sel": int(rng.integers(0, 1 << 32))}) for _ in range(600)]
    syms = SymbolTable(interpret_keccak=True)
    tb0, syms0, ok0 = lower_batch(roots, syms)
    ref, _ = cref.first_hit(tb0, serialize_models(models, syms0))
    syms = SymbolTable(interpret_keccak=True)
    tb, syms1, ok1 = lower_batch(roots, syms, hoist=True)
    assert ok0.all() and ok1.all() and tb.columns is not None
    mb = serialize_models(models, syms1)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.keccak_columns() == len(hs)
    fh = evaluator.first_hit(ct)
    v, _ = evaluator.verdicts(tb)
    assert (fh == ref).all() and 0 < (ref >= 0).sum() < len(ref)
    assert (v == cref.verdicts(tb0, serialize_models(models, syms0))).all()
    monkeypatch.setenv("MQ_NO_KECCAK_COLUMNS", "1")
    ct2 = evaluator.compile(tb)
    assert ct2.keccak_columns() == 0 and (evaluator.first_hit(ct2) == ref).all()


@pytest.mark.gpu
def test_address_key_mapping_uses_keccak_columns(evaluator):
    from mythril_amd.lower import SymbolTable, lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    rng = np.random.default_rng(6)
    from test_lowering import _address_key_roots
    roots, xs, keys, hs = _address_key_roots(rng)
    models = [Model({f"a{i}": int.from_bytes(rng.bytes(32), "little") for i in range(3)}) for _ in range(700)]
    tb0, syms0, _ = lower_batch(roots, SymbolTable(interpret_keccak=True))
    ref, _ = cref.first_hit(tb0, serialize_models(models, syms0))
    tb, syms1, ok = lower_batch(roots, SymbolTable(interpret_keccak=True), hoist=True)
    evaluator.upload_models(serialize_models(models, syms1))
    ct = evaluator.compile(tb)
    assert ct.keccak_columns() == len(hs)
    assert (evaluator.first_hit(ct) == ref).all() and (ref >= 0).any()


@pytest.mark.parametrize("seed", range(3))
def test_wide_key_chunk_lookups_match_oracle(evaluator, seed):
    """keccak256_4096 / _2560 keys matched 256 bits at a time (G_UFK0 / G_UFK / G_UFKV on the
    assembly interpreter, h_ufk / h_ufkv on the C++ one): verdicts equal the oracle's and the
    independent term evaluator's (tests/test_wide_keys.py)."""
    import random
    import term_eval
    from test_wide_keys import _wide_cases
    from mythril_amd.lower import lower_batch, serialize_models
    exprs, models = _wide_cases(random.Random(40 + seed))
    tb, syms, ok = lower_batch(exprs)
    assert ok.all()
    mb = serialize_models(models, syms)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    v, fh = evaluator.verdicts(ct)
    want = np.array([[term_eval.is_true(e, m) for m in models] for e in exprs])
    assert (v == want).all(), np.argwhere(v != want)[:5]
    assert (v == cref.verdicts(tb, mb)).all()
    assert (fh == cref.first_hit(tb, mb)[0]).all() and (fh != -2).all()


def test_wide_key_over_64_entries_is_unsupported_only_where_looked_up(evaluator):
    import random
    from test_wide_keys import _wide_cases
    from mythril_amd import smt as S
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    rng = random.Random(9)
    exprs, models = _wide_cases(rng)
    exprs = exprs + [S.BitVecSym("w0", 256) == 1]
    big = dict(models[3].functions["keccak256_4096"][0])
    while len(big) <= 64:
        big[(rng.getrandbits(4096),)] = rng.getrandbits(256)
    models[3] = Model(models[3].assignment, {**models[3].functions, "keccak256_4096": (big, 0)})
    tb, syms, _ = lower_batch(exprs)
    mb = serialize_models(models, syms)
    evaluator.upload_models(mb)
    ref, _ = cref.first_hit(tb, mb)
    assert (ref == -2).any() and (ref != -2).any()
    assert (evaluator.first_hit(tb) == ref).all()


def test_gpu_engine_answers_states_after_a_long_sha3_input():
    """The product VerdictEngine: states carrying keccak256_4096 axioms are answered on the
    device (hits equal to the reference loop's), none unsupported."""
    import random
    import term_eval
    from oracle_engine import ReferenceLoopCache
    from mythril_amd import smt as S
    from mythril_amd import support as sp
    from mythril_amd.function_managers import KeccakFunctionManager
    from mythril_amd.smt_model import Model
    km = KeccakFunctionManager(hasher=keccak_ref.keccak256)
    w = [S.BitVecSym(f"w{i}", 256) for i in range(16)]
    msg = S.Concat(*w)
    km.create_keccak(msg)
    cond = km.create_conditions()
    lo = (km.interval(4096)[0] + 63) // 64 * 64
    rng = random.Random(3)
    gpu, ref = sp.ModelCache(sp.VerdictEngine()), ReferenceLoopCache()
    for i in range(20):
        vals = {f"w{j}": rng.getrandbits(8) for j in range(16)}
        key = term_eval.evaluate(msg, Model(vals))
        v = lo + 64 * rng.randrange(1, 100) + (0 if i % 3 else 1)
        m = Model(vals, {"keccak256_4096": ({(key,): v}, 0), "keccak256_4096-1": ({(v,): key}, 0)})
        gpu.put(m, 1)
        ref.put(m, 1)
    qs = [S.And(cond, S.ULT(w[i], w[i + 1])) for i in range(8)] + [S.And(cond, w[2] == 300 % 256)]
    for q in qs:
        assert gpu.check_quick_sat(q) is ref.check_quick_sat(q)
    assert gpu.stats["unsupported"] == 0 and gpu.stats["hits"] > 0
