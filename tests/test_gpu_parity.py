"""GPU parity: the HIP evaluator (through the C-ABI) against the oracle on the same seeded
inputs — bit-exact verdicts and first-hit indices (integer work: no tolerance)."""
import numpy as np
import pytest

import cref
import keccak_ref
from golden_util import check_tape, constraint_tape, load, power_models
from unsupported import supported_exactly
from mythril_amd.models import FuncSpec, ModelBatch
from mythril_amd.synth import c2_workload, fuzz_workload
from mythril_amd.tape import Tape, TapeBatch

pytestmark = pytest.mark.gpu


def _one_model():
    return ModelBatch([8], np.zeros((1, 1), np.uint32))


def test_golden_exp_constraints_on_gpu(evaluator):
    """The VMTests EXP programs' Power constraints (product create_condition + lowering): verdicts
    under the model with the Power table and under the empty one, against the oracle."""
    kats = [e for e in load("vmtests_kats.json") if "constraint" in e]
    tb = TapeBatch([constraint_tape(e) for e in kats])
    mb = power_models(kats)
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    assert (fh != -2).all()
    assert v[:, 0].all()
    assert (v == cref.verdicts(tb, mb)).all()
    want_empty = np.array([all(int(r, 16) == 0 for _, _, r in e["power"]) for e in kats])
    assert (v[:, 1] == want_empty).all()


def test_golden_vectors_on_gpu(evaluator):
    """EIP-145 shift vectors + VMTests KATs: EQ(value, expected) true, EQ(value, expected^1) false."""
    entries = load("shift_vectors.json") + load("vmtests_kats.json")
    tapes = []
    for e in entries:
        exp = int(e["expected"], 16)
        tapes.append(check_tape(e, exp))
        tapes.append(check_tape(e, exp, negate=True))
    tb = TapeBatch(tapes)
    evaluator.upload_models(_one_model())
    v, fh = evaluator.verdicts(tb)
    bad = [entries[i]["name"] for i in np.flatnonzero(~v[0::2, 0])]
    assert not bad, bad
    assert not v[1::2, 0].any()
    fh2 = evaluator.first_hit(tb)
    assert list(fh2[0::2]) == [0] * len(entries)
    assert list(fh2[1::2]) == [-1] * len(entries)


@pytest.mark.parametrize("seed,max_width", [(0, 256), (1, 256), (2, 512), (3, 256), (4, 512), (5, 256)])
def test_fuzz_verdicts_match_oracle(evaluator, seed, max_width):
    tb, mb = fuzz_workload(100 + seed, 60, 150, max_width=max_width, depth=4)
    evaluator.upload_models(mb)
    v_gpu, fh_gpu = evaluator.verdicts(tb)
    v_ref = cref.verdicts(tb, mb)
    fh_ref, _ = cref.first_hit(tb, mb)
    sup = supported_exactly(tb, fh_gpu, max_width)
    unsup = ~sup
    mism = np.argwhere(v_gpu[sup] != v_ref[sup])
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    assert (fh_gpu[sup] == fh_ref[sup]).all()
    fh = evaluator.first_hit(tb)
    assert (fh[sup] == fh_ref[sup]).all()
    assert (fh[unsup] == -2).all()


def test_unsupported_tapes_are_exactly_the_named_limits(evaluator):
    """A batch mixing supported fuzz tapes with tapes past each named limit (a 2056-bit value, a
    1024-bit multiplication, a 1024-bit overflow predicate): -2 exactly on the latter, every other
    answer equal to the oracle's."""
    tb0, mb = fuzz_workload(41, 30, 120, max_width=512, depth=4)
    extra = []
    t = Tape()
    extra.append(t.finish(t.eq(t.zext(1800, t.var(0, 256)), t.const(3, 2056))))
    t = Tape()
    a = t.zext(768, t.var(0, 256))
    extra.append(t.finish(t.eq(t.mul(a, a), t.const(9, 1024))))
    t = Tape()
    a = t.zext(768, t.var(1, 256))
    extra.append(t.finish(t.umul_noovfl(a, a)))
    tx = TapeBatch(extra)
    nx = tx.nodes.copy()
    nx["a"][nx["op"] == 1] += np.uint32(tb0.consts.size)    # CONST nodes index the joined pool
    both = TapeBatch.from_arrays(np.concatenate([tb0.nodes, nx]),
                                 np.concatenate([tb0.offsets, tb0.offsets[-1] + tx.offsets[1:]]),
                                 np.concatenate([tb0.consts, tx.consts]))
    n0 = tb0.n_tapes
    order = list(range(5)) + [n0] + list(range(5, 17)) + [n0 + 1] + list(range(17, n0)) + [n0 + 2]
    tb = both.subset(order)
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    sup = supported_exactly(tb, fh)
    assert (~sup).sum() == 3 and not sup[5] and not sup[18] and not sup[-1]
    assert (v[sup] == cref.verdicts(tb.subset(np.flatnonzero(sup)), mb)).all()
    fh1 = evaluator.first_hit(tb)
    assert (fh1[~sup] == -2).all()
    assert (fh1[sup] == cref.first_hit(tb.subset(np.flatnonzero(sup)), mb)[0]).all()


def test_c2_first_hit(evaluator):
    tb, mb, exp = c2_workload(400, 5000, seed=2)
    evaluator.upload_models(mb)
    fh, st = evaluator.first_hit(tb, with_stats=True)
    assert (fh == exp).all()
    ref, _ = cref.first_hit(tb, mb)
    assert (fh == ref).all()
    assert st.n_unsupported == 0 and st.n_hits == int((exp >= 0).sum())


def test_first_hit_is_minimum_with_many_satisfiers(evaluator):
    """Every model from index k on satisfies: first hit must be exactly k even though many
    waves find hits concurrently (atomicMin + early exit)."""
    M = 3000
    rng = np.random.default_rng(7)
    vals = rng.integers(0, 1000, size=M)
    mb = ModelBatch([256], np.vstack([vals.astype(np.uint32)] + [np.zeros(M, np.uint32)] * 7))
    tapes, exps = [], []
    for thr in (0, 1, 5, 500, 998, 999, 1000):
        t = Tape()
        tapes.append(t.finish(t.ult(t.var(0, 256), t.const(thr, 256))))
        idx = np.flatnonzero(vals < thr)
        exps.append(int(idx[0]) if len(idx) else -1)
    tb = TapeBatch(tapes)
    evaluator.upload_models(mb)
    assert list(evaluator.first_hit(tb)) == exps


@pytest.mark.parametrize("M", [1, 63, 64, 65, 255, 257, 1000])
def test_ragged_model_counts(evaluator, M):
    tb, mb = fuzz_workload(77, 20, M, max_width=256, depth=3)
    evaluator.upload_models(mb)
    fh = evaluator.first_hit(tb)
    ref, _ = cref.first_hit(tb, mb)
    sup = fh != -2
    assert (fh[sup] == ref[sup]).all()


def test_index_base_shard(evaluator):
    tb, mb, exp = c2_workload(100, 2000, seed=9)
    shard = mb.shard(1000, 2000)
    evaluator.upload_models(shard)
    fh = evaluator.first_hit(tb)
    want = np.where(exp >= 1000, exp, -1)
    ref, _ = cref.first_hit(tb, shard)
    assert (fh == ref).all()
    assert (fh == want).all()


def test_empty_batch(evaluator):
    evaluator.upload_models(_one_model())
    assert len(evaluator.first_hit(TapeBatch([]))) == 0


def test_uf_and_arrays(evaluator):
    f = [FuncSpec(1, 256, (256,)), FuncSpec(2, 256, (256, 256))]
    models = []
    for m in range(200):
        models.append({"vars": {0: m, 1: 2 * m},
                       "funcs": {0: ({(m,): 1000 + m, (7,): 5}, 77), 1: ({(3, m): m * m}, 1)}})
    mb = ModelBatch.from_python([256, 256], models, f)
    t = Tape()
    x, y = t.var(0, 256), t.var(1, 256)
    c1 = t.eq(t.uf(0, 256, x), t.add(x, t.const(1000, 256)))          # entry hit
    c2 = t.eq(t.select(t.array_var(0, 256), t.const(8, 256)), t.const(77, 256))  # else value
    c3 = t.eq(t.uf(1, 256, t.const(3, 256), x), t.mul(x, x))
    arr = t.store(t.const_array(t.const(0, 256)), y, x)
    c4 = t.eq(t.select(arr, t.add(x, x)), x)
    tapes = [t.finish(t.and_(c1, c2, c3, c4))]
    t2 = Tape()
    x2 = t2.var(0, 256)
    tapes.append(t2.finish(t2.eq(t2.uf(0, 256, t2.const(7, 256)), t2.const(5, 256))))
    t3 = Tape()
    tapes.append(t3.finish(t3.and_(t3.ult(t3.const(150, 256), t3.var(0, 256)),
                                   t3.eq(t3.uf(1, 256, t3.const(4, 256), t3.var(0, 256)), t3.const(1, 256)))))
    tb = TapeBatch(tapes)
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    assert (v == cref.verdicts(tb, mb)).all()
    assert list(fh) == [0, 0, 151]


@pytest.mark.parametrize("host_blocks", [0, None])
def test_keccak_kernel(evaluator, host_blocks):
    """host_blocks 0: every batch on the GPU kernel; None: the default threshold (this small batch
    is hashed on the host path of mq_keccak256)."""
    kats = load("keccak_kats.json")
    msgs = [bytes.fromhex(k["data"]) for k in kats]
    rng = np.random.default_rng(3)
    extra = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in (1, 31, 32, 64, 135, 136, 137, 300)]
    if host_blocks is not None:
        evaluator.set_option(evaluator.OPT_KECCAK_HOST_BLOCKS, host_blocks)
    try:
        out = evaluator.keccak256(msgs + extra)
    finally:
        evaluator.set_option(evaluator.OPT_KECCAK_HOST_BLOCKS, 128)
    for k, d in zip(kats, out):
        assert d.hex() == k["digest"], k["name"]
    for m, d in zip(extra, out[len(msgs):]):
        assert d == keccak_ref.keccak256(m)


# ---------------------------------------------------------------- assembly interpreter (qsa)
def test_asm_interpreter_loaded(evaluator):
    assert evaluator.asm_ready, "gfx950 assembly interpreter failed to load its handler table"


def test_c2_runs_on_asm_path(evaluator):
    tb, mb, exp = c2_workload(200, 3000, seed=4)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    n_asm, n_l8, n_l16 = ct.split()
    assert (n_asm, n_l8, n_l16) == (200, 0, 0)
    assert (evaluator.first_hit(ct) == exp).all()


@pytest.mark.parametrize("seed", range(6))
def test_asm_fuzz_matches_oracle_and_generic(evaluator, seed):
    from mythril_amd.synth import fuzz_workload as fw
    tb, mb = fw(500 + seed, 80, 700, depth=6, asm_only=True)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    # tapes deeper than the assembly interpreter's 6-slot stack run on the HIP C++ kernel
    assert ct.split()[0] >= 0.9 * tb.n_tapes
    v_asm, fh_asm = evaluator.verdicts(tb)
    ref = cref.verdicts(tb, mb)
    mism = np.argwhere(v_asm != ref)
    assert len(mism) == 0, f"{len(mism)} asm mismatches, first {mism[:5]}"
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()
    evaluator.use_asm(False)
    try:
        v_gen, _ = evaluator.verdicts(tb)
        assert (evaluator.first_hit(ct) == fh_ref).all()
    finally:
        evaluator.use_asm(True)
    assert (v_gen == ref).all()


def _leaf_pair_tapes(rng, n_tapes, n_vars=8):
    """256-bit tapes whose binary ops have two leaf operands (var/var, const/var, var/const) under
    ADD/SUB/AND/OR/XOR/MUL, combined and compared: the P translator's leaf-pair fusions."""
    ops = ("add", "sub", "band", "bor", "bxor", "mul")
    tapes = []
    for _ in range(n_tapes):
        t = Tape()

        def leaf(kind):
            if kind == "v":
                return t.var(int(rng.integers(n_vars)), 256)
            return t.const(int.from_bytes(rng.bytes(32), "little") >> int(rng.integers(0, 250)), 256)

        def pair():
            a, b = [("v", "v"), ("c", "v"), ("v", "c")][int(rng.integers(3))]
            return getattr(t, ops[int(rng.integers(len(ops)))])(leaf(a), leaf(b))

        cmps = []
        for _ in range(3):
            x = t.add(pair(), pair()) if rng.random() < 0.5 else t.mul(pair(), pair())
            y = pair()
            cmps.append(t.ult(x, y) if rng.random() < 0.7 else t.not_(t.eq(x, y)))
        tapes.append(t.finish(t.and_(*cmps)))
    return TapeBatch(tapes)


@pytest.mark.parametrize("seed", range(3))
def test_p_leaf_pair_fusions_match_oracle(evaluator, seed):
    """Both-leaf operations run as one P handler (kindVV / MULVV / kindCV, the right variable
    addressed through M0): bit-exact verdicts and first hits against the oracle."""
    rng = np.random.default_rng(100 + seed)
    tb = _leaf_pair_tapes(rng, 300)
    M = 777
    mb = ModelBatch([256] * 8, rng.integers(0, 1 << 32, (64, M), dtype=np.uint64).astype(np.uint32))
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, _ = evaluator.verdicts(tb)
    ref = cref.verdicts(tb, mb)
    assert 0 < ref.sum() < ref.size
    mism = np.argwhere(v != ref)
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()
    assert ct.asm_split()[0] == tb.n_tapes
    hist = ct.handler_histogram(0)
    for kind in ("ADDVV", "SUBVV", "BANDVV", "BORVV", "BXORVV", "MULVV", "ADDCV", "SUBCV", "BANDCV", "BORCV",
                 "BXORCV", "MULCV"):
        # (constant handlers may run as their prefetched-constant PF_ variant)
        assert hist.get(kind, 0) + hist.get("PF_" + kind, 0) > 0, (kind, hist)
    assert sum(v for k, v in hist.items() if k.startswith("PF_")) > 0, hist


def test_p_constant_prefetch_runs_match_oracle(evaluator):
    """Runs of consecutive constant handlers (x + c1) * c2 & c3 - c4 ... on the P interpreter:
    the translator alternates prefetched (PF_) and self-loading handlers; a PF_ handler whose
    successor is not one re-loads its own constant.  Bit-exact against the oracle."""
    rng = np.random.default_rng(31)
    tapes = []
    for i in range(200):
        t = Tape()
        acc = t.var(int(rng.integers(8)), 256)
        for k in range(int(rng.integers(1, 12))):
            c = t.const(int.from_bytes(rng.bytes(32), "little") >> int(rng.integers(0, 255)), 256)
            op = ("add", "mul", "band", "sub", "bor", "bxor")[int(rng.integers(6))]
            acc = getattr(t, op)(acc, c)
            if rng.random() < 0.2:   # a variable operand between runs
                acc = t.add(acc, t.var(int(rng.integers(8)), 256))
        bound = t.const(int.from_bytes(rng.bytes(32), "little"), 256)
        tapes.append(t.finish(t.ult(acc, bound) if i % 2 else t.not_(t.eq(acc, bound))))
    tb = TapeBatch(tapes)
    M = 641
    mb = ModelBatch([256] * 8, rng.integers(0, 1 << 32, (64, M), dtype=np.uint64).astype(np.uint32))
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, _ = evaluator.verdicts(tb)
    assert (v == cref.verdicts(tb, mb)).all()
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()
    hist, pairs = ct.handler_histogram(0, pairs=True)
    assert ct.asm_split()[0] == tb.n_tapes
    pf = sum(n for k, n in hist.items() if k.startswith("PF_"))
    assert pf > 0 and sum(n for (a, b), n in pairs.items() if a.startswith("PF_") and b.startswith("PF_")) == 0


def test_golden_vectors_generic_kernel(evaluator):
    """The same golden fixtures with the assembly path disabled (HIP C++ interpreter only)."""
    entries = load("shift_vectors.json") + load("vmtests_kats.json")
    tapes = []
    for e in entries:
        exp = int(e["expected"], 16)
        tapes.append(check_tape(e, exp))
        tapes.append(check_tape(e, exp, negate=True))
    tb = TapeBatch(tapes)
    evaluator.upload_models(_one_model())
    evaluator.use_asm(False)
    try:
        v, _ = evaluator.verdicts(tb)
    finally:
        evaluator.use_asm(True)
    assert v[0::2, 0].all() and not v[1::2, 0].any()


def test_asm_with_temps_and_bool_sharing(evaluator):
    """Shared BV and Bool subterms go through LDS temps in the assembly interpreter."""
    rng = np.random.default_rng(11)
    M = 500
    words = rng.integers(0, 1 << 32, size=(64, M), dtype=np.uint64).astype(np.uint32)
    mb = ModelBatch([256] * 8, words)
    tapes = []
    for k in range(20):
        t = Tape()
        x, y, z = t.var(k % 8, 256), t.var((k + 3) % 8, 256), t.var((k + 5) % 8, 256)
        s = t.mul(t.add(x, y), z)                   # shared BV subterm
        c = t.ult(s, t.bnot(s))                      # shared Bool subterm
        root = t.and_(t.or_(c, t.eq(s, x)), t.not_(t.and_(c, t.eq(t.band(s, y), t.const(k, 256)))),
                      t.bite(c, t.ule(x, s), t.slt(s, y)))
        tapes.append(t.finish(root))
    tb = TapeBatch(tapes)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.split()[0] == len(tapes)
    v, _ = evaluator.verdicts(tb)
    assert (v == cref.verdicts(tb, mb)).all()


# ---------------------------------------------------------------- EVM-shaped C3 tapes (HIP C++ interpreter)
def test_c3_evm_tapes_match_oracle(evaluator):
    from mythril_amd.synth_evm import c3_workload
    tb, mb, exp, _ = c3_workload(80, 4000, seed=3, planted_frac=0.3)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    fh = evaluator.first_hit(ct)
    ref, _ = cref.first_hit(tb, mb)
    assert (ref == exp).all()
    assert (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    v, fh2 = evaluator.verdicts(tb)
    assert (v == cref.verdicts(tb, mb)).all()
    assert (fh2 == ref).all()


def test_c3_shard_index_base(evaluator):
    from mythril_amd.synth_evm import c3_workload
    tb, mb, exp, _ = c3_workload(40, 3000, seed=5, planted_frac=0.5, shard=(1100, 2900))
    assert mb.index_base == 1100
    evaluator.upload_models(mb)
    fh = evaluator.first_hit(tb)
    ref, _ = cref.first_hit(tb, mb)
    assert (fh == ref).all()
    inside = (exp >= 1100) & (exp < 2900)
    assert (fh[inside] == exp[inside]).all()


def test_many_shared_subterms_use_hbm_temps(evaluator):
    """> 16 live shared sub-terms: temps in per-wave HBM scratch (persistent C++ kernel)."""
    rng = np.random.default_rng(3)
    M = 777
    mb = ModelBatch([256] * 4, rng.integers(0, 1 << 32, (32, M), dtype=np.uint64).astype(np.uint32))
    tapes = []
    for k in range(12):
        t = Tape()
        v = [t.var(i, 256) for i in range(4)]
        shared = [t.mul(v[i % 4], t.add(v[(i + 1) % 4], t.const(i + k, 256))) for i in range(40)]
        # every shared product is used by two comparisons of the root: all 40 live at once
        pairs = [t.ult(shared[i], shared[i + 1]) for i in range(39)]
        root = t.or_(t.and_(*pairs[: 3 + k]), t.xor(pairs[-1], t.and_(*pairs[3 + k:])))
        tapes.append(t.finish(root))
    tb = TapeBatch(tapes)
    from mythril_amd.evaluator import compile_info
    assert max(compile_info(tb, i).n_temps for i in range(tb.n_tapes)) > 16
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    assert (fh != -2).all()
    assert (v == cref.verdicts(tb, mb)).all()
    ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(tb) == ref).all()


# ---------------------------------------------------------------- C4: keccak-heavy, in-kernel keccak-f
def _gpu_hasher(evaluator):
    return evaluator.keccak256_array


@pytest.mark.parametrize("interpret", [False, True])
def test_c4_keccak_tapes_match_oracle(evaluator, interpret):
    from mythril_amd.synth_evm import c4_workload
    tb, mb, exp, syms = c4_workload(40, 1500, seed=4, planted_frac=0.4, hasher_many=evaluator.keccak256_array,
                                    interpret_keccak=interpret)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    if interpret:
        assert ct.split()[2] == tb.n_tapes  # all on the L=16 keccak kernel
    fh = evaluator.first_hit(ct)
    ref, _ = cref.first_hit(tb, mb)
    assert (ref == exp).all()
    assert (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    v, _ = evaluator.verdicts(tb)
    assert (v == cref.verdicts(tb, mb)).all()


def test_keccak_op_all_widths(evaluator):
    """Interpreted keccak of 1..64-byte arguments (the padding byte moves through every lane
    position, including the 64-byte case where it leaves the value registers)."""
    rng = np.random.default_rng(11)
    widths = [8 * k for k in range(1, 65)]
    M = 70
    mb = ModelBatch(widths, np.vstack([rng.integers(0, 1 << 32, ((w + 31) // 32, M), dtype=np.uint64).astype(np.uint32)
                                       for w in widths]))
    tapes = []
    for v, w in enumerate(widths):
        t = Tape()
        k = t.keccak(t.var(v, w))
        # compare against the model-0 digest computed by the oracle, plus a low-byte predicate
        # raw words are NOT masked to the width: the upload must reduce them mod 2^w
        val = sum(int(mb.var_words[int(mb.var_word_offsets()[v]) + i, 0]) << (32 * i) for i in range((w + 31) // 32))
        val &= (1 << w) - 1
        dig = int.from_bytes(keccak_ref.keccak256(val.to_bytes(w // 8, "big")), "big")
        tapes.append(t.finish(t.eq(k, t.const(dig, 256))))
        t2 = Tape()
        k2 = t2.keccak(t2.var(v, w))
        tapes.append(t2.finish(t2.ult(t2.extract(7, 0, k2), t2.const(100, 8))))
    tb = TapeBatch(tapes)
    evaluator.upload_models(mb)
    v_gpu, fh = evaluator.verdicts(tb)
    assert (fh != -2).all()
    assert v_gpu[0::2, 0].all()
    assert (v_gpu == cref.verdicts(tb, mb)).all()


@pytest.mark.parametrize("hoist", [False, True])
def test_c5_deep_tapes_match_oracle(evaluator, hoist):
    """C5 at the stated depth (-t 5, ~4 096 DAG nodes per conjunction): first hits and the full
    verdict matrix against the oracle on the unhoisted lowering."""
    from mythril_amd.synth_evm import c3_workload
    kw = dict(planted_frac=0.5, n_tx=5, checks_per_tx=(18, 24), n_args=5)
    ptb, pmb, exp, _ = c3_workload(16, 3000, seed=5, **kw)
    assert ptb.sizes().mean() > 3900
    tb, mb, exp2, _ = c3_workload(16, 3000, seed=5, hoist=hoist, **kw)
    assert (exp == exp2).all()
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    fh = evaluator.first_hit(ct)
    ref, _ = cref.first_hit(ptb, pmb)
    assert (ref == exp).all() and (fh == ref).all()
    v, _ = evaluator.verdicts(ct)
    assert (v == cref.verdicts(ptb, pmb)).all()


# ---------------------------------------------------------------- batch-level hoisting (column programs)
@pytest.mark.parametrize("col_min_nodes", ["0", None, "8"])
def test_c3_hoisted_columns_match_unhoisted_oracle(evaluator, monkeypatch, col_min_nodes):
    """col_min_nodes "0": every column on the G assembly kernel (mode 3) or the kernels that take
    their shapes (flat Bool columns: fc_kernel; calldata words: the bit-gather kernel); None: the
    default split; "8": columns under 8 nodes on the HIP C++ column kernel, the rest on G, in one
    launch (G then writes its Bool columns' 0/1 rows too, and only the C++ columns' masks are
    packed)."""
    from mythril_amd.synth_evm import c3_workload
    if col_min_nodes is not None:
        monkeypatch.setenv("MQ_G_COL_MIN_NODES", col_min_nodes)
    plain = c3_workload(60, 3000, seed=3, planted_frac=0.3)
    tb, mb, exp, _ = c3_workload(60, 3000, seed=3, planted_frac=0.3, hoist=True)
    assert tb.columns.n > 0
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0 and ct.n_columns == tb.columns.n
    fh = evaluator.first_hit(ct)
    ref, _ = cref.first_hit(plain[0], plain[1])
    assert (ref == exp).all() and (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    n_cols_asm, cols_live = ct.column_asm_split()
    n_flat_cols = ct.flat_split()[1]
    if col_min_nodes == "0":
        assert cols_live and n_cols_asm + n_flat_cols >= 0.5 * tb.columns.n, (n_cols_asm, n_flat_cols, tb.columns.n)
        assert ct.gather_columns() > 0
    if col_min_nodes == "8":
        assert cols_live and 0 < n_cols_asm < tb.columns.n, (n_cols_asm, tb.columns.n)
    vref = cref.verdicts(plain[0], plain[1])
    v, _ = evaluator.verdicts(ct)
    assert (v == vref).all()
    # runs of hoisted Bool columns AND-ed into the conjunction are fused (PKBN_A: one wait for
    # up to four mask loads)
    hist = ct.handler_histogram(1)
    assert hist.get("PKBN_A", 0) > 0, hist
    # pushes of a model variable compared with a constant and AND-ed: one M/SEQK*_A handler
    assert sum(v for k, v in hist.items() if k[1:4] == "EQK" and k[0] in "MS") > 0, hist
    # the same columns on the HIP C++ column kernel
    evaluator.use_asm(False)
    try:
        v2, _ = evaluator.verdicts(ct)
        assert ct.column_asm_split() == (0, False) and (v2 == vref).all()
    finally:
        evaluator.use_asm(True)


def test_hoisting_nested_levels_on_gpu(evaluator, monkeypatch):
    monkeypatch.setenv("MQ_G_COL_MIN_NODES", "0")
    from mythril_amd import smt as S
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    x, y = S.BitVecSym("x", 256), S.BitVecSym("y", 256)
    inner = (x * y + x) * (y + x) + (x ^ y)
    outer = (inner * inner + x) * (inner - y) + (inner & y)
    b8 = S.Extract(7, 0, inner)
    roots = [S.ULT(outer, S.BitVecVal(1 << (250 - i), 256)) for i in range(4)] + \
            [S.ULT(inner, S.BitVecVal(1 << 255, 256)), S.And(b8 == 3, S.ULT(outer, x)), S.ULT(b8, S.BitVecVal(100, 8))]
    rng = np.random.default_rng(5)
    models = [Model({"x": int(rng.integers(1 << 62)) << 190, "y": int(rng.integers(1 << 62))}) for _ in range(500)]
    tb, syms, _ = lower_batch(roots, hoist=True, hoist_min_nodes=3)
    assert tb.columns.n >= 2 and tb.columns.level.max() >= 1
    tb2, syms2, _ = lower_batch(roots)
    evaluator.upload_models(serialize_models(models, syms))
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    ref = cref.verdicts(tb2, serialize_models(models, syms2))
    assert (v == ref).all()
    assert ct.column_asm_split()[1]


def test_c4_hoisted_in_kernel_keccak(evaluator):
    from mythril_amd.synth_evm import c4_workload
    plain = c4_workload(30, 1200, seed=14, planted_frac=0.4, hasher_many=evaluator.keccak256_array)
    tb, mb, exp, _ = c4_workload(30, 1200, seed=14, planted_frac=0.4, hasher_many=evaluator.keccak256_array,
                                 interpret_keccak=True, hoist=True)
    evaluator.upload_models(mb)
    fh = evaluator.first_hit(tb)
    ref, _ = cref.first_hit(plain[0], plain[1])
    assert (ref == exp).all() and (fh == ref).all()


@pytest.mark.parametrize("variant", ["fused", "no_predicates", "no_keccak_columns", "cpp_columns", "no_mask_index"])
def test_c4_keccak_predicates_in_the_keccak_column_kernel(evaluator, monkeypatch, variant):
    """The keccak manager's predicates over keccak columns (lo <= h, h < hi, h urem 64 == 0,
    h == h_c; keccak_function_manager.py:150-179) evaluated by the keccak column kernel from the
    digest in registers, their lane masks stored directly: full verdict matrix and first hits
    against the oracle on the UNhoisted lowering.  Variants: predicates on the interpreters, keccak
    columns on the interpreters (predicate columns then run one level later), and the G column
    path off (the kernel then also writes the 0/1 rows the HIP C++ kernels read); no Bool
    variable with a lane-mask index (MQ_BMASK_CAP=0, as past the 65 535-mask cap): G-only launches
    read the predicate columns' 0/1 rows, which the keccak kernel must then write."""
    from mythril_amd.synth_evm import c4_workload
    if variant == "no_mask_index":
        monkeypatch.setenv("MQ_BMASK_CAP", "0")
    if variant == "no_predicates":
        monkeypatch.setenv("MQ_NO_KECCAK_PREDICATES", "1")
    if variant == "no_keccak_columns":
        monkeypatch.setenv("MQ_NO_KECCAK_COLUMNS", "1")
    plain = c4_workload(40, 1500, seed=24, planted_frac=0.4, hasher_many=evaluator.keccak256_array)
    tb, mb, exp, _ = c4_workload(40, 1500, seed=24, planted_frac=0.4, hasher_many=evaluator.keccak256_array,
                                 interpret_keccak=True, hoist=True)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    if variant == "cpp_columns":
        evaluator.use_asm(False)
    try:
        fh = evaluator.first_hit(ct)
        v, _ = evaluator.verdicts(ct)
    finally:
        evaluator.use_asm(True)
    kp = ct.keccak_predicate_columns()
    if variant in ("fused", "cpp_columns", "no_mask_index"):
        assert kp >= 8 and ct.keccak_columns() >= 4, (kp, ct.keccak_columns())
    else:
        assert kp == 0
    ref, _ = cref.first_hit(plain[0], plain[1])
    assert (ref == exp).all() and (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    assert (v == cref.verdicts(plain[0], plain[1])).all()


def _calldata_roots(n_roots: int, seed: int):
    """Conjunctions over one tx's calldata words (calldata.py:48-55 / 234-247 as lower.py sees
    them): the selector (Extract(255, 224) of word 0), an address word masked to 160 bits, full
    words, a 31-byte tail, and a word whose top is another column (a 248-bit prefix)."""
    from mythril_amd import smt as S
    rng = np.random.default_rng(seed)
    cds = S.BitVecSym("1_calldatasize", 256)
    cd = S.Array("1_calldata", 256, 8)

    def byte(i):
        return S.If(S.BitVecVal(i, 256) < cds, cd[S.BitVecVal(i, 256)], S.BitVecVal(0, 8))

    def word(off, n=32):
        return S.Concat(*[byte(off + j) for j in range(n)])

    sel = S.Extract(255, 224, word(0))
    addr = word(4) & S.BitVecVal((1 << 160) - 1, 256)
    w36, tail = word(36), word(68, 31)
    glued = S.Concat(tail, byte(99))
    roots = []
    for j in range(n_roots):
        c = [int(x) for x in rng.integers(0, 1 << 62, 4)]
        roots.append(S.And(sel == S.BitVecVal(0xA9059CBB if j % 3 else 0x23B872DD, 32),
                           S.ULT(addr, S.BitVecVal(c[0] << 100 | c[1], 256)),
                           S.ULT(w36, S.BitVecVal(c[2] << 190, 256)),
                           S.Not(glued == S.BitVecVal(c[3], 256)),
                           S.ULT(S.BitVecVal(j, 248), tail)))
    return roots


def _calldata_models(n: int, seed: int):
    """Models whose calldatasize crosses every gate: around the word offsets, 2^31 +- 1, >= 2^32,
    negative (signed `<`: every byte reads 0), and bytes only partly present."""
    from mythril_amd.smt_model import Model
    rng = np.random.default_rng(seed)
    sizes = [0, 3, 4, 5, 35, 36, 37, 67, 68, 69, 98, 99, 100, 1000, (1 << 31) - 1, 1 << 31, (1 << 32) + 5,
             1 << 200, 1 << 255, (1 << 256) - 1, (1 << 255) + 77]
    out = []
    for i in range(n):
        cds = sizes[i % len(sizes)] if i % 2 else int(rng.integers(0, 110))
        present = 100 if i % 5 else int(rng.integers(0, 100))
        entries = {k: int(rng.integers(0, 256)) for k in range(present)}
        if i % 3 == 0:
            entries.update({0: 0xA9, 1: 0x05, 2: 0x9C, 3: 0xBB})
        for k in range(4, 16):
            if i % 4 == 0 and k in entries:
                entries[k] = 0   # address words with clean top bytes
        out.append(Model({"1_calldatasize": cds}, {"1_calldata": (entries, 0)}))
    return out


@pytest.mark.parametrize("variant", ["gather", "no_gather"])
def test_calldata_word_columns_on_the_gather_kernel(evaluator, monkeypatch, variant):
    """Hoisted calldata words (selector extract, masked address, full words, a 31-byte tail and
    a word with a column prefix) on the bit-gather column kernel (cw.hip) vs the oracle on the
    UNhoisted lowering: full verdict matrix and first hits, calldatasize across every gate
    (signed compare: a negative size reads no byte).  no_gather: the same columns on the
    interpreters (MQ_NO_GATHER_COLUMNS=1)."""
    from mythril_amd.lower import lower_batch, serialize_models
    if variant == "no_gather":
        monkeypatch.setenv("MQ_NO_GATHER_COLUMNS", "1")
    roots = _calldata_roots(24, 7)
    models = _calldata_models(3000, 8)
    tb, syms, _ = lower_batch(roots, hoist=True, hoist_min_nodes=3)
    tb2, syms2, _ = lower_batch(roots)
    assert tb.columns.n >= 5
    evaluator.upload_models(serialize_models(models, syms))
    ct = evaluator.compile(tb)
    assert ct.n_unsupported == 0
    v, fh = evaluator.verdicts(ct)
    mb2 = serialize_models(models, syms2)
    vref = cref.verdicts(tb2, mb2)
    assert (v == vref).all(), np.argwhere(v != vref)[:10]
    ref, _ = cref.first_hit(tb2, mb2)
    assert (evaluator.first_hit(ct) == ref).all()
    assert vref.any() and not vref.all()
    if variant == "gather":
        assert ct.gather_columns() >= 5, ct.gather_columns()
    else:
        assert ct.gather_columns() == 0
    # the HIP C++ kernels read the gather columns' rows too
    evaluator.use_asm(False)
    try:
        v3, _ = evaluator.verdicts(ct)
    finally:
        evaluator.use_asm(True)
    assert (v3 == vref).all()


# ---------------------------------------------------------------- assembly interpreters: P and G kernels
@pytest.mark.parametrize("seed", range(4))
def test_asm_const_ops_and_lookups_match_oracle(evaluator, seed):
    """Shifts / divisions by constants, extract / concat / sext, masks below 256 bits and array
    lookups, translated to the P (preloaded variables) and G (general) assembly kernels."""
    from mythril_amd.synth import const_op_workload
    tb, mb = const_op_workload(700 + seed, 150, 700)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    n_p, n_g, live = ct.asm_split()
    ref = cref.verdicts(tb, mb)
    mism = np.argwhere(v != ref)
    assert len(mism) == 0, f"{len(mism)} mismatches (P {n_p}, G {n_g}), first {mism[:5]}"
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()
    # wide divisors, variable shifts and signed ops below 256 bits stay on the HIP C++ kernel
    assert live and n_p > 0 and n_g > 0 and n_p + n_g >= 0.4 * tb.n_tapes, (n_p, n_g, live)


def test_c3_tapes_run_on_general_asm_kernel(evaluator):
    """C3's hoisted tapes run without the HIP C++ interpreter (on the assembly interpreters)."""
    from mythril_amd import synth_evm
    tb, mb, exp, _ = synth_evm.c3_workload(60, 3000, seed=9, hoist=True)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    fh = evaluator.first_hit(ct)
    n_p, n_g, live = ct.asm_split()
    n_flat = ct.flat_split()[0]
    assert live and n_p + n_g + n_flat >= 0.8 * tb.n_tapes, (n_p, n_g, n_flat, ct.split())
    assert (fh == exp).all()
    evaluator.use_asm(False)
    try:
        assert (evaluator.first_hit(ct) == exp).all()
    finally:
        evaluator.use_asm(True)


@pytest.mark.parametrize("stage_kb", ["0", "4", "32", "96"])
def test_g_kernel_lds_staged_rows_match_oracle(evaluator, monkeypatch, stage_kb):
    """G kernel with 0 / a few / many model rows staged in LDS per workgroup (MQ_G_STAGE_KB;
    96 KB exceeds the 64 KB default dynamic LDS): identical first hits to the oracle."""
    from mythril_amd.synth_evm import c3_workload
    monkeypatch.setenv("MQ_G_STAGE_KB", stage_kb)
    tb, mb, exp, _ = c3_workload(24, 3000, seed=13, planted_frac=0.5)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    fh = evaluator.first_hit(ct)
    assert ct.asm_split()[1] > 0          # the G kernel ran
    ref, _ = cref.first_hit(tb, mb)
    assert (ref == exp).all() and (fh == ref).all()
    v, _ = evaluator.verdicts(ct)
    assert (v == cref.verdicts(tb, mb)).all()


# ---------------------------------------------------------------- G kernel: packed Bool masks, fused Bool handlers
def _bool_heavy_workload(n_tapes, M, seed):
    """Conjunctions / disjunctions of Bool variables (not preloaded: 24 of them) and compares
    with constants: PUSH_PKB, PUSH_*_A / _O and the NOT-of-compare peephole on the G kernel."""
    from mythril_amd.models import ModelBatch
    from mythril_amd.tape import Tape, TapeBatch
    rng = np.random.default_rng(seed)
    NB, NW = 24, 12
    words = np.concatenate([rng.integers(0, 1 << 32, (8 * NW, M), dtype=np.uint64).astype(np.uint32),
                            (rng.random((NB, M)) < 0.8).astype(np.uint32) * rng.integers(1, 1 << 32, (NB, M), dtype=np.uint64).astype(np.uint32)])
    mb = ModelBatch([256] * NW + [0] * NB, words)
    tapes = []
    for t in range(n_tapes):
        tp = Tape()
        leaves = []
        for i in range(int(rng.integers(3, 12))):
            k = int(rng.integers(0, 6))
            v = int(rng.integers(0, NW))
            if k <= 1:
                leaves.append(tp.var(NW + int(rng.integers(0, NB)), 0))
            elif k == 2:
                leaves.append(tp.not_(tp.var(NW + int(rng.integers(0, NB)), 0)))
            elif k == 3:
                leaves.append(tp.not_(tp.ult(tp.var(v, 256), tp.const(int(rng.integers(0, 1 << 62)) << 190, 256))))
            elif k == 4:
                leaves.append(tp.or_(tp.var(NW + int(rng.integers(0, NB)), 0),
                                     tp.eq(tp.var(v, 256), tp.const(int(words[8 * v, t % M]), 256))))
            else:
                leaves.append(tp.not_(tp.eq(tp.var(v, 256), tp.const(12345, 256))))
        tapes.append(tp.finish(tp.and_(*leaves)))
    return TapeBatch(tapes), mb


@pytest.mark.parametrize("M", [1000, 4096])
def test_g_kernel_bool_masks_and_fused_handlers_match_oracle(evaluator, M):
    tb, mb = _bool_heavy_workload(120, M, seed=M)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    fh = evaluator.first_hit(ct)
    n_p, n_g, live = ct.asm_split()
    assert live and n_g > 0, (n_p, n_g)
    hist = ct.handler_histogram(1)
    assert hist.get("PUSH_PKB", 0) + hist.get("PUSH_PKB_A", 0) + hist.get("PUSH_PKB_O", 0) > 0, hist
    assert any(k.endswith("_A") for k in hist), hist
    ref, _ = cref.first_hit(tb, mb)
    assert (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    v, _ = evaluator.verdicts(ct)
    assert (v == cref.verdicts(tb, mb)).all()


def test_bool_columns_repacked_per_level(evaluator, monkeypatch):
    """Hoisted Bool sub-terms at two nesting levels: level-1 columns and the tapes read the
    level-0 Bool columns as packed lane masks, repacked after each level ran."""
    monkeypatch.setenv("MQ_G_COL_MIN_NODES", "0")
    from mythril_amd import smt as S
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    x, y, z = (S.BitVecSym(n, 256) for n in "xyz")
    c1 = S.ULT(x * y + z, S.BitVecVal(1 << 255, 256))
    c2 = S.And(c1, S.ULT(x, y + z), S.Not(S.ULT(z ^ x, y)))
    roots = [S.And(c2, S.ULT(x + S.BitVecVal(i, 256), y)) for i in range(3)] + \
            [S.Or(c1, S.Not(c2), x == S.BitVecVal(i, 256)) for i in range(3)] + [S.And(c1, S.Not(c2))]
    rng = np.random.default_rng(11)
    models = [Model({n: int.from_bytes(rng.bytes(32), "little") >> int(rng.integers(0, 256)) for n in "xyz"})
              for _ in range(777)]
    tb, syms, _ = lower_batch(roots, hoist=True, hoist_min_nodes=2)
    assert tb.columns.n >= 2 and tb.columns.level.max() >= 1
    tb2, syms2, _ = lower_batch(roots)
    evaluator.upload_models(serialize_models(models, syms))
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    ref = cref.verdicts(tb2, serialize_models(models, syms2))
    assert (v == ref).all()
    fh2 = evaluator.first_hit(ct)
    ref_fh, _ = cref.first_hit(tb2, serialize_models(models, syms2))
    assert (fh2 == ref_fh).all()


# ---------------------------------------------------------------- G kernel: division by a variable
def _var_division_workload(M, seed):
    """x / y and x % y with variable (and wide-constant / zero-constant) divisors at 256 and 64
    bits, against per-model quotients q and remainders r (perturbed in ~30 % of the models),
    plus the SafeMath multiplication check: zero, one, equal, larger and multi-limb divisors."""
    from mythril_amd.models import ModelBatch
    from mythril_amd.tape import Tape, TapeBatch
    rng = np.random.default_rng(seed)

    def draw(bits, n):
        kind = rng.integers(0, 6, n)
        out = []
        for k in kind:
            if k == 0:
                out.append(0)
            elif k == 1:
                out.append(1)
            elif k == 2:
                out.append(int(rng.integers(2, 1 << 16)))
            elif k == 3:
                out.append(int(rng.integers(1, 1 << 62)) << int(rng.integers(0, bits - 62)))
            else:
                out.append(int.from_bytes(rng.bytes(bits // 8), "little"))
        return out

    cols = {}
    for w in (256, 64):
        mask = (1 << w) - 1
        xs, ys = draw(w, M), draw(w, M)
        for m in range(M):
            if rng.random() < 0.15:
                ys[m] = xs[m]
            elif rng.random() < 0.1:
                ys[m] = (xs[m] + int(rng.integers(1, 1000))) & mask
        qs = [mask if y == 0 else x // y for x, y in zip(xs, ys)]
        rs = [x if y == 0 else x % y for x, y in zip(xs, ys)]
        for arr in (qs, rs):
            for m in range(M):
                if rng.random() < 0.3:
                    arr[m] = (arr[m] + 1) & mask
        cols[w] = (xs, ys, qs, rs)
    widths, rows = [], []
    for w in (256, 64):
        for vals in cols[w]:
            widths.append(w)
            nl = w // 32
            rows += [[(v >> (32 * l)) & 0xFFFFFFFF for v in vals] for l in range(nl)]
    mb = ModelBatch(widths, np.asarray(rows, np.uint32))
    big = (1 << 200) + 12345
    tapes = []
    for i, w in enumerate((256, 64)):
        x, y, q, r = (4 * i + k for k in range(4))
        for form in range(6):
            tp = Tape()
            X, Y, Q, R = tp.var(x, w), tp.var(y, w), tp.var(q, w), tp.var(r, w)
            if form == 0:
                root = tp.eq(tp.udiv(X, Y), Q)
            elif form == 1:
                root = tp.eq(tp.urem(X, Y), R)
            elif form == 2:
                root = tp.and_(tp.eq(tp.udiv(X, Y), Q), tp.not_(tp.eq(tp.urem(X, Y), R)))
            elif form == 3:   # SafeMath: x == 0 or (x * y) / x == y
                root = tp.or_(tp.eq(X, tp.const(0, w)), tp.eq(tp.udiv(tp.mul(X, Y), X), Y))
            elif form == 4:   # wide and zero constant divisors
                root = tp.and_(tp.ult(tp.udiv(X, tp.const(big & ((1 << w) - 1), w)), Q),
                               tp.eq(tp.udiv(X, tp.const(0, w)), tp.const((1 << w) - 1, w)))
            else:
                root = tp.ule(tp.urem(tp.add(X, Q), tp.udiv(Y, tp.const(3, w))), R)
            tapes.append(tp.finish(root))
        # divisors forced above 2^k in every lane (the limb-skipping start of G's division):
        # q * d + r == x and r < d hold in every model iff the division is right
        for k in ((200, 255, 40, 33) if w == 256 else (40, 63, 33)):
            tp = Tape()
            X, Y = tp.var(x, w), tp.var(y, w)
            D = tp.bor(Y, tp.const(1 << k, w))
            q_, r_ = tp.udiv(X, D), tp.urem(X, D)
            tapes.append(tp.finish(tp.and_(tp.eq(tp.add(tp.mul(q_, D), r_), X), tp.ult(r_, D))))
    return TapeBatch(tapes), mb


@pytest.mark.parametrize("M", [64, 1000])
def test_g_kernel_variable_division_matches_oracle(evaluator, M):
    tb, mb = _var_division_workload(M, seed=M)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    n_p, n_g, live = ct.asm_split()
    assert live and n_g >= 8, (n_p, n_g, ct.split())
    hist = ct.handler_histogram(1)
    assert hist.get("UDIVV", 0) > 0 and hist.get("UREMV", 0) > 0, hist
    ref = cref.verdicts(tb, mb)
    mism = np.argwhere(v != ref)
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    assert ref.any(axis=1).sum() >= 6 and (~ref).any(axis=1).sum() >= 6
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()


def _signed_division_workload(M, seed):
    """bvsdiv / bvsrem / bvsmod by a variable at 256 bits: the identities a = q * b + r and
    smod = srem (+ b when the signs differ and srem != 0), and compares against a third
    variable, over zero, +-1, MIN, small and full-width operands of both signs."""
    from mythril_amd.models import ModelBatch
    from mythril_amd.tape import Tape, TapeBatch
    rng = np.random.default_rng(seed)
    MIN, MASK = 1 << 255, (1 << 256) - 1

    def draw(n):
        out = []
        for k in rng.integers(0, 7, n):
            if k == 0:
                out.append(0)
            elif k == 1:
                out.append(int(rng.choice([1, MASK, MIN])))
            elif k == 2:
                out.append(int(rng.integers(1, 1 << 20)))
            elif k == 3:
                out.append((-int(rng.integers(1, 1 << 20))) & MASK)
            else:
                out.append(int.from_bytes(rng.bytes(32), "little"))
        return out

    cols = [draw(M), draw(M), draw(M)]
    rows = [[(v >> (32 * l)) & 0xFFFFFFFF for v in vals] for vals in cols for l in range(8)]
    mb = ModelBatch([256, 256, 256], np.asarray(rows, np.uint32))
    tapes = []
    for form in range(7):
        tp = Tape()
        X, Y, Z = tp.var(0, 256), tp.var(1, 256), tp.var(2, 256)
        q, r, md = tp.sdiv(X, Y), tp.srem(X, Y), tp.smod(X, Y)
        zero = tp.const(0, 256)
        if form == 0:
            root = tp.eq(tp.add(tp.mul(q, Y), r), X)
        elif form == 1:
            same = tp.eq(tp.slt(X, zero), tp.slt(Y, zero))
            root = tp.eq(md, tp.ite(tp.or_(tp.eq(r, zero), same), r, tp.add(r, Y)))
        elif form == 2:
            root = tp.slt(q, Z)
        elif form == 3:
            root = tp.slt(r, Z)
        elif form == 4:
            root = tp.sle(md, Z)
        elif form == 5:
            root = tp.eq(tp.sdiv(X, Z), tp.sdiv(Y, Z))
        else:
            root = tp.ult(tp.smod(Z, Y), tp.srem(Z, X))
        tapes.append(tp.finish(root))
    return TapeBatch(tapes), mb


@pytest.mark.parametrize("M", [64, 700])
def test_g_kernel_signed_variable_division_matches_oracle(evaluator, M):
    tb, mb = _signed_division_workload(M, seed=M + 1)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    n_p, n_g, live = ct.asm_split()
    assert live and n_g == tb.n_tapes, (n_p, n_g, ct.split())
    hist = ct.handler_histogram(1)
    assert all(hist.get(k, 0) > 0 for k in ("SDIVV", "SREMV", "SMODV")), hist
    ref = cref.verdicts(tb, mb)
    assert ref[:2].all()                      # the identities hold in every model (oracle)
    mism = np.argwhere(v != ref)
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()



@pytest.mark.parametrize("M", [64, 700])
def test_g_kernel_signed_division_by_wide_and_zero_constants(evaluator, M):
    """bvsdiv / bvsrem / bvsmod by a constant divisor that is 0 or of magnitude >= 2^32:
    G runs them as SDIVV / SREMV / SMODV on the pushed constant (no tape left on the C++ kernel),
    bit-exact with the oracle; the 32-bit constant path (SDIVC*) stays for small divisors."""
    rng = np.random.default_rng(M + 9)
    MASK = (1 << 256) - 1
    xs = [int.from_bytes(rng.bytes(32), "little") if i % 3 else (-int(rng.integers(1, 1 << 40))) & MASK
          for i in range(M)]
    zs = [int.from_bytes(rng.bytes(32), "little") for _ in range(M)]
    rows = [[(v >> (32 * l)) & 0xFFFFFFFF for v in vals] for vals in (xs, zs) for l in range(8)]
    mb = ModelBatch([256, 256], np.asarray(rows, np.uint32))
    consts = [0, 1 << 32, (1 << 32) + 7, (-(1 << 40)) & MASK, (-((1 << 32) + 1)) & MASK, 1 << 255,
              MASK, (1 << 200) + 12345, 3, (-5) & MASK]
    tapes = []
    for c in consts:
        for op in ("sdiv", "srem", "smod"):
            tp = Tape()
            X, Z = tp.var(0, 256), tp.var(1, 256)
            tapes.append(tp.finish(tp.slt(getattr(tp, op)(X, tp.const(c, 256)), Z)))
    tb = TapeBatch(tapes)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    n_p, n_g, live = ct.asm_split()
    assert live and n_p + n_g == tb.n_tapes, (n_p, n_g, ct.split())
    hist = ct.handler_histogram(1)
    assert all(hist.get(k, 0) > 0 for k in ("SDIVV", "SREMV", "SMODV")), hist
    ref = cref.verdicts(tb, mb)
    mism = np.argwhere(v != ref)
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    assert 0.05 < ref.mean() < 0.95

SHIFT_WIDTHS = (256, 160, 64, 8)


def _shift_amounts(rng, w, M):
    """Per-model shift amounts at width w: the edge amounts 0, 1, 31, 32, 33, 63, 64, 255, 256,
    257, W-1, W, W+1, 2^32, 2^32+1, 2^64, 2^255 (reduced mod 2^W), uniform amounts below W + 10
    and amounts with high limbs set."""
    edge = [0, 1, 31, 32, 33, 63, 64, 255, 256, 257, w - 1, w, w + 1, 1 << 32, (1 << 32) + 1, 1 << 64, 1 << 255]
    out = []
    for m in range(M):
        r = rng.random()
        if m < len(edge):
            a = edge[m]
        elif r < 0.5:
            a = int(rng.integers(0, w + 10))
        elif r < 0.8:
            a = edge[int(rng.integers(0, len(edge)))]
        else:
            a = int.from_bytes(rng.bytes(32), "little")
        out.append(a & ((1 << w) - 1))
    return out


def _variable_shift_workload(M, seed):
    """shl / lshr / ashr by a per-model amount at widths 256, 160, 64 and 8 (_shift_amounts):
    the identity (x >> a) << a == x & (ones << a), compares with a third variable (sensitive
    verdicts, checked against the oracle), and EVM SIGNEXTEND's shape at 256 bits
    (instructions.py:645-672: testbit = 8 * s + 7, shl(1, testbit) masks, ite on s <= 31)."""
    from mythril_amd.models import ModelBatch
    from mythril_amd.tape import Tape, TapeBatch
    rng = np.random.default_rng(seed)
    widths, rows = [], []
    for w in SHIFT_WIDTHS:
        xs = [int.from_bytes(rng.bytes(32), "little") & ((1 << w) - 1) for _ in range(M)]
        zs = [int.from_bytes(rng.bytes(32), "little") & ((1 << w) - 1) for _ in range(M)]
        amts = _shift_amounts(rng, w, M)
        for vals in (xs, zs, amts):
            widths.append(w)
            rows += [[(v >> (32 * l)) & 0xFFFFFFFF for v in vals] for l in range((w + 31) // 32)]
    mb = ModelBatch(widths, np.asarray(rows, np.uint32))
    tapes, identities = [], []
    for i, w in enumerate(SHIFT_WIDTHS):
        ones = (1 << w) - 1
        for form in range(6 if w == 256 else 4):
            tp = Tape()
            X, Z, A = tp.var(3 * i, w), tp.var(3 * i + 1, w), tp.var(3 * i + 2, w)
            if form == 0:
                identities.append(len(tapes))
                root = tp.eq(tp.shl(tp.lshr(X, A), A), tp.band(X, tp.shl(tp.const(ones, w), A)))
            elif form == 1:
                root = tp.ult(tp.lshr(X, A), tp.lshr(Z, tp.const(min(3, w - 1), w)))
            elif form == 2:
                root = tp.ult(tp.shl(X, A), Z)
            elif form == 3:
                root = tp.eq(tp.lshr(tp.shl(X, A), A), tp.lshr(tp.shl(Z, A), A))
            elif form == 4:
                root = tp.slt(tp.ashr(X, A), tp.ashr(Z, tp.const(7, w)))
            else:
                # SIGNEXTEND(s = A & 31, x = X) compared with Z's low byte sign-extended
                s = tp.band(A, tp.const(31, w))
                testbit = tp.add(tp.mul(s, tp.const(8, w)), tp.const(7, w))
                bit = tp.shl(tp.const(1, w), testbit)
                setm = tp.sub(bit, tp.const(1, w))
                neg = tp.distinct(tp.band(X, bit), tp.const(0, w))
                se = tp.ite(neg, tp.bor(X, tp.bnot(setm)), tp.band(X, setm))
                root = tp.ule(se, Z)
            tapes.append(tp.finish(root))
    return TapeBatch(tapes), mb, identities


@pytest.mark.parametrize("M", [64, 700])
def test_g_kernel_variable_shifts_match_oracle(evaluator, M):
    """Shifts by a variable amount run on G's SHLV / LSHRV / ASHRV handlers (no tape left on the
    HIP C++ interpreter) and match the oracle bit for bit."""
    tb, mb, identities = _variable_shift_workload(M, seed=M + 2)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    n_p, n_g, live = ct.asm_split()
    assert live and n_p + n_g == tb.n_tapes, (n_p, n_g, ct.split())
    hist = ct.handler_histogram(1)
    for kind in ("SHLV", "LSHRV", "ASHRV"):
        assert hist.get(kind, 0) > 0, (kind, hist)
    ref = cref.verdicts(tb, mb)
    for t in identities:
        assert ref[t].all()          # the identity holds in every model (oracle)
    mism = np.argwhere(v != ref)
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()


@pytest.mark.parametrize("dense", [True, False])
@pytest.mark.parametrize("max_entries", [3, 9, 20])
def test_table_lookups_dense_and_csr_match_oracle(evaluator, monkeypatch, dense, max_entries):
    """UF / array lookups on G through both table layouts: dense slot-major rows (functions with
    at most 16 entries per model, mq_models_upload) and the CSR entry lists (more entries, or
    MQ_NO_DENSE_TABLES=1); keys found at every slot, absent keys (else value), empty tables."""
    import random
    from mythril_amd import smt as S
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    if not dense:
        monkeypatch.setenv("MQ_NO_DENSE_TABLES", "1")
    rng = random.Random(max_entries)
    f = S.Function("inv", [256], 256)
    g = S.Function("bal", [160], 64)
    x, y = S.BitVecSym("x", 256), S.BitVecSym("y", 160)
    exprs = [f(x) == S.BitVecVal(7, 256), S.ULT(f(x), S.BitVecVal(1 << 200, 256)),
             g(y) == S.BitVecVal(5, 64), S.And(f(x) == S.ZeroExt(192, g(y)), S.ULT(x, S.BitVecVal(1 << 255, 256)))]
    models = []
    for m in range(300):
        n = rng.randrange(max_entries + 1)
        keys = [rng.getrandbits(256) for _ in range(n)]
        xv = rng.choice(keys) if keys and rng.random() < 0.7 else rng.getrandbits(256)
        ft = {(k,): rng.choice([7, rng.getrandbits(256), rng.getrandbits(64)]) for k in keys}
        gk = [rng.getrandbits(160) for _ in range(rng.randrange(max_entries + 1))]
        yv = rng.choice(gk) if gk and rng.random() < 0.7 else rng.getrandbits(160)
        gt = {(k,): rng.choice([5, rng.getrandbits(64)]) for k in gk}
        models.append(Model({"x": xv, "y": yv}, {"inv": (ft, rng.choice([0, 7])), "bal": (gt, rng.choice([0, 5]))}))
    tb, syms, ok = lower_batch(exprs)
    assert ok.all()
    mb = serialize_models(models, syms)
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    assert (v == cref.verdicts(tb, mb)).all()
    assert (fh == cref.first_hit(tb, mb)[0]).all()
    assert 0 < v.mean() < 1


@pytest.mark.parametrize("dense", [True, False])
def test_table_lookups_with_shared_first_key_limb(evaluator, monkeypatch, dense):
    """Table keys that agree in their first 32-bit limb and differ above it (small integers
    and their 2^32 offsets): the dense scan's candidate (lowest slot whose limb 0 matches) is then
    often the wrong entry, so the lookup must fall back to its per-slot pass — keys at every slot,
    absent keys, more than 8 slots (two scan rounds), values of 1, 2 and 8 limbs."""
    import random
    from mythril_amd import smt as S
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    if not dense:
        monkeypatch.setenv("MQ_NO_DENSE_TABLES", "1")
    rng = random.Random(11)
    f = S.Function("inv", [256], 256)
    g = S.Function("narrow", [256], 32)
    h = S.Function("mid", [256], 64)
    x = S.BitVecSym("x", 256)
    exprs = [f(x) == S.BitVecVal(7, 256), S.ULT(f(x), S.BitVecVal(1 << 200, 256)), g(x) == S.BitVecVal(5, 32),
             S.ULT(h(x), S.BitVecVal(1 << 40, 64)), S.And(g(x) == S.BitVecVal(9, 32), S.ULT(f(x), S.BitVecVal(100, 256)))]
    models = []
    for m in range(400):
        n = rng.randrange(1, 15)
        low = rng.choice([3, 0xFFFFFFFF, rng.getrandbits(32)])
        keys = list({low | (rng.getrandbits(224) << 32 if rng.random() < 0.8 else rng.randrange(4) << 32) for _ in range(n)})
        rng.shuffle(keys)
        r = rng.random()
        xv = keys[-1] if r < 0.5 else (rng.choice(keys) if r < 0.8 else low | (rng.getrandbits(224) << 32))
        ft = {(k,): rng.choice([7, rng.getrandbits(256), rng.randrange(100)]) for k in keys}
        gt = {(k,): rng.choice([5, 9, rng.getrandbits(32)]) for k in keys}
        ht = {(k,): rng.getrandbits(rng.choice([20, 64])) for k in keys}
        models.append(Model({"x": xv}, {"inv": (ft, rng.choice([0, 7])), "narrow": (gt, rng.choice([0, 5])),
                                        "mid": (ht, rng.getrandbits(64))}))
    tb, syms, ok = lower_batch(exprs)
    assert ok.all()
    mb = serialize_models(models, syms)
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    assert (v == cref.verdicts(tb, mb)).all()
    assert (fh == cref.first_hit(tb, mb)[0]).all()
    assert 0 < v.mean() < 1


# ---------------------------------------------------------------- G kernel: calldata words, signed compares with constants
def _calldata_word_workload(n_tapes, M, seed):
    """Mythril's symbolic calldata words (laser/ethereum/state/calldata.py: a word is the Concat
    of 32 ``If(i < size, cd[i], 0)`` bytes, ``<`` signed) and their neighbours: signed compares
    of a variable with a constant in both operand orders (16-bit, two-word and eight-word
    constants, negative ones), ite with a zero else, concatenations whose low operand is 8, 31,
    40, 72 or 100 bits wide.  Sizes include 0, values around the byte offsets, huge positive
    and negative (bit 255 set) ones."""
    from mythril_amd.models import ModelBatch
    from mythril_amd.tape import Tape, TapeBatch
    rng = np.random.default_rng(seed)
    NB = 48
    widths = [256] + [8] * NB + [256] * 4 + [40, 72, 100, 31]
    rows = []
    size = np.zeros((8, M), dtype=np.uint32)
    kind = rng.integers(0, 10, M)
    size[0] = np.where(kind < 6, rng.integers(0, NB + 8, M), rng.integers(0, 1 << 32, M, dtype=np.uint64)).astype(np.uint32)
    size[7] = np.where(kind == 8, rng.integers(1 << 31, 1 << 32, M, dtype=np.uint64),
                       np.where(kind == 9, rng.integers(0, 1 << 31, M), 0)).astype(np.uint32)
    rows.append(size)
    rows.append(rng.integers(0, 256, (NB, M)).astype(np.uint32))
    w256 = rng.integers(0, 1 << 32, (4 * 8, M), dtype=np.uint64).astype(np.uint32)
    w256[7::8][:, : M // 3] |= np.uint32(1 << 31)          # negative words
    rows.append(w256)
    for w in (40, 72, 100, 31):
        nl = (w + 31) // 32
        r = rng.integers(0, 1 << 32, (nl, M), dtype=np.uint64).astype(np.uint32)
        if w % 32:
            r[nl - 1] &= np.uint32((1 << (w % 32)) - 1)
        rows.append(r)
    mb = ModelBatch(widths, np.concatenate(rows))
    W0, N0 = 1 + NB, 1 + NB + 4

    def kconst():
        c = int(rng.integers(0, 4))
        if c == 0:
            return int(rng.integers(0, 1 << 16))
        if c == 1:
            return int(rng.integers(0, 1 << 62))
        if c == 2:
            return (1 << 256) - int(rng.integers(1, 1 << 40))     # negative
        return int.from_bytes(rng.bytes(32), "little")

    tapes = []
    for t in range(n_tapes):
        tp = Tape()
        preds = []
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.integers(0, 5))
            if k <= 1:   # a calldata word at a random offset
                off = int(rng.integers(0, NB - 31))
                sz = tp.var(0, 256)
                word = tp.concat(*[tp.ite(tp.slt(tp.const(off + i, 256), sz), tp.var(1 + off + i, 8), tp.const(0, 8))
                                   for i in range(32)])
                thr = int.from_bytes(rng.bytes(32), "little")
                preds.append(tp.ult(word, tp.const(thr, 256)) if k == 0 else
                             tp.not_(tp.eq(tp.extract(255, 224, word), tp.const(0, 32))))
            elif k == 2:  # signed compares with a constant, either side
                x = tp.var(int(rng.integers(0, 1)) if rng.random() < 0.3 else W0 + int(rng.integers(0, 4)), 256)
                c = tp.const(kconst(), 256)
                preds.append([tp.slt(x, c), tp.slt(c, x), tp.sgt(x, c), tp.sge(c, x)][int(rng.integers(0, 4))])
            elif k == 3:  # concatenations of wider low operands
                a = tp.var(W0 + int(rng.integers(0, 4)), 256)
                lo = N0 + int(rng.integers(0, 4))
                lw = widths[lo]
                hi = tp.extract(255 - lw, 0, a)
                cat = tp.concat(hi, tp.var(lo, lw))
                preds.append(tp.ult(cat, tp.const(int.from_bytes(rng.bytes(32), "little"), 256)))
            else:         # ite with a zero else
                a, b = tp.var(W0 + int(rng.integers(0, 4)), 256), tp.var(W0 + int(rng.integers(0, 4)), 256)
                c = tp.ult(b, tp.const(int.from_bytes(rng.bytes(32), "little"), 256))
                preds.append(tp.ult(tp.ite(c, a, tp.const(0, 256)), tp.const(int.from_bytes(rng.bytes(32), "little"), 256)))
        tapes.append(tp.finish(tp.and_(*preds)))
    return TapeBatch(tapes), mb


@pytest.mark.parametrize("stage_kb", ["0", "26"])
def test_g_kernel_calldata_words_and_signed_constant_compares(evaluator, monkeypatch, stage_kb):
    """SLTK / SGTK, their staged-variable forms S{SLT,SGT}K{2,8}, ITEZ and SHLOR on the G
    kernel (rows read from global memory with MQ_G_STAGE_KB=0, from LDS otherwise): verdicts and
    first hits identical to the oracle's."""
    monkeypatch.setenv("MQ_G_STAGE_KB", stage_kb)
    tb, mb = _calldata_word_workload(160, 3000, seed=int(stage_kb) + 5)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, _ = evaluator.verdicts(ct)
    n_p, n_g, live = ct.asm_split()
    assert live and n_g >= 0.9 * tb.n_tapes, (n_p, n_g, ct.split())
    hist = ct.handler_histogram(1)
    base = {k.split("_")[0] for k in hist}
    assert "SHLOR" in base and {"ITEZ", "ITEZS"} & base, hist
    if stage_kb != "0":
        assert "ITEZS" in base, hist
    assert {"SLTK", "SGTK"} & base, hist
    if stage_kb != "0":
        assert {"SSLTK2", "SSGTK2", "SSLTK8", "SSGTK8"} & base, hist
    ref = cref.verdicts(tb, mb)
    mism = np.argwhere(v != ref)
    assert len(mism) == 0, f"{len(mism)} mismatches, first {mism[:5]}"
    assert 0.02 < v.mean() < 0.98
    fh_ref, _ = cref.first_hit(tb, mb)
    assert (evaluator.first_hit(ct) == fh_ref).all()


# ---------------------------------------------------------------- flat conjunctions (fc.hip)
@pytest.mark.parametrize("bmask_cap", [None, "0", "3"])
def test_flat_conjunctions_match_oracle(evaluator, monkeypatch, bmask_cap):
    """ANDs of Bool variables and variable-constant compares (every predicate, constant on either
    side, NOT, widths ending inside a limb) on the flat-conjunction kernel: first hits and the
    verdict matrix against the oracle, and against the same batch on the interpreters
    (MQ_NO_FLAT=1).  bmask_cap "0" / "3": none / some of the Bool variables have a packed lane
    mask, the others are read from their 0/1 rows."""
    from mythril_amd.synth import flat_workload
    if bmask_cap is not None:
        monkeypatch.setenv("MQ_BMASK_CAP", bmask_cap)
    tb, mb = flat_workload(31, 300, 1000)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    fh = evaluator.first_hit(ct)
    n_flat, _ = ct.flat_split()
    # (Bool variables read from rows take LDS staging slots: past the kernel's budget the tapes
    # reading them stay on the interpreter -- parity either way)
    assert n_flat >= (0.9 if bmask_cap is None else 0.3) * tb.n_tapes, n_flat
    ref, _ = cref.first_hit(tb, mb)
    assert (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    assert (ref >= 0).mean() > 0.4
    v, fh2 = evaluator.verdicts(ct)
    vref = cref.verdicts(tb, mb)
    assert (v == vref).all() and (fh2 == ref).all()
    monkeypatch.setenv("MQ_NO_FLAT", "1")
    ct2 = evaluator.compile(tb)
    assert (evaluator.first_hit(ct2) == ref).all() and ct2.flat_split()[0] == 0
    ct.free()
    ct2.free()


@pytest.mark.parametrize("variant", ["two_phase_segments", "one_phase"])
def test_flat_kernel_forms_match_oracle(evaluator, monkeypatch, variant):
    """The two-phase flat kernel (fca_kernel: distinct compares into LDS masks, then one lane per
    tape) over more distinct compares than one launch's atom budget (several launches), and the
    one-phase fc_kernel (MQ_FC_ONEPHASE=1): first hits and verdicts against the oracle."""
    from mythril_amd.synth import flat_workload
    if variant == "one_phase":
        monkeypatch.setenv("MQ_FC_ONEPHASE", "1")
    tb, mb = flat_workload(31, 900, 700, max_items=14, or_frac=0.3)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    fh = evaluator.first_hit(ct)
    assert ct.flat_split()[0] >= 0.9 * tb.n_tapes, ct.flat_split()
    ref, _ = cref.first_hit(tb, mb)
    assert (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    v, _ = evaluator.verdicts(ct)
    assert (v == cref.verdicts(tb, mb)).all()


def test_flat_disjunctions_match_oracle(evaluator, monkeypatch):
    """ORs of atoms, NOT of an AND, and OR(NOT(AND), atoms...) run on the flat kernel as negated
    conjunctions (De Morgan); an OR over a multi-atom AND is not flat and stays on the
    interpreters.  First hits and verdicts against the oracle and against MQ_NO_FLAT=1."""
    from mythril_amd.synth import flat_workload
    tb, mb = flat_workload(31, 300, 1000, or_frac=0.6)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    fh = evaluator.first_hit(ct)
    assert ct.flat_split()[0] >= 0.9 * tb.n_tapes, ct.flat_split()
    ref, _ = cref.first_hit(tb, mb)
    assert (fh == ref).all(), np.flatnonzero(fh != ref)[:10]
    v, _ = evaluator.verdicts(ct)
    vref = cref.verdicts(tb, mb)
    assert (v == vref).all() and 0.05 < vref.mean() < 0.95
    monkeypatch.setenv("MQ_NO_FLAT", "1")
    ct2 = evaluator.compile(tb)
    assert (evaluator.first_hit(ct2) == ref).all() and ct2.flat_split()[0] == 0


def test_flat_conjunctions_ragged_and_sharded(evaluator):
    """Model counts that end inside a tile, and a shard with a nonzero index base."""
    from mythril_amd.synth import flat_workload
    for M in (1, 63, 65, 200):
        tb, mb = flat_workload(32 + M, 80, M)
        evaluator.upload_models(mb)
        fh = evaluator.first_hit(tb)
        assert (fh == cref.first_hit(tb, mb)[0]).all(), M
    tb, mb = flat_workload(40, 120, 700)
    sh = mb.shard(300, 700)
    evaluator.upload_models(sh)
    assert (evaluator.first_hit(tb) == cref.first_hit(tb, sh)[0]).all()


def test_c4_tapes_on_the_flat_kernel(evaluator, monkeypatch):
    """C4's hoisted tapes (ANDs of keccak-predicate / calldata Bool columns and word compares) run
    on the flat-conjunction kernel; first hits and verdicts equal the unhoisted oracle's, with the
    flat path on and off."""
    from mythril_amd.synth_evm import c4_workload
    plain = c4_workload(40, 1500, seed=24, planted_frac=0.4, hasher_many=evaluator.keccak256_array)
    tb, mb, exp, _ = c4_workload(40, 1500, seed=24, planted_frac=0.4, hasher_many=evaluator.keccak256_array,
                                 interpret_keccak=True, hoist=True)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    fh = evaluator.first_hit(ct)
    # tapes, and the flat Bool columns of every level (ORs of compares among them)
    assert ct.flat_split()[0] >= 0.9 * tb.n_tapes, ct.flat_split()
    assert ct.flat_split()[1] >= 6, ct.flat_split()
    ref, _ = cref.first_hit(plain[0], plain[1])
    assert (ref == exp).all() and (fh == ref).all()
    v, _ = evaluator.verdicts(ct)
    assert (v == cref.verdicts(plain[0], plain[1])).all()
    monkeypatch.setenv("MQ_NO_FLAT", "1")
    ct2 = evaluator.compile(tb)
    assert (evaluator.first_hit(ct2) == ref).all() and ct2.flat_split() == (0, 0)


@pytest.mark.parametrize("n_tapes,n_models", [(48, 3000), (90, 100_000)])
def test_verdict_matrix_readback_small_and_large(evaluator, n_tapes, n_models):
    """Verdict matrices read back through the pinned staging buffer (up to 8 MB of verdict
    bytes) and straight into host memory (past it: 90 x 10^5 = 9 MB), bit-exact against the
    oracle, with first hits consistent with each row."""
    tb, mb, expected = c2_workload(n_tapes, n_models, seed=11)
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    ref = cref.verdicts(tb, mb)
    assert v.shape == ref.shape and (v == ref).all()
    first = np.where(v.any(axis=1), v.argmax(axis=1), -1)
    assert (fh == first).all()
    assert all(fh[t] == p for t, p in enumerate(expected) if p >= 0)


@pytest.mark.parametrize("hoist", [False, True])
def test_state_merge_array_ite_matches_oracle(evaluator, hoist):
    """The state-merge plugin's array-valued If (merge_states.py:27-29,95-107), lowered by
    pushing selects through the merged arrays (lower.py _select_merged): GPU verdicts and first
    hits against the oracle on the unhoisted lowering, and against the direct term evaluator."""
    import term_eval
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.synth_evm import merge_workload
    exprs, recs = merge_workload(64, 300, seed=9)
    tb, syms, ok = lower_batch(exprs, hoist=hoist)
    assert ok.all()
    mb = serialize_models(recs, syms)
    tb0, syms0, _ = lower_batch(exprs)
    mb0 = serialize_models(recs, syms0)
    evaluator.upload_models(mb)
    v, fh = evaluator.verdicts(tb)
    assert (fh != -2).all()
    v_ref = cref.verdicts(tb0, mb0)
    assert (v == v_ref).all()
    assert (fh == cref.first_hit(tb0, mb0)[0]).all()
    direct = np.array([[term_eval.is_true(e, m) for m in recs[:40]] for e in exprs])
    assert (v[:, :40] == direct).all()
    assert v.any() and (~v).any()


def test_p_section_lengths_every_residue_with_packed_g_columns(evaluator):
    """The r05ak fault class (packed column programs): G's program windows are the
    buffer's aligned 64-word blocks and the G section follows the P section, so a P section of any
    length mod 64 must leave G's programs (and the packed column programs, which start mid-block)
    decoding their own words.  One mixed batch per P-section length — EVM-shaped paths (G tapes,
    hoisted columns on G / the gather / flat kernels) plus P tapes whose handler count steps by
    one — over every residue mod 64, verdicts against the oracle on the unhoisted lowering."""
    from mythril_amd import smt as S
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    from mythril_amd.synth_evm import dropin_workload
    paths, recs, _ = dropin_workload(12, 200, seed=17, planted_frac=0.5)
    p = [S.BitVecSym(f"p{i}", 256) for i in range(3)]
    rng = np.random.default_rng(3)
    recs = [Model({**r.assignment, **{f"p{i}": int(rng.integers(0, 1 << 20)) for i in range(3)}}, r.functions)
            for r in recs]
    residues = set()
    for k in range(64):
        acc = p[0] * p[1]
        for j in range(k):
            acc = acc + S.BitVecVal(int(rng.integers(1, 1 << 30)), 256)
        # (two P tapes that share no sub-term: nothing of them is hoisted into a column)
        ptapes = [S.ULT(acc, p[2] * S.BitVecVal(1 << 20, 256)), S.ULT(p[1] + p[2], p[0] * S.BitVecVal(3, 256))]
        roots = ptapes + paths
        # (p0..p2 first in the symbol table: P preloads variables 0-7)
        from mythril_amd.lower import SymbolTable
        syms = SymbolTable()
        for i in range(3):
            syms.var(f"p{i}", 256)
        tb, syms, ok = lower_batch(roots, syms=syms, hoist=True)
        assert ok.all() and tb.columns is not None and tb.columns.n > 0
        mb = serialize_models(recs, syms)
        tb0, syms0, _ = lower_batch(roots)
        mb0 = serialize_models(recs, syms0)
        evaluator.upload_models(mb)
        ct = evaluator.compile(tb)
        v, fh = evaluator.verdicts(ct)
        n_p, n_g, live = ct.asm_split()
        assert live and n_p >= 1 and n_g > 0, (n_p, n_g, live)
        assert ct.column_asm_split()[0] > 0
        residues.add(int(sum(ct.handler_histogram(0).values())) % 64)
        vref = cref.verdicts(tb0, mb0)
        assert (v == vref).all(), (k, np.argwhere(v != vref)[:5])
        assert (fh == cref.first_hit(tb0, mb0)[0]).all()
        ct.free()
    assert len(residues) == 64, sorted(set(range(64)) - residues)


def _unary_atom_workload(seed, n_tapes=160, M=700):
    """Tapes that are ANDs / ORs of compares of a constant with a UNARY function of one variable
    (zero / sign extension, extract, shifts by constants — 0, mid, >= the width — and division /
    remainder by small constants, signed ones negative too; chains of two or three steps), the
    constants drawn from the functions' values under the models so the verdicts split."""
    import term_eval
    from mythril_amd import smt as S
    from mythril_amd.lower import lower_batch, serialize_models
    from mythril_amd.smt_model import Model
    rng = np.random.default_rng(seed)
    widths = (8, 64, 160, 256)
    xs = {w: [S.BitVecSym(f"u{w}_{i}", w) for i in range(2)] for w in widths}
    bools = [S.BoolSym(f"ub{i}") for i in range(2)]

    def val(w):
        k = int(rng.integers(6))
        if k == 0:
            return int(rng.integers(0, 4))
        if k == 1:
            return (1 << w) - 1 - int(rng.integers(0, 3))
        if k == 2:
            return (1 << (w - 1)) + int(rng.integers(-2, 3)) % (1 << w)
        return int.from_bytes(rng.bytes(32), "little") & ((1 << w) - 1)

    models = []
    for _ in range(M):
        asg = {f"u{w}_{i}": val(w) for w in widths for i in range(2) if rng.random() < 0.95}
        asg.update({f"ub{i}": bool(rng.integers(2)) for i in range(2)})
        models.append(Model(asg))

    def step(t):
        w = t.width
        k = int(rng.integers(11))
        if k == 0:
            return S.SignExt(int(rng.integers(1, 257 - w)), t) if w < 256 else t
        if k == 1 and w > 1:
            lo = int(rng.integers(0, w))
            hi = int(rng.integers(lo, w))
            return S.Extract(hi, lo, t)
        if k in (2, 3, 4):
            sh = int(rng.choice([0, 1, 7, 31, 32, 33, w - 1, w, w + 5, 1 << 40])) % (1 << w) if w < 64 else \
                int(rng.choice([0, 1, 7, 31, 32, 33, w - 1, w, w + 5, 1 << 40]))
            c = S.BitVecVal(sh, w)
            return [S.LShR(t, c), t << c, t >> c][k - 2]
        if k in (5, 6, 7, 8, 9):
            d = int(rng.choice([1, 2, 3, 7, 10, 255, 256, 1000, (1 << 21) - 1, (1 << 20) + 3]))
            d = d % (1 << w) or 1
            if k >= 7 and w < 256:
                k -= 2   # (signed division below 256 bits has no assembly handler: the tape
                #         would run on the HIP C++ kernel, which the flat path does not take from)
            if k >= 7 and rng.random() < 0.5:
                d = (-d) % (1 << w)   # a negative signed divisor
            c = S.BitVecVal(d, w)
            return [S.URem(t, c), S.UDiv(t, c), S.SMod(t, c), S.SRem(t, c), t / c][k - 5]
        return S.ZeroExt(int(rng.integers(1, 257 - w)), t) if w < 256 else t

    def atom():
        w = widths[int(rng.integers(4))]
        t = xs[w][int(rng.integers(2))]
        for _ in range(int(rng.integers(1, 4))):
            t = step(t)
        w = t.width
        base = term_eval.evaluate(t, models[int(rng.integers(M))])
        c = S.BitVecVal((base + int(rng.choice([0, 0, 1, -1]))) % (1 << w), w)
        k = int(rng.integers(6))
        e = [t == c, S.ULT(t, c), S.Not(S.ULT(c, t)), t < c, t <= c, S.UGT(t, c)][k]
        return S.Not(e) if rng.random() < 0.2 else e

    exprs = []
    for _ in range(n_tapes):
        parts = [atom() for _ in range(int(rng.integers(1, 5)))]
        if rng.random() < 0.3:
            parts.append(bools[int(rng.integers(2))])
        e = S.And(*parts) if rng.random() < 0.75 else S.Or(*parts)
        exprs.append(e)
    tb, syms, ok = lower_batch(exprs)
    assert ok.all()
    return exprs, models, tb, serialize_models(models, syms)


@pytest.mark.parametrize("seed", range(4))
def test_flat_unary_atoms_match_oracle(evaluator, monkeypatch, seed):
    """fca_kernel's unary atoms (fc.hip fx_apply; mq_api.cpp fc_match with unary steps; opt-in
    MQ_FC_UNARY=1): the workload's tapes run on the flat kernel, and their verdicts and first
    hits are the oracle's (and the direct term evaluator's)."""
    import term_eval
    monkeypatch.setenv("MQ_FC_UNARY", "1")   # (opt-in: read per compile)
    exprs, models, tb, mb = _unary_atom_workload(seed)
    evaluator.upload_models(mb)
    ct = evaluator.compile(tb)
    v, fh = evaluator.verdicts(ct)
    n_flat = ct.flat_split()[0]
    vref = cref.verdicts(tb, mb)
    bad = np.argwhere(v != vref)
    assert len(bad) == 0, (len(bad), bad[:5], [repr(exprs[i]) for i in sorted(set(bad[:3, 0]))])
    assert (fh == cref.first_hit(tb, mb)[0]).all()
    fh1 = evaluator.first_hit(ct)
    assert (fh1 == cref.first_hit(tb, mb)[0]).all()
    # (nearly) every tape the assembly path takes is flat — not one whose sub-term is used twice
    # (a temp); the others (signed division below 256 bits and the like) run on the HIP C++ kernel,
    # which the flat path does not take from
    n_asm = ct.split()[0]
    assert n_flat >= 0.9 * n_asm and n_flat >= 0.4 * tb.n_tapes, (n_flat, ct.split(), ct.asm_split())
    assert v.any() and (~v).any()
    direct = np.array([[term_eval.is_true(e, m) for m in models[:50]] for e in exprs])
    assert (v[:, :50] == direct).all()
    ct.free()
