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
