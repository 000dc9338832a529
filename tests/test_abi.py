"""CPU tests of the C-ABI boundary: libmq.so loads, exports every symbol include/mq.h declares,
the Python opcode/struct mirrors match the header, and the host-side tape compiler (no GPU)
produces the expected programs."""
import ctypes
import os
import re

import numpy as np
import pytest

from mythril_amd import evaluator
from mythril_amd._abi import MqFuncDesc, MqModelBatch, MqNode, MqStats, MqTapeBatch
from mythril_amd.synth import c2_workload, fuzz_workload
from mythril_amd.tape import Op, Tape, TapeBatch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = open(os.path.join(ROOT, "include", "mq.h")).read()


def test_library_exports_every_declared_symbol():
    lib = evaluator.load_library()
    declared = re.findall(r"^\s*(?:int|void|double|const char\*)\s+(mq_\w+)\s*\(", HEADER, re.M)
    assert len(declared) >= 14
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.mq_version().startswith(b"mq ")
    assert lib.mq_strerror(-1) == b"invalid argument"


def test_opcodes_match_header():
    hdr = dict((m[0], int(m[1])) for m in re.findall(r"MQ_OP_(\w+)\s*=\s*(\d+)", HEADER))
    assert hdr == {op.name: int(op) for op in Op}


def test_struct_layouts():
    assert ctypes.sizeof(MqNode) == 16
    assert ctypes.sizeof(MqFuncDesc) == 8
    assert ctypes.sizeof(MqTapeBatch) == 40
    assert ctypes.sizeof(MqModelBatch) == 112
    assert ctypes.sizeof(MqStats) == 40


def test_ctx_create_without_gpu_fails_loudly():
    """No CPU fallback: with no gfx950 device the evaluator refuses to exist."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(evaluator.EvaluatorError):
        evaluator.Evaluator(0)


def test_compile_c2_tapes():
    tb, mb, exp = c2_workload(50, 100, seed=2)
    for t in range(tb.n_tapes):
        ci = evaluator.compile_info(tb, t)
        assert ci.supported, ci.why
        assert ci.limbs == 8
        assert 2 <= ci.depth <= 8
        assert ci.n_temps <= 4  # hash-consing shares repeated subterms
        assert evaluator.tape_alg_ops(tb, t) > 0


def test_compile_fuzz_tapes_supported():
    """Every fuzz tape compiles (the fuzz stays inside the named limits of tests/unsupported.py),
    and the 256-bit ones onto 8 limbs."""
    from unsupported import expected_unsupported
    for seed, mw in ((0, 256), (1, 512), (5, 512), (7, 512)):
        tb, mb = fuzz_workload(seed, 60, 4, max_width=mw)
        assert not expected_unsupported(tb).any()
        infos = [evaluator.compile_info(tb, t) for t in range(tb.n_tapes)]
        assert all(i.limbs == 8 for i in infos) if mw == 256 else all(i.limbs in (8, 16) for i in infos)


def test_compile_supports_values_up_to_2048_bits():
    """Keccak inputs longer than 64 bytes (WalletLibrary.sol:134 keccak256(msg.data): 544 bits;
    abi.encode of 3 words: 768; one full block: 1088) compile onto the 1024 / 2048-bit stacks."""
    for w, L in ((544, 32), (768, 32), (1024, 32), (1088, 64), (2048, 64)):
        t = Tape()
        x = t.var(0, w)
        root = t.and_(t.eq(x, t.const(3, w)), t.ult(t.keccak(x), t.const(5, 256)))
        ci = evaluator.compile_info(TapeBatch([t.finish(root)]), 0)
        assert ci.supported and ci.limbs == L, (w, ci)
    t = Tape()   # a > 512-bit UF result (keccak256_<n>-1) extracted back to a selector
    inv = t.uf(1, 1088, t.var(0, 256))
    ci = evaluator.compile_info(TapeBatch([t.finish(t.eq(t.extract(1087, 1056, inv), t.const(7, 32)))]), 0)
    assert ci.supported and ci.limbs == 64


def test_compile_rejects_what_it_cannot_do():
    t = Tape()
    x = t.var(0, 2056)
    tb = TapeBatch([t.finish(t.eq(x, t.const(3, 2056)))])
    ci = evaluator.compile_info(tb, 0)
    assert not ci.supported and "2048" in ci.why
    t = Tape()
    a = t.var(0, 1024)        # multiplication / division stop at 512 bits
    tb = TapeBatch([t.finish(t.eq(t.mul(a, a), t.const(3, 1024)))])
    ci = evaluator.compile_info(tb, 0)
    assert not ci.supported and "512" in ci.why
    t = Tape()
    k = t.keccak(t.var(0, 2056))
    tb = TapeBatch([t.finish(t.eq(k, t.const(3, 256)))])
    assert not evaluator.compile_info(tb, 0).supported


def test_interpreted_keccak_compiles_to_the_l16_kernel():
    t = Tape()
    k = t.keccak(t.var(0, 512))
    tb = TapeBatch([t.finish(t.eq(k, t.const(3, 256)))])
    ci = evaluator.compile_info(tb, 0)
    assert ci.supported and ci.limbs == 16


def test_shared_subterms_use_temps():
    t = Tape()
    a = t.mul(t.var(0, 256), t.var(1, 256))
    root = t.and_(t.ult(a, t.const(5, 256)), t.eq(t.add(a, a), t.const(6, 256)))
    tb = TapeBatch([t.finish(root)])
    ci = evaluator.compile_info(tb, 0)
    assert ci.supported and ci.n_temps == 1


def test_alg_ops_cost_table():
    """add = L, mul = L(L+1), eq = L, bool and = 1 (L = 8 at 256 bits)."""
    t = Tape()
    x, y = t.var(0, 256), t.var(1, 256)
    root = t.and_(t.eq(t.add(x, y), t.mul(x, y)), t.ult(x, y))
    tb = TapeBatch([t.finish(root)])
    assert evaluator.tape_alg_ops(tb, 0) == 8 + 72 + 8 + 8 + 1


@pytest.mark.parametrize("world", [1, 2, 3, 7])
def test_models_shard_matches_python_shard_and_covers_the_batch(world):
    """mq_models_shard (what mq_models_upload gives each device of a multi-device context) equals
    ModelBatch.shard, and the shards' cref first hits MIN-merge to the unsharded first hits
    (the RCCL ncclMin of the library, restated on the host; support_utils.py:62 order)."""
    import cref
    from mythril_amd import dist
    tb, mb = fuzz_workload(31, 25, 50, max_width=512)
    ref, _ = cref.first_hit(tb, mb)
    parts = []
    for r in range(world):
        lo, hi = dist.shard_bounds(mb.n_models, r, world)
        a, b = evaluator.shard_models(mb, lo, hi), mb.shard(lo, hi)
        assert a.index_base == b.index_base == lo and a.n_models == hi - lo
        assert (a.var_words == b.var_words).all()
        for m in range(hi - lo):
            for f in range(len(mb.funcs)):
                assert a.func_table(f, m) == b.func_table(f, m) == mb.func_table(f, lo + m)
        parts.append(dist.encode_local(cref.first_hit(tb, a)[0]))
    assert (dist.decode_global(np.minimum.reduce(parts)) == ref).all()


def test_host_keccak_path_matches_the_kats_and_the_oracle():
    """mq_keccak256's host path (small batches, no GPU) against the keccak KATs and the oracle at
    every length around the 136-byte block boundary."""
    import keccak_ref
    from golden_util import load
    from mythril_amd.evaluator import keccak256_host
    kats = load("keccak_kats.json")
    out = keccak256_host([bytes.fromhex(k["data"]) for k in kats])
    assert [d.hex() for d in out] == [k["digest"] for k in kats]
    msgs = [bytes((i * 13 + n) & 0xFF for i in range(n)) for n in list(range(0, 300)) + [1000, 4096]]
    assert keccak256_host(msgs) == [keccak_ref.keccak256(m) for m in msgs]
    assert keccak256_host([]) == []


def test_keccak_op_count_is_the_first_principles_count():
    """keccak-f[1600] is charged 6 514 ops per 136-byte block (tape_compiler.h: 135 two-input
    64-bit lane ops per round with lane complementing, on 32-bit halves, x 24 rounds + 34 absorb
    XORs): a 64-byte key ++ slot message is one block, a 200-byte one two."""
    for nbytes, blocks in ((64, 1), (135, 1), (136, 2), (200, 2)):
        t = Tape()
        x = t.var(0, 8 * nbytes)
        root = t.eq(t.keccak(x), t.const(1, 256))
        tb = TapeBatch([t.finish(root)])
        assert evaluator.tape_alg_ops(tb, 0) == 6514 * blocks + 8, nbytes
    assert 24 * 2 * (55 + 24 + 55 + 1) + 34 == 6514
