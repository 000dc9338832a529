"""Candidate serialization (mythril_amd/candidates.py) on CPU: the host extension's row builder
(csrc/lowerwalk.cpp candidate_rows), its numpy fallback and a literal per-block loop agree, and
every generated candidate's rows equal its materialized model's serialization."""
import numpy as np
import pytest

from mythril_amd import candidates as C
from mythril_amd.lower import IncrementalLowering
from mythril_amd.synth_evm import fork_workload
from mythril_amd.tape import limbs


def _literal_rows(lru, blocks, syms):
    """The patch semantics written out per block and element (values in order, then floors)."""
    off = lru.var_word_offsets()
    sizes = [len(b) for _, b in blocks]
    base = np.concatenate([b for _, b in blocks])
    gen = lru.var_words[:, np.where(base >= 0, base, 0)].copy()
    pos = 0
    for (patch, _), n_k in zip(blocks, sizes):
        sl = slice(pos, pos + n_k)
        pos += n_k
        for v, lo, n, bits in [p for p in patch if p[1] >= 0] + [p for p in patch if p[1] < 0]:
            r0, nl = int(off[v]), limbs(syms.var_widths[v])
            if lo < 0:
                for k in range(sl.start, sl.stop):
                    if not gen[r0 + 1:r0 + nl, k].any() and gen[r0, k] < bits:
                        gen[r0, k] = bits
                continue
            for k in range(sl.start, sl.stop):
                val = 0
                for i in range(nl):
                    val |= int(gen[r0 + i, k]) << (32 * i)
                val = (val & ~(((1 << n) - 1) << lo)) | (bits << lo)
                for i in range(nl):
                    gen[r0 + i, k] = (val >> (32 * i)) & 0xFFFFFFFF
    return gen


@pytest.mark.parametrize("fill", [False, True])
def test_candidate_rows_native_numpy_and_literal_agree(monkeypatch, fill):
    exprs, recs, _ = fork_workload(24, 40, seed=5)
    inc = IncrementalLowering()
    db, ok = inc.lower(exprs)
    lru = inc.serialize(recs)
    captured = []
    real = C.CandidateGenerator._serialize

    def spy(self, lru_b, blocks, syms, models):
        captured.append((lru_b, blocks, syms))
        return real(self, lru_b, blocks, syms, models)
    monkeypatch.setattr(C.CandidateGenerator, "_serialize", spy)
    cs = C.CandidateGenerator(6000, seed=2, fill=fill).generate(db, inc.syms, lru, recs)
    lru_b, blocks, syms = captured[-1]
    assert cs.n_generated > 1000 and any(p[1] < 0 for b, _ in blocks for p in b)   # floors occur
    native = cs.batch.var_words[:, cs.n_lru:]
    monkeypatch.setenv("MQ_PY_CANDIDATES", "1")
    py = C.CandidateGenerator(6000, seed=2, fill=fill).generate(db, inc.syms, lru, recs).batch.var_words[:, cs.n_lru:]
    assert (native == py).all()
    assert (native == _literal_rows(lru_b, blocks, syms)).all()
    # a candidate's rows are its materialized model's rows
    ks = np.random.default_rng(0).integers(cs.n_lru, cs.batch.n_models, 40)
    mats = [cs.materialize(int(k)) for k in ks]
    ser = inc.serialize(mats)
    assert (ser.var_words == cs.batch.var_words[:, ks]).all()


def test_candidate_function_tables_match_materialized_models():
    """A generated candidate's function tables (its base model's entries plus the entries of the
    derived calldata bytes its patch changed) read like its materialized model's: the oracle's
    verdicts of the workload's tapes agree on both serializations."""
    import cref
    exprs, recs, _ = fork_workload(24, 40, seed=6)
    inc = IncrementalLowering()
    db, ok = inc.lower(exprs)
    cs = C.CandidateGenerator(6000, seed=4, fill=True).generate(db, inc.syms, inc.serialize(recs), recs)
    assert cs.batch.funcs
    tb = db.to_tapes()
    fh, _ = cref.first_hit(tb, cs.batch)
    hits = [int(h) for h in fh if h >= cs.n_lru]
    assert hits
    ks = np.asarray(hits[:30] + list(np.random.default_rng(1).integers(cs.n_lru, cs.batch.n_models, 30)), np.int64)
    mats = [cs.materialize(int(k)) for k in ks]
    ser = inc.serialize(mats)
    v_mat = cref.verdicts(tb, ser)
    for i, k in enumerate(ks):
        one = cs.batch.shard(int(k), int(k) + 1)
        assert (cref.verdicts(tb, one)[:, 0] == v_mat[:, i]).all(), int(k)
    assert v_mat.any()
