"""The EVM-shaped workload generators (C3/C4/C5 substitutes) on CPU: planted first
hits are what the oracle finds, shards reproduce the global candidate set, and the C4 tapes give
identical verdicts with keccak as a UF table lookup (z3 semantics) and as in-kernel keccak-f."""
import numpy as np
import pytest

import cref
from mythril_amd.synth_evm import c3_workload, c4_workload


def hasher_many(arr):
    return np.array([np.frombuffer(cref.keccak256(bytes(r)), np.uint8) for r in np.asarray(arr, np.uint8)],
                    np.uint8).reshape(-1, 32)


def test_c3_planted_first_hits():
    tb, mb, exp, _ = c3_workload(60, 2500, seed=3, planted_frac=0.3)
    fh, _ = cref.first_hit(tb, mb)
    assert (fh == exp).all() and (exp >= 0).sum() >= 10


def test_c3_shards_are_slices_of_the_global_set():
    full = c3_workload(20, 1500, seed=9, planted_frac=0.5)
    part = c3_workload(20, 1500, seed=9, planted_frac=0.5, shard=(700, 1300))
    assert (full[0].nodes == part[0].nodes).all() and (full[2] == part[2]).all()
    assert (full[1].var_words[:, 700:1300] == part[1].var_words).all() and part[1].index_base == 700
    v_full, v_part = cref.verdicts(full[0], full[1]), cref.verdicts(part[0], part[1])
    assert (v_full[:, 700:1300] == v_part).all()


def test_c5_deep_tapes_planted():
    """C5's shape (bench.py): -t 5, five ABI words per call, ~4 096 DAG nodes per conjunction."""
    tb, mb, exp, _ = c3_workload(12, 800, seed=5, planted_frac=0.5, n_tx=5, checks_per_tx=(18, 24), n_args=5)
    assert 3900 < tb.sizes().mean() < 4300
    fh, _ = cref.first_hit(tb, mb)
    assert (fh == exp).all()


@pytest.mark.parametrize("seed", [4, 14])
def test_c4_uf_lookup_equals_in_kernel_keccak(seed):
    a = c4_workload(30, 1200, seed=seed, planted_frac=0.4, hasher_many=hasher_many)
    b = c4_workload(30, 1200, seed=seed, planted_frac=0.4, hasher_many=hasher_many, interpret_keccak=True)
    assert "keccak256_512" in a[3].func_names and "keccak256_512" not in b[3].func_names
    va, vb = cref.verdicts(a[0], a[1]), cref.verdicts(b[0], b[1])
    assert (va == vb).all()
    fh, _ = cref.first_hit(b[0], b[1])
    assert (fh == b[2]).all() and (b[2] >= 0).any()
