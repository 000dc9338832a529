"""Multi-GPU from ONE process through the C-ABI: mq_ctx_create(n_dev, dev_ids)
shards the candidate axis inside mq_models_upload and MIN-reduces per-tape first hits with an
in-library RCCL all-reduce.  On a one-GPU box the RCCL path runs with a single rank and the
two-device case is skipped; empty model shards (fewer candidates than devices) are exercised
directly."""
import numpy as np
import pytest

import cref
from unsupported import supported_exactly
from mythril_amd import dist
from mythril_amd.evaluator import Evaluator
from mythril_amd.models import ModelBatch
from mythril_amd.synth import c2_workload, fuzz_workload

pytestmark = pytest.mark.gpu


def _n_devices() -> int:
    import torch
    return torch.cuda.device_count()


def test_rccl_path_single_rank():
    ev = Evaluator(0, use_rccl=True)
    try:
        assert ev.rccl_active
        tb, mb, exp = c2_workload(200, 3000, seed=2)
        ev.upload_models(mb)
        fh = ev.first_hit(tb)
        ref, _ = cref.first_hit(tb, mb)
        assert (fh == ref).all() and (fh == exp).all()
        tb2, mb2 = fuzz_workload(7, 30, 130, max_width=512)
        ev.upload_models(mb2)
        v, fh2 = ev.verdicts(tb2)
        sup = supported_exactly(tb2, fh2)
        assert (v[sup] == cref.verdicts(tb2, mb2)[sup]).all()
        assert (ev.first_hit(tb2)[sup] == cref.first_hit(tb2, mb2)[0][sup]).all()
    finally:
        ev.close()


@pytest.mark.skipif("_n_devices() < 2")
@pytest.mark.parametrize("n_models", [1, 777, 5000])
def test_two_devices_one_context(n_models):
    """Global MRU-first order survives the shard + MIN merge (support_utils.py:62): identical
    first hits and verdict matrices to the unsharded oracle, ragged and empty shards included."""
    ev = Evaluator(devices=[0, 1])
    try:
        assert ev.rccl_active
        tb, mb = fuzz_workload(8, 40, n_models, max_width=512)
        ev.upload_models(mb)
        ref, _ = cref.first_hit(tb, mb)
        fh = ev.first_hit(tb)
        sup = supported_exactly(tb, fh)
        assert (fh[sup] == ref[sup]).all()
        v, fhv = ev.verdicts(tb)
        assert (v[sup] == cref.verdicts(tb, mb)[sup]).all() and (fhv[sup] == ref[sup]).all()
    finally:
        ev.close()


@pytest.mark.parametrize("world", [3, 5])
def test_empty_shards_report_no_hit(evaluator, world):
    """with fewer candidates than ranks some shards are empty; their launch must
    succeed and report "no hit" so the MIN all-reduce of every rank completes."""
    tb, mb = fuzz_workload(9, 30, 2, max_width=256)
    ref, _ = cref.first_hit(tb, mb)
    parts = []
    for r in range(world):
        lo, hi = dist.shard_bounds(mb.n_models, r, world)
        evaluator.upload_models(mb.shard(lo, hi))
        parts.append(dist.encode_local(evaluator.first_hit(tb)))
    merged = dist.decode_global(np.minimum.reduce(parts))
    sup = supported_exactly(tb, merged, 256)
    assert (merged[sup] == ref[sup]).all()


def test_zero_model_upload(evaluator):
    tb, _ = fuzz_workload(10, 12, 4, max_width=256)
    evaluator.upload_models(ModelBatch([256], np.zeros((8, 0), np.uint32)))
    fh = evaluator.first_hit(tb)
    assert set(fh.tolist()) <= {-1, -2}
    v, fhv = evaluator.verdicts(tb)
    assert v.shape == (tb.n_tapes, 0)
