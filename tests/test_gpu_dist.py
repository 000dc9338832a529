"""The product multi-GPU path (mythril_amd.dist.ShardedEvaluator) with world size 2 and 3 on the
one GPU of the box: each rank holds its contiguous model shard in HBM, launches into a device
int32[N], MIN-all-reduces it in place on its stream (gloo here; RCCL on a multi-GPU node) and
finalizes.  The combined first hits must equal the oracle's on the unsharded batch
(support_utils.py:62-66: global MRU-first order survives the merge), including empty shards."""
import multiprocessing as mp
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, seed, n_tapes, n_models, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from mythril_amd.dist import ShardedEvaluator
    from mythril_amd.evaluator import Evaluator
    from mythril_amd.synth import c2_workload
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tb, mb, _ = c2_workload(n_tapes, n_models, seed=seed)
        sev = ShardedEvaluator(Evaluator(0), rank, world)
        sev.upload_models(mb)
        got = sev.first_hit(tb)
        q.put((rank, got.tolist()))
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_tapes,n_models", [(2, 200, 3001), (3, 60, 2)])
def test_sharded_evaluator_matches_unsharded_oracle(world, n_tapes, n_models):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cref
    from mythril_amd.synth import c2_workload
    tb, mb, _ = c2_workload(n_tapes, n_models, seed=9)
    ref, _ = cref.first_hit(tb, mb)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 9, n_tapes, n_models, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, v = q.get(timeout=100)
            res[r] = v
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert isinstance(res[r], list), res[r]
        assert res[r] == ref.tolist(), f"rank {r} differs from the unsharded oracle"
