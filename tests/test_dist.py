"""Multi-rank model-axis sharding on CPU (gloo, world sizes 2 and 3): each rank evaluates its
contiguous candidate shard (oracle here; the HIP evaluator on the GPU box), one MIN all-reduce
combines them, and the result equals the unsharded first hit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mythril_amd.dist import INT32_MAX, decode_global, encode_local, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_ragged():
    for M in (0, 1, 2, 7, 100, 1001):
        for W in (1, 2, 3, 8):
            rs = [shard_bounds(M, r, W) for r in range(W)]
            assert rs[0][0] == 0 and rs[-1][1] == M
            assert all(rs[i][1] == rs[i + 1][0] for i in range(W - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_encoding_roundtrip():
    fh = np.array([-1, -2, 0, 5, INT32_MAX - 1], np.int32)
    enc = encode_local(fh)
    assert enc[0] == INT32_MAX and enc[1] == -2
    assert (decode_global(enc) == fh).all()


def _worker(rank, world, port, seed, n_models, unsup, q):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import cref
    from mythril_amd.dist import allreduce_first_hit, shard_bounds
    from mythril_amd.synth import fuzz_workload
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tb, mb = fuzz_workload(seed, 40, n_models, max_width=256, depth=3)
        lo, hi = shard_bounds(mb.n_models, rank, world)
        local, _ = cref.first_hit(tb, mb.shard(lo, hi))
        local[unsup] = -2  # tape-level property: identical on every rank
        got = allreduce_first_hit(local)
        if rank == 0:
            full, _ = cref.first_hit(tb, mb)
            full[unsup] = -2
            q.put((got.tolist(), full.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_models", [(2, 301), (3, 2), (2, 1)])
def test_gloo_sharded_first_hit_equals_unsharded(world, n_models):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    unsup = [3, 17]
    procs = [ctx.Process(target=_worker, args=(r, world, port, 11, n_models, unsup, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, full = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == full
    assert any(v >= 0 for v in full) and -1 in full
