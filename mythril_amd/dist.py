"""Model-axis sharding over GPUs: one process per GPU, candidates split
contiguously in global candidate order, tapes replicated, per-tape first hits combined by ONE
min-allreduce of int32[N] (RCCL over xGMI on MI355X; gloo on CPU for tests).

Why a min-reduce is exact: rank g holds global candidates [lo_g, hi_g); its local first hit is
the smallest satisfying GLOBAL index inside its range, so the global first hit of
``check_quick_sat`` (support_utils.py:62-66, MRU-first order) is the minimum over ranks.  "No hit"
is encoded as INT32_MAX so it never wins; UNSUPPORTED (-2) is a property of the tape, identical
on every rank, and being negative it survives the MIN unchanged.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

INT32_MAX = np.iinfo(np.int32).max
NO_HIT = -1
UNSUPPORTED = -2


def shard_bounds(n_models: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous range of global candidates owned by ``rank`` (ragged M allowed)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return n_models * rank // world, n_models * (rank + 1) // world


def encode_local(first_hit: np.ndarray) -> np.ndarray:
    """Local first-hit (global indices, -1 none, -2 unsupported) -> reduce encoding."""
    out = np.asarray(first_hit, np.int32).copy()
    out[out == NO_HIT] = INT32_MAX
    return out


def decode_global(reduced: np.ndarray) -> np.ndarray:
    out = np.asarray(reduced, np.int32).copy()
    out[out == INT32_MAX] = NO_HIT
    return out


def allreduce_first_hit(local_first_hit: np.ndarray, group=None) -> np.ndarray:
    """Host-side combine (gloo / any backend with CPU tensors): MIN over ranks."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(encode_local(local_first_hit))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return decode_global(t.numpy())


class ShardedEvaluator:
    """The product multi-GPU path: this rank's shard resident in HBM, the launch writes the
    reduce encoding straight into a device int32[N] (``mq_launch_first_hit``), RCCL MIN-reduces
    it in place on the same HIP stream, and ``mq_finalize_first_hit`` maps the sentinels back.
    No host round trip between the kernel and the collective."""

    def __init__(self, evaluator, rank: int, world: int, group=None):
        import torch
        self.ev, self.rank, self.world, self.group = evaluator, rank, world, group
        self.device = torch.device("cuda", evaluator.device)
        self.stream = torch.cuda.Stream(self.device)
        self.n_models_global = 0

    def upload_models(self, global_batch) -> Tuple[int, int]:
        lo, hi = shard_bounds(global_batch.n_models, self.rank, self.world)
        self.ev.upload_models(global_batch.shard(lo, hi))
        self.n_models_global = global_batch.n_models
        return lo, hi

    def upload_shard(self, shard_batch, n_models_global: int) -> None:
        """Each rank built only its own shard (index_base = its global offset)."""
        self.ev.upload_models(shard_batch)
        self.n_models_global = n_models_global

    def launch(self, compiled, out):
        """Enqueue kernel + collective + finalize on this rank's stream (async)."""
        import torch
        import torch.distributed as dist
        with torch.cuda.stream(self.stream):
            self.ev.launch_first_hit(compiled, out.data_ptr(), self.stream.cuda_stream)
            if self.world > 1:
                dist.all_reduce(out, op=dist.ReduceOp.MIN, group=self.group)
            self.ev.finalize_first_hit(compiled, out.data_ptr(), self.stream.cuda_stream)

    def first_hit(self, tapes) -> np.ndarray:
        import torch
        ct = tapes if hasattr(tapes, "handle") else self.ev.compile(tapes)
        out = torch.empty(ct.n_tapes, dtype=torch.int32, device=self.device)
        self.launch(ct, out)
        self.stream.synchronize()
        return out.cpu().numpy()
