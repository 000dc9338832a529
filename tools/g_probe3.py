#!/usr/bin/env python3
"""G-kernel per-node cost by tape shape (diagnostic): conjunctions of K leaves of one kind over
2^20 models, timed on the general assembly kernel; prints SIMD-cycles per evaluated node-wave
(2.4 GHz, 1024 SIMDs).  Leaves: Bool variables, var == 256-bit const, var == small const,
var < const, var ^ var chains."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402
from mythril_amd.tape import Tape, TapeBatch  # noqa: E402

M, N, NB, NW = 1 << 20, 512, 16, 16
rng = np.random.default_rng(3)
words = np.concatenate([rng.integers(0, 1 << 32, (8 * NW, M), dtype=np.uint64).astype(np.uint32),
                        np.ones((NB, M), np.uint32)])
mb = ModelBatch([256] * NW + [0] * NB, words)
ev = Evaluator(0)
ev.upload_models(mb)
BIG = (1 << 255) | 0x1234567


def shape(kind, K):
    out = []
    for t in range(N):
        tp = Tape()
        leaves = []
        for i in range(K):
            v = (t * 5 + i * 3) % 16
            if kind == "boolvar":
                leaves.append(tp.var(NW + v, 0))
            elif kind == "eqbig":
                leaves.append(tp.not_(tp.eq(tp.var(v, 256), tp.const(BIG + i, 256))))
            elif kind == "eqsmall":
                leaves.append(tp.not_(tp.eq(tp.var(v, 256), tp.const(1000 + i, 256))))
            elif kind == "ult":
                leaves.append(tp.ult(tp.var(v, 256), tp.const(BIG + i, 256)))
        root = tp.and_(*leaves, tp.eq(tp.var(0, 256), tp.const(7, 256)))
        out.append(tp.finish(root))
    return TapeBatch(out)


for kind in ("boolvar", "eqbig", "eqsmall", "ult"):
    for K in (8, 32):
        tb = shape(kind, K)
        nodes = float(np.mean(tb.sizes()))
        for kb in ("0", "32"):
            os.environ["MQ_G_STAGE_KB"] = kb
            ct = ev.compile(tb)
            ev.first_hit(ct)
            ev.time_kernels(True)
            for _ in range(3):
                ev.first_hit(ct)
            ms = float(np.mean(ev.kernel_times(reset=True)))
            ev.time_kernels(False)
            cyc = ms * 1e-3 * 1024 * 2.4e9 / (N * M / 64 * nodes)
            print(f"{kind} K={K} nodes/tape={nodes:.0f} stage_kb={kb}: {ms:.3f} ms, {cyc:.1f} SIMD-cycles per node-wave, "
                  f"split {ct.asm_split()}", flush=True)
            ct.free()
