#!/usr/bin/env python3
"""G-kernel fixed-cost probe: K-node tapes (K = 1, 32) on the general assembly kernel with the
tape-group size (MQ_G_TPG), LDS staging (MQ_G_STAGE_KB) and early exit varied.  Diagnostic."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402
from mythril_amd.tape import Tape, TapeBatch  # noqa: E402

M, N, NV = 1 << 20, 512, 16
rng = np.random.default_rng(2)
mb = ModelBatch([256] * NV, rng.integers(0, 1 << 32, (8 * NV, M), dtype=np.uint64).astype(np.uint32))
ev = Evaluator(0)
ev.upload_models(mb)


def tapes(K):
    out = []
    for t in range(N):
        tp = Tape()
        acc = tp.var(8 + t % 8, 256)
        for i in range(K):
            acc = tp.bxor(acc, tp.var(8 + (t * 7 + i * 3) % 8, 256))
        out.append(tp.finish(tp.eq(acc, tp.const(12345, 256))))
    return TapeBatch(out)


for K in (1, 32):
    tb = tapes(K)
    for tpg in ("16", "64", "256"):
        for kb in ("0", "32"):
            for ee in (1, 0):
                os.environ["MQ_G_TPG"], os.environ["MQ_G_STAGE_KB"] = tpg, kb
                ev.set_option(Evaluator.OPT_EARLY_EXIT, ee)
                ct = ev.compile(tb)
                ev.first_hit(ct)
                ev.time_kernels(True)
                for _ in range(3):
                    ev.first_hit(ct)
                ms = float(np.mean(ev.kernel_times(reset=True)))
                ev.time_kernels(False)
                print(f"K={K} tpg={tpg} stage_kb={kb} early_exit={ee}: {ms:.3f} ms, "
                      f"{ms * 1e3 / (N * M / 64) * 1024:.3f} SIMD-us per tape-wave, split {ct.asm_split()}", flush=True)
                ct.free()
