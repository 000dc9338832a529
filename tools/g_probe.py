#!/usr/bin/env python3
"""G-kernel (qsg_kernel) cost probe on MI355X: tapes of K nodes over 16 model variables (so
they run on the general assembly kernel), N tapes x M models; prints microseconds per
(tape, 64-model wave) for several K, separating the fixed per-tape cost (descriptor, early-exit
read, program window) from the per-node cost.  Diagnostic only."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402
from mythril_amd.tape import Tape, TapeBatch  # noqa: E402

M = int(os.environ.get("PROBE_M", str(1 << 20)))
N = int(os.environ.get("PROBE_N", "512"))
NV = 16
rng = np.random.default_rng(2)
words = rng.integers(0, 1 << 32, (8 * NV, M), dtype=np.uint64).astype(np.uint32)
mb = ModelBatch([256] * NV, words)
ev = Evaluator(0)
ev.upload_models(mb)
out = {}
for kind in ("xor_mem", "xor_const"):
    for K in (1, 8, 32, 128):
        tapes = []
        for t in range(N):
            tp = Tape()
            acc = tp.var((t + 8) % NV, 256)
            for i in range(K):
                if kind == "xor_mem":
                    x = tp.var((t * 7 + i * 3 + 8) % NV, 256)
                else:
                    x = tp.const(int(rng.integers(1, 1 << 62)), 256)
                acc = tp.bxor(acc, x)
            tapes.append(tp.finish(tp.eq(acc, tp.const(12345, 256))))
        ct = ev.compile(TapeBatch(tapes))
        ev.first_hit(ct)
        ev.time_kernels(True)
        reps = 3
        for _ in range(reps):
            ev.first_hit(ct)
        ms = float(np.mean(ev.kernel_times(reset=True)))
        ev.time_kernels(False)
        p, g, live = ct.asm_split()
        waves = N * (M // 64)
        out[f"{kind}_K{K}"] = {"kernel_ms": ms, "us_per_tape_wave": ms * 1e3 / waves * 1024,
                               "note": "x1024 SIMDs: SIMD-microseconds per tape-wave", "on_g": g, "on_p": p}
        print(kind, K, round(ms, 3), "ms", out[f"{kind}_K{K}"]["us_per_tape_wave"], "SIMD-us/tape-wave", "G", g, "P", p, flush=True)
print(json.dumps(out))
