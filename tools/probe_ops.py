#!/usr/bin/env python3
"""Per-op cost probe of the HIP C++ interpreter on MI355X: for each node kind, 64 tapes that are
each a chain of K nodes of that kind, evaluated on M models with the assembly path disabled.
Prints ns per (node x 64-model wave) and lane-ops/s.  Diagnostic only (not a parity test)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402
from mythril_amd.tape import Tape, TapeBatch  # noqa: E402

K = int(os.environ.get("PROBE_K", "200"))
M = int(os.environ.get("PROBE_M", "262144"))
rng = np.random.default_rng(1)
W = [256] * 4 + [8] * 4
words = np.vstack([rng.integers(0, 1 << 32, (8, M), dtype=np.uint64).astype(np.uint32) for _ in range(4)] +
                  [rng.integers(0, 256, (1, M), dtype=np.uint64).astype(np.uint32) for _ in range(4)])
mb = ModelBatch(W, words)


def chain(kind: str, seed: int) -> Tape:
    t = Tape()
    r = np.random.default_rng(seed)
    v = [t.var(i, 256) for i in range(4)]
    b = [t.var(4 + i, 8) for i in range(4)]
    acc = v[0]
    acc8 = b[0]
    for i in range(K):
        x = v[i % 4]
        if kind == "add":
            acc = t.add(acc, x)
        elif kind == "mul":
            acc = t.mul(acc, x)
        elif kind == "and":
            acc = t.band(acc, x)
        elif kind == "udiv_small":
            acc = t.add(t.udiv(acc, t.const(int(r.integers(2, 1000)), 256)), x)
        elif kind == "udiv_big":
            acc = t.add(t.udiv(acc, t.bor(x, t.const(1 << 200, 256))), x)
        elif kind == "lshr_const":
            acc = t.bxor(t.lshr(acc, t.const(int(r.integers(1, 255)), 256)), x)
        elif kind == "ite8":
            acc8 = t.ite(t.ult(b[i % 4], t.const(128, 8)), acc8, b[(i + 1) % 4])
        elif kind == "concat":
            acc8 = t.extract(7, 0, t.concat(acc8, b[i % 4]))
        elif kind == "slt_ite_concat":   # a calldata byte feeding a word (C3's dominant shape)
            byte = t.ite(t.slt(t.const(i, 256), v[1]), b[i % 4], t.const(0, 8))
            acc = t.extract(255, 0, t.concat(t.extract(247, 0, acc), byte))
        elif kind == "push_var":
            acc = t.bxor(acc, t.bxor(x, v[(i + 1) % 4]))
    root = t.ult(acc, v[3]) if kind not in ("ite8", "concat") else t.eq(acc8, t.const(300 % 256, 8))
    return t.finish(root)


def main():
    ev = Evaluator(0)
    ev.use_asm(False)
    ev.upload_models(mb)
    out = {}
    for kind in ["add", "and", "push_var", "mul", "lshr_const", "ite8", "concat", "slt_ite_concat", "udiv_small", "udiv_big"]:
        tb = TapeBatch([chain(kind, s) for s in range(64)])
        ct = ev.compile(tb)
        ev.set_option(ev.OPT_EARLY_EXIT, 0)
        ev.first_hit(ct)
        ev.time_kernels(True)
        t0 = time.perf_counter()
        ev.first_hit(ct)
        dt = time.perf_counter() - t0
        ms = ev.kernel_times(reset=True)[0]
        ev.time_kernels(False)
        nodes = float(tb.sizes().mean())
        waves = 64 * M / 64
        ns_per_node_wave = ms * 1e6 / (waves * nodes) * 1024  # per SIMD (1024 SIMDs)
        out[kind] = {"kernel_ms": ms, "nodes_per_tape": nodes, "ns_per_node_wave_per_simd": ns_per_node_wave,
                     "node_evals_per_s": 64 * M * nodes / (ms * 1e-3)}
        print(json.dumps({kind: out[kind]}), flush=True)
    ev.close()


if __name__ == "__main__":
    main()
