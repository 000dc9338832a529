#!/usr/bin/env python3
"""Per-dispatch cost of the P interpreter (qsa_kernel) on MI355X — diagnostic, not a parity test.

For each op kind, N tapes that are each a chain of K nodes of that kind over 8 preloaded 256-bit
variables, rooted in an EQ against a random constant (never true: no early exit), on M models.
Prints cycles per (dispatch x wave) at 2.4 GHz over the kernel time of the launch (HIP events),
next to the handler's VALU issue cost from tools/issue_probe.py, so the dispatch overhead per node
(program-entry load, s_setpc, frame) is the difference."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402
from mythril_amd.tape import Tape, TapeBatch  # noqa: E402

K = int(os.environ.get("PROBE_K", "60"))
N = int(os.environ.get("PROBE_N", "4096"))
M = int(os.environ.get("PROBE_M", "65536"))
KINDS = sys.argv[1:] or ["andv", "addv", "mulv", "pushvar_and", "addc", "andc"]


def chain(kind: str, seed: int) -> Tape:
    t = Tape()
    r = np.random.default_rng(seed)
    v = [t.var(i, 256) for i in range(8)]
    acc = v[seed % 8]
    for i in range(K):
        x = v[(i + seed) % 8]
        c = t.const(int.from_bytes(r.bytes(32), "little"), 256)
        if kind == "andv":
            acc = t.band(acc, x)
        elif kind == "addv":
            acc = t.add(acc, x)
        elif kind == "mulv":
            acc = t.mul(acc, x)
        elif kind == "pushvar_and":      # x & y pushed as a pair: PUSH_VAR + BANDV, then BAND
            acc = t.band(acc, t.band(x, v[(i + seed + 3) % 8]))
        elif kind == "addc":
            acc = t.add(acc, c)
        elif kind == "andc":
            acc = t.band(acc, c)
    return t.finish(t.eq(acc, t.const(int.from_bytes(r.bytes(32), "little"), 256)))


def main():
    rng = np.random.default_rng(1)
    mb = ModelBatch([256] * 8, rng.integers(0, 1 << 32, (64, M), dtype=np.uint64).astype(np.uint32))
    ev = Evaluator(0)
    ev.upload_models(mb)
    out = []
    for kind in KINDS:
        tb = TapeBatch([chain(kind, s) for s in range(N)])
        ct = ev.compile(tb)
        ev.first_hit(ct)
        assert ct.asm_split()[0] == N, ct.asm_split()
        hist = ct.handler_histogram(0)
        disp = sum(hist.values()) / N
        ev.time_kernels(True)
        reps = 3
        for _ in range(reps):
            fh = ev.first_hit(ct)
        kt = ev.kernel_times(reset=True)
        ev.time_kernels(False)
        assert (fh == -1).all()
        ms = min(kt)
        waves_per_simd = (M / 64) / 1024.0
        cyc = ms * 1e-3 * 2.4e9
        per = cyc / (waves_per_simd * disp)
        out.append({"kind": kind, "dispatches_per_model": disp, "ms": ms, "cycles_per_dispatch_per_wave": per,
                    "hist": {k: v for k, v in sorted(hist.items(), key=lambda kv: -kv[1])[:6]}})
        print(json.dumps(out[-1]), flush=True)
        ct.free()
    ev.close()


if __name__ == "__main__":
    main()
