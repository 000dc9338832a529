#!/usr/bin/env python3
"""Handler-kind mix of the assembly translation of a bench workload (diagnostic): dispatches per
(tape, model) pair by kind and the most frequent (kind, next kind) pairs of the G tapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
M = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
n_tapes, _, seed = bench.WORKLOADS[cfg][:3]
tb, mb, _ = bench.build_workload(cfg, n_tapes, M, seed, 0, 1)
ev = Evaluator(0)
ev.upload_models(mb)
ct = ev.compile(tb)
ev.first_hit(ct)
print("split", ct.asm_split(), "columns", ct.column_asm_split())
for which, name in ((0, "P tapes"), (1, "G tapes"), (2, "G columns")):
    h = ct.handler_histogram(which)
    tot = sum(h.values())
    print(f"== {name}: {tot} dispatches per model")
    for k, v in sorted(h.items(), key=lambda kv: -kv[1])[:30]:
        print(f"  {k:16s} {v:9d} {100 * v / max(tot, 1):5.1f}%")
for which, name in ((0, "P"), (1, "G")):
    h, pr = ct.handler_histogram(which, pairs=True)
    tot = sum(pr.values())
    print(f"== {name} bigrams ({tot})")
    for (a, b), v in sorted(pr.items(), key=lambda kv: -kv[1])[:40]:
        print(f"  {a:16s} -> {b:16s} {v:9d} {100 * v / max(tot, 1):5.1f}%")
