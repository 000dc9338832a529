#!/usr/bin/env python3
"""Which G handlers precede (and follow) a given handler kind in a bench workload's translated
tapes (WHICH = 1) or column programs (WHICH = 2): (kind, next kind) dispatch counts per (tape,
model) pair from the translator's histogram (diagnostic).
usage: tools/g_pairs.py CONFIG KIND [WHICH] [models]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402

cfg, kind = sys.argv[1], sys.argv[2]
which = int(sys.argv[3]) if len(sys.argv) > 3 else 1
M = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
n_tapes, _, seed = bench.WORKLOADS[cfg][:3]
tb, mb, _ = bench.build_workload(cfg, n_tapes, M, seed, 0, 1)
ev = Evaluator(0)
ev.upload_models(mb)
ct = ev.compile(tb)
ev.first_hit(ct)
h, pr = ct.handler_histogram(which, pairs=True, wait_variants=True)
tot = sum(h.values())
match = lambda k: k == kind or (k.startswith(kind) and k[len(kind)].isdigit())   # noqa: E731  (EQK0, EQK1 ...)
print(f"{cfg}: {tot} G dispatches per pair-sum; {kind}: {sum(v for k, v in h.items() if match(k))}")
print("kinds:", sorted(((v, k) for k, v in h.items()), reverse=True)[:40])
before = sorted(((v, a, b) for (a, b), v in pr.items() if match(b)), reverse=True)
after = sorted(((v, a, b) for (a, b), v in pr.items() if match(a)), reverse=True)
print("before:", before[:15])
print("after:", after[:15])
# (with KIND = PUSH_MEM: a following stack reader without the _L form waits for the load)
waits = sum(v for (a, b), v in pr.items() if a.startswith(kind) and not b.endswith("_L") and not b.startswith("PUSH"))
print(f"pairs {kind} -> a waiting reader: {waits}; all pairs: {sum(pr.values())}")
