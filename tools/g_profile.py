#!/usr/bin/env python3
"""Per-handler-kind cycle profile of the G kernel on a bench workload (diagnostic; needs the
profile build: QSA_PROF=1 python -c 'import mythril_amd.build as b; b.build(force=True)').
Each dispatch charges the cycles since the previous handler ended (its dispatch jump, body and
any wait it hit) to its kind; FRAME = the tape loop between tapes (header, early-exit check,
program window).  usage: tools/g_profile.py [c3|c5] [models]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
M = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
n_tapes, _, seed = bench.WORKLOADS[cfg][:3]
tb, mb, _ = bench.build_workload(cfg, n_tapes, M, seed, 0, 1)
ev = Evaluator(0)
ev.upload_models(mb)
ct = ev.compile(tb)
ev.first_hit(ct)
ev.qsa_profile(reset=True)
ev.time_kernels(True)
ev.first_hit(ct)
ms = ev.kernel_times(reset=True)
prof = ev.qsa_profile(reset=True)
if not prof:
    sys.exit("not a profile build (QSA_PROF=1)")
tot = sum(c for c, _ in prof.values())
print(f"{cfg} M={M}: kernels {[round(x, 2) for x in ms]} ms; total charged {tot:.3e} wave-cycles")
print(f"{'kind':18s} {'dispatches':>12s} {'cycles':>14s} {'cyc/disp':>9s} {'share':>6s}")
for k, (c, n) in sorted(prof.items(), key=lambda kv: -kv[1][0]):
    print(f"{k:18s} {n:12d} {c:14d} {c / n:9.1f} {100 * c / tot:5.1f}%")
