#!/usr/bin/env python3
"""The fork-stream drop-in cell in a loop (diagnostic, e.g. under rocprofv3 --hip-trace): N parent
paths over M cached models, then K rounds of their 2N JUMPI children (synth_evm.fork_children with
a new seed each round: one new branch conjunct per child).  Prints the median wall time per round
and the engine / library stage split.   usage: stream_loop.py N M K"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from mythril_amd import support as sp  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.synth_evm import dropin_workload, fork_children  # noqa: E402

n, m, k = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1, 16, 200)))
ev = Evaluator(0)
eng = sp.VerdictEngine(ev)
warm, recs, _ = dropin_workload(n, m, seed=7)
cache = sp.ModelCache(eng)
for r in reversed(recs):
    cache.put(r, 1)
cache.check_quick_sat_batch(warm)
rounds = [fork_children(warm, seed=100 + i) for i in range(k)]
for kids in rounds[:10]:
    cache.check_quick_sat_batch(kids)
before = dict(eng.timing)
ev.host_times(reset=True)
ts = []
for kids in rounds[10:]:
    t0 = time.perf_counter()
    cache.check_quick_sat_batch(kids)
    ts.append(time.perf_counter() - t0)
r = len(ts)
print(json.dumps({"n_parents": n, "n_models": m, "rounds": r, "median_ms": float(np.median(ts) * 1e3),
                  "mean_ms": float(np.mean(ts) * 1e3),
                  "stage_ms": {s: (eng.timing[s] - before[s]) * 1e3 / r for s in eng.timing},
                  "library_phase_ms": {s: v * 1e3 / r for s, v in ev.host_times(reset=True).items()}}))
