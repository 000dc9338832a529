#!/usr/bin/env python3
"""cProfile of one fresh drop-in cell (bench.dropin_leg's timed call only; diagnostic).
usage: dropin_profile.py N M"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd import support as sp  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.synth_evm import dropin_workload  # noqa: E402

n, m = (int(x) for x in sys.argv[1:3])
ev = Evaluator(0)
for rep in range(3):
    eng = sp.VerdictEngine(ev)
    warm, recs, _ = dropin_workload(n, m, seed=7)
    cache = sp.ModelCache(eng)
    for r in reversed(recs):
        cache.put(r, 1)
    cache.check_quick_sat_batch(warm)
    exprs, _, _ = dropin_workload(n, m, seed=7, query_seed=1)
    cache = sp.ModelCache(eng)
    for r in reversed(recs):
        cache.put(r, 1)
    before = dict(eng.timing)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    if rep == 2:
        pr.enable()
    cache.check_quick_sat_batch(exprs)
    pr.disable()
    print("wall ms", round((time.perf_counter() - t0) * 1e3, 2),
          {k: round((eng.timing[k] - before[k]) * 1e3, 2) for k in eng.timing}, flush=True)
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
