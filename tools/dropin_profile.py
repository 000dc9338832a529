#!/usr/bin/env python3
"""cProfile of drop-in cells (diagnostic).
usage: dropin_profile.py N M        one fresh cell (bench.dropin_leg's timed call)
       dropin_profile.py sN M [R]   R fork-stream batches of N parents' 2N successors, each with
                                    new branch conditions (bench.dropin_stream_leg's shape)"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd import support as sp  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.synth_evm import dropin_workload, fork_children  # noqa: E402

stream = sys.argv[1].startswith("s")
n, m = int(sys.argv[1].lstrip("s")), int(sys.argv[2])
ev = Evaluator(0)
pr = cProfile.Profile()
if stream:
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    eng = sp.VerdictEngine(ev)
    warm, recs, _ = dropin_workload(n, m, seed=7)
    cache = sp.ModelCache(eng)
    for r in reversed(recs):
        cache.put(r, 1)
    cache.check_quick_sat_batch(warm)
    sets = [fork_children(warm, seed=1000 + i) for i in range(reps)]
    for kids in sets[:20]:
        cache.check_quick_sat_batch(kids)
    before = dict(eng.timing)
    t0 = time.perf_counter()
    pr.enable()
    for kids in sets[20:]:
        cache.check_quick_sat_batch(kids)
    pr.disable()
    k = reps - 20
    print("ms per batch", round((time.perf_counter() - t0) * 1e3 / k, 3),
          {x: round((eng.timing[x] - before[x]) * 1e3 / k, 3) for x in eng.timing}, flush=True)
else:
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
        t0 = time.perf_counter()
        if rep == 2:
            pr.enable()
        cache.check_quick_sat_batch(exprs)
        pr.disable()
        print("wall ms", round((time.perf_counter() - t0) * 1e3, 2),
              {k: round((eng.timing[k] - before[k]) * 1e3, 2) for k in eng.timing}, flush=True)
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
