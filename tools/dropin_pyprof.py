"""Host-side (Python) cost of the drop-in quick-sat path with the device stages stubbed out:
``python tools/dropin_pyprof.py N M [--prof]`` times ``check_quick_sat_batch`` on the 2N JUMPI
children of N EVM-shaped parent paths over M cached models (bench.py dropin_stream's shape) with
an evaluator that returns at once, so what remains is ModelCache / VerdictEngine bookkeeping,
lowering and serialization.  Diagnostic only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from mythril_amd import support as sp  # noqa: E402
from mythril_amd import evaluator as E  # noqa: E402
from mythril_amd.synth_evm import dropin_workload, fork_children  # noqa: E402


class CT:
    def __init__(self, n):
        self.n_tapes = n

    def free(self):
        pass


class NullEv:
    upload_seq = 1

    def upload_models(self, mb):
        self.M = mb.n_models

    def compile(self, tb):
        return CT(tb.n_tapes)

    def verdicts(self, ct):
        return np.zeros((ct.n_tapes, self.M), bool), np.full(ct.n_tapes, -1, np.int32)


def fresh(n, m):
    """bench.py dropin_leg's cell: warm the engine with one batch, then time a batch of NEW paths
    (another query seed) through a new ModelCache over the same models, per query seed."""
    E.CompiledTapes = CT
    ts, stages = [], []
    for q in range(1, 21):
        eng = sp.VerdictEngine(NullEv())
        warm, recs, _ = dropin_workload(n, m, seed=7)
        cache = sp.ModelCache(eng)
        for r in reversed(recs):
            cache.put(r, 1)
        cache.check_quick_sat_batch(warm)
        exprs, _, _ = dropin_workload(n, m, seed=7, query_seed=q)
        cache = sp.ModelCache(eng)
        for r in reversed(recs):
            cache.put(r, 1)
        before = dict(eng.timing)
        t0 = time.perf_counter()
        cache.check_quick_sat_batch(exprs)
        ts.append(time.perf_counter() - t0)
        stages.append({k: (eng.timing[k] - before[k]) * 1e3 for k in eng.timing})
    st = {k: round(float(np.median([s[k] for s in stages])), 4) for k in stages[0]}
    print(f"fresh: median {np.median(ts) * 1e3:.4f} ms per batch of {n} queries, M={m}; engine stages (median) {st}")


def main():
    n, m = int(sys.argv[1]), int(sys.argv[2])
    if "--fresh" in sys.argv:
        return fresh(n, m)
    E.CompiledTapes = CT
    eng = sp.VerdictEngine(NullEv())
    warm, recs, _ = dropin_workload(n, m, seed=7)
    cache = sp.ModelCache(eng)
    for r in reversed(recs):
        cache.put(r, 1)
    cache.check_quick_sat_batch(warm)
    batches = [fork_children(warm, seed=7 + n + rep) for rep in range(60)]
    ts = []
    t_before = dict(eng.timing)
    for kids in batches[:40]:
        t0 = time.perf_counter()
        cache.check_quick_sat_batch(kids)
        ts.append(time.perf_counter() - t0)
    st = {k: round((eng.timing[k] - t_before[k]) * 1e3 / 40, 4) for k in eng.timing}
    print(f"median {np.median(ts) * 1e3:.4f} ms per batch of {2 * n} children, M={m}; engine stages (mean) {st}")
    if "--prof" in sys.argv:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for kids in batches[40:]:
            cache.check_quick_sat_batch(kids)
        pr.disable()
        pstats.Stats(pr).sort_stats(sys.argv[4] if len(sys.argv) > 4 else "cumulative").print_stats(40)


if __name__ == "__main__":
    main()
