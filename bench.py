#!/usr/bin/env python3
"""bench.py — MI355X quick-sat evaluator on BASELINE.json's metric.

Metric: 256-bit constraint-node x model evaluations per second (+ z3 calls avoided).
Workload (N=1): config C2 = BASELINE.json configs[1]: 10^4 synthetic constraint tapes
(~64 DAG nodes over ADD/MUL/AND/EQ/ULT, Bool-AND root) x 10^5 random 256-bit models per GPU
(seed 2, 10 % planted).  One step = one pass of the hot path (check_quick_sat,
reference mythril/support/support_utils.py:60-67, batched): first-hit over all tapes x all
models resident in HBM, + (N>1) the RCCL min-allreduce of the per-tape first-hit index.

Multi-GPU (weak scaling): rank r holds candidates [r*M, (r+1)*M) of a global N*M candidate
list (contiguous model-axis shard); tapes are replicated; first-hit indices
are global and combined with dist.all_reduce(MIN) over RCCL.

Prints one JSON line (rank 0).  `value` counts the node-evals the GPUs actually performed
(device counters; first-hit early exit skips (tape, model-block) pairs above a found hit).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X INT32 VALU peak: 256 CU x 64 lane-ops/clk x 2.4 GHz = 39.3 TOPS.
# Confirmed by mythril_amd/csrc/valu_peak.hip on MI355X: v_add_u32 37.9, v_add_co/addc 36.9,
# v_mad_u64_u32 35.2 T lane-ops/s (profiles/r01_valu_peak.json).  The FP32 figure of
# MI355X_MICROARCH.md (SIMD-32, 157 TF with FMA) would imply 78.6 T; integer ops do not reach it.
VALU_PEAK_TOPS = 256 * 64 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0


# config -> (default tapes, default models per GPU, seed, workload text, kernel that dominates)
WORKLOADS = {
    "c2": (10_000, 100_000, 2, "C2: synthetic 10^4 constraint tapes (ADD/MUL/AND/EQ/ULT, Bool-AND root) x 10^5 "
           "random 256-bit models per GPU, seed 2, 10% planted", "mq::qsa_kernel (gfx950 threaded-code interpreter)"),
    "c3": (1_000, 1_000_000, 3, "C3 substitute: 10^3 EVM-shaped path conjunctions over 3 txs (calldata bytes/words, "
           "dispatch, SafeMath udiv/urem/smod, shifts, extract/concat/signext, balance table, storage store chains; "
           "~1060 DAG nodes) x 10^6 models per GPU, seed 3, 10% planted",
           "mq::qsg_kernel (gfx950 assembly interpreter: tapes, and hoisted columns in mode 3)"),
    "c4": (200, 1_000_000, 4, "C4: 200 keccak-heavy token-transfer paths over 2 txs (balances[key] = storage at "
           "keccak256(key ++ slot), store chains, keccak UF axioms of keccak_function_manager) x 10^6 "
           "keccak-consistent models per GPU, keccak256_512 evaluated IN-KERNEL (keccak-f[1600]), seed 4, 10% planted",
           "mq::qsg_kernel (G tapes + mode-3 columns) + keccak_column_kernel (keccak-f[1600] columns); "
           "whole-step alg ops / kernel time"),
    "c5": (256, 1_250_000, 5, "C5: 256 deep EVM-shaped paths over 5 txs (-t 5), 5 ABI words per call, 18-24 checks "
           "per tx (~4090 DAG nodes per conjunction before hoisting) x 1.25*10^6 models per GPU (10^7 over 8 GPUs), "
           "seed 5, 10% planted",
           "mq::qsg_kernel (gfx950 assembly interpreter: tapes, and hoisted columns in mode 3)"),
}


def build_workload(cfg: str, n_tapes: int, M: int, seed: int, rank: int, world: int, hoist: bool = True):
    """(tapes, this rank's model shard, expected global first hits)."""
    if cfg == "c2":
        from mythril_amd.synth import c2_workload
        tb, mb_all, expected = c2_workload(n_tapes, M * world, seed=seed)
        return tb, (mb_all.shard(rank * M, (rank + 1) * M) if world > 1 else mb_all), expected
    from mythril_amd import synth_evm
    shard = (rank * M, (rank + 1) * M)
    # EVM-shaped batches are lowered with batch-level hoisting: sub-terms shared by several tapes
    # (calldata words, selectors, storage reads, keccak axioms) are evaluated once per model into
    # derived columns, inside every timed step, and counted as evaluated nodes
    if cfg == "c4":
        from mythril_amd.evaluator import default_evaluator
        tb, mb, expected, _ = synth_evm.c4_workload(n_tapes, M * world, seed=seed, shard=shard, interpret_keccak=True,
                                                    hasher_many=default_evaluator().keccak256_array, hoist=hoist)
    elif cfg == "c5":
        tb, mb, expected, _ = synth_evm.c3_workload(n_tapes, M * world, seed=seed, shard=shard, n_tx=5,
                                                    checks_per_tx=(18, 24), n_args=5, hoist=hoist)
    else:
        tb, mb, expected, _ = synth_evm.c3_workload(n_tapes, M * world, seed=seed, shard=shard, hoist=hoist)
    return tb, mb, expected


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", choices=sorted(WORKLOADS), default="c2",
                   help="c2 = BASELINE configs[1] (the metric's workload); c3/c5 = EVM-shaped parity/scaling cases")
    p.add_argument("--tapes", type=int, default=None)
    p.add_argument("--models", type=int, default=None, help="candidate models per GPU")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="nccl (= RCCL over xGMI, the product path); gloo stages the 4N-byte reduce through "
                        "the host and lets a 1-GPU box rehearse N>1 with --device 0")
    p.add_argument("--device", type=int, default=None, help="override LOCAL_RANK -> device mapping (rehearsal)")
    p.add_argument("--no-hoist", action="store_true", help="c3/c4/c5: lower without batch-level hoisting")
    p.add_argument("--no-dropin", action="store_true", help="skip the drop-in leg (ModelCache at N<=256, M<=100)")
    p.add_argument("--no-early-exit", action="store_true", help="diagnostic: evaluate every (tape, model) pair")
    p.add_argument("--context", action="store_true",
                   help="drive the GPUs through one multi-device mq_ctx even at --gpus 1 (in-library RCCL with "
                        "one rank: a 1-GPU rehearsal of the one-process N-GPU path)")
    p.add_argument("--engine", choices=["gpu", "oracle"], default="gpu",
                   help="oracle: CPU rehearsal of the N-rank protocol (shards, MIN all-reduce over gloo, the line's "
                        "keys) with oracle/cref.c in place of the GPU -- a test of bench.py itself, never a measurement")
    return p.parse_args()


def host_cores():
    """CPU counts of this host: ``nproc`` (os.cpu_count), the CPUs this process may run on
    (sched_getaffinity) and the cgroup CPU quota; the OpenMP leg uses every core this job can
    actually use = min(affinity, quota)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, period = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
        except (OSError, ValueError):
            pass
    usable = min(aff, quota) if quota else aff
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "usable": usable}


def _timed_first_hit(cref, tb, mb, target_s: float, threads: int):
    """The first n tapes x the first m models, grown until the oracle runs ~target_s: a short
    calibration on 4 tapes x <= 4096 models, then all models when the budget allows (else as many
    as fit) and as many tapes as fit."""
    n, m = min(tb.n_tapes, 4), min(mb.n_models, 4096)
    sub = tb.subset(range(n))
    t0 = time.perf_counter()
    cref.first_hit(sub, mb.shard(0, m) if m < mb.n_models else mb, nthreads=threads)
    per_pair = max(time.perf_counter() - t0, 1e-4) / (n * m)
    m = int(min(mb.n_models, max(m, target_s / per_pair / max(4, min(tb.n_tapes, 16)))))
    n = int(min(tb.n_tapes, max(4, target_s / per_pair / m)))
    while True:
        sub, msub = tb.subset(range(n)), (mb.shard(0, m) if m < mb.n_models else mb)
        print(f"[cpu_baseline] {n} tapes x {m} models, {threads} threads", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        fh, pairs = cref.first_hit(sub, msub, nthreads=threads)
        dt = time.perf_counter() - t0
        if dt >= target_s * 0.5 or n >= tb.n_tapes:
            break
        n = min(tb.n_tapes, int(n * max(2.0, target_s / max(dt, 1e-3))))
    mb = msub
    sizes = sub.sizes()
    # node-evals the oracle performed: the full M for tapes without a hit, first hit + 1 otherwise
    # (cref stops a tape at its first satisfying model, support_utils.py:62-66)
    node_evals = 0.0
    for t in range(sub.n_tapes):
        evals = mb.n_models if fh[t] < 0 else (fh[t] - mb.index_base + 1)
        node_evals += float(evals) * float(sizes[t])
    return node_evals / dt, (n, mb.n_models), dt


def cpu_baseline(tb, mb, target_s: float):
    """Oracle C restatement (oracle/cref.c) timed on bounded samples of the SAME workload, once on
    every usable host core (OpenMP over tapes) and once single-core (BASELINE.md CPU plan)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cref  # oracle: checker / CPU baseline only
    hc = host_cores()
    cores = hc["usable"]
    v_all, n_all, dt_all = _timed_first_hit(cref, tb, mb, target_s * 2 / 3, cores)
    v_one, n_one, dt_one = _timed_first_hit(cref, tb, mb, target_s / 3, 1)
    return {"value": v_all, "unit": "node-evals/s", "cores": cores, "kind": "port",
            "sample": f"first {n_all[0]} of {tb.n_tapes} tapes x first {n_all[1]} of {mb.n_models} models of the same "
                      f"workload, oracle/cref.c OpenMP over {cores} threads, {dt_all:.1f} s; single core: first "
                      f"{n_one[0]} tapes x {n_one[1]} models, {dt_one:.1f} s",
            "single_core_value": v_one, "host": hc, "seconds": dt_all + dt_one}


DROPIN_REPS = 5   # timed batches per drop-in cell (each one never seen before); the line reports the median


def _median_rep(reps):
    """The cell entry of the median-wall repetition, with every repetition's wall time beside it
    (one batch is a sub-millisecond sample: the first of a cell pays allocator / page-fault /
    thread-pool warm-up that a LASER run pays once)."""
    walls = [r["ms_per_batch"] for r in reps]
    k = sorted(range(len(reps)), key=walls.__getitem__)[len(reps) // 2]
    out = dict(reps[k])
    out["ms_samples"] = [round(w, 4) for w in walls]
    out["ms_min"] = min(walls)
    out["answers_match_reference_loop"] = all(r["answers_match_reference_loop"] for r in reps)
    out["timed_batches"] = len(reps)
    return out


def _reference_replay(cref, tb, mb, n, order_models):
    """Answers of the reference loop (support_utils.py:62-66: first hit in the current order, bump
    to MRU) replayed on the oracle's verdicts of the lowered tapes x models; the models are
    ``order_models`` (MRU first)."""
    v = cref.verdicts(tb, mb)
    order, ref = list(range(len(order_models))), []
    for q in range(n):
        hit = next((i for i in order if v[q, i]), None)
        if hit is not None:
            order.remove(hit)
            order.insert(0, hit)
        ref.append(False if hit is None else order_models[hit])
    return ref


def _timed_batch(ev, eng, cache, exprs):
    before, st0 = dict(eng.timing), dict(eng.stats)
    ev.time_kernels(True)
    ev.host_times(reset=True)
    t0 = time.perf_counter()
    answers = cache.check_quick_sat_batch(exprs)
    wall = time.perf_counter() - t0
    kt = ev.kernel_times(reset=True)
    ev.time_kernels(False)
    cell = {"ms_per_batch": wall * 1e3, "ms_per_query": wall * 1e3 / max(1, len(exprs)),
            "stage_ms": {k: (eng.timing[k] - before[k]) * 1e3 for k in eng.timing},
            "library_phase_ms": {k: v * 1e3 for k, v in ev.host_times(reset=True).items()},
            "kernel_ms": float(sum(kt)), "hits": int(sum(a is not False for a in answers)),
            "conjuncts_evaluated": eng.stats["conjuncts_evaluated"] - st0["conjuncts_evaluated"],
            "conjuncts_cached": eng.stats["conjuncts_cached"] - st0["conjuncts_cached"]}
    return answers, cell


def dropin_leg(ev, grid=((1, 16), (1, 100), (32, 16), (32, 100), (256, 16), (256, 100)), seed: int = 7,
               reps: int = DROPIN_REPS):
    """The drop-in path at the reference's own shape: ``ModelCache.
    check_quick_sat_batch`` end to end over N EVM-shaped path conjunctions x M <= 100 cached
    models, through the product VerdictEngine (DAG lowering, model serialization, upload, compile,
    launch, readback) — NOT part of the headline metric.  Each cell first warms the run-level
    caches with one batch of queries, then times ``reps`` fresh batches from the same contract
    shape, each of paths never seen before (what a LASER run looks like after its first
    transaction); the cell reports the median batch.  The CPU column is the oracle (cref, one
    thread) evaluating the same lowered tapes x models: the evaluation stage only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cref  # oracle: CPU comparison only
    from mythril_amd import support as sp
    from mythril_amd.synth_evm import dropin_workload
    out = []
    for n, m in grid:
        eng = sp.VerdictEngine(ev)
        warm, recs, _ = dropin_workload(n, m, seed=seed)
        cache = sp.ModelCache(eng)
        for r in reversed(recs):
            cache.put(r, 1)
        cache.check_quick_sat_batch(warm)
        cells = []
        for rep in range(reps):
            exprs, _, planted = dropin_workload(n, m, seed=seed, query_seed=1 + rep)   # new paths, same models
            cache = sp.ModelCache(eng)
            for r in reversed(recs):
                cache.put(r, 1)
            answers, cell = _timed_batch(ev, eng, cache, exprs)
            # the oracle on the same lowered tapes x models (candidate index = position in recs,
            # MRU first), then the reference loop replayed on its verdicts
            db, ok = eng.incremental.lower(exprs)
            tb = db.to_tapes()
            mb = eng.incremental.serialize(recs)
            if rep == 0:
                t1 = time.perf_counter()
                cref.first_hit(tb, mb, nthreads=1)
                cpu_eval = time.perf_counter() - t1
            ref = _reference_replay(cref, tb, mb, n, recs)
            cell.update({"n_queries": n, "n_models": m, "avg_tape_nodes": float(tb.sizes().mean()),
                         "cpu_oracle_eval_ms_1thread": cpu_eval * 1e3,
                         "answers_match_reference_loop": all((a is False and b is False) or a is b
                                                             for a, b in zip(answers, ref))})
            cells.append(cell)
        out.append(_median_rep(cells))
        eng.close()
    return out


def dropin_stream_leg(ev, grid=((1, 16), (1, 100), (16, 100), (128, 100)), seed: int = 7,
                      reps: int = DROPIN_REPS):
    """The drop-in path on a LASER-shaped stream (svm.py:351-358): N parent paths are checked
    (``check_quick_sat_batch``), then their 2N JUMPI successors (parent + cond, parent +
    Not(cond); synth_evm.fork_children) are timed — what the next fork / transaction round asks.
    ``reps`` rounds per cell on one engine, each with parents never seen before; the cell reports
    the median round.  Answers are compared with the reference loop replayed on the oracle's
    verdicts."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cref  # oracle: CPU comparison only
    from mythril_amd import support as sp
    from mythril_amd.synth_evm import dropin_workload, fork_children
    out = []
    for n, m in grid:
        eng = sp.VerdictEngine(ev)
        cells = []
        for rep in range(reps):
            warm, recs_r, _ = dropin_workload(n, m, seed=seed, query_seed=None if rep == 0 else 100 + rep)
            recs = recs_r if rep == 0 else recs   # (the same models every round: the first round's records)
            cache = sp.ModelCache(eng)
            for r in reversed(recs):
                cache.put(r, 1)
            cache.check_quick_sat_batch(warm)
            kids = fork_children(warm, seed=seed + n + 1000 * rep)
            order_before = list(reversed(cache.model_cache.lru_cache.keys()))
            answers, cell = _timed_batch(ev, eng, cache, kids)
            db, ok = eng.incremental.lower(kids)
            tb = db.to_tapes()
            mb = eng.incremental.serialize(order_before)
            if rep == 0:
                t1 = time.perf_counter()
                cref.first_hit(tb, mb, nthreads=1)
                cpu_eval = time.perf_counter() - t1
            ref = _reference_replay(cref, tb, mb, len(kids), order_before)
            cell.update({"n_parents": n, "n_queries": len(kids), "n_models": m,
                         "cpu_oracle_eval_ms_1thread": cpu_eval * 1e3,
                         "answers_match_reference_loop": all((a is False and b is False) or a is b
                                                             for a, b in zip(answers, ref))})
            cells.append(cell)
        out.append(_median_rep(cells))
        eng.close()
    return out


def dropin_stream_z3stub_leg(ev, grid=((1, 16), (1, 100), (16, 100), (128, 100)), seed: int = 7):
    """``dropin_stream`` on the path a Mythril install takes: the queries are z3 ``BoolRef`` ASTs
    (model.py:101) and the cached models ``z3.ModelRef``s wrapped like mythril ``Model``s — here
    built in the z3 STAND-IN (tests/fake_z3.py; no z3 on the box) from the same workload
    (tests/z3_bridge.py).  Times are stand-in timings: the stand-in's AST accessors are plain
    Python calls, z3py's go through ctypes.  Per cell: the same stage split as dropin_stream, the
    z3 ASTs the engine translated for the timed children (only new ones are walked), and the
    answers against the reference loop replayed on the stand-in's own evaluator
    (z3_quick_sat_loop, support_utils.py:62-66)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fake_z3  # z3 stand-in: bench leg only
    saved = fake_z3.install()
    try:
        import z3_bridge as B
        import mythril_amd.lower_z3 as lz3
        from mythril_amd import support as sp
        from mythril_amd.synth_evm import dropin_workload, fork_children
        out = []
        for n, m in grid:
            warm_t, recs, _ = dropin_workload(n, m, seed=seed)
            kids_t = fork_children(warm_t, seed=seed + n)
            sig, to = B.signature(warm_t + kids_t), B.ToZ3()
            warm, kids = [to(e) for e in warm_t], [to(e) for e in kids_t]
            models = [B.model_to_z3(r, sig) for r in recs]
            eng = sp.VerdictEngine(ev)
            cache = sp.ModelCache(eng)
            for r in reversed(models):
                cache.put(r, 1)
            cache.check_quick_sat_batch(warm)
            order_before = list(reversed(cache.model_cache.lru_cache.keys()))
            before, st0, tr0 = dict(eng.timing), dict(eng.stats), eng._z3.translated
            ev.time_kernels(True)
            ev.host_times(reset=True)
            t0 = time.perf_counter()
            answers = cache.check_quick_sat_batch(kids)
            wall = time.perf_counter() - t0
            kt = ev.kernel_times(reset=True)
            ev.time_kernels(False)
            stages = {k: (eng.timing[k] - before[k]) * 1e3 for k in eng.timing}
            lib_ms = {k: v * 1e3 for k, v in ev.host_times(reset=True).items()}
            ref, _ = B.reference_replay(kids, order_before, lz3)
            out.append({"n_parents": n, "n_queries": len(kids), "n_models": m, "ms_per_batch": wall * 1e3,
                        "ms_per_query": wall * 1e3 / len(kids), "stage_ms": stages, "library_phase_ms": lib_ms,
                        "kernel_ms": float(sum(kt)),
                        "z3_asts_translated": eng._z3.translated - tr0,
                        "conjuncts_evaluated": eng.stats["conjuncts_evaluated"] - st0["conjuncts_evaluated"],
                        "conjuncts_cached": eng.stats["conjuncts_cached"] - st0["conjuncts_cached"],
                        "hits": int(sum(a is not False for a in answers)),
                        "answers_match_reference_loop": bool(all(a is b for a, b in zip(answers, ref))),
                        "timing": "z3 stand-in (tests/fake_z3.py), not real z3"})
            eng.close()
        return out
    finally:
        fake_z3.uninstall(saved)


def calls_avoided_leg(ev, n_forks: int = 256, n_models: int = 100, seed: int = 21, budget: int = 100_000):
    """"z3 solver calls avoided", counted where SURVEY Appendix E says: at ``get_model``
    (``support.counters``: calls, answers from quick-sat at model.py:101-103, answers from
    generated candidates, calls that reach ``solver_worker`` model.py:28).

    Stream: the per-fork check of svm.py:351-358 on ``n_forks`` JUMPIs
    (synth_evm.fork_stream_workload): each fork's parent path is satisfied by a cached model
    (100 models in the LRU, MRU first); of its two successors one is satisfied by the parent's
    model, the other needs a different third argument.  All 2 * n_forks states go through
    ``is_possible_batch`` (one launch, answers sequentially exact), with
    ``Args.quick_sat_candidates`` off (the reference's behaviour) and on.  There is no z3 on the
    box: the solver stand-in (support.WitnessSolver) answers every state it is asked with the
    known satisfying model, which get_model caches in the LRU like z3's (model.py:124-126), so
    both arms run under the reference's insertion semantics and the LRU evolves alike."""
    from mythril_amd import support as sp
    from mythril_amd.synth_evm import fork_stream_workload
    states, wits, recs = fork_stream_workload(n_forks, n_models, seed=seed)
    out = {"stream": f"svm.py:351-358 fork checks: {n_forks} forks x 2 successors over {n_models} cached models "
                     f"(fork_stream_workload seed {seed}); solver stand-in returns each state's known witness, "
                     f"cached like z3's sat model (model.py:124-126)"}
    saved = (sp.model_cache, sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget)
    try:
        for cand in (False, True):
            sp.reset_caches()
            sp.model_cache = sp.ModelCache(sp.VerdictEngine(ev))
            solver = sp.WitnessSolver(states, wits)
            sp.set_solver_backend(solver)
            sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget = cand, budget
            for m in reversed(recs):
                sp.model_cache.put(m, 1)
            cs = [sp.Constraints(st) for st in states]
            eng = sp.model_cache.engine
            lib_times = getattr(ev, "host_times", lambda reset=True: {})
            lib_times(reset=True)
            e0, l0 = sum(eng.timing.values()), eng.launches
            t_stage0 = dict(eng.timing)
            t0 = time.perf_counter()
            alive = sp.is_possible_batch(cs)
            dt = time.perf_counter() - t0
            c = dict(sp.counters)
            mc = sp.model_cache.stats
            avoided = c["get_model_calls"] - c["solver_calls"]
            engine_s = sum(eng.timing.values()) - e0
            stage_ms = {k: (eng.timing[k] - t_stage0[k]) * 1e3 / len(cs) for k in eng.timing}
            pool_s = sp.timing["solver_pool"]
            out["candidates_on" if cand else "candidates_off"] = {
                **c, "states_alive": int(sum(alive)), "solver_calls_avoided": avoided,
                "fraction_avoided": avoided / max(c["get_model_calls"], 1), "ms_per_state": dt * 1e3 / len(cs),
                # the per-state cost split: the verdict engine's host stages and launches
                # (lower / serialize / upload / compile / evaluate), get_model's ThreadPool +
                # solver stand-in, and the rest (the reference loop's Python: memo, LRU, answers)
                "engine_ms_per_state": engine_s * 1e3 / len(cs),
                "solver_pool_ms_per_state": pool_s * 1e3 / len(cs),
                "other_ms_per_state": (dt - engine_s - pool_s) * 1e3 / len(cs),
                "engine_launches": eng.launches - l0, "engine_stage_ms_per_state": stage_ms,
                "library_phase_ms_per_state": {k: v * 1e3 / len(cs) for k, v in lib_times(reset=True).items()},
                "conjunct_batches_reused": eng.stats.get("conjunct_batches_reused", 0),
                "late_fills": mc.get("late_fills", 0), "late_fill_exprs": mc.get("late_fill_exprs", 0),
                "candidate_budget": budget if cand else 0, "solver_stand_in_calls": solver.calls,
                "models_inserted_by_solver": solver.sat_calls}
    finally:
        sp.model_cache, sp.args.quick_sat_candidates, sp.args.quick_sat_candidate_budget = saved
        sp.set_solver_backend(None)
    return out


def keccak_leg(ev, sizes=(1, 4, 16, 64, 256, 4096, 262144), msg_bytes: int = 64):
    """Concrete keccak service (mythril_amd.keccak_service): mq_keccak256 per-call latency by
    batch size — as shipped (batches of <= MQ_OPT_KECCAK_HOST_BLOCKS blocks hashed by the library's
    host keccak, larger ones by the GPU kernel) and with every batch forced onto the GPU — vs the
    per-call CPU keccak the reference uses (eth_hash from Python, here the oracle's C keccak called
    from Python per message: oracle/cref.c, one core)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cref  # oracle: CPU comparison only
    rng = np.random.default_rng(5)
    out = []
    default_blocks = 128

    def per_call(msgs, reps):
        for _ in range(2):   # the first calls at a size grow the device buffers and the runtime's staging
            ev.keccak256_array(msgs)
        t0 = time.perf_counter()
        for _ in range(reps):
            dg = ev.keccak256_array(msgs)
        return (time.perf_counter() - t0) / reps, dg

    for n in sizes:
        msgs = rng.integers(0, 256, (n, msg_bytes), dtype=np.uint8)
        reps = max(5, min(200, 20000 // n))
        service, dg = per_call(msgs, reps)
        ev.set_option(ev.OPT_KECCAK_HOST_BLOCKS, 0)
        try:
            gpu, dg2 = per_call(msgs, reps)
        finally:
            ev.set_option(ev.OPT_KECCAK_HOST_BLOCKS, default_blocks)
        k = min(n, 20000)
        t0 = time.perf_counter()
        ref = [cref.keccak256(bytes(m)) for m in msgs[:k]]
        cpu = (time.perf_counter() - t0) / k * n
        ok = all(bytes(dg[i]) == ref[i] and bytes(dg2[i]) == ref[i] for i in range(min(k, 256)))
        out.append({"messages": n, "bytes_each": msg_bytes,
                    "path": "host" if n * (msg_bytes // 136 + 1) <= default_blocks else "gpu",
                    "service_ms_per_call": service * 1e3, "gpu_kernel_path_ms_per_call": gpu * 1e3,
                    "service_us_per_hash": service / n * 1e6, "cpu_us_per_hash_1core": cpu / n * 1e6,
                    "service_over_cpu": cpu / service, "gpu_path_over_cpu": cpu / gpu, "digests_match": bool(ok)})
    return out


def pmc_traffic(workload_key: str):
    """HBM bytes per launch of the evaluation kernel from the committed rocprofv3 PMC summary of
    this exact workload (profiles/, FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; see
    tools/rocpd_summary.py).  None if no summary matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            table = json.load(f)
    except OSError:
        return None
    e = table.get(workload_key)
    return None if e is None else {"bytes": e["fetch_bytes"] + e["write_bytes"], "source": e["source"]}


class OracleRehearsal:
    """``--engine oracle``: the evaluator calls bench.py's timed loop makes, answered by the oracle
    (oracle/cref.c) on the host -- so a CPU test can run the N-rank protocol end to end (shards,
    reduce encoding, gloo MIN all-reduce, per-rank timing keys).  Test infrastructure only: the
    line it prints carries ``"engine": "oracle"`` and is not a measurement."""

    rccl_active = False

    def __init__(self, n_devices: int = 1):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cref  # oracle: rehearsal only
        self.cref = cref
        self.mb = None
        self.n_devices = n_devices   # a one-process context over n "devices": contiguous model shards
        self._counts = [0.0, 0.0, 0.0]
        self._times = []
        self._dev_times = [[] for _ in range(n_devices)]
        self._launch = ([], [], [])

    def upload_models(self, mb):
        from mythril_amd.dist import shard_bounds
        self.mb = mb
        self.shards = [mb.shard(*shard_bounds(mb.n_models, g, self.n_devices)) for g in range(self.n_devices)]

    def compile(self, tb):
        from mythril_amd.evaluator import tape_alg_ops
        self.tb, self.alg = tb, np.array([tape_alg_ops(tb, t) for t in range(tb.n_tapes)])

    def launch_first_hit(self, best):
        # each "device" evaluates its shard (global indices), then the MIN over devices: the
        # in-library protocol of mq_launch_first_hit on a multi-device context
        t0 = time.perf_counter()
        enc = []
        for g, sb in enumerate(self.shards):
            t = time.perf_counter()
            f, _ = self.cref.first_hit(self.tb, sb)
            self._dev_times[g].append((time.perf_counter() - t) * 1e3)
            enc.append(np.where(f < 0, np.iinfo(np.int32).max, f).astype(np.int32))
        t1 = time.perf_counter()
        fh = np.minimum.reduce(enc)
        t2 = time.perf_counter()
        self._times.append((t2 - t0) * 1e3)
        self._launch[0].append((t2 - t1) * 1e3)
        self._launch[1].append((t2 - t0) * 1e3)
        self._launch[2].append((t1 - t0) * 1e3 - self._dev_times[0][-1])
        fh = np.where(fh == np.iinfo(np.int32).max, -1, fh)
        best.copy_(torch_tensor(np.where(fh < 0, np.iinfo(np.int32).max, fh).astype(np.int32)))
        sizes = self.tb.sizes()
        evals = np.where(fh < 0, self.mb.n_models, fh - self.mb.index_base + 1).astype(np.float64)
        self._counts[0] += float(evals.sum())
        self._counts[1] += float((evals * sizes).sum())
        self._counts[2] += float((evals * self.alg).sum())

    @staticmethod
    def finalize_first_hit(best):
        best[best == np.iinfo(np.int32).max] = -1

    def counters(self, reset=False):
        c = tuple(self._counts)
        if reset:
            self._counts = [0.0, 0.0, 0.0]
        return c

    def kernel_times(self, reset=True):
        t = list(self._times)
        if reset:
            self._times = []
        return t

    def time_kernels(self, on=True):
        self._times = []
        self._dev_times = [[] for _ in range(self.n_devices)]
        self._launch = ([], [], [])

    def kernel_times_device(self, g, reset=False):
        t = list(self._dev_times[g])
        if reset:
            self._dev_times[g] = []
        return t

    def launch_times(self, reset=True):
        t = tuple(list(x) for x in self._launch)
        if reset:
            self._launch = ([], [], [])
        return t


def torch_tensor(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a))


def launch_mode(args):
    """How the N GPUs of ``--gpus N`` are driven:
    * ``torchrun``: WORLD_SIZE > 1 in the environment (the driver's N > 1 launch): one process per
      GPU, torch.distributed over RCCL, this process is one rank;
    * ``context``: ``--gpus N > 1`` without WORLD_SIZE: ONE process drives N devices through one
      multi-device ``mq_ctx`` (mq_ctx_create(N, ids): the candidate axis is sharded inside
      mq_models_upload, first hits are MIN-reduced by an in-library ncclAllReduce) — the way
      Mythril itself, a single process (mythril_analyzer.py:136-185), would use N GPUs;
    * ``single``: one GPU.
    Returns (mode, n_gpus); exits non-zero with a message when N cannot be honoured."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        if args.gpus not in (1, world):
            raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}")
        return "torchrun", world
    if args.gpus > 1 or getattr(args, "context", False):
        if getattr(args, "engine", "gpu") == "oracle":
            return "context", args.gpus   # (the CPU rehearsal: shards stand in for devices)
        import torch
        have = torch.cuda.device_count()   # does not initialise the GPU
        if have < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} requested but only {have} GPU device(s) are visible")
        return "context", args.gpus
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus}: need at least one GPU")
    return "single", 1


def main():
    args = parse()
    mode, n_gpus = launch_mode(args)
    rank = int(os.environ.get("RANK", "0"))
    world = n_gpus if mode == "torchrun" else 1     # processes
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device is not None:
        local = args.device
    import torch
    import torch.distributed as dist
    oracle = args.engine == "oracle"
    if oracle:
        args.dist_backend = "gloo"
    if world > 1:
        if not oracle:
            torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    def all_reduce(t, op):
        if world == 1:
            return
        if args.dist_backend == "nccl" or t.device.type == "cpu":
            dist.all_reduce(t, op=op)
        else:
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)

    from mythril_amd.evaluator import Evaluator

    d_tapes, d_models, d_seed, workload_text, kernel_name = WORKLOADS[args.config]
    args.tapes = args.tapes or d_tapes
    args.models = args.models or d_models
    args.seed = d_seed if args.seed is None else args.seed
    t_gen = time.perf_counter()
    M = args.models
    if mode == "context":
        # the whole global candidate list (n_gpus x M); mq_models_upload shards it over the devices
        tb, mb, expected = build_workload(args.config, args.tapes, M * n_gpus, args.seed, 0, 1, hoist=not args.no_hoist)
    else:
        tb, mb, expected = build_workload(args.config, args.tapes, M, args.seed, rank, world, hoist=not args.no_hoist)
    t_gen = time.perf_counter() - t_gen

    if oracle:
        ev = OracleRehearsal(n_gpus if mode == "context" else 1)
        ev.upload_models(mb)
        ev.compile(tb)
        ct = None
        dev = torch.device("cpu")
        best = torch.empty(tb.n_tapes, dtype=torch.int32)
        stream = None
    else:
        ev = Evaluator(devices=list(range(n_gpus)), use_rccl=True) if mode == "context" else Evaluator(local)
        if args.no_early_exit:
            ev.set_option(Evaluator.OPT_EARLY_EXIT, 0)
        ev.upload_models(mb)
        ct = ev.compile(tb)
        if ct.n_unsupported:
            raise SystemExit(f"{ct.n_unsupported} {args.config} tapes unsupported by the evaluator")
        dev = torch.device("cuda", local)
        best = torch.empty(tb.n_tapes, dtype=torch.int32, device=dev)
        # a dedicated (non-null) stream: the kernels, the HIP events and RCCL all order on it
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        sptr = stream.cuda_stream
        assert sptr != 0
    # per timed step: the MIN all-reduce of the first hits, bracketed on the launch stream by
    # events (RCCL) or host clocks (gloo / the oracle rehearsal), apart from the kernels
    reduce_ms = []
    red_ev = None

    def step(i=None):
        if oracle:
            ev.launch_first_hit(best)
        else:
            ev.launch_first_hit(ct, best.data_ptr(), sptr)
        if world > 1 and i is not None and red_ev is not None:
            red_ev[i][0].record(stream)
            all_reduce(best, dist.ReduceOp.MIN)
            red_ev[i][1].record(stream)
        elif world > 1 and i is not None:
            t0 = time.perf_counter()
            all_reduce(best, dist.ReduceOp.MIN)
            reduce_ms.append((time.perf_counter() - t0) * 1e3)
        else:
            all_reduce(best, dist.ReduceOp.MIN)
        if oracle:
            ev.finalize_first_hit(best)
        else:
            ev.finalize_first_hit(ct, best.data_ptr(), sptr)

    def sync_all():
        if oracle:
            return
        for d in (range(n_gpus) if mode == "context" else [local]):
            torch.cuda.synchronize(d)

    for _ in range(args.warmup):
        step()
    sync_all()
    # correctness gate on the benchmark workload itself (planted first hits)
    got = best.cpu().numpy()
    ok = bool((got == expected).all())
    if not ok:
        bad = np.flatnonzero(got != expected)
        print(f"[rank {rank}] first-hit mismatch on {len(bad)} tapes, e.g. {bad[:5]}", file=sys.stderr)

    # where the batch ran (after a launch): tapes on the P / G assembly interpreters vs the HIP C++
    # kernels, hoisted columns on G / the keccak and bit-gather column kernels / the C++ column kernel
    if oracle:
        kernel_split = {"tapes": tb.n_tapes, "engine": "oracle (CPU rehearsal)"}
    else:
        n_p, n_g, asm_live = ct.asm_split()
        n_cols = int(getattr(ct, "n_columns", 0))
        cols_g, cols_live = ct.column_asm_split() if n_cols else (0, False)
        kcols = int(ct.keccak_columns()) if n_cols else 0
        kpreds = int(ct.keccak_predicate_columns()) if n_cols else 0
        gcols = int(ct.gather_columns()) if n_cols else 0
        n_fc, cols_fc = ct.flat_split()
        kernel_split = {"tapes": tb.n_tapes, "tapes_p": n_p, "tapes_g": n_g, "tapes_flat": n_fc,
                        "tapes_cpp": tb.n_tapes - ((n_p + n_g + n_fc) if asm_live else 0),
                        "columns_flat": cols_fc,
                        "columns": n_cols, "columns_g": cols_g if cols_live else 0, "columns_keccak": kcols,
                        "columns_keccak_predicates": kpreds, "columns_gather": gcols,
                        "columns_cpp": n_cols - kcols - kpreds - gcols - cols_fc - (cols_g if cols_live else 0)}
    if world > 1 and not oracle and args.dist_backend == "nccl":
        red_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    ev.counters(reset=True)
    # HIP event pair recorded by libmq on `stream` around the evaluation kernel(s) of each launch
    ev.time_kernels(True)
    if world > 1:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    sync_all()
    t_sync = time.perf_counter()
    if world > 1:
        dist.barrier()
    t_end = time.perf_counter()
    elapsed = t_end - t0
    pairs, node_evals, alg_ops = ev.counters(reset=True)
    ctx_attr = None
    if mode == "context":
        # one process, N devices: each device's own kernel events, then the in-library reduce
        # (events on the lead stream around the ncclGroup) and the host time spent issuing
        dev_ms = [float(np.mean(ev.kernel_times_device(g, reset=False) or [0.0])) for g in range(n_gpus)]
        red_l, iss_l, peer_l = ev.launch_times(reset=True)
        ctx_attr = (dev_ms, red_l, iss_l, peer_l)
    ktimes = ev.kernel_times(reset=True)
    ev.time_kernels(False)
    assert len(ktimes) == args.steps, ktimes
    kern_ms = float(np.mean(ktimes))
    if red_ev is not None:
        reduce_ms = [a.elapsed_time(b) for a, b in red_ev]
    red_ms = float(np.mean(reduce_ms)) if reduce_ms else 0.0
    # this rank's wait in the closing barrier: how far it ran ahead of the slowest rank
    barrier_ms = (t_end - t_sync) * 1e3

    stats = torch.tensor([elapsed, node_evals, alg_ops, float(ok), kern_ms, red_ms, barrier_ms], dtype=torch.float64,
                         device=dev)
    per_rank = None
    if world > 1:
        mx = stats.clone()
        all_reduce(mx, dist.ReduceOp.MAX)
        sm = stats.clone()
        all_reduce(sm, dist.ReduceOp.SUM)
        mn = stats.clone()
        all_reduce(mn, dist.ReduceOp.MIN)
        elapsed, node_evals, alg_ops, ok = float(mx[0]), float(sm[1]), float(sm[2]), bool(mn[3] > 0)
        per_rank = {k: {"min": float(mn[j]), "max": float(mx[j])}
                    for j, k in ((4, "kernel_ms"), (5, "allreduce_ms"), (6, "barrier_wait_ms"))}
        per_rank["allreduce_timer"] = "hip events on the launch stream (RCCL)" if red_ev is not None else \
            "host clock around the gloo all_reduce"
    elif ctx_attr is not None:
        dev_ms, red_l, iss_l, peer_l = ctx_attr
        mean = lambda x: float(np.mean(x)) if x else 0.0  # noqa: E731
        per_rank = {"kernel_ms": {"min": min(dev_ms), "max": max(dev_ms)},
                    "kernel_ms_per_device": dev_ms,
                    "allreduce_ms": {"min": mean(red_l), "max": mean(red_l)},
                    "issue_ms": mean(iss_l), "peer_issue_ms": mean(peer_l),
                    "barrier_wait_ms": None,
                    "allreduce_timer": ("host clock around the MIN over shards (oracle rehearsal)" if oracle else
                                        "hip events on the lead stream around the in-library ncclGroup")}
    hits = int((got >= 0).sum())

    if rank == 0:
        per_launch_ops = alg_ops / args.steps / n_gpus
        achieved_tops = per_launch_ops / (kern_ms * 1e-3) / 1e12
        model_bytes = mb.var_words.nbytes
        tape_bytes = tb.nodes.nbytes + tb.consts.nbytes + 4 * tb.n_tapes
        hbm_gbs = (model_bytes + tape_bytes) / (kern_ms * 1e-3) / 1e9
        wkey = f"{args.config}:n{tb.n_tapes}:m{M}:s{args.seed}"
        traffic = pmc_traffic(wkey)
        out = {
            "metric": "256-bit constraint-node x model evals/s",
            "value": node_evals / elapsed,
            "unit": "node-evals/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {
                "workload": workload_text,
                "n_tapes": tb.n_tapes, "models_per_gpu": M, "models_total": M * n_gpus,
                "avg_tape_nodes": float(tb.sizes().mean()), "seed": args.seed,
                "avg_tape_nodes_unhoisted": float(np.mean(getattr(tb, "unhoisted_nodes", tb.sizes()))),
                "hoisted_columns": int(tb.columns.n) if getattr(tb, "columns", None) is not None else 0,
                "column_nodes_per_model": int(tb.columns.programs.sizes().sum()) if getattr(tb, "columns", None) is not None else 0,
                "keccak_columns": int(ct.keccak_columns()) if getattr(tb, "columns", None) is not None else 0,
                "parallelism": {"torchrun": f"one process per GPU x{n_gpus}: model-axis shard + torch.distributed RCCL "
                                            f"min-allreduce",
                                "context": f"one-process context x{n_gpus}: model-axis shard inside mq_models_upload + "
                                           f"in-library RCCL min (ncclAllReduce)",
                                "single": "single GPU"}[mode],
                "rccl_in_library": bool(ev.rccl_active),
            },
            "roofline": {
                "bound": "valu", "achieved": achieved_tops, "peak": VALU_PEAK_TOPS, "unit": "TOPS (int32 VALU)",
                "frac": achieved_tops / VALU_PEAK_TOPS,
                "traffic": traffic["bytes"] if traffic else None,
                "traffic_source": traffic["source"] if traffic else None,
                "kernel": kernel_name, "kernel_ms": kern_ms,
                "alg_bytes_per_launch": model_bytes + tape_bytes,
                "alg_ops_per_launch": per_launch_ops,
                "hbm_alg_GBps": hbm_gbs, "hbm_frac": hbm_gbs / HBM_PEAK_GBS,
            },
            "planted_first_hits": {"hits": hits, "tapes": tb.n_tapes},
            "kernel_split": kernel_split,
            # N > 1: per-rank kernel time (mean over steps), the MIN all-reduce of the first hits
            # and each rank's wait in the closing barrier, as (min, max) over ranks
            "per_rank": per_rank,
            "parity_ok": ok,
            "pairs_evaluated": pairs,
            "nominal_node_evals_per_step": float(tb.sizes().sum()) * M * n_gpus,
            "gen_seconds": t_gen,
        }
        if oracle:
            out["engine"] = "oracle (CPU rehearsal of the protocol; not a measurement)"
        if n_gpus == 1 and not args.no_cpu_baseline and not oracle:
            if getattr(tb, "columns", None) is not None:
                # the reference evaluates every conjunction in full per model: time the oracle on
                # the same conjunctions lowered without hoisting
                ptb, pmb, _ = build_workload(args.config, args.tapes, M, args.seed, rank, world, hoist=False)
                cb = cpu_baseline(ptb, pmb, args.cpu_seconds)
            else:
                cb = cpu_baseline(tb, mb, args.cpu_seconds)
            out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample", "single_core_value", "host")}
            out["gpu_over_cpu"] = out["value"] / cb["value"]
        if n_gpus == 1 and not args.no_dropin and not oracle:
            out["dropin"] = dropin_leg(ev)
            out["dropin_stream"] = dropin_stream_leg(ev)
            out["dropin_stream_z3stub"] = dropin_stream_z3stub_leg(ev)
            out["z3_calls_avoided"] = calls_avoided_leg(ev)
            out["keccak_service"] = keccak_leg(ev)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
