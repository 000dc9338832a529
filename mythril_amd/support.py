"""Drop-in mirrors of the reference's quick-sat boundary, backed by the MI355X evaluator.

Reference interface, kept name for name:

* ``LRUCache``            ``mythril/support/support_utils.py:34-53``
* ``ModelCache``          ``support_utils.py:56-70`` — ``check_quick_sat(constraints)`` returns the
  first cached model (MRU first) under which the conjunction evaluates to literally ``true``,
  bumps it to MRU, and is memoized per ``(self, constraints)`` by ``functools.lru_cache(2**10)``
  (a memoized ``False`` or hit is returned again without re-evaluation and without a bump);
* ``get_model``           ``mythril/support/model.py:68-130`` (gating, exceptions, quick-sat iff no
  minimize/maximize, solver fallback in a ``ThreadPool(1)`` with timeout, cache insert on sat),
  memoized by ``lru_cache(2**23)``;
* ``model_cache``         ``model.py:25`` (the process-global instance).

What changes is HOW ``check_quick_sat`` decides: instead of ``deepcopy(model).eval(...)`` per model
in a Python loop (support_utils.py:62-64), the conjunction is lowered to a tape and evaluated against
every cached model in one launch of the HIP kernels (``mq_eval_verdicts``, include/mq.h); the
first-hit/bump/memo logic then runs exactly as the reference's loop would.

Batching without changing semantics: :meth:`ModelCache.prefetch` evaluates N
pending conjunctions against the current cache in ONE launch.  The queries are still answered
one at a time, in the caller's order, through the unchanged ``check_quick_sat``: a bump reorders
candidates exactly as in the sequential loop, and a model inserted mid-batch (a z3 fallback) is
evaluated lazily for every still-pending conjunction in one more launch.  The answers are
therefore identical to the sequential reference for any interleaving.

Fail closed: a conjunction the lowering or the tape compiler cannot express is answered by the
reference's own z3 eval loop where z3 exists (:mod:`mythril_amd.lower_z3`); without z3 it gets no
quick answer (``False``) and goes to the solver, which is what a quick-sat miss does anyway.
There is no CPU evaluator: if the HIP library or the GPU is missing, :class:`EvaluatorError` is
raised.
"""
from __future__ import annotations

import logging
import math
import os
import sys
import threading
import time
from collections import OrderedDict
from functools import lru_cache
from multiprocessing import TimeoutError as _PoolTimeout
from multiprocessing.pool import ThreadPool
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import smt as S
from .exceptions import LoweringError, SolverTimeOutException, UnsatError, fail_closed  # noqa: F401
#   (fail_closed: queries routed to z3 because a conjunct did not lower, by reason -- array equality, ...)
from .exceptions import note_fail_closed as fail_closed_note
from .lower import DagBatch
from .smt_model import Model, as_record

log = logging.getLogger(__name__)


# ---------------------------------------------------------------------------- support_utils.py
class Singleton(type):
    """support_utils.py:14-31 (not thread-safe, as documented there)."""
    _instances: Dict = {}

    def __call__(cls, *args, **kwargs):
        if cls not in cls._instances:
            cls._instances[cls] = super().__call__(*args, **kwargs)
        return cls._instances[cls]


class LRUCache:
    """support_utils.py:34-53: ``get`` moves the key to MRU (or returns -1); ``put`` re-inserts at
    MRU and evicts the LRU entry when a NEW key arrives at capacity."""

    def __init__(self, size: int):
        self.size = size
        self.lru_cache: "OrderedDict" = OrderedDict()
        self.version = 0   # (not in the reference) bumped when the order or the contents change

    def get(self, key):
        if key not in self.lru_cache:
            return -1
        self.lru_cache.move_to_end(key)
        self.version += 1
        return self.lru_cache[key]

    def put(self, key, value) -> None:
        if key in self.lru_cache:
            del self.lru_cache[key]
        elif len(self.lru_cache) >= self.size:
            self.lru_cache.popitem(last=False)
        self.lru_cache[key] = value
        self.version += 1


class Args(metaclass=Singleton):
    """The hot-path subset of ``Args`` (mythril/support/support_args.py:5-27)."""

    def __init__(self):
        self.solver_timeout = 10000
        self.pruning_factor = None
        self.solver_log = None
        self.parallel_solving = False
        # build extension (not a reference flag): on a quick-sat miss, a verdict-only caller
        # (Constraints.is_possible) also tries generated candidates (mythril_amd.candidates)
        self.quick_sat_candidates = False
        self.quick_sat_candidate_budget = 100_000


args = Args()


class TimeHandler(metaclass=Singleton):
    """``time_handler`` (mythril/laser/ethereum/time_handler.py:5-18).  Before
    ``start_execution`` the budget is unbounded (the reference would fail on ``None``)."""

    def __init__(self):
        self._start_time = None
        self._execution_time = None

    def start_execution(self, execution_time) -> None:
        self._start_time = int(time.time() * 1000)
        self._execution_time = execution_time * 1000

    def time_remaining(self):
        if self._start_time is None:
            return math.inf
        return self._execution_time - (int(time.time() * 1000) - self._start_time)


time_handler = TimeHandler()


# ---------------------------------------------------------------------------- verdict engine
def split_conjuncts(db: DagBatch, groups: int) -> Tuple[DagBatch, Optional[np.ndarray]]:
    """Each tape of ``db`` (a conjunction: its list of conjunct roots) as up to ``groups``
    tapes over contiguous runs of its conjuncts (consecutive conjuncts of a path share the most
    sub-terms).  Returns the split batch and the index of each original tape's first group, or
    ``(db, None)`` when nothing splits."""
    offs = db.root_offsets
    n_conj = np.diff(offs)
    k = np.minimum(n_conj, max(1, int(groups)))
    if groups <= 1 or not np.any(k > 1):
        return db, None
    new = [0]
    for q in range(db.n_tapes):
        a, kq = int(offs[q]), int(max(k[q], 1))
        bounds = a + (np.arange(1, kq + 1) * int(n_conj[q])) // kq
        new.extend(int(x) for x in bounds)
    starts = np.concatenate(([0], np.cumsum(np.maximum(k, 1))[:-1])).astype(np.int64)
    return DagBatch(db.nodes, db.consts, np.asarray(new, np.int64), db.roots), starts


class ConjunctRows:
    """Verdicts of single conjuncts under single models, kept across calls: ``R[row, slot]`` is
    -1 (not evaluated), 0 or 1 for the conjunct DAG node of ``row`` under the model in ``slot``
    (:class:`~mythril_amd.lower.IncrementalLowering` slots).  A conjunction is true under a model
    iff each of its conjuncts is, so a query whose conjuncts were all seen before (a forked path's
    parent constraints, svm.py:351-358; the keccak axioms riding on every query,
    constraints.py:127-128) needs no device work for the models already evaluated.  Valid for one
    DAG generation and slot epoch (``key``); past ``MAX_ROWS`` conjuncts it starts over."""

    MAX_ROWS = 1 << 16

    def __init__(self) -> None:
        self.reset(None)

    def reset(self, key) -> None:
        self.key = key
        self.n_rows = 0
        self.row_of = np.full(1024, -1, np.int64)   # DAG node -> row (-1: none yet)
        self.R = np.full((256, 128), -1, np.int8)
        self.bad: set = set()   # conjunct nodes whose tape the evaluator does not support

    def sync(self, key) -> None:
        if key != self.key or self.n_rows > self.MAX_ROWS:
            self.reset(key)

    def ensure(self, n_nodes: int, n_rows: int, n_slots: int) -> None:
        """Capacity for node ids < n_nodes, n_rows rows and n_slots slots (grown geometrically)."""
        if n_nodes > len(self.row_of):
            grow = np.full(max(2 * len(self.row_of), n_nodes), -1, np.int64)
            grow[:len(self.row_of)] = self.row_of
            self.row_of = grow
        nr, ns = self.R.shape
        if n_rows > nr or n_slots > ns:
            grow = np.full((max(nr, 2 * n_rows) if n_rows > nr else nr,
                            max(ns, 2 * n_slots) if n_slots > ns else ns), -1, np.int8)
            grow[:nr, :ns] = self.R
            self.R = grow

    def rows_for(self, nodes: np.ndarray, n_slots: int) -> np.ndarray:
        """Rows of the conjunct nodes (new rows numbered in order of first appearance)."""
        nodes = np.asarray(nodes, np.int64)
        if len(nodes) and int(nodes.max()) >= len(self.row_of):
            self.ensure(int(nodes.max()) + 1, 0, 0)
        out = self.row_of[nodes]
        new = out < 0
        if new.any():
            u, first = np.unique(nodes[new], return_index=True)
            u = u[np.argsort(first)]   # first-appearance order
            self.row_of[u] = self.n_rows + np.arange(len(u))
            self.n_rows += len(u)
            out = self.row_of[nodes]
        nr, ns = self.R.shape
        if self.n_rows > nr or n_slots > ns:
            grow = np.full((max(nr, 2 * self.n_rows) if self.n_rows > nr else nr,
                            max(ns, 2 * n_slots) if n_slots > ns else ns), -1, np.int8)
            grow[:nr, :ns] = self.R
            self.R = grow
        return out


class VerdictEngine:
    """Lowers conjunctions + candidate models and evaluates them on the GPU.

    ``rows(exprs, models)`` -> one ``bool[len(models)]`` verdict row per expression (``None`` =
    unsupported: fail closed).  Works on z3-free terms (:mod:`mythril_amd.smt`) and, on a z3 host,
    on z3 ``BoolRef``, translated once per AST into the same terms (:meth:`_rows_z3`).

    The drop-in path (the LRU's <= 100 models) keeps three things across calls:
    the hash-consed DAG of every lowered term, the candidate models' serialized rows (resident on
    the device in slot order, so an LRU bump re-uploads nothing), and per-conjunct verdict rows
    (:class:`ConjunctRows`).  A call evaluates only the conjuncts not yet known under the current
    models, one tape each, when there are at most ``conj_tapes`` of them; a batch of mostly new
    paths is evaluated as whole conjunctions instead (split into conjunct groups when small).

    ``timing`` accumulates host seconds per stage of every call (lower, serialize, upload,
    compile, evaluate = launch + readback) — the drop-in leg of bench.py reports it."""

    # batch-level hoisting pays off when the device work dominates: many conjunctions x many
    # candidates (generated candidates); at the LRU's <= 100 models the host stages dominate and
    # the incremental lowering (cached conjunct fragments and model rows) is used instead
    hoist_min_batch = 8
    hoist_min_models = 1024
    # a small batch of new paths leaves the GPU idle and a single conjunction is one wave's
    # serial walk over its ~1 000 nodes: its conjuncts are split into up to ``split_tapes // N``
    # contiguous groups, each its own tape (one wave each), and the group verdict rows are AND-ed.
    # Shared sub-terms are then re-evaluated per group — more work (and compile time), less
    # latency (profiles/r02lat*, r02sp); from N = 32 the compile cost outweighs it; 0 disables
    split_tapes = int(os.environ.get("MQ_SPLIT_TAPES", "32"))
    # at most this many unknown conjuncts are evaluated one tape each (and cached); more are
    # evaluated as whole conjunctions.  One tape per conjunct re-evaluates shared sub-terms per
    # conjunct, yet it measured no slower on batches of new paths either (one wave per short
    # tape; profiles/r03c) and it is what lets forked paths reuse their parents' rows, so the
    # default is unbounded.  0 disables the conjunct cache
    conj_tapes = int(os.environ.get("MQ_CONJ_TAPES", str(1 << 30)))
    # launches of at most this many waves run the G kernel one tape per wave (MQ_OPT_LATENCY_WAVES)
    latency_waves = int(os.environ.get("MQ_LATENCY_WAVES", "4096"))
    STAGES = ("lower", "serialize", "upload", "compile", "evaluate")
    # a compiled conjunct batch is launched again for a subset of its conjuncts up to this size
    REUSE_MAX = 4096

    def __init__(self, evaluator=None):
        from .lower import IncrementalLowering
        self._ev = evaluator
        self.launches = 0
        self.pairs = 0
        self.timing = dict.fromkeys(self.STAGES, 0.0)
        self.incremental = IncrementalLowering()
        self.conjuncts = ConjunctRows()
        self.stats = {"conjuncts_evaluated": 0, "conjuncts_cached": 0, "whole_query_batches": 0,
                      "conjunct_batches_reused": 0}
        self._resident = None   # (model key, evaluator upload_seq) of the batch on the device
        # the last compiled batch of conjunct tapes: (DAG generation, sorted roots, CompiledTapes).
        # A model inserted mid-batch (a solver answer, model.py:125) needs the still-pending
        # conjuncts under it alone; they are a subset of what the previous launch compiled, so
        # that compiled batch is launched again (all of it: the extra rows are cached too) instead
        # of compiling the subset (~4 ms per fill on the fork stream, profiles/r04k)
        self._conj_ct = None
        self._owner = threading.get_ident()   # the thread whose HIP context owns _conj_ct
        self._z3 = None   # lower_z3.Z3Terms of the z3 queries seen (created on the first one)

    @property
    def evaluator(self):
        if self._ev is None:
            from .evaluator import default_evaluator
            self._ev = default_evaluator()
        return self._ev

    def _lower(self, exprs, models, hoist: bool):
        """``(tapes, models, supported mask)`` of z3-free terms, for a whole-batch launch."""
        clock = time.perf_counter
        t0 = clock()
        if not hoist:
            inc = self.incremental
            tb, ok = inc.lower(exprs)
            t1 = clock()
            mb = inc.serialize(models)
        else:
            from .lower import lower_batch, serialize_models
            # states forked from a common parent share constraint prefixes: hoist what a batch
            # shares into once-per-model columns (lower.py lower_batch)
            records = [as_record(m) for m in models]
            tb, syms, ok = lower_batch(exprs, hoist=hoist)
            t1 = clock()
            mb = serialize_models(records, syms)
        self.timing["lower"] += t1 - t0
        self.timing["serialize"] += clock() - t1
        return tb, mb, ok

    def _rows_z3(self, exprs: Sequence, models: Sequence) -> List[Optional[np.ndarray]]:
        """z3 ``BoolRef`` queries (model.py:101 hands quick-sat ``simplify(And(*c)).raw``): each is
        translated into interned terms (:class:`mythril_amd.lower_z3.Z3Terms`, memoized by z3 AST
        id, so only ASTs never seen before are walked) and then takes the z3-free path — the
        persistent DAG, the resident model rows (each z3 model read once, when it gets its slot)
        and the per-conjunct verdict rows: the top-level ``And``'s children are the conjuncts, so
        a forked state's parent conjuncts and the keccak axioms are answered from cached rows.
        A query that does not translate is unsupported (``None``: the z3 loop answers it); a
        cached model whose interpretation is not literal makes the whole batch unsupported."""
        t0 = time.perf_counter()
        if self._z3 is None:
            from .lower_z3 import Z3Terms
            self._z3 = Z3Terms()
        out: List[Optional[np.ndarray]] = [None] * len(exprs)
        terms, idx = [], []
        for i, e in enumerate(exprs):
            if isinstance(e, S.Term):
                terms.append(e)
                idx.append(i)
                continue
            try:
                terms.append(self._z3.term(e))
                idx.append(i)
            except LoweringError as err:
                fail_closed_note(err)
        self.timing["lower"] += time.perf_counter() - t0
        if terms:
            try:
                rows = self.rows(terms, models)
            except LoweringError:
                return out
            for i, r in zip(idx, rows):
                out[i] = r
        return out

    @staticmethod
    def _latency_mode(ev, waves: Optional[int]) -> Optional[int]:
        """Set the evaluator's latency-mode threshold; returns the previous value (None: the
        evaluator has no such option).  ``waves=None`` leaves it unchanged."""
        if not hasattr(ev, "OPT_LATENCY_WAVES"):
            return None
        prev = ev.option(ev.OPT_LATENCY_WAVES) if hasattr(ev, "option") else 0
        if waves is not None:
            ev.set_option(ev.OPT_LATENCY_WAVES, waves)
        return prev

    def _compile(self, tb):
        """Device hook: the compiled batch ``_evaluate`` accepts in place of ``tb``."""
        return self.evaluator.compile(tb)

    @staticmethod
    def _free(ct) -> None:
        free = getattr(ct, "free", None)
        if free is not None:
            free()

    def close(self) -> None:
        """Free the device buffers this engine keeps across calls (the reused conjunct batch)."""
        prev, self._conj_ct = self._conj_ct, None
        if prev is not None:
            self._free(prev[2])

    def __del__(self):
        # libmq context calls are not thread-safe and the HIP device is per thread: a finalizer
        # run by another thread (a GC pass on the solver worker) only queues the buffer, which
        # the next engine call on the owning thread frees
        prev = getattr(self, "_conj_ct", None)
        if prev is None:
            return
        self._conj_ct = None
        if threading.get_ident() == getattr(self, "_owner", None):
            try:
                self._free(prev[2])
            except Exception:   # (interpreter shutdown: the library may be gone)
                pass
        else:
            _DEFERRED_FREES.append((self._owner, prev[2]))

    def _drain_deferred(self) -> None:
        if _DEFERRED_FREES:
            me = threading.get_ident()
            keep = []
            while _DEFERRED_FREES:
                owner, ct = _DEFERRED_FREES.pop()
                if owner == me:
                    self._free(ct)
                else:
                    keep.append((owner, ct))
            _DEFERRED_FREES.extend(keep)

    def _evaluate(self, tb, mb, upload: bool = True):
        """Device hook: (verdicts [n_tapes, M], first hits) of ``tb`` over ``mb``; ``upload``
        False when ``mb`` is already the evaluator's resident batch."""
        clock = time.perf_counter
        ev = self.evaluator
        t0 = clock()
        if upload:
            ev.upload_models(mb)
        t1 = clock()
        from .evaluator import CompiledTapes
        own = not isinstance(tb, CompiledTapes)   # (a compiled batch the caller keeps)
        ct = ev.compile(tb) if own else tb
        t2 = clock()
        prev = self._latency_mode(ev, self.latency_waves)
        try:
            v, fh = ev.verdicts(ct)
        finally:
            self._latency_mode(ev, prev)   # (the caller's own setting, not 0)
            if own:
                ct.free()
        self.timing["upload"] += t1 - t0
        self.timing["compile"] += t2 - t1
        self.timing["evaluate"] += clock() - t2
        return v, fh

    def _evaluate_resident(self, tb, slots):
        """``_evaluate`` over the models of ``slots`` (sorted), uploading them only when the
        evaluator no longer holds the batch this engine last uploaded for the same slots."""
        t0 = time.perf_counter()
        key = self.incremental.model_key(slots)
        seq = getattr(self._ev, "upload_seq", None)
        if self._resident is not None and self._resident[:2] == (key, seq) and seq is not None:
            mb, upload = self._resident[2], False
        else:
            mb, upload = self.incremental.batch_of_slots(slots), True
        self.timing["serialize"] += time.perf_counter() - t0
        v, fh = self._evaluate(tb, mb, upload)
        if upload:
            self._resident = (key, getattr(self._ev, "upload_seq", None), mb)
        return v, fh

    def candidate_first_hits(self, exprs: Sequence, models: Sequence, generator):
        """First hits of ``exprs`` over the LRU ``models`` followed by generated candidates (one
        launch): ``(int32[N] global indices / -1 / -2, CandidateSet)``.  z3-free terms only."""
        clock = time.perf_counter
        t0 = clock()
        inc = self.incremental
        db, ok = inc.lower(exprs)
        t1 = clock()
        cs = generator.generate(db, inc.syms, inc.serialize(models), models)
        t2 = clock()
        fh, t3, t4 = self._first_hit(db, cs.batch)
        self.timing["lower"] += t1 - t0
        self.timing["serialize"] += t2 - t1
        self.timing["upload"] += t3 - t2
        self.timing["compile"] += t4 - t3
        self.timing["evaluate"] += clock() - t4
        self.launches += 1
        self.pairs += len(exprs) * cs.batch.n_models
        fh = np.where(ok, fh, -2)
        return fh, cs

    def _first_hit(self, tb, mb):
        """Upload + compile + first-hit launch; returns (first hits, time after upload, time
        after compile)."""
        clock = time.perf_counter
        ev = self.evaluator
        ev.upload_models(mb)
        t3 = clock()
        ct = ev.compile(tb)
        t4 = clock()
        prev = self._latency_mode(ev, self.latency_waves)
        try:
            fh = ev.first_hit(ct)
        finally:
            self._latency_mode(ev, prev)
            ct.free()
        return fh, t3, t4

    def rows(self, exprs: Sequence, models: Sequence) -> List[Optional[np.ndarray]]:
        if not exprs:
            return []
        if not models:
            return [np.zeros(0, bool) for _ in exprs]
        self._drain_deferred()
        if not all(isinstance(e, S.Term) for e in exprs):
            return self._rows_z3(exprs, models)
        hoist = len(exprs) >= self.hoist_min_batch and len(models) >= self.hoist_min_models
        if not hoist and all(isinstance(e, S.Term) for e in exprs):
            return self._rows_incremental(exprs, models)
        tb, mb, ok = self._lower(exprs, models, hoist)
        try:
            v, fh = self._evaluate(tb, mb)
        except Exception:
            if getattr(tb, "columns", None) is None:
                raise
            # a column program the compiler rejects (mq_tapes_set_columns -> MQ_ERR_TAPE):
            # evaluate the batch without hoisting instead
            tb, mb, ok = self._lower(exprs, models, False)
            v, fh = self._evaluate(tb, mb)
        self._resident = None
        self.launches += 1
        self.pairs += len(exprs) * mb.n_models
        return [v[i].copy() if ok[i] and fh[i] != -2 else None for i in range(len(exprs))]

    def _rows_incremental(self, exprs: Sequence, models: Sequence) -> List[Optional[np.ndarray]]:
        clock = time.perf_counter
        inc = self.incremental
        t0 = clock()
        db, ok = inc.lower(exprs)
        t1 = clock()
        slots = np.asarray(inc.slots(models, live=getattr(self, "live_models", 0)), np.int64)
        dev_slots = sorted(set(slots.tolist()))
        self.timing["lower"] += t1 - t0
        self.timing["serialize"] += clock() - t1
        cache = self.conjuncts
        cache.sync((inc.dag_gen, inc.slot_epoch))
        from .lower import _walker
        walker = _walker()
        if walker is not None:
            return self._rows_incremental_native(walker, exprs, db, ok, slots, dev_slots)
        uroots, inv = np.unique(db.roots, return_inverse=True)
        urows = cache.rows_for(uroots, int(slots.max()) + 1)
        unk = (cache.R.take(urows, 0).take(slots, 1) < 0).any(axis=1)   # (take: 3x np.ix_)
        n_unk = int(unk.sum())
        self.stats["conjuncts_cached"] += int(len(uroots) - n_unk)
        if n_unk > self.conj_tapes:
            return self._rows_whole(db, ok, slots, dev_slots, len(exprs))
        if n_unk:
            self._conjunct_launch(db, uroots[unk], slots, dev_slots)
        # each query: the AND of its conjuncts' rows, in the caller's model order
        occ = (cache.R.take(urows, 0).take(slots, 1) > 0)[inv]
        offs = db.root_offsets
        lens = np.diff(offs)
        rows = np.ones((len(exprs), len(slots)), bool)   # And() of nothing: true
        full = lens > 0
        if full.any():
            # (the segments of the non-empty queries, back to back: empty ones add no conjuncts)
            rows[full] = np.logical_and.reduceat(occ, offs[:-1][full], axis=0)
        bad = cache.bad
        out: List[Optional[np.ndarray]] = list(rows)
        for q in np.flatnonzero(~np.asarray(ok, bool)).tolist():
            out[q] = None
        if bad:
            for q in range(len(exprs)):
                if out[q] is not None and any(int(x) in bad for x in db.roots[offs[q]:offs[q + 1]]):
                    out[q] = None
        return out

    def _conjunct_launch(self, db, todo: np.ndarray, slots: np.ndarray, dev_slots) -> np.ndarray:
        """Evaluate the unknown conjuncts ``todo`` (one tape each, one launch) under the models of
        ``dev_slots`` and store their verdict rows; returns the conjunct nodes evaluated (a reused
        compiled batch: a superset of ``todo``)."""
        from .lower import DagBatch
        clock = time.perf_counter
        inc, cache = self.incremental, self.conjuncts
        n_unk = len(todo)
        prev = self._conj_ct
        # (the evaluator that compiled it is part of the key: a batch is bound to its context)
        gen = (inc.dag_gen, inc.slot_epoch, id(self._ev))
        # (a superset launch costs device microseconds per extra conjunct; compiling the subset
        # costs ~1 ms: reuse while the superset is at most REUSE_MAX conjuncts)
        if prev is not None and prev[0] == gen and len(prev[1]) <= max(4 * n_unk + 64, self.REUSE_MAX) and \
                prev[3].issuperset(todo.tolist()):
            todo, ct = prev[1], prev[2]
            self.stats["conjunct_batches_reused"] += 1
        else:
            if prev is not None:
                self._free(prev[2])
                self._conj_ct = None
            tb = DagBatch(db.nodes, db.consts, np.arange(n_unk + 1, dtype=np.int64), todo)
            t2 = clock()
            ct = self._compile(tb)
            self.timing["compile"] += clock() - t2
            self._conj_ct = (gen, todo, ct, set(todo.tolist()))
        v, fh = self._evaluate_resident(ct, dev_slots)
        trows = cache.rows_for(todo, int(slots.max()) + 1)
        cache.R[np.ix_(trows, np.asarray(dev_slots, np.int64))] = v.astype(np.int8)
        for x in todo[fh == -2].tolist():
            cache.bad.add(int(x))
        self.stats["conjuncts_evaluated"] += len(todo)
        self.launches += 1
        self.pairs += len(todo) * len(dev_slots)
        return todo

    def _rows_incremental_native(self, walker, exprs, db, ok, slots, dev_slots) -> List[Optional[np.ndarray]]:
        """``_rows_incremental``'s bookkeeping in the host extension (csrc/lowerwalk.cpp
        conj_rows / conj_answer): the conjuncts' rows, the unknown ones, and each query's AND of
        its conjuncts' rows in the caller's model order — a few calls instead of ~30 numpy ones
        per batch (the drop-in path's fixed cost at the reference's shape)."""
        cache = self.conjuncts
        roots = db.roots
        n = len(roots)
        cache.ensure(int(roots.max()) + 1 if n else 0, cache.n_rows + n, int(slots.max()) + 1)
        rows = np.empty(n, np.int64)
        cache.n_rows, todo = walker.conj_rows(roots, cache.row_of, cache.n_rows, cache.R, slots, rows)
        n_unk = len(todo)
        self.stats["conjuncts_cached"] += len(set(roots.tolist())) - n_unk
        if n_unk > self.conj_tapes:
            return self._rows_whole(db, ok, slots, dev_slots, len(exprs))
        if n_unk:
            self._conjunct_launch(db, np.asarray(todo, np.int64), slots, dev_slots)
        out_b = np.empty((len(exprs), len(slots)), np.uint8)
        walker.conj_answer(cache.R, rows, db.root_offsets, slots, out_b)
        out: List[Optional[np.ndarray]] = list(out_b.view(bool))
        if not ok.all():
            for q in np.flatnonzero(~np.asarray(ok, bool)).tolist():
                out[q] = None
        bad = cache.bad
        if bad:
            offs = db.root_offsets
            for q in range(len(exprs)):
                if out[q] is not None and any(int(x) in bad for x in roots[offs[q]:offs[q + 1]]):
                    out[q] = None
        return out

    def _rows_whole(self, db, ok, slots, dev_slots, n_exprs) -> List[Optional[np.ndarray]]:
        """Whole conjunctions, one tape each (a small batch: conjunct groups, rows AND-ed), on the
        resident model batch; nothing is cached per conjunct."""
        tb, starts = db, None
        if self.split_tapes:
            tb, starts = split_conjuncts(db, self.split_tapes // n_exprs)
        v, fh = self._evaluate_resident(tb, dev_slots)
        if starts is not None:
            v = np.logical_and.reduceat(v, starts, axis=0)
            fh = np.where(np.minimum.reduceat(fh, starts) == -2, -2, 0)
        pos = {s: i for i, s in enumerate(dev_slots)}
        v = v[:, [pos[s] for s in slots.tolist()]]
        self.stats["whole_query_batches"] += 1
        self.launches += 1
        self.pairs += n_exprs * len(dev_slots)   # (queries, not the conjunct groups split_conjuncts made)
        return [v[i].copy() if ok[i] and fh[i] != -2 else None for i in range(n_exprs)]


_UNSUPPORTED = object()
# (owner thread, compiled batch) freed by the next engine call on that thread (VerdictEngine.__del__)
_DEFERRED_FREES: List[Tuple[int, object]] = []


# ---------------------------------------------------------------------------- ModelCache
class ModelCache:
    """support_utils.py:56-70 with the GPU verdict engine behind ``check_quick_sat``."""

    MEMO_SIZE = 2 ** 10   # @lru_cache(maxsize=2**10) on check_quick_sat (support_utils.py:60)
    LOOKAHEAD_MIN = 4     # pending conjunctions a late fill always carries besides its query

    def __init__(self, engine: Optional[VerdictEngine] = None):
        self.model_cache = LRUCache(size=100)
        self.engine = engine or VerdictEngine()
        # expr -> int8 verdict row over model slots (-1: not evaluated yet) for conjunctions
        # evaluated ahead of their check_quick_sat call, or _UNSUPPORTED
        self._rows: Dict[object, object] = {}
        self._slot: Dict[int, int] = {}      # id(model) -> slot of the rows above
        self._slot_model: List[object] = []  # keeps those models (and their ids) alive
        self._order_v = None                 # (LRU version, MRU-first order, its slots)
        self._pending: "OrderedDict[object, None]" = OrderedDict()
        # the memo of check_quick_sat: functools.lru_cache semantics (a hit moves to MRU, the LRU
        # entry is evicted past MEMO_SIZE, exceptions are not cached), kept as a dict so prefetch
        # can tell which conjunctions will never reach the evaluator again
        self._memo: "OrderedDict[object, object]" = OrderedDict()
        self._cand: Dict[object, object] = {}   # prefetched generated-candidate answers
        self.stats = {"queries": 0, "hits": 0, "unsupported": 0,
                      # launches for models a query found unevaluated (a solver model inserted
                      # since its prefetch), and the conjunctions they carried
                      "late_fills": 0, "late_fill_exprs": 0}
        # pending conjunctions that ride along when a query meets a model inserted after their
        # prefetch: doubles while late fills keep serving later queries, reset when a query
        # arrives after another insertion (on a fork stream nearly every miss inserts a model,
        # and evaluating every pending conjunction per insertion was the per-state cost)
        self._lookahead = 0
        self._served_since_fill = 0

    def check_quick_sat(self, constraints):
        """support_utils.py:60-67, memoized per ``(self, constraints)`` like the reference's
        ``@lru_cache(maxsize=2**10)``: a memoized ``False`` or model is returned again without
        re-evaluation and without an LRU bump."""
        memo = self._memo
        if constraints in memo:
            memo.move_to_end(constraints)
            return memo[constraints]
        result = self._check_quick_sat(constraints)
        memo[constraints] = result
        if len(memo) > self.MEMO_SIZE:
            memo.popitem(last=False)
        return result

    def _order(self):
        """The candidate order (MRU first, support_utils.py:62) and its row slots, recomputed
        only when the LRU changed."""
        lru = self.model_cache
        if not self._rows and len(self._slot_model) > 4 * lru.size + 256:
            # no pending row refers to a slot: forget the models that left the cache
            self._slot, self._slot_model, self._order_v = {}, [], None
        if self._order_v is None or self._order_v[0] != lru.version or len(self._order_v[1]) != len(lru.lru_cache):
            order = list(reversed(lru.lru_cache.keys()))
            self._order_v = (lru.version, order, self._slots_of(order))
        return self._order_v[1], self._order_v[2]

    def _slots_of(self, models) -> np.ndarray:
        slot, keep = self._slot, self._slot_model
        try:
            # every model seen before (the LRU reordered after a hit): keep holds each model with
            # a slot alive, so no other object can carry its id
            return np.fromiter(map(slot.__getitem__, map(id, models)), np.int64, len(models))
        except KeyError:
            pass
        out = np.empty(len(models), np.int64)
        for i, m in enumerate(models):
            s = slot.get(id(m))
            if s is None or keep[s] is not m:
                s = slot[id(m)] = len(keep)
                keep.append(m)
            out[i] = s
        return out

    def _check_quick_sat(self, constraints):
        self.stats["queries"] += 1
        order, slots = self._order()
        row = self._verdicts(constraints, order, slots)
        if row is _UNSUPPORTED:
            self.stats["unsupported"] += 1
            self._record(constraints, order, -2)
            return self._fallback(constraints, order)
        i = int(np.argmax(row)) if len(row) else 0
        if len(row) and row[i]:
            model = order[i]
            self._record(constraints, order, i)
            self.model_cache.put(model, self.model_cache.get(model) + 1)
            self.stats["hits"] += 1
            return model
        self._record(constraints, order, -1)
        return False

    recorder = None  # corpus.Recorder: harvest every evaluated query (enable_dump)

    def _record(self, constraints, order, answer: int) -> None:
        if self.recorder is not None and order:
            self.recorder.record(constraints, order, answer)

    def put(self, key, value) -> None:
        self.model_cache.put(key, value)

    # -------------------------------------------------------------- batching
    def prefetch(self, exprs: Iterable) -> None:
        """Evaluate pending conjunctions against the current cache in one launch (a10).
        Conjunctions the memo already answers never reach the evaluator again: they are skipped."""
        exprs = [e for e in dict.fromkeys(exprs) if e not in self._rows and e not in self._memo]
        order, slots = self._order()
        for e in exprs:
            self._rows[e] = self._empty_row()
            self._pending[e] = None
        if exprs and order:
            self._fill(exprs, order, slots)

    # -------------------------------------------------------------- generated candidates
    def candidates(self, exprs: Sequence) -> list:
        """Verdict-only extension (``Args.quick_sat_candidates``): for conjunctions quick-sat did
        not answer, search the LRU models followed by up to ``quick_sat_candidate_budget``
        generated candidates in ONE launch.  Returns per expression a satisfying model (an LRU
        model, or a generated candidate materialized as a Model: never inserted into the cache)
        or False.  get_model caches a candidate answer in the LRU as the solver's model would be
        (model.py:125), so the model differs from z3's: see INTEGRATION.md, "Generated candidates"."""
        from .candidates import CandidateGenerator
        exprs = list(exprs)
        out = [False] * len(exprs)
        todo = [i for i, e in enumerate(exprs) if isinstance(e, S.Term)]
        if not todo:
            return out
        order = list(reversed(self.model_cache.lru_cache.keys()))
        gen = CandidateGenerator(args.quick_sat_candidate_budget, seed=len(self.stats) + self.stats["queries"])
        fh, cs = self.engine.candidate_first_hits([exprs[i] for i in todo], order, gen)
        for i, h in zip(todo, fh):
            if h < 0:
                continue
            out[i] = order[h] if h < cs.n_lru else cs.materialize(int(h))
            self.stats["candidate_hits"] = self.stats.get("candidate_hits", 0) + 1
        return out

    def prefetch_candidates(self, exprs: Iterable) -> None:
        """Batch form: the candidates search of every conjunction the prefetched LRU rows already
        show as a miss, in one launch; consumed by :meth:`candidate_for`."""
        miss = []
        for e in dict.fromkeys(exprs):
            d = self._rows.get(e)
            if isinstance(d, np.ndarray) and (d >= 0).any() and not (d > 0).any() and e not in self._cand:
                miss.append(e)
        for e, r in zip(miss, self.candidates(miss)):
            self._cand[e] = r

    def candidate_for(self, expr):
        """A generated candidate satisfying ``expr`` (a quick-sat miss), or False.  A miss the
        batch prefetch did not foresee (its LRU hit was evicted by a model inserted meanwhile) is
        searched together with up to 63 other pending conjunctions not searched yet, whose answers
        wait in the prefetch table (a candidate is any satisfying model: an older LRU order as its
        base changes which one is found, never whether it satisfies)."""
        if expr in self._cand:
            return self._cand.pop(expr)
        more = [e for e in self._pending if e is not expr and e not in self._cand and isinstance(e, S.Term)][:63]
        res = self.candidates([expr] + more)
        for e, r in zip(more, res[1:]):
            self._cand[e] = r
        return res[0]

    def discard(self, exprs: Iterable) -> None:
        """Forget prefetched rows of conjunctions whose check_quick_sat never ran (their answer
        came from get_model's own memo): they must not ride along in later launches."""
        for e in exprs:
            self._rows.pop(e, None)
            self._pending.pop(e, None)

    def check_quick_sat_batch(self, exprs: Sequence) -> list:
        """``[check_quick_sat(e) for e in exprs]`` with one GPU launch for the whole batch."""
        self.prefetch(exprs)
        try:
            return [self.check_quick_sat(e) for e in exprs]
        finally:
            self.discard(exprs)

    def _empty_row(self) -> np.ndarray:
        return np.full(max(len(self._slot_model), 16), -1, np.int8)

    def _fill(self, exprs: List, models: List, slots: np.ndarray) -> None:
        # the engine's model slots outlive a batch: tell it how many models stay candidates (the
        # LRU's capacity), so it does not start its slots over every few hundred solver models
        self.engine.live_models = max(getattr(self.engine, "live_models", 0), self.model_cache.size)
        rows = self.engine.rows(exprs, models)
        n = len(self._slot_model)
        for e, r in zip(exprs, rows):
            d = self._rows[e]
            if d is _UNSUPPORTED:
                continue
            if r is None:
                self._rows[e] = _UNSUPPORTED
                continue
            if len(d) < n:
                d = self._rows[e] = np.concatenate([d, np.full(max(n, 2 * len(d)) - len(d), -1, np.int8)])
            d[slots] = r

    def _verdicts(self, expr, order, slots):
        if expr not in self._rows:
            self._rows[expr] = self._empty_row()
            self._pending[expr] = None
        d = self._rows[expr]
        if d is not _UNSUPPORTED:
            got = d[slots] if slots.size and int(slots.max()) < len(d) else None
            if got is None or (got < 0).any():
                # the query, and the next few pending conjunctions, against the models it has not
                # seen, in one launch; the window grows while such fills keep answering later
                # queries and shrinks to the query alone when models keep arriving in between
                known = np.zeros(len(slots), bool) if got is None else got >= 0
                miss = np.flatnonzero(~known)
                self._lookahead = max(self.LOOKAHEAD_MIN, 2 * self._served_since_fill)
                batch = [expr]
                for e in self._pending:
                    if len(batch) > self._lookahead:
                        break
                    if e is not expr and self._rows.get(e) is not _UNSUPPORTED:
                        batch.append(e)
                self._fill(batch, [order[i] for i in miss], slots[miss])
                self.stats["late_fills"] += 1
                self.stats["late_fill_exprs"] += len(batch)
                self._served_since_fill = 0
                d = self._rows[expr]
            else:
                self._served_since_fill += 1
        self._rows.pop(expr, None)
        self._pending.pop(expr, None)
        if d is _UNSUPPORTED:
            return _UNSUPPORTED
        return d[slots] > 0

    def _fallback(self, constraints, order):
        """Unsupported conjunction: the reference's own loop where z3 exists, else no quick answer."""
        if isinstance(constraints, S.Term):
            return False
        from .lower_z3 import z3_quick_sat_loop
        model = z3_quick_sat_loop(constraints, order)
        if model is not False:
            self.model_cache.put(model, self.model_cache.get(model) + 1)
        return model


# ---------------------------------------------------------------------------- model.py
class SolverBackend:
    """What ``solver_worker`` needs from an SMT solver (model.py:28-65): ``solve`` returns
    ``(status, model_factory)`` with status in {"sat", "unsat", "unknown"} and ``model_factory()``
    producing a fresh model object (``s.model()``, called twice at model.py:125-126)."""

    def solve(self, constraints, minimize, maximize, timeout_ms) -> Tuple[str, Optional[Callable]]:
        raise NotImplementedError


class NoSolver(SolverBackend):
    """No SMT solver available (this container / the GPU box have no z3): every miss is
    ``unknown`` -> SolverTimeOutException, i.e. what the reference does when z3 gives up."""

    def solve(self, constraints, minimize, maximize, timeout_ms):
        return "unknown", None


class WitnessSolver(SolverBackend):
    """A stand-in SMT solver for states whose satisfying model is known in advance (synthetic
    streams, synth_evm.fork_stream_workload): ``sat`` with that witness, which get_model caches
    in the LRU as it caches z3's model (model.py:124-126); ``unknown`` for any other state.  So
    a benchmark without z3 keeps the reference's insertion semantics on every miss."""

    def __init__(self, states: Sequence, witnesses: Sequence):
        self.known = {frozenset(c for c in st if c.kind != S.TRUE): w for st, w in zip(states, witnesses) if w is not None}
        self.calls = 0
        self.sat_calls = 0   # calls answered sat: each inserts its model into the LRU

    def solve(self, constraints, minimize, maximize, timeout_ms):
        self.calls += 1
        w = self.known.get(frozenset(c for c in constraints if c.kind != S.TRUE))
        if w is None:
            return "unknown", None
        self.sat_calls += 1
        return "sat", lambda: w


def _default_backend() -> SolverBackend:
    try:
        from .lower_z3 import Z3Backend
        return Z3Backend()
    except ImportError:
        return NoSolver()


model_cache = ModelCache()
solver_backend: SolverBackend = None  # type: ignore[assignment]
counters = {"get_model_calls": 0, "quick_sat_answers": 0, "candidate_answers": 0, "solver_calls": 0}
# host seconds of get_model's solver path: the worker-thread hand-off around the solver
# (model.py:104-113) and the solver itself
timing = {"solver_pool": 0.0}

# model.py:104-113 creates a ThreadPool(1) per solver call and terminates it afterwards (~0.7 ms of
# thread start-up per call).  The solver runs on one persistent worker instead; a call that times
# out or raises discards that worker (as terminate() does), so a hung solver never blocks the next
# call.  Answers, exceptions and timeouts are the reference's.
_solver_pool: Optional[ThreadPool] = None
_solver_pool_pid = None


def _pool() -> ThreadPool:
    global _solver_pool, _solver_pool_pid
    if _solver_pool is None or _solver_pool_pid != os.getpid():   # (a forked child starts its own)
        _solver_pool, _solver_pool_pid = ThreadPool(1), os.getpid()
    return _solver_pool


def _discard_pool() -> None:
    global _solver_pool
    if _solver_pool is not None:
        _solver_pool.terminate()
    _solver_pool = None


def set_solver_backend(backend: Optional[SolverBackend]) -> None:
    global solver_backend
    solver_backend = backend


def solver_worker(constraints, minimize=(), maximize=(), solver_timeout=None):
    """model.py:28-65 (the ``--solver-log`` dump is the harvest hook of :mod:`mythril_amd.corpus`)."""
    backend = solver_backend or _default_backend()
    return backend.solve(constraints, minimize, maximize, solver_timeout)


def simplify(expr):
    """``simplify`` (smt/expression.py:64-71).  Lowering does not depend on z3's rewrites
    (equivalence-preserving), so on z3-free terms this is the identity."""
    return expr


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), solver_timeout=None, verdict_only=False):
    """model.py:68-130.  ``verdict_only`` (build extension, default off): the caller only uses
    whether a model exists (``Constraints.is_possible``); with ``Args.quick_sat_candidates`` a
    quick-sat miss then also tries generated candidates before the solver."""
    counters["get_model_calls"] += 1
    asked, asked_timeout = constraints, solver_timeout
    solver_timeout = solver_timeout or args.solver_timeout
    solver_timeout = min(solver_timeout, time_handler.time_remaining())
    if solver_timeout <= 0:
        raise SolverTimeOutException
    for constraint in constraints:
        if isinstance(constraint, bool) and not constraint:
            raise UnsatError
    if not isinstance(constraints, tuple):
        constraints = constraints.get_all_constraints()
    constraints = [c for c in constraints if not isinstance(c, bool)]

    if len(maximize) + len(minimize) == 0:
        ret_model = model_cache.check_quick_sat(simplify(S.And(*constraints)))
        # the reference's cached models are mythril ``Model`` wrappers (smt/model.py:6-18), which
        # define neither __len__ nor __bool__: any model is truthy, exactly like ours
        if ret_model:
            counters["quick_sat_answers"] += 1
            return ret_model
        if verdict_only and args.quick_sat_candidates:
            cand = model_cache.candidate_for(simplify(S.And(*constraints)))
            if cand is not False:
                counters["candidate_answers"] += 1
                # the candidate stands in for the solver's sat answer, and is cached as that
                # answer would be (model.py:125): later quick-sat queries see it in the LRU
                model_cache.put(cand, 1)
                return cand
            # a candidate miss goes to the solver under the plain get_model key, so that a later
            # Constraints.get_model() of the same state finds the answer in this memo as the
            # reference's would (the verdict-only key is an extension the reference does not have)
            counters["get_model_calls"] -= 1
            # (same call form as Constraints.get_model: lru_cache keys depend on it)
            return get_model(asked, solver_timeout=asked_timeout)
    counters["solver_calls"] += 1
    t_pool = time.perf_counter()
    ok = False
    try:
        res = _pool().apply_async(solver_worker, args=(constraints, minimize, maximize, solver_timeout))
        try:
            # model.py:110 hands the millisecond timeout to AsyncResult.get(), which reads it as
            # seconds: the pool wait never pre-empts the solver's own timeout.  Kept as is.
            status, factory = res.get(None if math.isinf(solver_timeout) else solver_timeout)
            ok = True
        except _PoolTimeout:
            status, factory = "unknown", None
        except Exception:
            log.warning("Encountered an exception while solving expression")
            status, factory = "unknown", None
    finally:
        if not ok:
            _discard_pool()
        timing["solver_pool"] += time.perf_counter() - t_pool

    if status == "sat":
        model_cache.model_cache.put(factory(), 1)
        return factory()
    if status == "unknown":
        raise SolverTimeOutException
    raise UnsatError


# ---------------------------------------------------------------------------- constraints.py
class Constraints(list):
    """``Constraints`` (mythril/laser/ethereum/state/constraints.py:12-131) over z3-free terms."""

    def __init__(self, constraint_list=None):
        super().__init__(self._get_smt_bool_list(constraint_list or []))

    def is_possible(self, solver_timeout=None) -> bool:
        """constraints.py:28-43: a timeout under the default timeout prunes the state."""
        try:
            if args.quick_sat_candidates:
                get_model(self, solver_timeout=solver_timeout, verdict_only=True)
            else:
                get_model(self, solver_timeout=solver_timeout)
        except SolverTimeOutException:
            return solver_timeout is not None
        except UnsatError:
            return False
        return True

    def get_model(self, solver_timeout=None):
        try:
            return get_model(self, solver_timeout=solver_timeout)
        except UnsatError:  # includes SolverTimeOutException
            return None

    def append(self, constraint) -> None:
        super().append(simplify(constraint) if isinstance(constraint, S.Term) else S.BoolVal(constraint))

    @property
    def as_list(self):
        return self.get_all_constraints()

    def get_all_constraints(self):
        from .function_managers import keccak_function_manager
        return self[:] + [keccak_function_manager.create_conditions()]

    def __copy__(self):
        return Constraints(list.copy(self))

    def copy(self):
        return self.__copy__()

    def __deepcopy__(self, memodict=None):
        return Constraints(list(self))  # terms are immutable and interned

    def __add__(self, constraints):
        return Constraints(list(self) + self._get_smt_bool_list(constraints))

    def __iadd__(self, constraints):
        super().__iadd__(self._get_smt_bool_list(constraints))
        return self

    @staticmethod
    def _get_smt_bool_list(constraints):
        return [c if isinstance(c, S.Term) else S.BoolVal(c) for c in constraints]

    def __hash__(self):
        return tuple(self[:]).__hash__()


def quick_sat_expr(constraints) -> Optional[S.Term]:
    """The conjunction ``get_model`` hands to quick-sat for ``constraints`` (model.py:92-101),
    or None when get_model would not reach quick-sat (a Python ``False`` constraint)."""
    for c in constraints:
        if isinstance(c, bool) and not c:
            return None
    cs = constraints if isinstance(constraints, tuple) else constraints.get_all_constraints()
    return simplify(S.And(*[c for c in cs if not isinstance(c, bool)]))


def is_possible_batch(states: Sequence[Constraints], solver_timeout=None) -> List[bool]:
    """Batched ``[c.is_possible(solver_timeout) for c in states]`` — the per-transaction
    reachability loop (svm.py:278-283) and per-fork pruning (svm.py:351-358) with one GPU launch
    for all quick-sat queries.  Answers are identical to the sequential loop (see module doc)."""
    exprs = [e for e in (quick_sat_expr(c) for c in states) if e is not None]
    model_cache.prefetch(exprs)
    if args.quick_sat_candidates:
        model_cache.prefetch_candidates(exprs)
    try:
        return [c.is_possible(solver_timeout=solver_timeout) for c in states]
    finally:
        # a state whose get_model call was answered by get_model's own memo never reached
        # check_quick_sat: drop its prefetched row so it does not ride along in later launches
        model_cache.discard(exprs)
        for e in exprs:
            model_cache._cand.pop(e, None)


def enable_dump(directory: Optional[str]) -> None:
    """Harvest hook next to ``--solver-log`` (model.py:51-62): record every quick-sat query of the
    process-global cache into ``directory`` (mythril_amd.corpus format); None disables it."""
    from .corpus import Recorder
    model_cache.recorder = Recorder(directory) if directory else None


def reset_caches() -> None:
    """Tests only: clear both memo layers and the candidate cache (the reference never does)."""
    global model_cache
    get_model.cache_clear()
    engine = model_cache.engine
    engine.close()
    model_cache = ModelCache(engine)
    for k in counters:
        counters[k] = 0
    for k in timing:
        timing[k] = 0.0
