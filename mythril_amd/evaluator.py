"""ctypes binding of libmq.so — the MI355X quick-sat evaluator (include/mq.h).

This is the product path: there is no CPU fallback.  If ``libmq.so`` is missing or no
gfx950 device is present, constructing :class:`Evaluator` raises :class:`EvaluatorError`
(the ``get_model`` adapter then keeps the reference behaviour of going to z3 — it never
evaluates tapes on the CPU).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from ._abi import MqDagBatch, MqModelBatch, MqNode, MqStats, MqTapeBatch, as_dag_batch, as_model_batch, as_tape_batch
from .models import ModelBatch
from .tape import TapeBatch

# MQ_LIB: another build of the library (diagnostic A/B runs of generator variants)
LIB_PATH = os.environ.get("MQ_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmq.so")
NO_HIT = -1
UNSUPPORTED = -2

_lib = None
_lib_lock = threading.Lock()


class EvaluatorError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load libmq.so (built in-tree by ``python -m mythril_amd.build``); raises if absent."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise EvaluatorError(f"{path} not built: run `python -m mythril_amd.build` (hipcc, gfx950)")
        L = C.CDLL(path)
        P = C.c_void_p
        L.mq_version.restype = C.c_char_p
        L.mq_strerror.argtypes = [C.c_int]
        L.mq_strerror.restype = C.c_char_p
        L.mq_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(P)]
        L.mq_ctx_destroy.argtypes = [P]
        L.mq_ctx_destroy.restype = None
        L.mq_models_upload.argtypes = [P, C.POINTER(MqModelBatch)]
        L.mq_tapes_upload.argtypes = [P, C.POINTER(MqTapeBatch), C.POINTER(P), C.POINTER(C.c_int32)]
        L.mq_tapes_free.argtypes = [P]
        L.mq_tapes_free.restype = None
        L.mq_eval_first_hit.argtypes = [P, C.POINTER(MqTapeBatch), C.POINTER(C.c_int32), C.POINTER(MqStats)]
        L.mq_eval_tapes_first_hit.argtypes = [P, P, C.POINTER(C.c_int32), C.POINTER(MqStats)]
        L.mq_launch_first_hit.argtypes = [P, P, P, P]
        L.mq_finalize_first_hit.argtypes = [P, P, P, P]
        L.mq_counters.argtypes = [P, C.POINTER(C.c_double), C.c_int]
        L.mq_ctx_set_option.argtypes = [P, C.c_int, C.c_int]
        L.mq_kernel_times.argtypes = [P, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_int32), C.c_int]
        L.mq_kernel_times_device.argtypes = [P, C.c_int32, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_int32),
                                             C.c_int]
        L.mq_launch_times.argtypes = [P, C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                      C.c_int32, C.POINTER(C.c_int32), C.c_int]
        L.mq_host_times.argtypes = [P, C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_int32), C.c_int]
        L.mq_tapes_info.argtypes = [P] + [C.POINTER(C.c_int32)] * 3
        L.mq_tapes_qsa_split.argtypes = [P] + [C.POINTER(C.c_int32)] * 3
        L.mq_tapes_column_split.argtypes = [P] + [C.POINTER(C.c_int32)] * 2
        L.mq_tapes_flat_split.argtypes = [P] + [C.POINTER(C.c_int32)] * 2
        L.mq_tapes_column_keccak.argtypes = [P, C.POINTER(C.c_int32)]
        L.mq_tapes_column_gather.argtypes = [P, C.POINTER(C.c_int32)]
        L.mq_tapes_qsa_histogram.argtypes = [P, C.c_int32, C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_int64),
                                             C.POINTER(C.c_int32)]
        L.mq_qsa_kind_name.argtypes = [C.c_int32]
        L.mq_qsa_kind_name.restype = C.c_char_p
        L.mq_qsa_profile.argtypes = [P, C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_int32), C.c_int]
        L.mq_eval_verdicts.argtypes = [P, C.POINTER(MqTapeBatch), C.POINTER(C.c_uint8), C.POINTER(C.c_int32)]
        L.mq_eval_tapes_verdicts.argtypes = [P, P, C.POINTER(C.c_uint8), C.POINTER(C.c_int32)]
        L.mq_tapes_set_columns.argtypes = [P, C.POINTER(MqTapeBatch), C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int32]
        L.mq_keccak256.argtypes = [P, C.POINTER(C.c_uint8), C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_uint8)]
        L.mq_keccak256_host.argtypes = [C.POINTER(C.c_uint8), C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_uint8)]
        L.mq_tape_alg_ops.argtypes = [C.POINTER(MqTapeBatch), C.c_int32]
        L.mq_tape_alg_ops.restype = C.c_double
        L.mq_tape_compile_info.argtypes = [C.POINTER(MqTapeBatch), C.c_int32] + [C.POINTER(C.c_int32)] * 5 + [C.c_char_p, C.c_int32]
        L.mq_tapes_column_keccak_predicates.argtypes = [P, C.POINTER(C.c_int32)]
        L.mq_tape_compile_info_g.argtypes = [C.POINTER(MqTapeBatch), C.c_int32] + [C.POINTER(C.c_int32)] * 3
        L.mq_tape_program.argtypes = [C.POINTER(MqTapeBatch), C.c_int32, C.POINTER(C.c_uint32), C.c_int32, C.POINTER(C.c_int32)]
        L.mq_tapes_upload_dag.argtypes = [P, C.POINTER(MqDagBatch), C.POINTER(P), C.POINTER(C.c_int32)]
        L.mq_dag_expand.argtypes = [C.POINTER(MqDagBatch), C.c_int32, P, C.c_int64, C.POINTER(C.c_int64)]
        L.mq_models_shard.argtypes = [C.POINTER(MqModelBatch), C.c_int64, C.c_int64, C.POINTER(MqModelBatch), C.POINTER(P)]
        L.mq_models_shard_free.argtypes = [P]
        L.mq_models_shard_free.restype = None
        _lib = L
        return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load_library().mq_strerror(rc).decode()
        raise EvaluatorError(f"{what}: {msg} ({rc})")


@dataclass
class EvalStats:
    kernel_ms: float
    node_evals: float
    alg_ops: float
    pairs_evaluated: int
    n_hits: int
    n_unsupported: int


@dataclass
class CompileInfo:
    supported: bool
    limbs: int
    depth: int
    n_temps: int
    prog_words: int
    why: str


def keccak256_host(messages: Sequence[bytes]) -> List[bytes]:
    """keccak256 of each message through the library's host path (``mq_keccak256_host``: what
    ``Evaluator.keccak256`` runs for small batches); no GPU needed."""
    msgs = [bytes(m) for m in messages]
    offs = np.zeros(len(msgs) + 1, np.int64)
    offs[1:] = np.cumsum([len(m) for m in msgs])
    data = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
    out = np.zeros(32 * len(msgs), np.uint8)
    _check(load_library().mq_keccak256_host(data.ctypes.data_as(C.POINTER(C.c_uint8)), offs.ctypes.data_as(C.POINTER(C.c_int64)),
                                            len(msgs), out.ctypes.data_as(C.POINTER(C.c_uint8))), "mq_keccak256_host")
    return [bytes(out[32 * i:32 * i + 32]) for i in range(len(msgs))]


def compile_info(tb: TapeBatch, t: int) -> CompileInfo:
    """Host-only report of how tape t compiles (no GPU needed)."""
    L = load_library()
    s, keep = as_tape_batch(tb)
    vals = [C.c_int32() for _ in range(5)]
    why = C.create_string_buffer(256)
    _check(L.mq_tape_compile_info(C.byref(s), t, *[C.byref(v) for v in vals], why, 256), "compile_info")
    return CompileInfo(bool(vals[0].value), vals[1].value, vals[2].value, vals[3].value, vals[4].value, why.value.decode())


def compile_info_g(tb: TapeBatch, t: int):
    """Host-only: (depth, LDS temps, program words) of the program the G assembly interpreter
    runs for tape t (mq_tape_compile_info_g: subtrees deeper than its stack spilled to temps)."""
    L = load_library()
    s, keep = as_tape_batch(tb)
    vals = [C.c_int32() for _ in range(3)]
    _check(L.mq_tape_compile_info_g(C.byref(s), t, *[C.byref(v) for v in vals]), "compile_info_g")
    return tuple(v.value for v in vals)


def tape_program(tb: TapeBatch, t: int) -> np.ndarray:
    """Host-only: the compiled stack program of tape t (gprog.h words), for inspection/tests."""
    L = load_library()
    s, keep = as_tape_batch(tb)
    n = C.c_int32()
    _check(L.mq_tape_program(C.byref(s), t, None, 0, C.byref(n)), "tape_program")
    out = np.zeros(n.value, np.uint32)
    _check(L.mq_tape_program(C.byref(s), t, out.ctypes.data_as(C.POINTER(C.c_uint32)), n.value, C.byref(n)), "tape_program")
    return out


def shard_models(mb: ModelBatch, lo: int, hi: int) -> ModelBatch:
    """Host-only: candidates [lo, hi) as their own batch (``mq_models_shard``) — the contiguous
    shard a device of a multi-device context, or one rank of the per-process path, holds."""
    L = load_library()
    s, keep = as_model_batch(mb)
    out = MqModelBatch()
    h = C.c_void_p()
    _check(L.mq_models_shard(C.byref(s), int(lo), int(hi), C.byref(out), C.byref(h)), "mq_models_shard")
    try:
        ms, F = hi - lo, len(mb.funcs)
        rows = int(mb.var_word_offsets()[-1])

        def arr(ptr, n, dtype):
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True) if n else np.zeros(0, dtype)

        words = arr(out.var_words, rows * ms, np.uint32).reshape(rows, ms)
        if not F:
            return ModelBatch(mb.var_widths, words, index_base=out.index_base)
        eptr = arr(out.entry_ptr, F * (ms + 1), np.int64).reshape(F, ms + 1)
        ebase = arr(out.entry_base, F, np.int64)
        ew = arr(out.entry_words, int(out.n_entry_words), np.uint32)
        elb = arr(out.else_base, F, np.int64)
        return ModelBatch(mb.var_widths, words, mb.funcs, eptr, ew, ebase, mb.else_words, elb, out.index_base)
    finally:
        L.mq_models_shard_free(h)


def dag_expand(db) -> TapeBatch:
    """Host-only: every tape of a DagBatch as a self-contained postfix block (``mq_dag_expand``)."""
    from .tape import NODE_DTYPE
    L = load_library()
    s, keep = as_dag_batch(db)
    chunks, offs = [], [0]
    n = C.c_int64()
    for t in range(db.n_tapes):
        _check(L.mq_dag_expand(C.byref(s), t, None, 0, C.byref(n)), "mq_dag_expand")
        out = np.zeros(n.value, NODE_DTYPE)
        _check(L.mq_dag_expand(C.byref(s), t, out.ctypes.data, n.value, C.byref(n)), "mq_dag_expand")
        chunks.append(out)
        offs.append(offs[-1] + n.value)
    nodes = np.concatenate(chunks) if chunks else np.zeros(0, NODE_DTYPE)
    return TapeBatch.from_arrays(nodes, np.asarray(offs, np.int64), db.consts)


def tape_alg_ops(tb: TapeBatch, t: int) -> float:
    s, keep = as_tape_batch(tb)
    return float(load_library().mq_tape_alg_ops(C.byref(s), t))


class CompiledTapes:
    """A tape batch compiled and resident on the device (``mq_tapes``)."""

    def __init__(self, ev: "Evaluator", tb: TapeBatch):
        self.ev = ev
        self.n_tapes = tb.n_tapes
        h = C.c_void_p()
        nu = C.c_int32()
        if hasattr(tb, "root_offsets"):   # a DagBatch (the drop-in query stream)
            s, keep = as_dag_batch(tb)
            _check(ev.lib.mq_tapes_upload_dag(ev.ctx, C.byref(s), C.byref(h), C.byref(nu)), "mq_tapes_upload_dag")
        else:
            s, keep = as_tape_batch(tb)
            _check(ev.lib.mq_tapes_upload(ev.ctx, C.byref(s), C.byref(h), C.byref(nu)), "mq_tapes_upload")
        self.handle = h
        self.n_unsupported = nu.value
        cols = getattr(tb, "columns", None)
        self.n_columns = 0
        if cols is not None and cols.n:
            cs, ckeep = as_tape_batch(cols.programs)
            vi = np.ascontiguousarray(cols.var_index, np.int32)
            lv = np.ascontiguousarray(cols.level, np.int32)
            _check(ev.lib.mq_tapes_set_columns(h, C.byref(cs), vi.ctypes.data_as(C.POINTER(C.c_int32)),
                                               lv.ctypes.data_as(C.POINTER(C.c_int32)), cols.n), "mq_tapes_set_columns")
            self.n_columns = cols.n

    def split(self):
        """(tapes on the assembly interpreter, generic 256-bit, wider generic kernels (512..2048-bit))."""
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        _check(self.ev.lib.mq_tapes_info(self.handle, C.byref(a), C.byref(b), C.byref(c)), "mq_tapes_info")
        return a.value, b.value, c.value

    def asm_split(self):
        """After a launch: (tapes on the preloaded-variable assembly kernel, on the general assembly
        kernel, whether the assembly path ran for the current model batch)."""
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        _check(self.ev.lib.mq_tapes_qsa_split(self.handle, C.byref(a), C.byref(b), C.byref(c)), "mq_tapes_qsa_split")
        return a.value, b.value, bool(c.value)

    def flat_split(self):
        """After a launch: (tapes, hoisted Bool columns) on the flat-conjunction kernel (fc.hip)."""
        a, b = C.c_int32(), C.c_int32()
        _check(self.ev.lib.mq_tapes_flat_split(self.handle, C.byref(a), C.byref(b)), "mq_tapes_flat_split")
        return a.value, b.value

    def column_asm_split(self):
        """After a launch: (hoisted columns on the general assembly kernel, whether that path ran)."""
        a, b = C.c_int32(), C.c_int32()
        _check(self.ev.lib.mq_tapes_column_split(self.handle, C.byref(a), C.byref(b)), "mq_tapes_column_split")
        return a.value, bool(b.value)

    def keccak_predicate_columns(self) -> int:
        """Bool columns over keccak columns evaluated by the keccak column kernel
        (mq_tapes_column_keccak_predicates)."""
        n = C.c_int32()
        _check(self.ev.lib.mq_tapes_column_keccak_predicates(self.handle, C.byref(n)), "mq_tapes_column_keccak_predicates")
        return n.value

    def gather_columns(self) -> int:
        """Hoisted columns computed by the bit-gather column kernel (cw.hip: calldata words,
        their extracts and masks; mq_tapes_column_gather)."""
        n = C.c_int32()
        _check(self.ev.lib.mq_tapes_column_gather(self.handle, C.byref(n)), "mq_tapes_column_gather")
        return n.value

    def keccak_columns(self) -> int:
        """Hoisted columns computed by the keccak-f[1600] column kernel (mq_tapes_column_keccak)."""
        n = C.c_int32()
        _check(self.ev.lib.mq_tapes_column_keccak(self.handle, C.byref(n)), "mq_tapes_column_keccak")
        return n.value

    def handler_histogram(self, which: int = 1, pairs: bool = False, wait_variants: bool = False):
        """After a launch: {handler kind: dispatches per (tape, model) pair, summed over tapes} of
        the assembly translation (which = 0 P tapes, 1 G tapes, 2 G column programs); with
        pairs, also {(kind, next kind): count} over the G tapes.  A G stack reader's "_L" variant
        (waits for LDS / scalar loads only, gen_qsa.py LGKMWAIT) counts as its kind unless
        ``wait_variants``.  Diagnostic."""
        if not wait_variants:
            fold = lambda k: k[:-2] if k.endswith("_L") else k   # noqa: E731
            res = self.handler_histogram(which, pairs, True)
            h = res[0] if pairs else res
            hf = {}
            for k, v in h.items():
                hf[fold(k)] = hf.get(fold(k), 0) + v
            if not pairs:
                return hf
            pf = {}
            for (a, b), v in res[1].items():
                pf[(fold(a), fold(b))] = pf.get((fold(a), fold(b)), 0) + v
            return hf, pf
        lib = self.ev.lib
        n = C.c_int32()
        _check(lib.mq_tapes_qsa_histogram(self.handle, which, None, 0, None, C.byref(n)), "mq_tapes_qsa_histogram")
        k = n.value
        hist = np.zeros(k, np.int64)
        pr = np.zeros(k * k, np.int64) if pairs else None
        _check(lib.mq_tapes_qsa_histogram(self.handle, which, hist.ctypes.data_as(C.POINTER(C.c_int64)), k,
                                          pr.ctypes.data_as(C.POINTER(C.c_int64)) if pairs else None, C.byref(n)),
               "mq_tapes_qsa_histogram")
        names = [lib.mq_qsa_kind_name(i).decode() for i in range(k)]
        h = {names[i]: int(hist[i]) for i in range(k) if hist[i]}
        if not pairs:
            return h
        pr = pr.reshape(k, k)
        return h, {(names[i], names[j]): int(pr[i, j]) for i, j in zip(*np.nonzero(pr))}

    def free(self) -> None:
        if self.handle:
            self.ev.lib.mq_tapes_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Evaluator:
    """An evaluator context (``mq_ctx``).  ``devices=[d0, d1, ...]`` drives several GPUs from this
    one process (Mythril is single-process): the candidate axis is sharded over them
    inside ``mq_models_upload`` and first hits are MIN-reduced over RCCL inside the library.
    ``use_rccl=True`` on one device runs that RCCL path with a single rank.  The alternative, one
    process per GPU under torch.distributed, uses single-device contexts (:mod:`mythril_amd.dist`)."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None, use_rccl: bool = False):
        self.lib = load_library()
        ids = [int(d) for d in devices] if devices is not None else [int(device)]
        ctx = C.c_void_p()
        arr = (C.c_int * len(ids))(*ids)
        _check(self.lib.mq_ctx_create(len(ids), arr, C.byref(ctx)), "mq_ctx_create")
        self.ctx = ctx
        self.devices = ids
        self.device = ids[0]
        self.n_models = 0
        self.index_base = 0
        self._opts = {}
        if use_rccl and len(ids) == 1:
            self.set_option(self.OPT_USE_RCCL, 1)

    OPT_USE_ASM, OPT_EARLY_EXIT, OPT_ASM_READY, OPT_TIME_KERNELS = 1, 2, 3, 4
    OPT_USE_RCCL, OPT_RCCL_ACTIVE, OPT_LATENCY_WAVES, OPT_KECCAK_HOST_BLOCKS = 5, 6, 7, 8

    @property
    def rccl_active(self) -> bool:
        return self.set_option(self.OPT_RCCL_ACTIVE, 0) == 1

    def set_option(self, option: int, value: int) -> int:
        rc = self.lib.mq_ctx_set_option(self.ctx, option, value)
        if rc < 0:
            _check(rc, "mq_ctx_set_option")
        self._opts[option] = value
        return rc

    def option(self, option: int, default: int = 0) -> int:
        """The last value this process set for a settable option (the library's default if none)."""
        return self._opts.get(option, default)

    @property
    def asm_ready(self) -> bool:
        return self.set_option(self.OPT_ASM_READY, 0) == 1

    def use_asm(self, on: bool) -> None:
        self.set_option(self.OPT_USE_ASM, 1 if on else 0)

    def close(self) -> None:
        if getattr(self, "ctx", None):
            self.lib.mq_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ models
    upload_seq = 0   # bumped by every upload: lets a caller tell its own batch is still resident

    def upload_models(self, mb: ModelBatch) -> None:
        s, keep = as_model_batch(mb)
        self.upload_seq += 1
        _check(self.lib.mq_models_upload(self.ctx, C.byref(s)), "mq_models_upload")
        self.n_models = mb.n_models
        self.index_base = mb.index_base

    # ------------------------------------------------------------ tapes
    def compile(self, tb: TapeBatch) -> CompiledTapes:
        return CompiledTapes(self, tb)

    def first_hit(self, tapes, with_stats: bool = False):
        """check_quick_sat over a batch: int32[N] of global candidate indices / -1 / -2."""
        own = not isinstance(tapes, CompiledTapes)
        ct = self.compile(tapes) if own else tapes
        out = np.zeros(ct.n_tapes, np.int32)
        st = MqStats()
        try:
            _check(self.lib.mq_eval_tapes_first_hit(self.ctx, ct.handle, out.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(st)),
                   "mq_eval_tapes_first_hit")
        finally:
            if own:
                ct.free()
        if with_stats:
            return out, EvalStats(st.kernel_ms, st.node_evals, st.alg_ops, st.pairs_evaluated, st.n_hits, st.n_unsupported)
        return out

    def launch_first_hit(self, ct: CompiledTapes, device_ptr: int, stream: int = 0) -> None:
        """Async: int32 first-hit (INT32_MAX = none) into device memory on a HIP stream."""
        _check(self.lib.mq_launch_first_hit(self.ctx, ct.handle, C.c_void_p(device_ptr), C.c_void_p(stream or None)),
               "mq_launch_first_hit")

    def finalize_first_hit(self, ct: CompiledTapes, device_ptr: int, stream: int = 0) -> None:
        _check(self.lib.mq_finalize_first_hit(self.ctx, ct.handle, C.c_void_p(device_ptr), C.c_void_p(stream or None)),
               "mq_finalize_first_hit")

    def time_kernels(self, on: bool = True) -> None:
        """Bracket the evaluation kernels of every launch with HIP events (clears old ones)."""
        self.set_option(self.OPT_TIME_KERNELS, 1 if on else 0)

    def qsa_profile(self, reset: bool = True) -> dict:
        """G profile build only (gen_qsa.py QSA_PROF=1): {kind: (cycles, dispatches)} charged
        since the last reset; {} in product builds."""
        n = C.c_int32()
        _check(self.lib.mq_qsa_profile(self.ctx, None, 0, C.byref(n), 0), "mq_qsa_profile")
        if n.value == 0:
            return {}
        out = np.zeros(n.value, np.int64)
        _check(self.lib.mq_qsa_profile(self.ctx, out.ctypes.data_as(C.POINTER(C.c_int64)), n.value, C.byref(n),
                                       1 if reset else 0), "mq_qsa_profile")
        res = {}
        for i in range(n.value // 2):
            if out[2 * i + 1]:
                res[self.lib.mq_qsa_kind_name(i).decode()] = (int(out[2 * i]), int(out[2 * i + 1]))
        return res

    def kernel_times(self, reset: bool = True) -> List[float]:
        """Per-launch device time (ms) of the evaluation kernels since the last reset."""
        n = C.c_int32()
        _check(self.lib.mq_kernel_times(self.ctx, None, 0, C.byref(n), 0), "mq_kernel_times")
        buf = (C.c_float * max(n.value, 1))()
        _check(self.lib.mq_kernel_times(self.ctx, buf, n.value, C.byref(n), 1 if reset else 0), "mq_kernel_times")
        return [float(buf[i]) for i in range(n.value)]

    def kernel_times_device(self, device_index: int, reset: bool = False) -> List[float]:
        """``kernel_times`` of one device of a multi-device context (0 = the lead)."""
        n = C.c_int32()
        f = self.lib.mq_kernel_times_device
        _check(f(self.ctx, device_index, None, 0, C.byref(n), 0), "mq_kernel_times_device")
        buf = (C.c_float * max(n.value, 1))()
        _check(f(self.ctx, device_index, buf, n.value, C.byref(n), 1 if reset else 0), "mq_kernel_times_device")
        return [float(buf[i]) for i in range(n.value)]

    def launch_times(self, reset: bool = True):
        """Per launch on an in-library-reducing context (mq_launch_times): (reduce ms on the lead
        stream, host issue ms of the whole launch call, host issue ms of the peers' loop)."""
        n = C.c_int32()
        f = self.lib.mq_launch_times
        _check(f(self.ctx, None, None, None, 0, C.byref(n), 0), "mq_launch_times")
        k = max(n.value, 1)
        red, iss, peer = (C.c_float * k)(), (C.c_double * k)(), (C.c_double * k)()
        _check(f(self.ctx, red, iss, peer, n.value, C.byref(n), 1 if reset else 0), "mq_launch_times")
        return [float(red[i]) for i in range(n.value)], [float(iss[i]) for i in range(n.value)], \
            [float(peer[i]) for i in range(n.value)]

    @property
    def n_devices(self) -> int:
        return len(self.devices)

    HOST_PHASES = ("compile", "translate_upload", "tape_upload", "translate_p", "translate_g", "program_upload",
                   "args_upload", "launch_readback", "model_upload", "tape_free")

    def host_times(self, reset: bool = True) -> dict:
        """Host seconds per phase of the library (mq_host_times; diagnostic)."""
        out = (C.c_double * 16)()
        n = C.c_int32()
        _check(self.lib.mq_host_times(self.ctx, out, 16, C.byref(n), 1 if reset else 0), "mq_host_times")
        return {self.HOST_PHASES[i] if i < len(self.HOST_PHASES) else str(i): float(out[i]) for i in range(n.value)}

    def counters(self, reset: bool = False):
        """(pairs evaluated, node-evals, algorithmic ops) accumulated on the device."""
        out = (C.c_double * 3)()
        _check(self.lib.mq_counters(self.ctx, out, 1 if reset else 0), "mq_counters")
        return float(out[0]), float(out[1]), float(out[2])

    def verdicts(self, tapes):
        """Full N x M verdict matrix (bool) and first-hit (parity dumps)."""
        own = not isinstance(tapes, CompiledTapes)
        ct = self.compile(tapes) if own else tapes
        n = ct.n_tapes * self.n_models
        bits = np.zeros((n + 7) // 8, np.uint8)
        fh = np.zeros(ct.n_tapes, np.int32)
        try:
            _check(self.lib.mq_eval_tapes_verdicts(self.ctx, ct.handle, bits.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                   fh.ctypes.data_as(C.POINTER(C.c_int32))), "mq_eval_tapes_verdicts")
        finally:
            if own:
                ct.free()
        v = np.unpackbits(bits, bitorder="little")[:n].reshape(ct.n_tapes, self.n_models).astype(bool)
        return v, fh

    # ------------------------------------------------------------ keccak
    def keccak256_array(self, msgs: np.ndarray) -> np.ndarray:
        """keccak256 of each row of a uint8 [n, len] array on the GPU -> uint8 [n, 32]."""
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        n, ln = msgs.shape
        out = np.zeros((n, 32), np.uint8)
        if n == 0:
            return out
        offs = np.arange(n + 1, dtype=np.int64) * ln
        data = msgs.reshape(-1) if msgs.size else np.zeros(1, np.uint8)
        _check(self.lib.mq_keccak256(self.ctx, data.ctypes.data_as(C.POINTER(C.c_uint8)), offs.ctypes.data_as(C.POINTER(C.c_int64)),
                                     n, out.ctypes.data_as(C.POINTER(C.c_uint8))), "mq_keccak256")
        return out

    def keccak256(self, messages: Sequence[bytes]) -> List[bytes]:
        msgs = [bytes(m) for m in messages]
        offs = np.zeros(len(msgs) + 1, np.int64)
        offs[1:] = np.cumsum([len(m) for m in msgs])
        data = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
        out = np.zeros(32 * len(msgs), np.uint8)
        _check(self.lib.mq_keccak256(self.ctx, data.ctypes.data_as(C.POINTER(C.c_uint8)), offs.ctypes.data_as(C.POINTER(C.c_int64)),
                                     len(msgs), out.ctypes.data_as(C.POINTER(C.c_uint8))), "mq_keccak256")
        return [bytes(out[32 * i:32 * i + 32]) for i in range(len(msgs))]


_default: Optional[Evaluator] = None


def default_evaluator() -> Evaluator:
    global _default
    if _default is None:
        _default = Evaluator(int(os.environ.get("LOCAL_RANK", "0")))
    return _default
