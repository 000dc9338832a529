"""ctypes mirror of the structs in ``include/mq.h`` (the C-ABI boundary).

``as_tape_batch`` / ``as_model_batch`` build the C structs over numpy buffers owned by
the returned keep-alive tuple; the library copies everything it needs.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .tape import TapeBatch
from .models import ModelBatch


class MqNode(C.Structure):
    _fields_ = [("op", C.c_uint16), ("width", C.c_uint16), ("a", C.c_uint32), ("b", C.c_uint32), ("c", C.c_uint32)]


class MqTapeBatch(C.Structure):
    _fields_ = [
        ("n_tapes", C.c_int32),
        ("tape_offsets", C.POINTER(C.c_int64)),
        ("nodes", C.c_void_p),
        ("const_words", C.POINTER(C.c_uint32)),
        ("n_const_words", C.c_int64),
    ]


class MqFuncDesc(C.Structure):
    _fields_ = [("arity", C.c_uint16), ("result_width", C.c_uint16), ("arg_width", C.c_uint16 * 2)]


class MqModelBatch(C.Structure):
    _fields_ = [
        ("n_models", C.c_int64),
        ("index_base", C.c_int64),
        ("n_vars", C.c_int32),
        ("var_width", C.POINTER(C.c_uint16)),
        ("var_words", C.POINTER(C.c_uint32)),
        ("n_funcs", C.c_int32),
        ("funcs", C.c_void_p),
        ("entry_ptr", C.POINTER(C.c_int64)),
        ("entry_base", C.POINTER(C.c_int64)),
        ("entry_words", C.POINTER(C.c_uint32)),
        ("n_entry_words", C.c_int64),
        ("else_base", C.POINTER(C.c_int64)),
        ("else_words", C.POINTER(C.c_uint32)),
        ("n_else_words", C.c_int64),
    ]


class MqStats(C.Structure):
    _fields_ = [
        ("kernel_ms", C.c_double),
        ("node_evals", C.c_double),
        ("alg_ops", C.c_double),
        ("pairs_evaluated", C.c_int64),
        ("n_hits", C.c_int32),
        ("n_unsupported", C.c_int32),
    ]


class MqDagBatch(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int64),
        ("nodes", C.c_void_p),
        ("const_words", C.POINTER(C.c_uint32)),
        ("n_const_words", C.c_int64),
        ("n_tapes", C.c_int32),
        ("root_offsets", C.POINTER(C.c_int64)),
        ("roots", C.POINTER(C.c_uint32)),
    ]


def _ptr(arr: np.ndarray, ctype):
    return arr.ctypes.data_as(C.POINTER(ctype))


def as_tape_batch(tb: TapeBatch):
    nodes = np.ascontiguousarray(tb.nodes)
    offs = np.ascontiguousarray(tb.offsets, dtype=np.int64)
    consts = np.ascontiguousarray(tb.consts, dtype=np.uint32)
    s = MqTapeBatch(tb.n_tapes, _ptr(offs, C.c_int64), nodes.ctypes.data, _ptr(consts, C.c_uint32), consts.size)
    return s, (nodes, offs, consts)


def as_model_batch(mb: ModelBatch):
    vw = np.ascontiguousarray(mb.var_widths, dtype=np.uint16)
    if vw.size == 0:
        vw = np.zeros(1, np.uint16)
    words = np.ascontiguousarray(mb.var_words, dtype=np.uint32)
    if words.size == 0:
        words = np.zeros(1, np.uint32)
    funcs = np.ascontiguousarray(mb.func_arr)
    eptr = np.ascontiguousarray(mb.entry_ptr, dtype=np.int64)
    ebase = np.ascontiguousarray(mb.entry_base, dtype=np.int64)
    ew = np.ascontiguousarray(mb.entry_words, dtype=np.uint32)
    elb = np.ascontiguousarray(mb.else_base, dtype=np.int64)
    elw = np.ascontiguousarray(mb.else_words, dtype=np.uint32)
    s = MqModelBatch(
        mb.n_models, mb.index_base, mb.n_vars, _ptr(vw, C.c_uint16), _ptr(words, C.c_uint32),
        len(mb.funcs), funcs.ctypes.data, _ptr(eptr, C.c_int64), _ptr(ebase, C.c_int64),
        _ptr(ew, C.c_uint32), ew.size, _ptr(elb, C.c_int64), _ptr(elw, C.c_uint32), elw.size)
    return s, (vw, words, funcs, eptr, ebase, ew, elb, elw)


def as_dag_batch(db):
    nodes = np.ascontiguousarray(db.nodes)
    consts = np.ascontiguousarray(db.consts, dtype=np.uint32)
    offs = np.ascontiguousarray(db.root_offsets, dtype=np.int64)
    roots = np.ascontiguousarray(db.roots, dtype=np.uint32)
    if roots.size == 0:
        roots = np.zeros(1, np.uint32)
    s = MqDagBatch(len(nodes), nodes.ctypes.data if len(nodes) else None, _ptr(consts, C.c_uint32), consts.size,
                   db.n_tapes, _ptr(offs, C.c_int64), _ptr(roots, C.c_uint32))
    return s, (nodes, consts, offs, roots)
