"""ORACLE (test infrastructure / CPU baseline only): ctypes wrapper of oracle/libcref.so,
the C restatement of ``ModelCache.check_quick_sat`` (support_utils.py:60-67) + z3
``model.eval(..., model_completion=True)`` semantics.  See oracle/cref.c."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from typing import List

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(_HERE))

from mythril_amd._abi import MqModelBatch, MqTapeBatch, as_model_batch, as_tape_batch  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402
from mythril_amd.tape import TapeBatch  # noqa: E402

_LIB = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return os.path.join(_HERE, "libcref.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libcref.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.cref_first_hit.argtypes = [C.POINTER(MqTapeBatch), C.POINTER(MqModelBatch), C.POINTER(C.c_int32), C.c_int]
        L.cref_first_hit.restype = C.c_int64
        L.cref_verdicts.argtypes = [C.POINTER(MqTapeBatch), C.POINTER(MqModelBatch), C.POINTER(C.c_uint8), C.c_int]
        L.cref_verdicts.restype = C.c_int
        L.cref_eval_tape.argtypes = [C.POINTER(MqTapeBatch), C.c_int32, C.POINTER(MqModelBatch), C.c_int64]
        L.cref_eval_tape.restype = C.c_int
        L.cref_eval_node.argtypes = [C.POINTER(MqTapeBatch), C.c_int32, C.POINTER(MqModelBatch), C.c_int64, C.c_int64, C.POINTER(C.c_uint32)]
        L.cref_eval_node.restype = C.c_int
        L.cref_keccak256.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_uint8)]
        L.cref_keccak256.restype = None
        _LIB = L
    return _LIB


def first_hit(tb: TapeBatch, mb: ModelBatch, nthreads: int = 0):
    """Returns (first_hit[int32 N], pairs_evaluated)."""
    ts, keep_t = as_tape_batch(tb)
    ms, keep_m = as_model_batch(mb)
    out = np.zeros(tb.n_tapes, np.int32)
    pairs = lib().cref_first_hit(C.byref(ts), C.byref(ms), out.ctypes.data_as(C.POINTER(C.c_int32)), nthreads)
    return out, int(pairs)


def verdicts(tb: TapeBatch, mb: ModelBatch, nthreads: int = 0) -> np.ndarray:
    ts, keep_t = as_tape_batch(tb)
    ms, keep_m = as_model_batch(mb)
    nbits = tb.n_tapes * mb.n_models
    bits = np.zeros((nbits + 7) // 8, np.uint8)
    lib().cref_verdicts(C.byref(ts), C.byref(ms), bits.ctypes.data_as(C.POINTER(C.c_uint8)), nthreads)
    return np.unpackbits(bits, bitorder="little")[:nbits].reshape(tb.n_tapes, mb.n_models).astype(bool)


def eval_tape(tb: TapeBatch, t: int, mb: ModelBatch, m: int) -> int:
    """Verdict of tape t on local model m (1 / 0, -2 unsupported)."""
    ts, k1 = as_tape_batch(tb)
    ms, k2 = as_model_batch(mb)
    return int(lib().cref_eval_tape(C.byref(ts), t, C.byref(ms), m))


def eval_node(tb: TapeBatch, t: int, mb: ModelBatch, m: int, node: int) -> int:
    ts, keep_t = as_tape_batch(tb)
    ms, keep_m = as_model_batch(mb)
    out = np.zeros(64, np.uint32)
    n = lib().cref_eval_node(C.byref(ts), t, C.byref(ms), m, node, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    if n < 0:
        raise ValueError("unsupported")
    return sum(int(out[i]) << (32 * i) for i in range(n))


def keccak256(data: bytes) -> bytes:
    out = (C.c_uint8 * 32)()
    lib().cref_keccak256(bytes(data), len(data), out)
    return bytes(out)
