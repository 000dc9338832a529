"""Candidate-model batches in the ``mq_model_batch`` layout (include/mq.h).

A batch is M serialized z3 models in global candidate order — index 0 is the MRU
model, i.e. the first one ``check_quick_sat`` tries (``reversed(lru_cache.keys())``,
reference ``mythril/support/support_utils.py:62``).  Interpretations are stored
WITHOUT model completion: an absent constant is 0 / false and an absent function has
no entries and else-value 0, which is exactly what ``eval(..., model_completion=True)``
assigns (``support_utils.py:63`` deep-copies because completion
mutates the model).

Scalar variables are SoA ``u32`` limbs, ``var_words[var_word_off[v] + limb, m]`` —
the layout the kernels stream coalesced (one model per lane).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from .tape import FUNC_DTYPE, limbs, to_words, from_words


@dataclass
class FuncSpec:
    """Signature of a model function: UF (``keccak256_<n>``, ``keccak256_<n>-1``,
    ``Power`` — keccak_function_manager.py:71-84, exponent_function_manager.py:21) or
    the as-array interpretation of a symbolic array (``balance``, ``Storage<addr>``,
    ``<tx>_calldata``)."""
    arity: int
    result_width: int
    arg_widths: Tuple[int, ...]

    @property
    def stride(self) -> int:
        return sum(limbs(w) for w in self.arg_widths) + limbs(self.result_width)


class ModelBatch:
    def __init__(self, var_widths: Sequence[int], var_words: np.ndarray,
                 funcs: Sequence[FuncSpec] = (), entry_ptr: Optional[np.ndarray] = None,
                 entry_words: Optional[np.ndarray] = None, entry_base: Optional[np.ndarray] = None,
                 else_words: Optional[np.ndarray] = None, else_base: Optional[np.ndarray] = None,
                 index_base: int = 0):
        self.var_widths = np.asarray(var_widths, dtype=np.uint16)
        self.var_words = np.ascontiguousarray(var_words, dtype=np.uint32)
        # limbs(w) per variable (Bool -> 1), vectorised: the drop-in path builds a batch per launch
        n_rows = int(np.maximum((self.var_widths.astype(np.int64) + 31) // 32, 1).sum())
        if self.var_words.ndim != 2 or self.var_words.shape[0] != n_rows:
            raise ValueError(f"var_words must be [{n_rows}, M], got {self.var_words.shape}")
        self.n_models = int(self.var_words.shape[1])
        self.funcs = list(funcs)
        F, M = len(self.funcs), self.n_models
        self.func_arr = np.zeros(max(F, 1), dtype=FUNC_DTYPE)
        for i, f in enumerate(self.funcs):
            self.func_arr[i]["arity"] = f.arity
            self.func_arr[i]["result_width"] = f.result_width
            aw = list(f.arg_widths) + [0] * (2 - len(f.arg_widths))
            self.func_arr[i]["arg_width"] = aw[:2]
        self.entry_ptr = np.ascontiguousarray(entry_ptr if entry_ptr is not None else np.zeros((max(F, 1), M + 1), np.int64), dtype=np.int64)
        self.entry_words = np.ascontiguousarray(entry_words if entry_words is not None else np.zeros(1, np.uint32), dtype=np.uint32)
        self.entry_base = np.ascontiguousarray(entry_base if entry_base is not None else np.zeros(max(F, 1), np.int64), dtype=np.int64)
        self.else_words = np.ascontiguousarray(else_words if else_words is not None else np.zeros(1, np.uint32), dtype=np.uint32)
        self.else_base = np.ascontiguousarray(else_base if else_base is not None else np.zeros(max(F, 1), np.int64), dtype=np.int64)
        if self.entry_words.size == 0:
            self.entry_words = np.zeros(1, np.uint32)
        if self.else_words.size == 0:
            self.else_words = np.zeros(1, np.uint32)
        self.index_base = int(index_base)

    @property
    def n_vars(self) -> int:
        return len(self.var_widths)

    def var_word_offsets(self) -> np.ndarray:
        off = np.zeros(self.n_vars + 1, np.int64)
        off[1:] = np.cumsum([limbs(int(w)) for w in self.var_widths])
        return off

    # ------------------------------------------------------------ python views (oracle/tests)
    def var_value(self, v: int, m: int) -> int:
        off = self.var_word_offsets()
        return from_words(self.var_words[off[v]:off[v + 1], m])

    def func_table(self, f: int, m: int) -> Tuple[Dict[Tuple[int, ...], int], int]:
        spec = self.funcs[f]
        lo, hi = int(self.entry_ptr[f, m]), int(self.entry_ptr[f, m + 1])
        table: Dict[Tuple[int, ...], int] = {}
        base = int(self.entry_base[f])
        for e in range(lo, hi):
            w0 = base + e * spec.stride
            args = []
            for aw in spec.arg_widths:
                n = limbs(aw)
                args.append(from_words(self.entry_words[w0:w0 + n]))
                w0 += n
            val = from_words(self.entry_words[w0:w0 + limbs(spec.result_width)])
            table.setdefault(tuple(args), val)
        nl = limbs(spec.result_width)
        eb = int(self.else_base[f]) + m * nl
        return table, from_words(self.else_words[eb:eb + nl])

    def shard(self, lo: int, hi: int) -> "ModelBatch":
        """Contiguous model-axis shard [lo, hi) in global candidate order."""
        F = len(self.funcs)
        new_ptr = np.zeros((max(F, 1), hi - lo + 1), np.int64)
        ew: List[np.ndarray] = []
        eb = np.zeros(max(F, 1), np.int64)
        elw: List[np.ndarray] = []
        elb = np.zeros(max(F, 1), np.int64)
        wpos = 0
        epos = 0
        for f, spec in enumerate(self.funcs):
            s = spec.stride
            a, b = int(self.entry_ptr[f, lo]), int(self.entry_ptr[f, hi])
            base = int(self.entry_base[f])
            eb[f] = wpos
            ew.append(self.entry_words[base + a * s: base + b * s])
            wpos += (b - a) * s
            new_ptr[f] = self.entry_ptr[f, lo:hi + 1] - a
            nl = limbs(spec.result_width)
            ebase = int(self.else_base[f])
            elb[f] = epos
            elw.append(self.else_words[ebase + lo * nl: ebase + hi * nl])
            epos += (hi - lo) * nl
        return ModelBatch(self.var_widths, self.var_words[:, lo:hi], self.funcs, new_ptr,
                          np.concatenate(ew) if ew else None, eb,
                          np.concatenate(elw) if elw else None, elb, self.index_base + lo)

    # ------------------------------------------------------------ construction from python values
    @classmethod
    def from_python(cls, var_widths: Sequence[int], models: Sequence[Mapping],
                    funcs: Sequence[FuncSpec] = (), index_base: int = 0) -> "ModelBatch":
        """``models[m] = {"vars": {v: int}, "funcs": {f: (entries{args_tuple: value}, else_value)}}``;
        anything missing is absent (completion default)."""
        M = len(models)
        off = np.zeros(len(var_widths) + 1, np.int64)
        off[1:] = np.cumsum([limbs(int(w)) for w in var_widths])
        words = np.zeros((int(off[-1]), M), np.uint32)
        for m, mod in enumerate(models):
            for v, val in mod.get("vars", {}).items():
                w = int(var_widths[v])
                words[off[v]:off[v + 1], m] = to_words(int(val) & ((1 << max(w, 1)) - 1), w)
        F = len(funcs)
        entry_ptr = np.zeros((max(F, 1), M + 1), np.int64)
        entry_words: List[int] = []
        entry_base = np.zeros(max(F, 1), np.int64)
        else_words: List[int] = []
        else_base = np.zeros(max(F, 1), np.int64)
        for f, spec in enumerate(funcs):
            entry_base[f] = len(entry_words)
            else_base[f] = len(else_words)
            count = 0
            for m, mod in enumerate(models):
                entry_ptr[f, m] = count
                table, els = mod.get("funcs", {}).get(f, ({}, 0))
                for args, val in table.items():
                    if not isinstance(args, tuple):
                        args = (args,)
                    for aw, av in zip(spec.arg_widths, args):
                        entry_words.extend(to_words(int(av), aw))
                    entry_words.extend(to_words(int(val), spec.result_width))
                    count += 1
                else_words.extend(to_words(int(els), spec.result_width))
            entry_ptr[f, M] = count
        return cls(var_widths, words, funcs, entry_ptr,
                   np.asarray(entry_words, np.uint32), entry_base,
                   np.asarray(else_words, np.uint32), else_base, index_base)
