"""Keccak and exponent uninterpreted-function managers over z3-free terms.

Mirrors ``KeccakFunctionManager`` (reference
``mythril/laser/ethereum/function_managers/keccak_function_manager.py:25-182``) and
``ExponentFunctionManager`` (``exponent_function_manager.py:10-63``): they decide which UF
applications and axioms appear in a quick-sat conjunction, so the synthetic
EVM-shaped workloads and the drop-in ``Constraints.get_all_constraints`` produce the same shapes
as Mythril.

Concrete keccak (``find_concrete_keccak``, kfm.py:56-69; a7) goes through ``hasher``; the product
default is the GPU keccak-f[1600] kernel (``mq_keccak256``).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

from . import smt as S

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30
EMPTY_KECCAK = 0xC5D2460186F7233C927E7DB2DCC703C0E500B653CA82273B7BFAD8045D85A470


def _gpu_keccak(data: bytes) -> bytes:
    from .evaluator import default_evaluator
    return default_evaluator().keccak256([data])[0]


class KeccakFunctionManager:
    """kfm.py:25-179.  ``keccak256_<n>`` (domain n -> 256) and its inverse ``keccak256_<n>-1``;
    symbolic inputs get injectivity + disjoint-interval + ``urem 64 == 0`` axioms, concrete
    inputs are hashed and pinned."""

    def __init__(self, hasher: Optional[Callable[[bytes], bytes]] = None):
        self.hasher = hasher
        self._index_counter = TOTAL_PARTS - 34534   # kfm.py:41, set once per manager
        self.reset()

    def reset(self) -> None:
        """kfm.py:48-54: forgets functions, intervals and inputs but keeps ``_index_counter``, so
        the interval of a size first seen after a reset differs from a fresh manager's."""
        self.store_function: Dict[int, Tuple[S.Function, S.Function]] = {}
        self.interval_hook_for_size: Dict[int, int] = {}
        self.hash_result_store: Dict[int, List[S.Term]] = {}
        self.concrete_hashes: Dict[S.Term, S.Term] = {}
        self.symbolic_inputs: Dict[int, List[S.Term]] = {}

    def find_concrete_keccak(self, data: S.Term) -> S.Term:
        digest = (self.hasher or _gpu_keccak)(data.value.to_bytes(data.size() // 8, "big"))
        return S.BitVecVal(int.from_bytes(digest, "big"), 256)

    def get_function(self, length: int) -> Tuple[S.Function, S.Function]:
        if length not in self.store_function:
            self.store_function[length] = (S.Function(f"keccak256_{length}", [length], 256),
                                           S.Function(f"keccak256_{length}-1", [256], length))
            self.hash_result_store[length] = []
        return self.store_function[length]

    @staticmethod
    def get_empty_keccak_hash() -> S.Term:
        return S.BitVecVal(EMPTY_KECCAK, 256)

    def create_keccak(self, data: S.Term) -> S.Term:
        length = data.size()
        func, _ = self.get_function(length)
        if not data.symbolic:
            h = self.find_concrete_keccak(data)
            self.concrete_hashes[data] = h
            return h
        self.symbolic_inputs.setdefault(length, []).append(data)
        self.hash_result_store[length].append(func(data))
        return func(data)

    def create_conditions(self) -> S.Term:
        cond = S.BoolVal(True)
        for inputs in self.symbolic_inputs.values():
            for x in inputs:
                cond = S.And(cond, self._create_condition(x))
        for data, h in self.concrete_hashes.items():
            func, inv = self.get_function(data.size())
            cond = S.And(cond, func(data) == h, inv(func(data)) == data)
        return cond

    def interval(self, length: int) -> Tuple[int, int]:
        if length not in self.interval_hook_for_size:
            self.interval_hook_for_size[length] = self._index_counter
            self._index_counter -= INTERVAL_DIFFERENCE
        lo = self.interval_hook_for_size[length] * PART
        return lo, lo + PART

    def _create_condition(self, func_input: S.Term) -> S.Term:
        length = func_input.size()
        func, inv = self.get_function(length)
        lo, hi = self.interval(length)
        fx = func(func_input)
        cond = S.And(inv(fx) == func_input,
                     S.ULE(S.BitVecVal(lo, 256), fx),
                     S.ULT(fx, S.BitVecVal(hi, 256)),
                     S.URem(fx, S.BitVecVal(64, 256)) == 0)
        concrete = S.BoolVal(False)
        for key, h in self.concrete_hashes.items():
            if key.size() == length:
                concrete = S.Or(concrete, S.And(fx == h, key == func_input))
        return S.And(inv(fx) == func_input, S.Or(cond, concrete))


class ExponentFunctionManager:
    """exponent_function_manager.py:10-60: ``Power(b, e)`` UF, ``Power > 0`` (SIGNED ``>``,
    bitvec.py:149-158) and 32 axioms ``Power(256, i) == 256^i``."""

    def __init__(self):
        power = S.Function("Power", [256, 256], 256)
        n256 = S.BitVecVal(256, 256)
        self.concrete_constraints = S.And(*[power(n256, S.BitVecVal(i, 256)) == S.BitVecVal(pow(256, i, 2 ** 256), 256)
                                            for i in range(32)])

    def create_condition(self, base: S.Term, exponent: S.Term) -> Tuple[S.Term, S.Term]:
        power = S.Function("Power", [256, 256], 256)
        exponentiation = power(base, exponent)
        if not exponent.symbolic and not base.symbolic:
            c = S.BitVecVal(pow(base.value, exponent.value, 2 ** 256), 256)
            return c, c == exponentiation
        constraint = S.And(exponentiation > 0, self.concrete_constraints)
        if base.value == 256:
            constraint = S.And(constraint, power(base, S.URem(exponent, S.BitVecVal(32, 256))) == power(base, exponent))
        return exponentiation, constraint


keccak_function_manager = KeccakFunctionManager()
exponent_function_manager = ExponentFunctionManager()
