"""Concrete keccak256 as a batched GPU service.

The reference hashes concrete byte strings one call at a time through eth_hash:
``find_concrete_keccak`` (keccak_function_manager.py:56-69) at constraint-build time and, after a
solver run, ``_replace_with_actual_sha`` (mythril/analysis/solver.py:131-167), which scans every
64-hex-digit slice of each concrete transaction's input for the ``hash_matcher`` prefix, looks the
slice up in the model's concrete hashes, reads its pre-image through the inverse UF, and replaces
the slice with the real keccak of that pre-image.

Here the same scan collects every pre-image first and hashes them in ONE launch of the
keccak-f[1600] kernel (``mq_keccak256``); the replacements are then applied in the reference's
order.  A launch costs tens of microseconds, so the GPU pays off from a few hundred hashes per
call; bench.py's keccak leg measures the crossover against a CPU keccak.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

HASH_MATCHER = "fffffff"   # keccak_function_manager.py:36


def keccak256_many(messages: Sequence[bytes], evaluator=None) -> List[bytes]:
    """keccak256 (Ethereum padding) of every message, one GPU launch."""
    if not messages:
        return []
    if evaluator is None:
        from .evaluator import default_evaluator
        evaluator = default_evaluator()
    return evaluator.keccak256(list(messages))


def _scan(tx_input: str, s_index: int, concrete_hashes, preimage):
    """Yield (slice position, pre-image, size) of every matching slice of an input."""
    for i in range(s_index, len(tx_input)):
        data_slice = tx_input[i:i + 64]
        if HASH_MATCHER not in data_slice or len(data_slice) != 64:
            continue
        find = int(data_slice, 16)
        found = None
        for size, values in concrete_hashes.items():   # the last matching size wins, as there
            if find not in values:
                continue
            found = (preimage(size, find), size)
        if found is not None and found[0] is not None:
            yield i, found[0], found[1]


def replace_with_actual_sha(concrete_transactions: List[Dict[str, str]], concrete_hashes: Dict[int, Sequence[int]],
                            preimage: Callable[[int, int], Optional[int]], code_bytecode: Optional[str] = None,
                            hasher: Callable[[Sequence[bytes]], List[bytes]] = keccak256_many) -> None:
    """solver.py:131-167 with batched hashing.

    ``concrete_hashes``: ``keccak_function_manager.get_concrete_hash_data(model)`` (size -> hash
    values the model assigns); ``preimage(size, hash)``: the model's inverse-UF value
    (``model.eval(inverse(hash)).as_long()``).  Pass 1 hashes every pre-image found in the inputs
    in one batch; pass 2 is the reference's loop verbatim (it re-reads each slice from the input
    as edited so far and replaces every occurrence), taking digests from pass 1 and hashing on
    demand only a pre-image that an earlier replacement brought into view."""
    def s_index_of(tx):
        return len(code_bytecode) + 2 if (code_bytecode is not None and code_bytecode in tx["input"]) else 10

    wanted = {}
    for tx in concrete_transactions:
        if HASH_MATCHER in tx["input"]:
            for _, v, size in _scan(tx["input"], s_index_of(tx), concrete_hashes, preimage):
                wanted[(v, size)] = None
    keys = list(wanted)
    memo = dict(zip(keys, hasher([v.to_bytes(size // 8, "big") for v, size in keys]))) if keys else {}

    def digest(v: int, size: int) -> bytes:
        if (v, size) not in memo:
            memo[(v, size)] = hasher([v.to_bytes(size // 8, "big")])[0]
        return memo[(v, size)]

    for tx in concrete_transactions:
        if HASH_MATCHER not in tx["input"]:
            continue
        s_index = s_index_of(tx)
        for i in range(s_index, len(tx["input"])):
            data_slice = tx["input"][i:i + 64]
            if HASH_MATCHER not in data_slice or len(data_slice) != 64:
                continue
            find = int(data_slice, 16)
            input_ = None
            for size, values in concrete_hashes.items():
                if find not in values:
                    continue
                input_ = (preimage(size, find), size)
            if input_ is None or input_[0] is None:
                continue
            hex_keccak = digest(*input_).hex().rjust(64, "0")
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(tx["input"][i:64 + i], hex_keccak)
