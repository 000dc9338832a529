"""Batched concrete keccak (mythril_amd.keccak_service) against a literal restatement of the
reference's _replace_with_actual_sha (mythril/analysis/solver.py:131-167), hashing with the CPU
keccak of the oracle (the GPU kernel itself is checked in test_gpu_parity.py)."""
import random

import keccak_ref
from mythril_amd.keccak_service import HASH_MATCHER, replace_with_actual_sha


def _reference(concrete_transactions, concrete_hashes, preimage, code_bytecode=None):
    for tx in concrete_transactions:
        if HASH_MATCHER not in tx["input"]:
            continue
        if code_bytecode is not None and code_bytecode in tx["input"]:
            s_index = len(code_bytecode) + 2
        else:
            s_index = 10
        for i in range(s_index, len(tx["input"])):
            data_slice = tx["input"][i: i + 64]
            if HASH_MATCHER not in data_slice or len(data_slice) != 64:
                continue
            find_input = int(data_slice, 16)
            input_ = None
            for size in concrete_hashes:
                if find_input not in concrete_hashes[size]:
                    continue
                input_ = (preimage(size, find_input), size)
            if input_ is None:
                continue
            hex_keccak = keccak_ref.keccak256(input_[0].to_bytes(input_[1] // 8, "big")).hex().rjust(64, "0")
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(tx["input"][i: 64 + i], hex_keccak)


def test_batched_replacement_matches_reference():
    rng = random.Random(5)
    hashes = {512: [], 256: []}
    pre = {}
    for size in (512, 256):
        for _ in range(4):
            h = (0xFFFFFFF << 228) | rng.getrandbits(228)
            hashes[size].append(h)
            pre[(size, h)] = rng.getrandbits(size)
    txs = []
    for _ in range(5):
        parts = ["0x", "a9059cbb"]
        for _ in range(rng.randrange(1, 5)):
            if rng.random() < 0.6:
                size = rng.choice([512, 256])
                parts.append(format(rng.choice(hashes[size]), "064x"))
            else:
                parts.append(format(rng.getrandbits(256), "064x"))
        txs.append({"input": "".join(parts)})
    ref = [dict(t) for t in txs]
    got = [dict(t) for t in txs]
    calls = []

    def hasher(msgs):
        calls.append(len(msgs))
        return [keccak_ref.keccak256(m) for m in msgs]

    _reference(ref, hashes, lambda s, h: pre[(s, h)])
    replace_with_actual_sha(got, hashes, lambda s, h: pre[(s, h)], hasher=hasher)
    assert got == ref
    assert calls and calls[0] > 1          # one batch for the pre-images found up front
