"""ORACLE (test infrastructure only — never imported by the product path).

Pure-Python keccak-f[1600] and keccak256 with Ethereum padding (0x01 ... 0x80), the
function the reference reaches through ``eth_hash.auto.keccak`` in
``mythril/support/support_utils.py:92-100`` and
``mythril/laser/ethereum/function_managers/keccak_function_manager.py:56-69``
(third-party dep ``eth-hash >=0.3.1,<0.4.0``, requirements.txt:13, absent here).
Published algorithm: FIPS-202 Keccak-f[1600] permutation; rate 1088 bits; the
pre-FIPS multi-rate padding ``pad10*1`` with domain byte 0x01.

Pinned by: ``keccak256(b"") == get_empty_keccak_hash()`` (kfm.py:86-93), the VMTests
vmSha3Test digests (tests/golden/keccak_kats.json) and, for the permutation itself,
SHA3-256 (domain byte 0x06) against ``hashlib.sha3_256``.
"""
from __future__ import annotations

_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
# rotation offsets r[x][y]
_ROT = [
    [0, 36, 3, 41, 18],
    [1, 44, 10, 45, 2],
    [62, 6, 43, 15, 61],
    [28, 55, 25, 21, 56],
    [27, 20, 39, 8, 14],
]
_M = (1 << 64) - 1


def _rol(v: int, n: int) -> int:
    n %= 64
    return ((v << n) | (v >> (64 - n))) & _M if n else v


def keccak_f1600(a):
    """a: list of 25 lanes, index x + 5*y.  Returns the permuted state."""
    a = list(a)
    for rnd in range(24):
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
        a = [a[i] ^ d[i % 5] for i in range(25)]
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = _rol(a[x + 5 * y], _ROT[x][y])
        a = [b[x + 5 * y] ^ ((~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]) for y in range(5) for x in range(5)]
        # list comprehension above iterates y outer, x inner -> index x + 5*y order preserved
        a[0] ^= _RC[rnd]
    return a


def _sponge(data: bytes, domain: int, rate: int = 136, out_len: int = 32) -> bytes:
    msg = bytearray(data)
    msg.append(domain)
    while len(msg) % rate:
        msg.append(0)
    msg[-1] |= 0x80
    state = [0] * 25
    for off in range(0, len(msg), rate):
        block = msg[off:off + rate]
        for i in range(rate // 8):
            state[i] ^= int.from_bytes(block[8 * i:8 * i + 8], "little")
        state = keccak_f1600(state)
    out = b"".join(s.to_bytes(8, "little") for s in state)
    return out[:out_len]


def keccak256(data: bytes) -> bytes:
    return _sponge(bytes(data), 0x01)


def sha3_256(data: bytes) -> bytes:
    return _sponge(bytes(data), 0x06)
