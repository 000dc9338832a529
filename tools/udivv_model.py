#!/usr/bin/env python3
"""Per-lane model of G's division by a variable (gen_qsa.py sub_udivv), instruction-shaped:
32-bit words, the fp64 reciprocal estimate + integer fix-up, Moller-Granlund 2-by-1 quotient
digits, Knuth D3 refinement, multiply-subtract with a rare add-back, in-place quotient digits.
Checked against Python big ints on random and adversarial operands (diagnostic; not product code,
not test infrastructure)."""
import random
import struct
import sys

B = 1 << 32
M32 = B - 1


def f64(x):
    return struct.unpack("<d", struct.pack("<d", x))[0]


def inv_estimate(d1, rcp_err=0.0):
    """inv = floor((B^2 - 1) / d1) - B for d1 in [2^31, 2^32): fp64 estimate + fix-up."""
    F = float(d1)
    R = f64(1.0 / F * (1.0 + rcp_err))          # v_rcp_f64 (approximate)
    E = f64(-F * R + 1.0)                       # v_fma_f64 (fused: one rounding; close enough)
    R = f64(R * E + R)
    R = f64(R * 2.0 ** 64)                      # v_ldexp_f64
    R = f64(R - 2.0 ** 32)                      # v_add_f64 with -2^32
    t = int(R) if R > 0 else 0                  # v_cvt_u32_f64: truncate, clamp
    t = min(max(t, 0), M32)
    p = t * d1 + (d1 << 32)                     # v_mad_u64_u32 with addend (0 : d1)
    if p >= B * B:                              # carry out: too big
        t = (t - 1) & M32
    else:
        if (p + d1) < B * B:                    # no overflow adding d1: too small
            t = (t + 1) & M32
    return t


def udiv2by1(n1, n0, d, v):
    """Moller-Granlund: (q, r) = divmod(n1:n0, d), n1 < d, d normalized, v = inv."""
    p = v * n1 + ((n1 << 32) | n0)
    q0, q1 = p & M32, (p >> 32) & M32
    q1 = (q1 + 1) & M32
    r = (n0 - q1 * d) & M32
    if r > q0:
        q1 = (q1 - 1) & M32
        r = (r + d) & M32
    if r >= d:
        q1 = (q1 + 1) & M32
        r = (r - d) & M32
    return q1, r


def udivv(u, v, stats=None):
    """u, v: 256-bit ints -> (q, r) with bvudiv / bvurem semantics (x / 0 = ones, x % 0 = x)."""
    U = [(u >> (32 * l)) & M32 for l in range(8)] + [0] * 8
    V = [(v >> (32 * l)) & M32 for l in range(8)]
    z = v == 0
    if z:
        V[0] = 1
    top, k = V[7], 0
    for l in range(6, -1, -1):
        if top == 0:
            top, k = V[l], k + 1
    b = 32 - top.bit_length()
    # limb shift by k (stages 4, 2, 1), then bit shift by b
    for st in (4, 2, 1):
        if k & st:
            U = [0] * st + U[:16 - st]
            V = [0] * st + V[:8 - st]
    if b:
        U = [((U[i] << b) | (U[i - 1] >> (32 - b))) & M32 if i else (U[0] << b) & M32 for i in range(16)]
        V = [((V[i] << b) | (V[i - 1] >> (32 - b))) & M32 if i else (V[0] << b) & M32 for i in range(8)]
    d1, d0 = V[7], V[6]
    assert d1 >> 31
    inv = inv_estimate(d1)
    assert inv == (B * B - 1) // d1 - B, (d1, inv)
    for j in range(7, -1, -1):
        n1, n0, n_ = U[j + 8], U[j + 7], U[j + 6]
        if n1 == 0 and n0 < d1:
            if stats is not None:
                stats["skip_lane"] = stats.get("skip_lane", 0) + 1
            continue                           # (wave-uniform only when every lane skips)
        if n1 >= d1:
            assert n1 == d1
            qh, rh = M32, n0 + d1
            ovf = rh >= B
            rh &= M32
        else:
            qh, rh = udiv2by1(n1, n0, d1, inv)
            ovf = False
        for _ in range(2):
            if not ovf and qh * d0 > ((rh << 32) | n_):
                qh = (qh - 1) & M32
                s = rh + d1
                ovf = s >= B
                rh = s & M32
        # multiply-subtract over the 9-limb window
        carry, borrow = 0, 0
        for i in range(8):
            p = qh * V[i] + carry
            carry = p >> 32
            t = U[j + i] - (p & M32) - borrow
            borrow = 1 if t < 0 else 0
            U[j + i] = t & M32
        t = U[j + 8] - carry - borrow
        borrow = 1 if t < 0 else 0
        if borrow:
            if stats is not None:
                stats["addback"] = stats.get("addback", 0) + 1
            qh = (qh - 1) & M32
            c = 0
            for i in range(8):
                s = U[j + i] + V[i] + c
                U[j + i], c = s & M32, s >> 32
        else:
            assert (t & M32) == 0
        U[j + 8] = qh
    # remainder: u'[0..7] >> (32k + b)
    W = [((U[i + 1] << 32 | U[i]) >> b) & M32 for i in range(7)] + [U[7] >> b]
    for st in (4, 2, 1):
        if k & st:
            W = W[st:] + [0] * st
    Q = U[8:16]
    if z:
        W, Q = Q, [M32] * 8
    q = sum(x << (32 * i) for i, x in enumerate(Q))
    r = sum(x << (32 * i) for i, x in enumerate(W))
    return q, r


def check(n=200000, seed=1):
    rng = random.Random(seed)
    ones = (1 << 256) - 1
    stats = {}

    def rnd():
        kind = rng.randrange(8)
        bits = rng.randrange(1, 257)
        if kind == 0:
            return 0
        if kind == 1:
            return rng.choice([1, 2, ones, 1 << 255, (1 << 255) - 1, B - 1, B, B + 1])
        if kind == 2:   # all-ones limbs (D3 / add-back territory)
            nl = rng.randrange(1, 9)
            return ((1 << (32 * nl)) - 1) ^ (rng.getrandbits(32) << (32 * rng.randrange(nl)))
        if kind == 3:   # top limb 0x8000.. / 0xffff..
            nl = rng.randrange(1, 9)
            return (rng.choice([0x80000000, 0xFFFFFFFF, 0x80000001]) << (32 * (nl - 1))) | rng.getrandbits(32 * (nl - 1))
        return rng.getrandbits(bits)
    for it in range(n):
        u, v = rnd(), rnd()
        if it % 3 == 0 and v:
            # dividends near multiples of the divisor: q * v + r with extreme digits
            q = rng.choice([ones // v, (ones // v) - 1, rng.getrandbits(rng.randrange(1, 257)) % (ones // v + 1)])
            r = rng.choice([0, v - 1, rng.randrange(v)])
            if q * v + r <= ones:
                u = q * v + r
        q, r = udivv(u, v, stats)
        if v == 0:
            assert q == ones and r == u
        else:
            assert (q, r) == divmod(u, v), (hex(u), hex(v), hex(q), hex(r))
    # Hacker's Delight add-back vectors (divmnu tests)
    for u, v in ((0x800000000000000000000003, 0x200000000000000000000001),
                 (0x0000800000000000fffe000000000000, 0x0000800000000000ffff),
                 (0x00008000fffffffe00000000, 0x00008000ffffffff)):
        assert udivv(u, v, stats) == divmod(u, v)
    # inverse over every d1 class edge
    for d1 in [B // 2, B // 2 + 1, B - 1, B - 2] + [rng.randrange(B // 2, B) for _ in range(100000)]:
        assert inv_estimate(d1) == (B * B - 1) // d1 - B, d1
        for e in (1e-15, -1e-15, 3e-16):
            assert inv_estimate(d1, e) == (B * B - 1) // d1 - B, (d1, e)
    print("ok", n, stats)


if __name__ == "__main__":
    check(int(sys.argv[1]) if len(sys.argv) > 1 else 200000)
