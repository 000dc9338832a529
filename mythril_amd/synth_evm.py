"""EVM-shaped synthetic workloads for configs C3 and C5.

Real harvesting (``myth analyze rubixi.sol / BECToken.sol -t 3`` with z3 + solc) is not possible
offline, so these generators reproduce the constraint SHAPES Mythril emits, built through the
z3-free term layer (:mod:`mythril_amd.smt`, the reference's constructor vocabulary) and lowered by
the product lowering pass:

* caller is an actor: ``Or(sender_k == CREATOR, == ATTACKER, == SOMEGUY)`` (transaction/symbolic.py:26-34, 217-219)
* calldata bytes ``If(i < k_calldatasize, k_calldata[i], 0)`` (SIGNED ``<``, calldata.py:234-246)
  and words ``Concat`` of 32 of them (calldata.py:48-55)
* dispatch ``Extract(255,224,w0) == sel`` / ``LShR(w0,224) & 0xffffffff`` / ``UDiv(w0, 2^224)`` (instructions.py:510-573)
* ``Not(ULT(calldatasize, 4))``, address cleanliness ``w & (2^160-1) == w``, range checks
* SafeMath: ``Or(a == 0, UDiv(a*b, a) == b)``, ``UGE(a+b, a)``, ``ULE(b, a)``
* ``URem``/``SMod``/``SDiv``, ``SHL``/``LSHR``/``ASHR`` by constants, SIGNEXTEND / BYTE shapes
* value transfer ``UGE(balance[sender], call_value)`` (symbolic index -> per-model table lookup)
* storage ``Select(Store(Store(K(0), s0, v0), s1, v1), slot)`` with values from earlier txs
* Bool->BV fork conditions ``If(c, 1, 0) == 1`` (util.py:75-92)

Each tape is one path's conjunction over ``n_tx`` transactions.  A fraction of tapes is PLANTED:
built so that one chosen candidate model satisfies it (every branch is taken the way that model
goes); the others are built from a ghost model outside the batch, so three 4-byte selector
equalities make them unsatisfiable by every candidate (probability ~M·2^-96) — the no-early-exit
worst case, as in C2.  Models are generated column-wise (numpy PCG64, committed seeds): senders
mostly actors, small call values, calldatasize in [4, 100), uniform calldata bytes, balance tables
with entries for the three actors.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import smt as S
from .lower import SymbolTable, lower_term
from .models import FuncSpec, ModelBatch
from .tape import TapeBatch, limbs

M256 = (1 << 256) - 1
ACTORS = [0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE, 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
          0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA]
N_BYTES = 68  # selector + two ABI words


def _to_limbs(vals: np.ndarray, nl: int = 8) -> np.ndarray:
    """uint64 column (values < 2^64) -> [nl, M] u32 limbs."""
    out = np.zeros((nl, len(vals)), np.uint32)
    out[0] = (vals & 0xFFFFFFFF).astype(np.uint32)
    out[1] = (vals >> np.uint64(32)).astype(np.uint32)
    return out


def _int_limbs(v: int, nl: int = 8) -> np.ndarray:
    return np.array([(v >> (32 * i)) & 0xFFFFFFFF for i in range(nl)], np.uint32)


BLOCK = 1 << 16  # models are generated in independently seeded blocks (any rank can rebuild any model)


class _Block:
    def __init__(self, seed: int, b: int, n: int, n_tx: int):
        rng = np.random.Generator(np.random.PCG64([seed, b]))
        self.sender, self.value, self.cds, self.cdata = [], [], [], []
        for _ in range(n_tx):
            who = rng.integers(0, 10, n)
            s = rng.integers(0, 1 << 32, (8, n), dtype=np.uint64).astype(np.uint32)
            for a, addr in enumerate(ACTORS):
                pick = (who // 3) == a
                s[:, pick] = _int_limbs(addr)[:, None]
            self.sender.append(s)
            v = rng.integers(0, 1 << 40, n, dtype=np.uint64)
            v[rng.random(n) < 0.4] = 0
            self.value.append(_to_limbs(v))
            self.cds.append(_to_limbs(rng.integers(4, 100, n, dtype=np.uint64)))
            self.cdata.append(rng.integers(0, 256, (N_BYTES, n), dtype=np.uint64).astype(np.uint8))
        # balance: entries for the three actors + else value, all < 2^62
        self.bal_vals = rng.integers(0, 1 << 62, (3, n), dtype=np.uint64)
        self.bal_else = rng.integers(0, 1 << 62, n, dtype=np.uint64)


class EvmModels:
    """Column store of candidate models [lo, hi) of a global set of M for ``n_tx`` transactions.
    Senders are actors 90 % of the time, call values are 0 (40 %) or < 2^40, calldatasize is
    uniform in [4, 100), calldata bytes are uniform, balances have entries for the 3 actors."""

    def __init__(self, seed: int, M: int, n_tx: int, lo: int = 0, hi: int = None):
        hi = M if hi is None else hi
        self.seed, self.M, self.n_tx, self.lo, self.hi = seed, M, n_tx, lo, hi
        blocks = [self._block(b) for b in range(lo // BLOCK, (hi + BLOCK - 1) // BLOCK)] if hi > lo else []
        off = lo - (lo // BLOCK) * BLOCK
        n = hi - lo

        def cat(get, axis=1):
            if not blocks:
                return None
            return np.ascontiguousarray(np.concatenate([get(b) for b in blocks], axis=axis)[..., off:off + n])
        self.sender = [cat(lambda b, k=k: b.sender[k]) for k in range(n_tx)]
        self.value = [cat(lambda b, k=k: b.value[k]) for k in range(n_tx)]
        self.cds = [cat(lambda b, k=k: b.cds[k]) for k in range(n_tx)]
        self.cdata = [cat(lambda b, k=k: b.cdata[k]) for k in range(n_tx)]
        self.bal_vals = cat(lambda b: b.bal_vals)
        self.bal_else = cat(lambda b: b.bal_else, axis=0)
        self._cache = {}

    def _block(self, b: int) -> _Block:
        n = min(BLOCK, self.M - b * BLOCK)
        return _Block(self.seed, b, n, self.n_tx)

    # witness values of GLOBAL model m as Python ints (any m: its block is regenerated)
    @staticmethod
    def w(arr: np.ndarray, m: int) -> int:
        return sum(int(arr[i, m]) << (32 * i) for i in range(arr.shape[0]))

    def witness(self, m: int) -> Dict:
        b = m // BLOCK
        if b not in self._cache:
            if len(self._cache) > 8:
                self._cache.clear()
            self._cache[b] = self._block(b)
        blk, j = self._cache[b], m - b * BLOCK
        d = {"sender": [], "value": [], "cds": [], "bytes": []}
        for k in range(self.n_tx):
            d["sender"].append(self.w(blk.sender[k], j))
            d["value"].append(self.w(blk.value[k], j))
            d["cds"].append(self.w(blk.cds[k], j))
            d["bytes"].append([int(x) for x in blk.cdata[k][:, j]])
        d["balance"] = ({ACTORS[a]: int(blk.bal_vals[a, j]) for a in range(3)}, int(blk.bal_else[j]))
        return d

    # ------------------------------------------------------------------ ModelBatch for a symbol table
    def batch(self, syms: SymbolTable) -> ModelBatch:
        """The stored shard [lo, hi) serialized for ``syms`` (index_base = lo)."""
        lo, hi, n = 0, self.hi - self.lo, self.hi - self.lo
        rows = []
        for (name, w), i in sorted(syms.vars.items(), key=lambda kv: kv[1]):
            nl = limbs(w)
            if i in syms.derived:
                fname, args = syms.derived[i]
                k = int(fname.split("_")[0]) - 1
                idx = args[0]
                col = self.cdata[k][idx, lo:hi].astype(np.uint32) if idx < N_BYTES else np.zeros(n, np.uint32)
                r = np.zeros((nl, n), np.uint32)
                r[0] = col
            elif name.startswith("sender_"):
                r = self.sender[int(name[7:]) - 1][:, lo:hi]
            elif name.startswith("call_value"):
                r = self.value[int(name[10:]) - 1][:, lo:hi]
            elif name.endswith("_calldatasize"):
                r = self.cds[int(name.split("_")[0]) - 1][:, lo:hi]
            else:
                r = np.zeros((nl, n), np.uint32)
            rows.append(np.ascontiguousarray(r[:nl]))
        words = np.concatenate(rows, axis=0) if rows else np.zeros((0, n), np.uint32)
        funcs, eptr, ewords, ebase, elw, elb = [], [], [], [], [], []
        wpos = epos = 0
        for f, fname in enumerate(syms.func_names):
            spec = syms.func_specs[f]
            funcs.append(spec)
            if fname != "balance":
                raise ValueError(f"EvmModels has no table for {fname}")
            # 3 entries per model: key = actor (8 limbs), value (8 limbs)
            ent = np.zeros((n, 3, 16), np.uint32)
            for a in range(3):
                ent[:, a, :8] = _int_limbs(ACTORS[a])[None, :]
                ent[:, a, 8] = (self.bal_vals[a, lo:hi] & 0xFFFFFFFF).astype(np.uint32)
                ent[:, a, 9] = (self.bal_vals[a, lo:hi] >> np.uint64(32)).astype(np.uint32)
            ebase.append(wpos)
            ewords.append(ent.reshape(-1))
            wpos += ent.size
            eptr.append(np.arange(n + 1, dtype=np.int64) * 3)
            # ModelBatch keeps else values model-major (else_base + m*limbs + l)
            elb.append(epos)
            els = np.ascontiguousarray(_to_limbs(self.bal_else[lo:hi]).T).reshape(-1)
            elw.append(els)
            epos += els.size
        if not funcs:
            return ModelBatch(syms.var_widths, words, index_base=self.lo)
        return ModelBatch(syms.var_widths, words, funcs, np.stack(eptr), np.concatenate(ewords),
                          np.asarray(ebase, np.int64), np.concatenate(elw), np.asarray(elb, np.int64), self.lo)


class _Tx:
    """Terms of transaction k (Mythril's symbol names, transaction/symbolic.py:125-143, calldata.py:230-231)."""

    def __init__(self, k: int):
        self.k = k
        self.sender = S.BitVecSym(f"sender_{k}", 256)
        self.value = S.BitVecSym(f"call_value{k}", 256)
        self.cds = S.BitVecSym(f"{k}_calldatasize", 256)
        self.cd = S.Array(f"{k}_calldata", 256, 8)
        self._bytes = {}

    def byte(self, i: int) -> S.Term:
        if i not in self._bytes:
            self._bytes[i] = S.If(S.BitVecVal(i, 256) < self.cds, self.cd[S.BitVecVal(i, 256)], S.BitVecVal(0, 8))
        return self._bytes[i]

    def word(self, off: int) -> S.Term:
        return S.Concat(*[self.byte(off + j) for j in range(32)])


def _word_val(bytes_: Sequence[int], cds: int, off: int) -> int:
    v = 0
    for j in range(32):
        i = off + j
        b = bytes_[i] if (i < cds and i < len(bytes_)) else 0
        v = (v << 8) | b
    return v


def _signed(x: int) -> int:
    return x - (1 << 256) if x >> 255 else x


def _smod(a: int, b: int) -> int:
    if b == 0:
        return a
    sa, sb = _signed(a), _signed(b)
    r = abs(sa) % abs(sb)
    if r == 0:
        return 0
    if sa < 0 and sb > 0:
        return (-r + sb) & M256
    if sa >= 0 and sb < 0:
        return (r + sb) & M256
    if sa < 0 and sb < 0:
        return (-r) & M256
    return r


def _holds(cond: S.Term, truth: bool) -> S.Term:
    """The branch the witness takes (instructions.py:1616-1622 forks on c / not c)."""
    return cond if truth else S.Not(cond)


def evm_path(rng: np.random.Generator, wit: Dict, n_tx: int, checks_per_tx: Tuple[int, int] = (3, 6)) -> S.Term:
    """One path conjunction whose every branch is the one ``wit`` takes."""
    cs: List[S.Term] = []
    storage = S.K(256, 256, 0)
    for k in range(n_tx):
        tx = _Tx(k + 1)
        snd, cv, cds, B = wit["sender"][k], wit["value"][k], wit["cds"][k], wit["bytes"][k]
        W0, W1, W2 = _word_val(B, cds, 0), _word_val(B, cds, 4), _word_val(B, cds, 36)
        w0, w1, w2 = tx.word(0), tx.word(4), tx.word(36)
        cs.append(_holds(S.Or(*[tx.sender == a for a in ACTORS]), snd in ACTORS))
        cs.append(_holds(S.ULT(tx.cds, S.BitVecVal(4, 256)), cds < 4))
        sel = W0 >> 224
        form = int(rng.integers(3))
        if form == 0:
            cs.append(S.Extract(255, 224, w0) == sel)
        elif form == 1:
            cs.append((S.LShR(w0, S.BitVecVal(224, 256)) & 0xFFFFFFFF) == sel)
        else:
            cs.append((S.UDiv(w0, S.BitVecVal(1 << 224, 256)) & 0xFFFFFFFF) == sel)
        n_checks = int(rng.integers(checks_per_tx[0], checks_per_tx[1] + 1))
        for _ in range(n_checks):
            c = int(rng.integers(14))
            if c == 0:
                m160 = (1 << 160) - 1
                cs.append(_holds((w1 & m160) == w1, W1 & m160 == W1))
            elif c == 1:
                t = int.from_bytes(rng.bytes(32), "little")
                cs.append(_holds(S.ULT(w1, S.BitVecVal(t, 256)), W1 < t))
            elif c == 2:
                prod = (W1 * W2) & M256
                ok = W1 == 0 or (prod // W1) == W2
                cs.append(_holds(S.Or(w1 == 0, S.UDiv(w1 * w2, w1) == w2), ok))
            elif c == 3:
                cs.append(_holds(S.UGE(w1 + w2, w1), ((W1 + W2) & M256) >= W1))
            elif c == 4:
                cs.append(_holds(S.ULE(w2, w1), W2 <= W1))
            elif c == 5:
                d = int(rng.integers(2, 1000))
                cs.append(S.URem(w1, S.BitVecVal(d, 256)) == (W1 % d))
            elif c == 6:
                d = int(rng.integers(2, 1 << 20)) * (1 if rng.random() < 0.5 else -1)
                cs.append(S.SMod(w2, S.BitVecVal(d, 256)) == _smod(W2, d & M256))
            elif c == 7:
                s1, s2 = int(rng.integers(0, 256)), int(rng.integers(0, 256))
                v = ((W2 >> s1) << s2) & M256
                cs.append((S.LShR(w2, S.BitVecVal(s1, 256)) << S.BitVecVal(s2, 256)) == v)
            elif c == 8:
                s1 = int(rng.integers(0, 256))
                t = int.from_bytes(rng.bytes(32), "little")
                v = (_signed(W1) >> s1) & M256
                cs.append(_holds(S.ULT(w1 >> S.BitVecVal(s1, 256), S.BitVecVal(t, 256)), v < t))
            elif c == 9:
                bal, els = wit["balance"]
                b = bal.get(snd, els)
                cs.append(_holds(S.UGE(S.Array("balance", 256, 256)[tx.sender], tx.value), b >= cv))
            elif c == 10:
                cs.append(_holds(tx.value == 0, cv == 0))
            elif c == 11:
                x = W1 & 0xFF
                sx = (x - 256 if x >> 7 else x) & M256
                cs.append(S.SignExt(248, S.Extract(7, 0, w1)) == sx)
            elif c == 12:
                o = 8 * int(rng.integers(0, 32))
                cs.append(S.Concat(S.BitVecVal(0, 248), S.Extract(o + 7, o, w2)) == ((W2 >> o) & 0xFF))
            else:
                cs.append(_holds(S.If(S.ULT(w1, w2), S.BitVecVal(1, 256), S.BitVecVal(0, 256)) == 1, W1 < W2))
        # storage written by this tx, read back by later ones
        if k > 0 and rng.random() < 0.7:
            slot = int(rng.integers(0, 4))
            cs.append(_holds(S.Select(storage, S.BitVecVal(slot, 256)) == 0, wit["_storage"].get(slot, 0) == 0))
        wit.setdefault("_storage", {})
        slot = int(rng.integers(0, 4))
        storage = S.Store(storage, S.BitVecVal(slot, 256), w1)
        wit["_storage"][slot] = W1
    wit.pop("_storage", None)
    return S.And(*cs)


def c3_workload(n_tapes: int = 1000, n_models: int = 1_000_000, seed: int = 3, planted_frac: float = 0.1,
                n_tx: int = 3, shard: Tuple[int, int] = None, checks_per_tx: Tuple[int, int] = (3, 6)):
    """Config C3 substitute: ``n_tapes`` EVM-shaped path conjunctions over ``n_tx`` transactions x
    ``n_models`` candidates.  ``shard=(lo, hi)`` materialises only candidates [lo, hi) (multi-GPU);
    tapes and expected first hits are global.  Returns (tapes, models, expected, symbols)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lo, hi = shard if shard else (0, n_models)
    models = EvmModels(seed, n_models, n_tx, lo, hi)
    ghost = EvmModels(seed + 1_000_003, max(1, n_tapes), n_tx, 0, 0)
    syms = SymbolTable()
    tapes, expected = [], np.full(n_tapes, -1, np.int32)
    planted = rng.random(n_tapes) < planted_frac
    for t in range(n_tapes):
        if planted[t]:
            p = int(rng.integers(n_models))
            wit = models.witness(p)
            expected[t] = p
        else:
            wit = ghost.witness(t)
        tapes.append(lower_term(evm_path(rng, wit, n_tx, checks_per_tx), syms))
    return TapeBatch(tapes), models.batch(syms), expected, syms
