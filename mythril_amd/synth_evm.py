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
from .lower import SymbolTable, lower_batch, lower_term, split_slice
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
    def __init__(self, seed: int, b: int, n: int, n_tx: int, address_args: bool = False, n_bytes: int = N_BYTES):
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
            self.cds.append(_to_limbs(rng.integers(4, n_bytes + 32, n, dtype=np.uint64)))
            cd = rng.integers(0, 256, (n_bytes, n), dtype=np.uint64).astype(np.uint8)
            if address_args:
                # first ABI argument is an address: 12 zero bytes + an actor (90 %) or random bytes
                cd[4:16] = 0
                who2 = rng.integers(0, 10, n)
                for a, addr in enumerate(ACTORS):
                    pick = (who2 // 3) == a
                    cd[16:36, pick] = np.frombuffer(addr.to_bytes(20, "big"), np.uint8)[:, None]
            self.cdata.append(cd)
        # balance: entries for the three actors + else value, all < 2^62
        self.bal_vals = rng.integers(0, 1 << 62, (3, n), dtype=np.uint64)
        self.bal_else = rng.integers(0, 1 << 62, n, dtype=np.uint64)


class EvmModels:
    """Column store of candidate models [lo, hi) of a global set of M for ``n_tx`` transactions.
    Senders are actors 90 % of the time, call values are 0 (40 %) or < 2^40, calldatasize is
    uniform in [4, 100), calldata bytes are uniform, balances have entries for the 3 actors."""

    def __init__(self, seed: int, M: int, n_tx: int, lo: int = 0, hi: int = None, address_args: bool = False,
                 n_bytes: int = N_BYTES):
        hi = M if hi is None else hi
        self.seed, self.M, self.n_tx, self.lo, self.hi = seed, M, n_tx, lo, hi
        self.address_args = address_args
        self.n_bytes = n_bytes   # calldata bytes per tx (selector + ABI words); calldatasize in [4, n_bytes + 32)
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
        return _Block(self.seed, b, n, self.n_tx, self.address_args, self.n_bytes)

    def derived_column(self, fname: str, args, nl: int, n: int) -> np.ndarray:
        """Interpretation of ``fname`` at constant ``args`` for every stored model."""
        r = np.zeros((nl, n), np.uint32)
        if fname.endswith("_calldata"):
            k, idx = int(fname.split("_")[0]) - 1, args[0]
            if idx < self.n_bytes:
                r[0] = self.cdata[k][idx].astype(np.uint32)
            return r
        raise ValueError(f"no derived column for {fname}{args}")

    def extra_table(self, fname: str, spec):
        return None

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
                r = self.derived_column(fname, args, nl, n)
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
                base, sl = split_slice(fname)
                t = self.extra_table(base, spec)
                if t is None:
                    raise ValueError(f"EvmModels has no table for {fname}")
                ptr, ent, els = t
                if sl is not None:   # a slice of the base function's values (lower.py _wide_eq)
                    kl = sum(limbs(w) for w in spec.arg_widths)
                    a, b = sl[0] // 32, sl[1] // 32
                    ent = np.concatenate([ent[..., :kl], ent[..., kl + a:kl + b]], axis=-1)
                    els = els[..., a:b]
                ebase.append(wpos)
                ewords.append(ent.reshape(-1))
                wpos += ent.size
                eptr.append(ptr)
                elb.append(epos)
                elw.append(els.reshape(-1))
                epos += els.size
                continue
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


def evm_path(rng: np.random.Generator, wit: Dict, n_tx: int, checks_per_tx: Tuple[int, int] = (3, 6),
             n_args: int = 2) -> S.Term:
    """One path conjunction whose every branch is the one ``wit`` takes.  ``n_args`` ABI words per
    call (at 4, 36, 68, ...); with more than two, every check draws the pair of words it relates
    (the default keeps the round-1/2 C3 stream bit for bit)."""
    cs: List[S.Term] = []
    storage = S.K(256, 256, 0)
    for k in range(n_tx):
        tx = _Tx(k + 1)
        snd, cv, cds, B = wit["sender"][k], wit["value"][k], wit["cds"][k], wit["bytes"][k]
        W0, W1, W2 = _word_val(B, cds, 0), _word_val(B, cds, 4), _word_val(B, cds, 36)
        w0, w1, w2 = tx.word(0), tx.word(4), tx.word(36)
        a_vals = [_word_val(B, cds, 4 + 32 * i) for i in range(n_args)]
        a_terms = [tx.word(4 + 32 * i) for i in range(n_args)]
        cs.append(S.Or(*[tx.sender == a for a in ACTORS]))  # always asserted (symbolic.py:217-219)
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
            if n_args > 2:
                i, j = (int(x) for x in rng.choice(n_args, 2, replace=False))
                W1, W2, w1, w2 = a_vals[i], a_vals[j], a_terms[i], a_terms[j]
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
        storage = S.Store(storage, S.BitVecVal(slot, 256), a_terms[0])
        wit["_storage"][slot] = a_vals[0]
    wit.pop("_storage", None)
    return S.And(*cs)


def c3_workload(n_tapes: int = 1000, n_models: int = 1_000_000, seed: int = 3, planted_frac: float = 0.1,
                n_tx: int = 3, shard: Tuple[int, int] = None, checks_per_tx: Tuple[int, int] = (3, 6),
                hoist: bool = False, n_args: int = 2):
    """Config C3 substitute: ``n_tapes`` EVM-shaped path conjunctions over ``n_tx`` transactions x
    ``n_models`` candidates (``n_args`` ABI words per call).  ``shard=(lo, hi)`` materialises only
    candidates [lo, hi) (multi-GPU); tapes and expected first hits are global.  Returns (tapes,
    models, expected, symbols)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lo, hi = shard if shard else (0, n_models)
    nb = 4 + 32 * n_args
    models = EvmModels(seed, n_models, n_tx, lo, hi, n_bytes=nb)
    ghost = EvmModels(seed + 1_000_003, max(1, n_tapes), n_tx, 0, 0, n_bytes=nb)
    syms = SymbolTable()
    roots, expected = [], np.full(n_tapes, -1, np.int32)
    planted = rng.random(n_tapes) < planted_frac
    for t in range(n_tapes):
        if planted[t]:
            while True:  # the caller is always an actor (transaction/symbolic.py:217-219)
                p = int(rng.integers(n_models))
                wit = models.witness(p)
                if all(x in ACTORS for x in wit["sender"]):
                    break
            expected[t] = p
        else:
            wit = ghost.witness(t)
        roots.append(evm_path(rng, wit, n_tx, checks_per_tx, n_args))
    tb, syms, ok = lower_batch(roots, syms, hoist=hoist)
    assert ok.all()
    # DAG nodes per conjunction as the reference evaluates it (no batch-level hoisting)
    tb.unhoisted_nodes = lower_batch(roots, SymbolTable())[0].sizes() if hoist else tb.sizes()
    return tb, models.batch(syms), expected, syms


# ====================================================================== C4: keccak-heavy mappings
def _be_bytes(words: np.ndarray) -> np.ndarray:
    """[nl, n] u32 little-endian limbs -> [n, 4*nl] big-endian bytes."""
    nl = words.shape[0]
    le = np.ascontiguousarray(words.T).view(np.uint8).reshape(-1, 4 * nl)
    return le[:, ::-1]


def _digest_limbs(dig: np.ndarray) -> np.ndarray:
    """[n, 32] digests (big-endian integers) -> [8, n] u32 limbs."""
    le = np.ascontiguousarray(dig[:, ::-1])
    return np.ascontiguousarray(le.view(np.uint32).T)


class KeccakModels(EvmModels):
    """Keccak-consistent candidates: for every mapping key the path hashes —
    ``sender_k ++ slot`` and ``to_k ++ slot`` (to = the address argument) — and for the concrete
    constructor key ``CREATOR ++ slot``, the model's ``keccak256_512`` table holds the TRUE
    keccak256 and ``keccak256_512-1`` the inverse entry.  UF table lookup (z3 semantics) and the
    in-kernel keccak-f[1600] then agree on every model."""

    SLOT = 1

    def __init__(self, seed, M, n_tx, lo=0, hi=None, hasher_many=None):
        super().__init__(seed, M, n_tx, lo, hi, address_args=True)
        self.hasher_many = hasher_many
        self._tables = None

    def keys(self) -> List[np.ndarray]:
        """[n, 64] big-endian 512-bit keys per stored model: the 3 actors, then per tx sender / to."""
        n = self.hi - self.lo
        slot = np.zeros((8, n), np.uint32)
        slot[0] = self.SLOT
        out = [np.concatenate([_be_bytes(np.repeat(_int_limbs(a)[:, None], n, 1)), _be_bytes(slot)], 1) for a in ACTORS]
        for k in range(self.n_tx):
            out.append(np.concatenate([_be_bytes(self.sender[k]), _be_bytes(slot)], 1))
            # address word: calldata bytes 4..35 (zero past calldatasize) masked to 160 bits
            to = np.zeros((32, n), np.uint8)
            idx = np.arange(16, 36)[:, None]
            to[12:32] = np.where(idx < self.cds[k][0][None, :], self.cdata[k][16:36], 0)
            out.append(np.concatenate([to.T, _be_bytes(slot)], 1))
        return out

    def _build(self):
        if self._tables is not None:
            return self._tables
        keys = self.keys()
        n = self.hi - self.lo
        E = len(keys)
        digests = [self.hasher_many(k) for k in keys]
        fwd = np.zeros((n, E, 24), np.uint32)   # key (16 limbs LE) + value (8 limbs)
        inv = np.zeros((n, E, 24), np.uint32)   # key (8) + value (16)
        for e, (k, dg) in enumerate(zip(keys, digests)):
            key_limbs = np.ascontiguousarray(k[:, ::-1]).view(np.uint32)      # [n, 16] LE limbs
            val_limbs = _digest_limbs(dg).T                                    # [n, 8]
            fwd[:, e, :16] = key_limbs
            fwd[:, e, 16:] = val_limbs
            inv[:, e, :8] = val_limbs
            inv[:, e, 8:] = key_limbs
        ptr = np.arange(n + 1, dtype=np.int64) * E
        self._tables = {"keccak256_512": (ptr, fwd, np.zeros((n, 8), np.uint32)),
                        "keccak256_512-1": (ptr, inv, np.zeros((n, 16), np.uint32))}
        return self._tables

    def extra_table(self, fname, spec):
        return self._build().get(fname)

    def derived_column(self, fname, args, nl, n):
        base, sl = split_slice(fname)
        if sl is not None and base in ("keccak256_512", "keccak256_512-1"):
            full = self.derived_column(base, args, 16 if base.endswith("-1") else 8, n)
            return np.ascontiguousarray(full[sl[0] // 32:sl[1] // 32][:nl])
        if fname in ("keccak256_512", "keccak256_512-1"):
            ptr, ent, els = self._build()[fname]
            kl = 16 if fname == "keccak256_512" else 8
            key = _int_limbs(args[0], kl)
            r = np.zeros((nl, n), np.uint32)
            found = np.zeros(n, bool)
            for e in range(ent.shape[1]):
                hit = (ent[:, e, :kl] == key[None, :]).all(1) & ~found
                r[:, hit] = ent[hit, e, kl:kl + nl].T
                found |= hit
            return r
        return super().derived_column(fname, args, nl, n)


def c4_path(rng: np.random.Generator, wit: Dict, n_tx: int, hasher_many) -> S.Term:
    """A token-transfer path per tx over ``balances[...]`` mappings (storage slot keccak256 of
    key ++ slot, instructions.py:1017-1055) plus the manager's axioms for every keccak input on
    the path (keccak_function_manager.py:116-179)."""
    from .function_managers import KeccakFunctionManager

    def h(v: int) -> int:
        return int.from_bytes(bytes(hasher_many(np.frombuffer(v.to_bytes(64, "big"), np.uint8)[None, :])[0]), "big")

    km = KeccakFunctionManager(hasher=lambda b: h(int.from_bytes(b, "big")).to_bytes(32, "big"))
    slot = S.BitVecVal(KeccakModels.SLOT, 256)
    # constructor: initial balances of the three actors (concrete keys -> concrete hashes)
    storage = S.K(256, 256, 0)
    wst = {}
    for a, addr in enumerate(ACTORS):
        amount = 10 ** 24 >> a
        storage = S.Store(storage, km.create_keccak(S.Concat(S.BitVecVal(addr, 256), slot)), amount)
        wst[h((addr << 256) | KeccakModels.SLOT)] = amount
    cs: List[S.Term] = []
    m160 = (1 << 160) - 1
    for k in range(n_tx):
        tx = _Tx(k + 1)
        snd, cds, B = wit["sender"][k], wit["cds"][k], wit["bytes"][k]
        W0, W1, W2 = _word_val(B, cds, 0), _word_val(B, cds, 4), _word_val(B, cds, 36)
        w0, w1, w2 = tx.word(0), tx.word(4), tx.word(36)
        cs.append(S.Or(*[tx.sender == a for a in ACTORS]))
        cs.append(_holds(S.ULT(tx.cds, S.BitVecVal(68, 256)), cds < 68))
        cs.append(S.Extract(255, 224, w0) == (W0 >> 224))
        to = w1 & m160
        TO = W1 & m160
        cs.append(_holds(to == 0, TO == 0))
        hf = km.create_keccak(S.Concat(tx.sender, slot))
        ht = km.create_keccak(S.Concat(to, slot))
        HF, HT = h((snd << 256) | KeccakModels.SLOT), h((TO << 256) | KeccakModels.SLOT)
        bal_f, bal_t = S.Select(storage, hf), S.Select(storage, ht)
        BF, BT = wst.get(HF, 0), wst.get(HT, 0)
        cs.append(_holds(S.UGE(bal_f, w2), BF >= W2))
        storage = S.Store(storage, hf, bal_f - w2)
        wst[HF] = (BF - W2) & M256
        BT = wst.get(HT, 0)
        bal_t = S.Select(storage, ht)
        cs.append(_holds(S.UGE(bal_t + w2, bal_t), ((BT + W2) & M256) >= BT))
        storage = S.Store(storage, ht, bal_t + w2)
        wst[HT] = (BT + W2) & M256
    # sender's balance after the path is read back (storage chain over every keccak key)
    cs.append(_holds(S.UGT(S.Select(storage, km.create_keccak(S.Concat(_Tx(1).sender, slot))), S.BitVecVal(0, 256)),
                     wst.get(h((wit["sender"][0] << 256) | KeccakModels.SLOT), 0) > 0))
    return S.And(*cs, km.create_conditions())


def c4_workload(n_tapes: int = 200, n_models: int = 1_000_000, seed: int = 4, planted_frac: float = 0.1,
                n_tx: int = 2, shard: Tuple[int, int] = None, hasher_many=None, interpret_keccak: bool = False,
                hoist: bool = False):
    """Config C4: keccak-heavy mapping/storage tapes x keccak-consistent models.

    ``interpret_keccak`` lowers ``keccak256_512(x)`` to the in-kernel keccak-f[1600]
    (MQ_OP_KECCAK) instead of the model's UF table; on these models both give the same verdicts.
    ``hasher_many``: uint8 [n, len] -> uint8 [n, 32] (the GPU keccak kernel in the product)."""
    if hasher_many is None:
        from .evaluator import default_evaluator
        hasher_many = default_evaluator().keccak256_array
    rng = np.random.Generator(np.random.PCG64(seed))
    lo, hi = shard if shard else (0, n_models)
    models = KeccakModels(seed, n_models, n_tx, lo, hi, hasher_many)
    ghost = EvmModels(seed + 1_000_003, max(1, n_tapes), n_tx, 0, 0, address_args=True)
    syms = SymbolTable(interpret_keccak=interpret_keccak,
                       keccak_of_constant=lambda b: bytes(hasher_many(np.frombuffer(b, np.uint8)[None, :])[0]))
    roots, expected = [], np.full(n_tapes, -1, np.int32)
    planted = rng.random(n_tapes) < planted_frac
    def hashed_keys_are_concrete(w) -> bool:
        # the manager's axioms hold under true hashes only for keys equal to a concrete (actor)
        # key; keccak-consistent witnesses therefore send to actors with a full address argument
        return all(w["cds"][k] >= 36 and _word_val(w["bytes"][k], w["cds"][k], 4) in ACTORS
                   and w["sender"][k] in ACTORS for k in range(n_tx))

    for t in range(n_tapes):
        if planted[t]:
            while True:
                p = int(rng.integers(n_models))
                wit = models.witness(p)
                if hashed_keys_are_concrete(wit):
                    break
            expected[t] = p
        else:
            wit = ghost.witness(t)
        roots.append(c4_path(rng, wit, n_tx, hasher_many))
    tb, syms, ok = lower_batch(roots, syms, hoist=hoist)
    assert ok.all()
    return tb, models.batch(syms), expected, syms


# ====================================================================== C4-wide: keccak of > 64 bytes
WIDE_SIZES = (544, 768, 1088)   # keccak256(msg.data) of a 2-argument call, abi.encode of 3 words, 136 B


def c4_wide_workload(n_tapes: int = 48, n_models: int = 2048, seed: int = 44, sizes: Sequence[int] = WIDE_SIZES,
                     planted_frac: float = 0.3, hasher=None, hoist: bool = False):
    """Keccak inputs LONGER than 64 bytes, the shape of ``WalletLibrary.sol:134``
    (``keccak256(msg.data)`` on ``changeOwner(address,address)``: 68 bytes = 544 bits) and of
    ``abi.encode`` of three words (768 bits), plus a 136-byte (one full keccak block) input.

    Mythril hashes ``Concat`` of memory bytes (instructions.py:1017-1052) through the UF
    ``keccak256_<n>``; the manager's axioms (keccak_function_manager.py:116-179) for EVERY input of
    the run ride on every query: ``inv(f(x)) == x`` at n bits, interval + ``urem 64`` on f(x), or a
    match with a concretely hashed input.  Candidate models are z3-shaped: ``keccak256_<n>`` maps the
    model's own input to a multiple of 64 inside the size's interval (what a solver picks) and each
    concrete input to its true digest; ``keccak256_<n>-1`` inverts both.  Paths: actor caller,
    selector dispatch, ``pending[h]`` storage reads keyed by the hash, interval comparisons on h
    and a selector re-read through the inverse (``Extract`` of a > 512-bit UF result).
    Returns ``(tapes, models, expected first hits, records)`` (``records`` = the Model objects)."""
    from .function_managers import KeccakFunctionManager
    from .lower import serialize_models
    from .smt_model import Model

    if hasher is None:
        from .evaluator import default_evaluator
        hasher = lambda b: default_evaluator().keccak256([b])[0]   # noqa: E731
    rng = np.random.Generator(np.random.PCG64(seed))
    km = KeccakFunctionManager(hasher=hasher)
    for n in sizes:                      # intervals in a fixed order (first use order in Mythril)
        km.interval(n)
    nmax = max(sizes) // 8
    tx = _Tx(1)
    data = {n: S.Concat(*[tx.byte(i) for i in range(n // 8)]) for n in sizes}
    # one concretely hashed input per size (constant keys: find_concrete_keccak, kfm.py:56-69)
    conc = {n: int.from_bytes(rng.bytes(n // 8), "big") for n in sizes}
    conc_h = {n: km.create_keccak(S.BitVecVal(conc[n], n)).value for n in sizes}
    hashes = {n: km.create_keccak(data[n]) for n in sizes}
    axioms = km.create_conditions()
    f = {n: km.get_function(n) for n in sizes}

    # candidate models
    records = []
    wit = []
    for m in range(n_models):
        who = int(rng.integers(0, 10))
        sender = ACTORS[who // 3] if who < 9 else int.from_bytes(rng.bytes(20), "big")
        cds = int(rng.integers(4, nmax + 24))
        cd = [int(x) for x in rng.integers(0, 256, nmax + 24)]
        funcs = {"1_calldata": ({(i,): cd[i] for i in range(len(cd))}, 0)}
        vals = {}
        for n in sizes:
            x = 0
            for i in range(n // 8):
                x = (x << 8) | (cd[i] if i < cds else 0)
            lo, hi = km.interval(n)
            v = (lo + 63) // 64 * 64 + 64 * int(rng.integers(0, 1 << 40))
            assert v < hi
            fwd, inv = f[n]
            funcs[fwd.name] = ({(x,): v, (conc[n],): conc_h[n]}, 0)
            funcs[inv.name] = ({(v,): x, (conc_h[n],): conc[n]}, 0)
            vals[n] = (x, v)
        records.append(Model({"sender_1": sender, "1_calldatasize": cds}, funcs))
        wit.append({"sender": sender, "cds": cds, "cd": cd, "vals": vals})

    def path(w, planted_: bool) -> S.Term:
        cs = [S.Or(*[tx.sender == a for a in ACTORS]),
              _holds(S.ULT(tx.cds, S.BitVecVal(4, 256)), w["cds"] < 4)]
        sel = _word_val(w["cd"], w["cds"], 0) >> 224
        cs.append(S.Extract(255, 224, tx.word(0)) == sel)
        pending = S.K(256, 256, 0)
        for n in sizes:
            pending = S.Store(pending, S.BitVecVal(conc_h[n], 256), 1)
        for n in sizes:
            if rng.random() < 0.25:
                continue
            h = hashes[n]
            x, v = w["vals"][n]
            cs.append(_holds(S.Select(pending, h) == 0, v not in conc_h.values()))
            t = int.from_bytes(rng.bytes(32), "big") | (1 << 255)
            cs.append(_holds(S.ULT(h, S.BitVecVal(t, 256)), v < t))
            # the selector read back through the inverse: a > 512-bit UF result, Extract'ed
            cs.append(S.Extract(n - 1, n - 32, f[n][1](h)) == (x >> (n - 32)))
        return S.And(*cs, axioms)

    roots, expected = [], np.full(n_tapes, -1, np.int32)
    planted = rng.random(n_tapes) < planted_frac
    for t in range(n_tapes):
        if planted[t]:
            while True:
                p = int(rng.integers(n_models))
                if wit[p]["sender"] in ACTORS and wit[p]["cds"] >= 4:
                    break
            roots.append(path(wit[p], True))
            expected[t] = p   # the first hit can be lower: fixed below against the oracle
        else:
            g = {"sender": ACTORS[0], "cds": 200, "cd": [int(x) for x in rng.integers(0, 256, nmax + 24)],
                 "vals": {n: (0, 0) for n in sizes}}
            roots.append(path(g, False))
    tb, syms, ok = lower_batch(roots, SymbolTable(), hoist=hoist)
    assert ok.all()
    return tb, serialize_models(records, syms), expected, records


# ====================================================================== the drop-in shape
def evm_model_record(wit: Dict, n_tx: int):
    """A candidate model as the z3 solver would return it for an EVM path (the LRU keys of
    ModelCache, support_utils.py:58): senders, call values, calldata sizes, the calldata arrays'
    as-array interpretations and the balance table (smt_model.Model, no completion)."""
    from .smt_model import Model
    asg, funcs = {}, {}
    for k in range(n_tx):
        asg[f"sender_{k + 1}"] = wit["sender"][k]
        asg[f"call_value{k + 1}"] = wit["value"][k]
        asg[f"{k + 1}_calldatasize"] = wit["cds"][k]
        funcs[f"{k + 1}_calldata"] = ({(i,): b for i, b in enumerate(wit["bytes"][k])}, 0)
    bal, els = wit["balance"]
    funcs["balance"] = ({(a,): v for a, v in bal.items()}, els)
    return Model(asg, funcs)


def dropin_workload(n_queries: int, n_models: int, seed: int = 7, n_tx: int = 3, planted_frac: float = 0.3,
                    checks_per_tx: Tuple[int, int] = (3, 6), query_seed: int = None):
    """Quick-sat at the reference's own shape: ``n_models`` <= 100 cached
    models (the LRU, MRU first) and ``n_queries`` EVM-shaped path conjunctions, a fraction of them
    satisfied by one of the cached models.  ``query_seed`` draws another query set over the same
    models (default: ``seed``).  Returns ``(exprs, records, planted index or -1)``."""
    rng = np.random.Generator(np.random.PCG64(seed if query_seed is None else (seed, query_seed)))
    models = EvmModels(seed, n_models, n_tx)
    ghost = EvmModels(seed + 1_000_003, max(1, n_queries), n_tx, 0, 0)
    records = [evm_model_record(models.witness(m), n_tx) for m in range(n_models)]
    exprs, planted = [], []
    for q in range(n_queries):
        if rng.random() < planted_frac:
            p = int(rng.integers(n_models))
            wit = models.witness(p)
            if all(x in ACTORS for x in wit["sender"]):
                exprs.append(evm_path(rng, wit, n_tx, checks_per_tx))
                planted.append(p)
                continue
        exprs.append(evm_path(rng, ghost.witness(q), n_tx, checks_per_tx))
        planted.append(-1)
    return exprs, records, planted


def fork_workload(n_queries: int, n_models: int, seed: int = 8, n_tx: int = 3,
                  checks_per_tx: Tuple[int, int] = (3, 6)):
    """Fork-pruning queries (svm.py:351-358): each query is a path that a cached model satisfies
    plus ONE new branch condition on the last transaction's calldata — the successor of a JUMPI —
    which that model falsifies.  These are the misses a candidate generator can answer without
    z3.  Returns ``(exprs, records, parent index)`` (records = the cached models, MRU first)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    models = EvmModels(seed, n_models, n_tx)
    records, wits = [], []
    for m in range(n_models):
        w = models.witness(m)
        w["sender"] = [ACTORS[int(rng.integers(3))] if s not in ACTORS else s for s in w["sender"]]
        wits.append(w)
        records.append(evm_model_record(w, n_tx))
    exprs, parents = [], []
    tx = _Tx(n_tx)
    for q in range(n_queries):
        p = int(rng.integers(n_models))
        wit = wits[p]
        path = evm_path(rng, dict(wit), n_tx, checks_per_tx)
        B, cds = wit["bytes"][n_tx - 1], wit["cds"][n_tx - 1]
        kind = int(rng.integers(4))
        if kind == 0:      # require(arg == c): the parent's argument differs
            c = int.from_bytes(rng.bytes(4), "big")
            cond = S.Extract(31, 0, tx.word(36)) == c
        elif kind == 1:    # if (arg < c) with the parent on the other side
            W = _word_val(B, cds, 36)
            c = int(rng.integers(1, 1 << 16))
            cond = S.ULT(tx.word(36), S.BitVecVal(c, 256)) if W >= c else S.Not(S.ULT(tx.word(36), S.BitVecVal(c, 256)))
        elif kind == 2:    # a flag byte of the first argument
            c = int(rng.integers(0, 256))
            cond = S.Extract(7, 0, tx.word(4)) == c
            if (_word_val(B, cds, 4) & 0xFF) == c:
                cond = S.Not(cond)
        else:              # calldata size branch
            c = int(rng.integers(4, 100))
            cond = S.ULT(tx.cds, S.BitVecVal(c, 256)) if cds >= c else S.Not(S.ULT(tx.cds, S.BitVecVal(c, 256)))
        exprs.append(S.And(*(path.args + (cond,))))
        parents.append(p)
    return exprs, records, parents


def fork_stream_workload(n_forks: int, n_models: int, seed: int = 21, n_tx: int = 3,
                         checks_per_tx: Tuple[int, int] = (3, 6)):
    """The per-fork check of svm.py:351-358 with a KNOWN witness for every successor, for the
    "z3 calls avoided" leg: each fork takes a path a cached model satisfies (evm_path over that
    model's witness) and branches on the last call's THIRD ABI argument (calldata bytes 68..99, a
    ``require(arg == c)``, ``if (arg < c)`` or flag-byte test; the path never reads those bytes).
    One successor is satisfied by the parent model (a quick-sat hit); the other is satisfiable
    too, by the parent's witness with the argument set and the calldata size raised to 100 (the
    bytes between the old size and 68 zeroed, so the path's words read the same): the model an
    SMT solver would return, which get_model then caches (model.py:124-126).

    Returns ``(states, witnesses, records)``: per successor its conjunct list and a satisfying
    Model (None never occurs: every successor is satisfiable), and the cached models (MRU
    first)."""
    import copy
    rng = np.random.Generator(np.random.PCG64(seed))
    models = EvmModels(seed, n_models, n_tx)
    records, wits = [], []
    for m in range(n_models):
        w = models.witness(m)
        w["sender"] = [ACTORS[int(rng.integers(3))] if s not in ACTORS else s for s in w["sender"]]
        wits.append(w)
        records.append(evm_model_record(w, n_tx))
    tx = _Tx(n_tx)
    arg = tx.word(68)
    states, witnesses = [], []
    for f in range(n_forks):
        p = int(rng.integers(n_models))
        path = evm_path(rng, dict(wits[p]), n_tx, checks_per_tx)
        conj = list(path.args) if path.kind == S.AND else [path]

        def witness(value: int):
            w = copy.deepcopy(wits[p])
            k = n_tx - 1
            b = list(w["bytes"][k]) + [0] * max(0, 100 - len(w["bytes"][k]))
            for i in range(min(w["cds"][k], 68), 68):
                b[i] = 0
            for i in range(32):
                b[68 + i] = (value >> (8 * (31 - i))) & 0xFF
            w["bytes"][k] = b
            w["cds"][k] = 100
            return evm_model_record(w, n_tx)

        kind = int(rng.integers(3))
        if kind == 0:      # require(arg == c): the parent's argument (0) differs
            c = int(rng.integers(1, 1 << 32))
            cond, sat_value = S.Extract(31, 0, arg) == c, c
        elif kind == 1:    # if (arg < c): the parent (0) takes the branch, the other side needs arg >= c
            c = int(rng.integers(1, 1 << 16))
            cond, sat_value = S.Not(S.ULT(arg, S.BitVecVal(c, 256))), c
        else:              # a flag byte of the argument
            c = int(rng.integers(1, 256))
            cond, sat_value = S.Extract(7, 0, arg) == c, c
        states += [conj + [S.Not(cond)], conj + [cond]]
        witnesses += [records[p], witness(sat_value)]
    return states, witnesses, records


def fork_children(parents: Sequence[S.Term], n_tx: int = 3, seed: int = 9) -> List[S.Term]:
    """The two successors of a JUMPI after each parent path (svm.py:351-358): ``parent + cond``
    and ``parent + Not(cond)``, with ``cond`` a branch condition on the last transaction's
    calldata (an argument compare, a flag byte or a calldata-size check).  The children reuse
    the parents' conjunct terms (interned), as LASER's forked states share their constraints."""
    rng = np.random.Generator(np.random.PCG64(seed))
    tx = _Tx(n_tx)
    out = []
    for p in parents:
        kind = int(rng.integers(3))
        if kind == 0:
            cond = S.ULT(tx.word(36), S.BitVecVal(int(rng.integers(1, 1 << 16)), 256))
        elif kind == 1:
            cond = S.Extract(7, 0, tx.word(4)) == int(rng.integers(0, 256))
        else:
            cond = S.ULT(tx.cds, S.BitVecVal(int(rng.integers(4, 100)), 256))
        conj = list(p.args) if p.kind == S.AND else [p]
        out += [S.And(*(conj + [cond])), S.And(*(conj + [S.Not(cond)]))]
    return out


def merge_workload(n_queries: int, n_models: int, seed: int = 31):
    """The state-merge plugin's shapes (laser/plugin/plugins/state_merge/merge_states.py): two
    world states joined under a merge condition, the balances as ``If(c, balances1, balances2)``
    (:27-29) and an account's storage as an If of the two storages (:95-107), read and written
    afterwards — selects through the merged arrays at symbolic and constant indices, stores over
    them, nested merges.  Models interpret the arrays ``as-array`` (smt_model.Model functions)
    with random tables.  Returns ``(exprs, records)``."""
    from .smt_model import Model
    rng = np.random.Generator(np.random.PCG64(seed))
    cond = [S.BoolSym("merge_cond_1"), S.BitVecSym("call_value1", 256) == 0]
    bal = [S.Array(f"balance_{i}", 256, 256) for i in range(3)]
    sto = [S.Array(f"Storage_{i}", 256, 256) for i in range(2)]
    addr = [S.BitVecSym(f"sender_{i}", 256) for i in range(1, 3)]
    keys = [0, 1, 2, 3, 0xAFFE, 0xDEADBEEF]
    cst = lambda v: S.BitVecVal(int(v), 256)  # noqa: E731
    exprs = []
    for _ in range(n_queries):
        c = cond[int(rng.integers(2))]
        merged = S.If(c, bal[0], bal[1])
        if rng.random() < 0.4:   # a transfer after the merge: stores over the merged balances
            a = addr[int(rng.integers(2))]
            v = cst(rng.integers(1, 50))
            merged = S.Store(S.Store(merged, a, merged[a] - v), cst(keys[int(rng.integers(6))]), merged[a] + v)
        if rng.random() < 0.3:   # a second merge over the first (a three-way join)
            merged = S.If(S.Not(cond[1] if c is cond[0] else cond[0]), merged, bal[2])
        storage = S.If(S.ULT(addr[0], cst(0x10000)), S.Store(S.K(256, 256, 0), cst(7), cst(70)), sto[0])
        if rng.random() < 0.5:
            storage = S.Store(storage, cst(keys[int(rng.integers(6))]), addr[1])
        conj = []
        for _ in range(int(rng.integers(1, 4))):
            kind = int(rng.integers(4))
            idx = addr[int(rng.integers(2))] if rng.random() < 0.5 else cst(keys[int(rng.integers(6))])
            if kind == 0:
                conj.append(S.UGE(merged[idx], cst(rng.integers(0, 40))))
            elif kind == 1:
                conj.append(S.ULT(merged[idx], merged[cst(keys[int(rng.integers(6))])]))
            elif kind == 2:
                conj.append(storage[idx] == cst(rng.integers(0, 4) * 35))
            else:
                conj.append(S.Not(storage[idx] == merged[idx]))
        exprs.append(S.And(*conj))
    records = []
    for _ in range(n_models):
        asg = {"merge_cond_1": bool(rng.integers(2)), "call_value1": int(rng.integers(0, 2)),
               "sender_1": keys[int(rng.integers(6))] if rng.random() < 0.8 else int(rng.integers(1 << 20)),
               "sender_2": keys[int(rng.integers(6))]}
        funcs = {}
        for name in ("balance_0", "balance_1", "balance_2", "Storage_0"):
            if rng.random() < 0.9:
                funcs[name] = ({(k,): int(rng.integers(0, 80)) for k in keys if rng.random() < 0.6},
                               int(rng.integers(0, 3)) * 35)
        records.append(Model(asg, funcs))
    return exprs, records
