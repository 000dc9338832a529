"""The z3 side of the lowering pass (mythril_amd/lower_z3.py) executed through a z3 stand-in
(tests/fake_z3.py: the SURVEY Appendix F surface, no z3 needed).

Every ``_lower_node`` kind, every model-reading form (constants, ``FuncInterp`` tables, arrays
as ``as-array`` / ``K`` / ``Store`` chains) and every fail-closed branch is driven here.  The
lowered tapes are evaluated by the oracle (oracle/cref.c) against the serialized models and
compared with the stand-in's own evaluator, which works on the stand-in's term objects and
shares no code with the tape IR.  Parity with real z3 remains UNPINNED (z3 is absent from every
host of this pipeline): this checks the lowering and the model reader, not z3's semantics.
"""
from __future__ import annotations

import dis
import os
import sys
import types

import numpy as np
import pytest

import cref
import fake_z3 as Z

C = Z.C


@pytest.fixture()
def lz3():
    saved = Z.install()
    try:
        import mythril_amd.lower_z3 as mod
        yield mod
    finally:
        Z.uninstall(saved)


# ----------------------------------------------------------------------------- term generator
WIDTHS = (8, 64, 160, 256)


class Gen:
    """Random stand-in terms over a fixed symbol set, every lowered kind reachable."""

    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)
        self.vars = {w: [Z.BitVec(f"x{w}_{i}", w) for i in range(3)] for w in WIDTHS}
        self.bools = [Z.Bool(f"b{i}") for i in range(2)]
        bv = Z.BitVecSort
        self.arr = {w: Z.Array(f"arr{w}", bv(w), bv(w)) for w in (8, 256)}
        self.barr = Z.Array("flags", bv(8), Z.BoolSort())
        self.f1 = Z.Function("keccak256_512", bv(512), bv(256))
        self.f1i = Z.Function("keccak256_512-1", bv(256), bv(512))
        self.f2 = Z.Function("Power", bv(256), bv(256), bv(256))
        self.fb = Z.Function("pred", bv(64), Z.BoolSort())

    def var(self, w):
        if w not in self.vars:
            self.vars[w] = [Z.BitVec(f"x{w}_{i}", w) for i in range(3)]
        return self.vars[w][self.r(3)]

    def r(self, n):
        return int(self.rng.integers(0, n))

    def const(self, w):
        c = self.r(6)
        if c == 0:
            v = self.r(4)
        elif c == 1:
            v = (1 << w) - 1 - self.r(3)
        elif c == 2:
            v = 1 << (w - 1)
        else:
            v = int.from_bytes(self.rng.bytes(64), "little")
        return Z.BitVecVal(v, w)

    def bv(self, w, d):
        if d <= 0 or self.r(5) == 0:
            return self.var(w) if self.r(3) else self.const(w)
        k = self.r(20)
        a = lambda: self.bv(w, d - 1)  # noqa: E731
        if k == 0:
            return Z.bv_op([C.Z3_OP_BADD, C.Z3_OP_BMUL, C.Z3_OP_BAND, C.Z3_OP_BOR, C.Z3_OP_BXOR][self.r(5)], a(), a(), a())
        if k in (1, 2, 3):
            ops = [C.Z3_OP_BADD, C.Z3_OP_BSUB, C.Z3_OP_BMUL, C.Z3_OP_BUDIV, C.Z3_OP_BUDIV_I, C.Z3_OP_BUREM,
                   C.Z3_OP_BUREM_I, C.Z3_OP_BSDIV, C.Z3_OP_BSDIV_I, C.Z3_OP_BSREM, C.Z3_OP_BSREM_I, C.Z3_OP_BSMOD,
                   C.Z3_OP_BSMOD_I, C.Z3_OP_BAND, C.Z3_OP_BOR, C.Z3_OP_BXOR, C.Z3_OP_BSHL, C.Z3_OP_BLSHR,
                   C.Z3_OP_BASHR, C.Z3_OP_BNAND, C.Z3_OP_BNOR, C.Z3_OP_BXNOR]
            return Z.bv_op(ops[self.r(len(ops))], a(), a())
        if k == 4:
            return Z.bv_op([C.Z3_OP_BNEG, C.Z3_OP_BNOT][self.r(2)], a())
        if k == 5:
            return Z.If(self.bool(d - 1), a(), a())
        if k == 6 and w >= 16:
            lo = self.r(w // 2)
            return Z.Concat(self.bv(w - lo, d - 1), self.bv(lo, d - 1)) if lo else a()
        if k == 7:
            src = WIDTHS[self.r(4)]
            if src > w:
                lo = self.r(src - w + 1)
                return Z.Extract(lo + w - 1, lo, self.bv(src, d - 1))
            if src < w:
                return (Z.ZeroExt if self.r(2) else Z.SignExt)(w - src, self.bv(src, d - 1))
            return a()
        if k == 8 and w % 8 == 0 and w <= 64:
            return Z.RepeatBitVec(w // 8, self.bv(8, d - 1))
        if k == 9 and w in self.arr:
            return Z.Select(self.array(w, d - 1), self.bv(w, d - 1))
        if k == 10 and w == 256:
            key = Z.Concat(self.bv(256, d - 1), self.bv(256, d - 1))
            return self.f1(key)
        if k == 11 and w == 256:
            return self.f2(self.bv(256, d - 1), self.bv(256, d - 1))
        if k == 12 and w == 256:
            return Z.Extract(255, 0, self.f1i(self.bv(256, d - 1)))
        return a()

    def array(self, w, d):
        base = self.arr[w] if self.r(3) else Z.K(Z.BitVecSort(w), self.bv(w, 0))
        for _ in range(self.r(3)):
            base = Z.Store(base, self.bv(w, max(d - 1, 0)), self.bv(w, max(d - 1, 0)))
        return base

    def bool(self, d):
        if d <= 0 or self.r(6) == 0:
            c = self.r(4)
            return self.bools[self.r(2)] if c < 2 else Z.BoolVal(c == 2)
        w = WIDTHS[self.r(4)]
        k = self.r(14)
        if k < 5:
            ops = [C.Z3_OP_ULT, C.Z3_OP_ULEQ, C.Z3_OP_UGT, C.Z3_OP_UGEQ, C.Z3_OP_SLT, C.Z3_OP_SLEQ, C.Z3_OP_SGT,
                   C.Z3_OP_SGEQ, C.Z3_OP_BUMUL_NO_OVFL, C.Z3_OP_BSMUL_NO_OVFL, C.Z3_OP_BSMUL_NO_UDFL]
            return Z.bool_op(ops[self.r(len(ops))], self.bv(w, d - 1), self.bv(w, d - 1))
        if k == 5:
            return Z.Eq(self.bv(w, d - 1), self.bv(w, d - 1))
        if k == 6:
            return Z.bool_op(C.Z3_OP_DISTINCT, self.bv(8, d - 1), self.bv(8, d - 1), self.bv(8, d - 1))
        if k == 7:
            return Z.And(*[self.bool(d - 1) for _ in range(2 + self.r(3))])
        if k == 8:
            return Z.Or(*[self.bool(d - 1) for _ in range(2 + self.r(3))])
        if k == 9:
            return Z.Not(self.bool(d - 1))
        if k == 10:
            return Z.bool_op([C.Z3_OP_XOR, C.Z3_OP_IMPLIES, C.Z3_OP_IFF][self.r(3)], self.bool(d - 1), self.bool(d - 1))
        if k == 11:
            return Z.If(self.bool(d - 1), self.bool(d - 1), self.bool(d - 1))
        if k == 12:
            return Z.Select(self.barr, self.bv(8, d - 1))
        return self.fb(self.bv(64, d - 1))

    # ------------------------------------------------------------------------- models
    def lit(self, sort):
        if sort.kind() == Z.Z3_BOOL_SORT:
            return Z.BoolVal(bool(self.r(2)))
        w = sort.size()
        return Z.BitVecVal(self.r(4) if self.r(2) else int.from_bytes(self.rng.bytes(64), "little"), w)

    def interp(self, decl, n):
        ents = [Z.FuncEntry([self.lit(decl.domain(j)) for j in range(decl.arity())], self.lit(decl.range()))
                for _ in range(n)]
        return Z.FuncInterp(decl.arity(), ents, self.lit(decl.range()))

    def model(self, exprs_terms=()):
        m = Z.ModelRef()
        for w in list(self.vars):
            for x in self.vars[w]:
                if self.r(5):                       # some constants absent: completion gives 0
                    m.set(x.decl(), self.lit(x.sort()))
        for b in self.bools:
            if self.r(3):
                m.set(b.decl(), self.lit(b.sort()))
        # UF tables, entries drawn so lookups of small arguments hit
        for f in (self.f1, self.f1i, self.f2, self.fb):
            if self.r(4):
                m.set(f, self.interp(f, self.r(4)))
        # arrays: as-array of a FuncInterp, K, Store chain over K
        for w, a in list(self.arr.items()) + [(8, self.barr)]:
            form = self.r(4)
            if form == 0:
                continue
            if form == 1:
                fdecl = Z.FuncDeclRef(f"{a.decl().name()}!as", C.Z3_OP_UNINTERPRETED, (), (a.sort().domain(),),
                                      a.sort().range())
                m.set(fdecl, self.interp(fdecl, 1 + self.r(4)))
                m.set(a.decl(), Z.AsArray(fdecl))
            elif form == 2:
                m.set(a.decl(), Z.K(a.sort().domain(), self.lit(a.sort().range())))
            else:
                v = Z.K(a.sort().domain(), self.lit(a.sort().range()))
                for _ in range(1 + self.r(3)):
                    v = Z.Store(v, self.lit(a.sort().domain()), self.lit(a.sort().range()))
                m.set(a.decl(), v)
        return m


class Wrapped:
    """A mythril ``Model`` wrapper: ``.raw`` = [ModelRef] (smt/model.py:13-18); hashed by
    identity, as the reference's LRU keys are."""

    def __init__(self, m):
        self.raw = [m]


def wrap(m):
    return Wrapped(m)


def fake_rows(exprs, models):
    return np.array([[Z.is_true(m.eval(e, model_completion=True)) for m in models] for e in exprs], bool)


# ----------------------------------------------------------------------------- exercises
def exercise_random(lz3, seed=0, n_exprs=160, n_models=24, depth=4):
    g = Gen(seed)
    exprs = [g.bool(depth) for _ in range(n_exprs)]
    models = [g.model() for _ in range(n_models)]
    tb, mb, ok = lz3.lower_batch_z3(exprs, [wrap(m) for m in models])
    assert ok.all()
    got = cref.verdicts(tb, mb)
    exp = fake_rows(exprs, models)
    bad = np.argwhere(got != exp)
    assert len(bad) == 0, (len(bad), exprs[bad[0][0]] if len(bad) else None)
    # both outcomes occur (the comparison is not vacuous)
    assert exp.any() and (~exp).any()
    return exprs, models, exp


def exercise_shapes(lz3):
    """EVM shapes of SURVEY Appendix D through the z3 side: actor constraint, calldata bytes from
    a symbolic array (signed bound), dispatch by LShR + Extract, a storage read from a Store chain
    over K, the keccak axioms' UF pair and Power."""
    bv = Z.BitVecSort
    sender = Z.BitVec("sender_1", 256)
    size = Z.BitVec("1_calldatasize", 256)
    cd = Z.Array("1_calldata", bv(256), bv(8))
    actors = [Z.BitVecVal(0xAFFE << 240, 256), Z.BitVecVal(0xDEADBEEF, 256)]
    actor = Z.Or(*[Z.Eq(sender, a) for a in actors])
    byte = lambda i: Z.If(Z.bool_op(C.Z3_OP_SLT, Z.BitVecVal(i, 256), size),  # noqa: E731
                          Z.Select(cd, Z.BitVecVal(i, 256)), Z.BitVecVal(0, 8))
    word0 = Z.Concat(*[byte(i) for i in range(32)])
    sel = Z.Eq(Z.Extract(31, 0, Z.bv_op(C.Z3_OP_BLSHR, word0, Z.BitVecVal(224, 256))), Z.BitVecVal(0xA9059CBB, 32))
    kf = Z.Function("keccak256_512", bv(512), bv(256))
    kfi = Z.Function("keccak256_512-1", bv(256), bv(512))
    key = Z.Concat(sender, Z.BitVecVal(1, 256))
    storage = Z.Store(Z.K(bv(256), Z.BitVecVal(0, 256)), kf(key), Z.BitVecVal(100, 256))
    bal = Z.Select(storage, kf(key))
    ax = Z.And(Z.Eq(kfi(kf(key)), key), Z.bool_op(C.Z3_OP_ULEQ, Z.BitVecVal(10, 256), kf(key)))
    pw = Z.Function("Power", bv(256), bv(256), bv(256))
    exp_c = Z.bool_op(C.Z3_OP_SGT, pw(Z.BitVecVal(256, 256), Z.BitVecVal(2, 256)), Z.BitVecVal(0, 256))
    exprs = [Z.And(actor, sel), Z.And(actor, Z.bool_op(C.Z3_OP_UGEQ, bal, Z.BitVecVal(50, 256))), ax, exp_c,
             Z.And(sel, ax, exp_c)]
    models = []
    for s_val, words, kv, pv in ((0xDEADBEEF, 0xA9059CBB, 11, 65536), (1, 0xA9059CBB, 5, 0), (0xAFFE << 240, 0, 10, 1)):
        m = Z.ModelRef()
        m.set(sender.decl(), Z.BitVecVal(s_val, 256))
        m.set(size.decl(), Z.BitVecVal(68, 256))
        f = Z.FuncDeclRef("cd!as", C.Z3_OP_UNINTERPRETED, (), (bv(256),), bv(8))
        ents = [Z.FuncEntry([Z.BitVecVal(i, 256)], Z.BitVecVal((words >> (8 * (3 - i))) & 0xFF, 8)) for i in range(4)]
        m.set(f, Z.FuncInterp(1, ents, Z.BitVecVal(0, 8)))
        m.set(cd.decl(), Z.AsArray(f))
        keyv = (s_val << 256) | 1
        m.set(kf, Z.FuncInterp(1, [Z.FuncEntry([Z.BitVecVal(keyv, 512)], Z.BitVecVal(kv, 256))], Z.BitVecVal(3, 256)))
        m.set(kfi, Z.FuncInterp(1, [Z.FuncEntry([Z.BitVecVal(kv, 256)], Z.BitVecVal(keyv, 512))], Z.BitVecVal(0, 512)))
        m.set(pw, Z.FuncInterp(2, [Z.FuncEntry([Z.BitVecVal(256, 256), Z.BitVecVal(2, 256)], Z.BitVecVal(pv, 256))],
                               Z.BitVecVal(0, 256)))
        models.append(m)
    tb, mb, ok = lz3.lower_batch_z3(exprs, [wrap(m) for m in models])
    assert ok.all()
    got = cref.verdicts(tb, mb)
    exp = fake_rows(exprs, models)
    assert (got == exp).all(), (got, exp)
    assert exp[0].tolist() == [True, False, False]       # selector + actor: only model 0
    assert exp[2].tolist() == [True, False, True]        # the keccak axiom pair
    return exprs, models, exp


def exercise_fail_closed(lz3):
    """Every kind outside the vocabulary is rejected (ok False), the rest of the batch lowers."""
    bv = Z.BitVecSort
    x = Z.BitVec("x", 256)
    good = Z.bool_op(C.Z3_OP_ULT, x, Z.BitVecVal(5, 256))
    a1, a2 = Z.Array("A", bv(256), bv(256)), Z.Array("B", bv(256), bv(256))
    barr = Z.Array("Bd", Z.BoolSort(), bv(8))
    f3 = Z.Function("f3", bv(8), bv(8), bv(8), bv(8))
    rej = [
        Z.ForAll(good),                                                     # quantifier
        Z.Eq(a1, a2),                                                       # array equality
        Z.Eq(Z._mk(C.Z3_OP_ROTATE_LEFT, bv(256), (x,), params=(3,)), x),    # kind outside the set
        Z.Eq(Z.Select(barr, Z.BoolVal(True)), Z.BitVecVal(0, 8)),           # array over a Bool domain
        Z.Eq(Z.Int("i"), Z.Int("j")),                                       # an Int sort
        Z.Eq(f3(Z.BitVecVal(1, 8), Z.BitVecVal(2, 8), Z.BitVecVal(3, 8)), Z.BitVecVal(0, 8)),   # arity 3
    ]
    exprs = [good] + rej + [good]
    m = Z.ModelRef()
    m.set(x.decl(), Z.BitVecVal(3, 256))
    from mythril_amd.exceptions import fail_closed
    before = dict(fail_closed)
    tb, mb, ok = lz3.lower_batch_z3(exprs, [wrap(m)])
    assert ok.tolist() == [True] + [False] * len(rej) + [True]
    # each rejected query is counted under its reason (the state-merge shapes by name)
    new = {k: fail_closed[k] - before.get(k, 0) for k in fail_closed if fail_closed[k] != before.get(k, 0)}
    assert sum(new.values()) == len(rej), new
    assert new.get("array equality") == 1, new
    v = cref.verdicts(tb, mb)
    assert v[0, 0] and v[-1, 0]
    # a model whose interpretation cannot be read routes the whole batch to the z3 loop
    bad = Z.ModelRef()
    bad.set(x.decl(), x)                                   # a value that is not a literal
    _, _, ok2 = lz3.lower_batch_z3([good], [wrap(bad)])
    assert not ok2.any()
    bad2 = Z.ModelRef()
    bad2.set(a1.decl(), Z.Store(Z.AsArray(Z.Function("g", bv(256), bv(256))), Z.BitVecVal(1, 256), Z.BitVecVal(2, 256)))
    with pytest.raises(Exception):
        lz3.model_record(wrap(bad2))


def exercise_loop_and_backend(lz3, exprs, models, exp):
    """z3_quick_sat_loop (support_utils.py:62-66) against the rows; Z3Backend (model.py:28-65)."""
    for e, row in zip(exprs[:40], exp[:40]):
        got = lz3.z3_quick_sat_loop(e, models)
        want = models[int(np.argmax(row))] if row.any() else False
        assert got is want
    be = lz3.Z3Backend()
    x = Z.BitVec("x64_0", 64)
    Z.Optimize.candidates = models
    Z.Optimize.exhaustive = False
    st, fac = be.solve([Z.bool_op(C.Z3_OP_ULT, x, Z.BitVecVal(1 << 63, 64))], [x], [], 250)
    assert st == "sat" and fac() is not None
    assert Z.Optimize.last.params == {"timeout": 250} and Z.Optimize.last.objectives[0][0] == "min"
    st, fac = be.solve([Z.BoolVal(False)], [], [x], 10)
    assert st == "unknown" and fac is None
    Z.Optimize.exhaustive = True
    st, _ = be.solve([Z.BoolVal(False)], [], [], 10)
    assert st == "unsat"
    # with mythril importable, the model comes back in the caller's Model wrapper
    mm = types.ModuleType("mythril.laser.smt.model")
    mm.Model = lambda raws: ("wrapped", raws)
    saved = {k: sys.modules.get(k) for k in ("mythril", "mythril.laser", "mythril.laser.smt", "mythril.laser.smt.model")}
    for k in saved:
        sys.modules[k] = mm if k.endswith("model") else types.ModuleType(k)
    try:
        st, fac = be.solve([Z.BoolVal(True)], [], [], 10)
        assert st == "sat" and fac()[0] == "wrapped"
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    Z.Optimize.candidates = []


def exercise_adapter(lz3):
    """The drop-in adapter's z3 branches on CPU: VerdictEngine lowering of z3 terms,
    ModelCache's fallback loop for an unsupported conjunction, the default solver backend."""
    from mythril_amd import support as sp
    g = Gen(3)
    exprs = [g.bool(3) for _ in range(6)]
    models = [wrap(g.model()) for _ in range(5)]
    eng = sp.VerdictEngine(evaluator=object())
    tb, mb, ok = lz3.lower_batch_z3(exprs, models)
    assert ok.all() and tb.n_tapes == 6 and mb.n_models == 5
    raw = [m.raw[0] for m in models]
    exp = fake_rows(exprs, raw)
    assert (cref.verdicts(tb, mb) == exp).all()
    # hoisted form (the generated-candidates batch shape): same verdicts
    tbh, mbh, okh = lz3.lower_batch_z3(exprs, models, hoist=True)
    assert okh.all()
    from oracle_engine import apply_columns
    assert (cref.verdicts(tbh, apply_columns(tbh, mbh) if tbh.columns is not None else mbh) == exp).all()
    mc = sp.ModelCache(eng)
    for m in models:
        mc.put(m, 1)
    order = list(reversed(mc.model_cache.lru_cache.keys()))
    q = int(np.argmax(exp.any(axis=1)))
    hit = mc._fallback(exprs[q], [m.raw[0] for m in order])
    assert hit is not False
    assert isinstance(sp._default_backend(), lz3.Z3Backend)


# ----------------------------------------------------------------------------- tests
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_terms_lower_and_evaluate_like_the_stand_in(lz3, seed):
    exercise_random(lz3, seed=seed)


def test_evm_shapes_through_the_z3_side(lz3):
    exercise_shapes(lz3)


def test_fail_closed_kinds(lz3):
    exercise_fail_closed(lz3)


def test_quick_sat_loop_and_backend(lz3):
    exercise_loop_and_backend(lz3, *exercise_random(lz3, seed=5, n_exprs=60, n_models=12))


def test_adapter_z3_branches(lz3):
    exercise_adapter(lz3)


def _executable_lines(path):
    with open(path) as f:
        code = compile(f.read(), path, "exec")
    lines, todo = set(), [code]
    while todo:
        co = todo.pop()
        if co is not code:                       # function bodies (module-level lines run at import)
            lines.update(ln for _, ln in dis.findlinestarts(co) if ln)
            lines.discard(co.co_firstlineno)     # the def line itself
        todo.extend(c for c in co.co_consts if isinstance(c, types.CodeType))
    return lines


def test_lower_z3_line_coverage(lz3):
    """The exercises above together execute >= 90 % of the function-body lines of lower_z3.py."""
    path = os.path.abspath(lz3.__file__)
    hit = set()

    def tracer(frame, event, arg):
        if frame.f_code.co_filename != path:
            return None
        if event == "line":
            hit.add(frame.f_lineno)
        return tracer

    old = sys.gettrace()
    sys.settrace(tracer)
    try:
        rows = exercise_random(lz3, seed=0, n_exprs=120)
        exercise_shapes(lz3)
        exercise_fail_closed(lz3)
        exercise_loop_and_backend(lz3, *rows)
        exercise_adapter(lz3)
    finally:
        sys.settrace(old)
    lines = _executable_lines(path)
    missed = sorted(lines - hit)
    frac = len(lines & hit) / len(lines)
    print(f"lower_z3.py line coverage {frac:.3f} ({len(lines & hit)}/{len(lines)}), missed {missed}")
    assert frac >= 0.90, f"coverage {frac:.3f}, missed lines {missed}"


@pytest.mark.gpu
def test_gpu_model_cache_on_z3_terms_matches_reference_loop(lz3, evaluator):
    """ModelCache.check_quick_sat over stand-in z3 terms (lowered by lower_z3, evaluated on the
    GPU) answers exactly as the reference loop (support_utils.py:62-66) replayed with
    z3_quick_sat_loop and the LRU bump; the final LRU order agrees too."""
    from mythril_amd import support as sp
    g = Gen(11)
    exprs = [g.bool(4) for _ in range(48)]
    raws = [g.model() for _ in range(20)]
    models = [wrap(m) for m in raws]
    mc = sp.ModelCache(sp.VerdictEngine(evaluator))
    ref_order = []
    for m in models:
        mc.put(m, 1)
        ref_order.insert(0, m)
    got = mc.check_quick_sat_batch(exprs[:24]) + [mc.check_quick_sat(e) for e in exprs[24:]]
    for e, ans in zip(exprs, got):
        hit = lz3.z3_quick_sat_loop(e, [m.raw[0] for m in ref_order])
        want = False if hit is False else next(m for m in ref_order if m.raw[0] is hit)
        assert ans is want
        if want is not False:
            ref_order.remove(want)
            ref_order.insert(0, want)
    assert list(reversed(mc.model_cache.lru_cache.keys())) == ref_order
    assert any(a is not False for a in got) and any(a is False for a in got)


# ----------------------------------------------------------------------------- the incremental z3 path
def _z3_fork_stream(n_parents=8, n_models=24, seed=11):
    """Parents (EVM-shaped paths) and their JUMPI children (svm.py:351-358) as stand-in z3 ASTs,
    the cached models as stand-in ModelRefs (the MRU-first LRU order)."""
    import z3_bridge as B
    from mythril_amd.synth_evm import dropin_workload, fork_children
    exprs, recs, _ = dropin_workload(n_parents, n_models, seed=seed)
    kids = fork_children(exprs)
    sig = B.signature(exprs + kids)
    to = B.ToZ3()
    return [to(e) for e in exprs], [to(e) for e in kids], [B.model_to_z3(r, sig) for r in recs]


def _run_z3_stream(lz3, engine, parents, kids, models):
    """check_quick_sat over the parents, then the children, through ModelCache on z3 ASTs; the
    answers and final LRU order against the reference loop replayed on the stand-in evaluator."""
    import z3_bridge as B
    from mythril_amd import support as sp
    mc = sp.ModelCache(engine)
    for m in reversed(models):
        mc.put(m, 1)
    got = mc.check_quick_sat_batch(parents)
    evaluated = engine.stats["conjuncts_evaluated"]
    translated = engine._z3.translated
    got += mc.check_quick_sat_batch(kids)
    want, order = B.reference_replay(parents + kids, models, lz3)
    assert all(a is b for a, b in zip(got, want)), [(a is b) for a, b in zip(got, want)]
    assert list(reversed(mc.model_cache.lru_cache.keys())) == order
    assert any(a is not False for a in got) and any(a is False for a in got)
    return got, evaluated, translated


def test_z3_fork_stream_takes_the_incremental_path(lz3):
    """model.py:101 hands quick-sat a z3 BoolRef.  A fork stream of such queries is translated
    once per AST into the persistent DAG: the children's parent conjuncts are answered from
    cached per-conjunct rows (conjuncts_cached > 0), only their new branch conditions reach the
    device, the z3 models are read once, and the answers and LRU order are the reference
    loop's (z3_quick_sat_loop, the stand-in's own evaluator)."""
    from oracle_engine import OracleEngine
    parents, kids, models = _z3_fork_stream()
    eng = OracleEngine()
    reads = []
    real = lz3.model_record

    def counting(m):
        reads.append(id(m))
        return real(m)
    lz3.model_record = counting
    try:
        _, evaluated, translated = _run_z3_stream(lz3, eng, parents, kids, models)
    finally:
        lz3.model_record = real
    st = eng.stats
    assert st["conjuncts_cached"] > 0
    # each child pair adds one branch condition and its negation: 2 new conjuncts per parent
    assert st["conjuncts_evaluated"] - evaluated <= 2 * len(parents)
    # the children's new ASTs: cond, Not(cond), two And roots and the condition's few sub-terms
    assert eng._z3.translated - translated <= 16 * len(parents)
    assert len(reads) == len(set(reads)) == len(models)   # every z3 model read once


def test_z3_state_merge_shapes_lower(lz3):
    """The state-merge plugin's array-valued If (merge_states.py:27-29,95-107) through the z3 side:
    selects read through the merged balances / storage, stores over the merge included."""
    bv = Z.BitVecSort
    c = Z.Bool("merge_cond")
    b1, b2 = Z.Array("balance_1", bv(256), bv(256)), Z.Array("balance_2", bv(256), bv(256))
    s1 = Z.Store(Z.K(bv(256), Z.BitVecVal(0, 256)), Z.BitVecVal(7, 256), Z.BitVecVal(70, 256))
    s2 = Z.Array("Storage_2", bv(256), bv(256))
    x = Z.BitVec("x", 256)
    merged_bal = Z.If(c, b1, b2)
    merged_st = Z.Store(Z.If(Z.bool_op(C.Z3_OP_ULT, x, Z.BitVecVal(9, 256)), s1, s2), Z.BitVecVal(3, 256), x)
    nested = Z.If(Z.Not(c), merged_bal, Z.Store(b1, x, Z.BitVecVal(1, 256)))
    exprs = [Z.bool_op(C.Z3_OP_UGEQ, Z.Select(merged_bal, x), Z.BitVecVal(5, 256)),
             Z.Eq(Z.Select(merged_st, Z.BitVecVal(7, 256)), Z.BitVecVal(70, 256)),
             Z.Eq(Z.Select(merged_st, Z.BitVecVal(3, 256)), Z.BitVecVal(2, 256)),
             Z.Eq(Z.Select(merged_st, x), Z.BitVecVal(0, 256)),
             Z.bool_op(C.Z3_OP_ULT, Z.Select(nested, Z.BitVecVal(2, 256)), Z.Select(merged_bal, Z.BitVecVal(2, 256)))]
    g = Gen(21)
    models = []
    for i in range(24):
        m = Z.ModelRef()
        if i % 3:
            m.set(c.decl(), Z.BoolVal(bool(i % 2)))
        m.set(x.decl(), Z.BitVecVal([0, 2, 3, 7, 8, 11][i % 6], 256))
        for a in (b1, b2, s2):
            f = Z.FuncDeclRef(f"{a.decl().name()}!as", C.Z3_OP_UNINTERPRETED, (), (bv(256),), bv(256))
            ents = [Z.FuncEntry([Z.BitVecVal(k, 256)], Z.BitVecVal(int(g.rng.integers(0, 12)), 256)) for k in (0, 2, 3, 7, 8, 11)
                    if g.r(2)]
            m.set(f, Z.FuncInterp(1, ents, Z.BitVecVal(g.r(3), 256)))
            m.set(a.decl(), Z.AsArray(f))
        models.append(m)
    tb, mb, ok = lz3.lower_batch_z3(exprs, [wrap(m) for m in models])
    assert ok.all()
    exp = fake_rows(exprs, models)
    assert (cref.verdicts(tb, mb) == exp).all()
    assert exp.any(axis=1).all() and (~exp).any(axis=1).all()   # every query splits the models


@pytest.mark.gpu
def test_gpu_z3_fork_stream_takes_the_incremental_path(lz3, evaluator):
    """The same z3 fork stream on the GPU through libmq: answers and LRU order equal the
    reference loop's; the children reuse their parents' conjunct rows."""
    from mythril_amd import support as sp
    parents, kids, models = _z3_fork_stream(n_parents=16, n_models=40, seed=13)
    eng = sp.VerdictEngine(evaluator)
    _, evaluated, _ = _run_z3_stream(lz3, eng, parents, kids, models)
    assert eng.stats["conjuncts_cached"] > 0
    assert eng.stats["conjuncts_evaluated"] - evaluated <= 2 * len(parents)
    eng.close()
