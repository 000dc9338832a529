"""Generate the golden fixtures in tests/golden/ from the reference's own test DATA.

Run in the build container (it reads /root/reference, which does not exist on the GPU box);
the JSON it writes is committed.  Nothing here imports or executes reference code: the
reference files are read as data (JSON test vectors, and the hex-string literals of the
EIP-145 parametrize tables) and re-expressed as constraint tapes with this repo's builder.

Outputs
  shift_vectors.json  — tests/instructions/{shl,shr,sar}_test.py concrete EIP-145 vectors
                        (shl_test.py:53-114, shr_test.py:56-117, sar_test.py:54-140):
                        mythril maps SHL -> bvshl (value << shift, bitvec.py:236-241),
                        SHR -> LShR (instructions.py:572), SAR -> bvashr (``>>``, bitvec.py:243-246).
  vmtests_kats.json   — VMTests vmArithmeticTest / vmBitwiseLogicOperation post-storage values
                        (tests/laser/evm_testsuite/VMTests, harness evm_test.py:178-189) for the
                        straight-line programs, each stored word lowered to a tape with
                        mythril's EVM->BV mapping (instructions.py:360-767).
                        EXP (0x0a) goes through the product's own
                        ``function_managers.exponent_function_manager.create_condition``
                        (exponent_function_manager.py:32-60, called at instructions.py:629-642):
                        concrete operands give pow(b, e, 2^256) and the constraint
                        ``c == Power(b, e)``; the conjunction of a program's constraints is lowered
                        by the product lowering (lower.py, Power a 2-argument model table looked up
                        on the GPU) into the entry's "constraint" tape, true under a model whose
                        Power table holds the entries listed in "power".  CALLDATALOAD (0x35) reads
                        the test's concrete calldata as Mythril's ConcreteCalldata does
                        (state/calldata.py:119-147: select over a store chain on K(0), the 32
                        bytes concatenated, get_word_at :48-55); CALLDATASIZE is its length.
                        Where Mythril needs a concrete value (EXP operands, BYTE index, SSTORE /
                        MSTORE keys) the operand expression is folded as z3's simplify folds it
                        (util.get_concrete_int): evaluated by the oracle (oracle/pyoracle.py);
                        the expected values stay the VMTests' own.
  keccak_kats.json    — VMTests vmSha3Test digests (keccak of zero/constant memory) plus
                        keccak("") = get_empty_keccak_hash() (keccak_function_manager.py:86-93).
"""
from __future__ import annotations

import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import pyoracle  # noqa: E402  (test infrastructure: folds constant operands)
from mythril_amd import smt as S  # noqa: E402
from mythril_amd.function_managers import exponent_function_manager  # noqa: E402
from mythril_amd.lower import SymbolTable, lower_term  # noqa: E402
from mythril_amd.models import ModelBatch  # noqa: E402
from mythril_amd.tape import Tape, TapeBatch  # noqa: E402

_NO_MODELS = ModelBatch([], np.zeros((0, 1), np.uint32))

REF = os.environ.get("MYTHRIL_REFERENCE", "/root/reference")
VMT = os.path.join(REF, "tests", "laser", "evm_testsuite", "VMTests")
M256 = (1 << 256) - 1


def dump_tape(t: Tape, value_node: int, **extra):
    arr, consts = t.packed()
    return dict(nodes=[[int(x) for x in row] for row in arr.tolist()], consts=[int(c) for c in consts],
                value_node=int(value_node), **extra)


# ---------------------------------------------------------------- EIP-145 shift vectors
def shift_vectors():
    out = []
    for name, opname in (("shl", "shl"), ("shr", "lshr"), ("sar", "ashr")):
        src = open(os.path.join(REF, "tests", "instructions", f"{name}_test.py")).read()
        body = src
        # the concrete vectors are the 3-tuples of hex strings
        triples = re.findall(r'\(\s*"(0x[0-9a-fA-F]+)",\s*"(0x[0-9a-fA-F]+)",\s*"(0x[0-9a-fA-F]+)",?\s*\)', body)
        for i, (val, sh, exp) in enumerate(triples):
            t = Tape()
            v = t.const(int(val, 16), 256)
            s = t.const(int(sh, 16), 256)
            r = getattr(t, opname)(v, s)
            out.append(dump_tape(t, r, name=f"{name}_{i}", op=name, value=val, shift=sh, expected=exp,
                                 source=f"tests/instructions/{name}_test.py"))
    return out


# ---------------------------------------------------------------- VMTests straight-line KATs
class Skip(Exception):
    pass


def lower_program(code: bytes, t: Tape, calldata: bytes = b"", exp_conditions=None, pre_storage=None):
    """Symbolically run straight-line EVM code building tape terms with mythril's mapping.
    Returns {storage_key_int: node}.  Raises Skip for control flow / unsupported opcodes.
    ``exp_conditions`` (a list) collects (base, exponent, result, condition term) per EXP.
    ``pre_storage`` ({key: value}): the account's storage before the program (the test's "pre"),
    what an SLOAD of a key the program has not stored reads."""
    stack = []
    store = {}
    mem = {}  # byte offset -> constant byte (sha3 tests only use constant memory)
    pc = 0
    zero = t.const(0, 256)
    one = t.const(1, 256)

    def pop():
        if not stack:
            raise Skip("stack underflow")
        return stack.pop()

    def as_bv(x):
        if isinstance(x, tuple):
            raise Skip("sha3 result used as an operand")
        # Bool on the EVM stack is If(b, 1, 0) when used as a word (instructions.py:369-375)
        if t.kind[x] == "bool":
            return t.ite(x, one, zero)
        return x

    def const_value(x):
        """The concrete value of a constant expression (z3's simplify folds it; util.get_concrete_int)."""
        if isinstance(x, tuple):
            raise Skip("sha3 result used as a concrete value")
        op, w, a, b, c = t.nodes[x]
        if op == 1:
            words = t.consts[a:a + (w + 31) // 32]
            return sum(int(v) << (32 * i) for i, v in enumerate(words))
        arr, consts = t.packed()
        return int(pyoracle.eval_nodes(arr[:x + 1], np.asarray(consts, np.uint32), _NO_MODELS, 0)[x])

    while pc < len(code):
        op = code[pc]
        pc += 1
        if 0x60 <= op <= 0x7F:
            n = op - 0x5F
            stack.append(t.const(int.from_bytes(code[pc:pc + n].ljust(n, b"\0"), "big"), 256))
            pc += n
            continue
        if 0x80 <= op <= 0x8F:
            k = op - 0x7F
            if len(stack) < k:
                raise Skip("dup underflow")
            stack.append(stack[-k])
            continue
        if 0x90 <= op <= 0x9F:
            k = op - 0x8F
            if len(stack) < k + 1:
                raise Skip("swap underflow")
            stack[-1], stack[-1 - k] = stack[-1 - k], stack[-1]
            continue
        if op == 0x00:
            break
        if op == 0x50:
            pop()
            continue
        if op in (0x01, 0x02, 0x03):  # ADD MUL SUB
            a, b = as_bv(pop()), as_bv(pop())
            stack.append({0x01: t.add, 0x02: t.mul, 0x03: t.sub}[op](a, b))
            continue
        if op in (0x04, 0x05, 0x06, 0x07):  # DIV SDIV MOD SMOD: concrete 0 divisor -> 0
            a, b = as_bv(pop()), as_bv(pop())
            fn = {0x04: t.udiv, 0x05: t.sdiv, 0x06: t.urem, 0x07: t.srem}[op]
            stack.append(t.ite(t.eq(b, zero), zero, fn(a, b)))
            continue
        if op in (0x08, 0x09):  # ADDMOD / MULMOD = URem(URem(a,n) op URem(b,n), n)
            a, b, n = as_bv(pop()), as_bv(pop()), as_bv(pop())
            inner = (t.add if op == 0x08 else t.mul)(t.urem(a, n), t.urem(b, n))
            stack.append(t.urem(inner, n))
            continue
        if op == 0x0B:  # SIGNEXTEND (instructions.py:645-672)
            s0, s1 = as_bv(pop()), as_bv(pop())
            testbit = t.add(t.mul(s0, t.const(8, 256)), t.const(7, 256))
            set_tb = t.shl(one, testbit)
            sign_set = t.not_(t.eq(t.band(s1, set_tb), zero))
            neg = t.bor(s1, t.sub(zero, set_tb))
            pos = t.band(s1, t.sub(set_tb, one))
            stack.append(t.ite(t.sle(s0, t.const(31, 256)), t.ite(sign_set, neg, pos), s1))
            continue
        if op in (0x10, 0x11, 0x12, 0x13):  # LT GT SLT SGT -> Bool
            a, b = as_bv(pop()), as_bv(pop())
            stack.append({0x10: t.ult, 0x11: t.ugt, 0x12: t.slt, 0x13: t.sgt}[op](a, b))
            continue
        if op == 0x14:
            a, b = as_bv(pop()), as_bv(pop())
            stack.append(t.eq(a, b))
            continue
        if op == 0x15:
            v = pop()
            e = t.not_(v) if t.kind[v] == "bool" else t.eq(v, zero)
            stack.append(t.ite(e, one, zero))
            continue
        if op in (0x16, 0x17, 0x18):
            a, b = as_bv(pop()), as_bv(pop())
            stack.append({0x16: t.band, 0x17: t.bor, 0x18: t.bxor}[op](a, b))
            continue
        if op == 0x19:  # NOT = TT256M1 - x (instructions.py:427)
            stack.append(t.sub(t.const(M256, 256), as_bv(pop())))
            continue
        if op == 0x0A:  # EXP (instructions.py:629-642 -> exponent_function_manager.create_condition)
            base, expo = as_bv(pop()), as_bv(pop())
            b_val, e_val = const_value(base), const_value(expo)
            res, cond = exponent_function_manager.create_condition(S.BitVecVal(b_val, 256), S.BitVecVal(e_val, 256))
            if res.symbolic:
                raise Skip("EXP result not concrete")
            if exp_conditions is None:
                raise Skip("EXP without a constraint sink")
            exp_conditions.append((b_val, e_val, res.value, cond))
            stack.append(t.const(res.value, 256))
            continue
        if op == 0x35:  # CALLDATALOAD over ConcreteCalldata (state/calldata.py:119-147, :48-55)
            off = const_value(pop())
            arr = t.const_array(t.const(0, 8))
            for i, byte in enumerate(calldata):
                arr = t.store(arr, t.const(i, 256), t.const(byte, 8))
            word = None
            for k in range(32):
                part = t.select(arr, t.const((off + k) & M256, 256))
                word = part if word is None else t.concat(word, part)
            stack.append(word)
            continue
        if op == 0x36:  # CALLDATASIZE (concrete calldata: its length)
            stack.append(t.const(len(calldata), 256))
            continue
        if op == 0x1A:  # BYTE with concrete index (instructions.py:431-458)
            i, x = pop(), as_bv(pop())
            idx = const_value(i)
            off = (31 - idx) * 8
            if off >= 0:
                stack.append(t.concat(t.const(0, 248), t.extract(off + 7, off, x)))
            else:
                stack.append(zero)
            continue
        if op in (0x1B, 0x1C, 0x1D):
            sh, v = as_bv(pop()), as_bv(pop())
            stack.append({0x1B: t.shl, 0x1C: t.lshr, 0x1D: t.ashr}[op](v, sh))
            continue
        if op == 0x52:  # MSTORE of a constant word (sha3 programs)
            off, v = const_value(pop()), const_value(pop())
            for k, byte in enumerate(v.to_bytes(32, "big")):
                mem[off + k] = byte
            continue
        if op == 0x53:
            off, v = const_value(pop()), const_value(pop())
            mem[off] = v & 0xFF
            continue
        if op == 0x20:  # SHA3 over constant memory: emitted as an interpreted keccak node
            off, size = const_value(pop()), const_value(pop())
            if size > 4096 or off > 1 << 32:   # (memory is sparse: only the size is read)
                raise Skip("sha3 region too large")
            data = bytes(mem.get(off + k, 0) for k in range(size))
            stack.append(("sha3", data))
            continue
        if op == 0x55:
            k, v = pop(), pop()
            key = const_value(k)
            store[key] = v
            continue
        if op == 0x54:  # SLOAD with a concrete key: the word stored earlier, else the pre-state's
            key = const_value(pop())
            if key in store:
                stack.append(store[key])
            else:
                stack.append(t.const(int((pre_storage or {}).get(key, 0)) & M256, 256))
            continue
        raise Skip(f"opcode 0x{op:02x}")
    return store


def vmtests():
    kats, sha = [], []
    skipped = {}
    for sub in ("vmArithmeticTest", "vmBitwiseLogicOperation", "vmSha3Test"):
        d = os.path.join(VMT, sub)
        for fn in sorted(os.listdir(d)):
            data = json.load(open(os.path.join(d, fn)))
            for name, case in data.items():
                post = case.get("post", {})
                addr = case["exec"]["address"]
                if not post or addr not in post:
                    continue
                expected = {int(k, 16): int(v, 16) for k, v in post[addr]["storage"].items()}
                if not expected:
                    continue
                code = bytes.fromhex(case["exec"]["code"][2:])
                calldata = bytes.fromhex(case["exec"].get("data", "0x")[2:])
                t = Tape()
                conds = []
                pre = {int(k, 16): int(v, 16) for k, v in case.get("pre", {}).get(addr, {}).get("storage", {}).items()}
                try:
                    store = lower_program(code, t, calldata, conds, pre)
                except Skip as e:
                    skipped[str(e)] = skipped.get(str(e), 0) + 1
                    continue
                extra = {}
                if conds:
                    # the program's EXP constraints, lowered by the product lowering with Power as
                    # a 2-argument model table (no host-side derivation of constant lookups)
                    syms = SymbolTable(derive_constant_lookups=False)
                    ct = lower_term(S.And(*[c for _, _, _, c in conds]), syms)
                    assert syms.func_names == ["Power"], syms.func_names
                    arr, consts = ct.packed()
                    extra = dict(constraint=dict(nodes=[[int(x) for x in row] for row in arr.tolist()],
                                                 consts=[int(c) for c in consts]),
                                 power=sorted({(f"{b:#x}", f"{e:#x}", f"{r:#x}") for b, e, r, _ in conds}))
                for key, exp in sorted(expected.items()):
                    node = store.get(key)
                    if node is None:
                        continue
                    if isinstance(node, tuple):  # ("sha3", data)
                        sha.append(dict(name=f"{sub}/{name}[{key}]", data=node[1].hex(), digest=f"{exp:064x}",
                                        source=f"tests/laser/evm_testsuite/VMTests/{sub}/{fn}"))
                        continue
                    if t.kind[node] == "bool":
                        node = t.ite(node, t.const(1, 256), t.const(0, 256))
                    kats.append(dump_tape(t, node, name=f"{sub}/{name}[{key}]", expected=f"0x{exp:064x}",
                                          source=f"tests/laser/evm_testsuite/VMTests/{sub}/{fn}", **extra))
    sha.append(dict(name="keccak_function_manager.get_empty_keccak_hash", data="",
                    digest=f"{89477152217924674838424037953991966239322087453347756267410168184682657981552:064x}",
                    source="mythril/laser/ethereum/function_managers/keccak_function_manager.py:86-93"))
    print("skipped programs:", skipped)
    return kats, sha


def main():
    sv = shift_vectors()
    kats, sha = vmtests()
    for fn, obj in (("shift_vectors.json", sv), ("vmtests_kats.json", kats), ("keccak_kats.json", sha)):
        with open(os.path.join(HERE, fn), "w") as f:
            json.dump(obj, f, indent=0, separators=(",", ":"))
            f.write("\n")
    print(f"shift vectors: {len(sv)}  vmtests kats: {len(kats)}  keccak kats: {len(sha)}")


if __name__ == "__main__":
    main()
