#!/usr/bin/env python3
"""Generate the gfx950 threaded-code tape interpreter ("QSA") as inline assembly.

Why assembly: the evaluator is an interpreter whose operand stack must live in statically
named VGPRs.  Expressed in HIP C++, every dispatch join made the register allocator shuffle
the whole stack (thousands of v_mov per tape, SGPR spills; profiles/r01_*): 137 VALU + 68 SALU
per tape node against ~18 algorithmic ops.  Here the register file is fixed by hand:

  VGPR  v1       LDS temp address (wave base + lane*8)
        v2       model byte offset m*4 (clamped)          v3 tid, v[4:7] scratch / MUL accumulator
        v[8:71]  the wave's 64 models' variables V[v][l] = v(8+8v+l), preloaded once
        v[72:119] operand stack S[d][l] = v(72+8d+l), d < 6 (256-bit values, 8 x u32 limbs)
        v[120:127] MUL partial-product column results
  SGPR  s[48:59] Bool stack B[d] = s[48+2d : 49+2d] as 64-lane masks (Bool ops are SALU)
        s[12:13] handler base, s[14:15] program pointer, s16 next word, s17 immediate

Programs are direct-threaded: each 32-bit word = (handler byte offset / 4) | imm << 16; every
handler ends with the dispatch tail NEXT (prefetch word n+2, decode word n+1, s_setpc).
Handler offsets are read back once per context by launching the kernel in mode 2.

gfx950 hazard rule respected throughout: a VALU that writes an SGPR/VCC is followed by >= 2
wait states before a VALU reads that SGPR (carry chains get s_nop 1; the MUL interleaves three
carry registers).

Outputs: qsa_gen.inc (the asm text as a C string literal + clobber list) and qsa_table.h
(handler enumeration used by the host-side translator in mq_api.cpp).
"""
from __future__ import annotations

import os
import sys

D = 6          # stack slots
NV = 8         # preloaded variables
L = 8          # limbs (256-bit)
VBASE, SBASE, TBASE = 8, 72, 120
BBASE = 48

HERE = os.path.dirname(os.path.abspath(__file__))


def S(d, l):
    return f"v{SBASE + 8 * d + l}"


def S2(d, l):  # even-aligned 64-bit pair starting at limb l
    r = SBASE + 8 * d + l
    return f"v[{r}:{r + 1}]"


def V2(v, l):
    r = VBASE + 8 * v + l
    return f"v[{r}:{r + 1}]"


def B(d):
    return f"s[{BBASE + 2 * d}:{BBASE + 2 * d + 1}]"


def T(k):
    return f"v{TBASE + k}"


NEXT = [
    "s_waitcnt lgkmcnt(0)",
    "s_and_b32 s18, s16, 0xffff",
    "s_lshr_b32 s17, s16, 16",
    "s_lshl_b32 s18, s18, 2",
    "s_add_u32 s18, s12, s18",
    "s_addc_u32 s19, s13, 0",
    "s_load_dword s16, s[14:15], 0x0",
    "s_add_u32 s14, s14, 4",
    "s_addc_u32 s15, s15, 0",
    "s_setpc_b64 s[18:19]",
]

handlers = []  # (key, body lines)


def H(key, body, tail=True):
    handlers.append((key, list(body) + (NEXT if tail else [])))


# ---------------------------------------------------------------- leaves
H(("END",), ["s_branch .Lqsa_tape_end"], tail=False)
for d in range(D):
    for v in range(NV):
        H(("PUSH_VAR", d, v), [f"v_mov_b64 {S2(d, l)}, {V2(v, l)}" for l in range(0, L, 2)])
    H(("PUSH_CONST", d), ["s_lshl_b32 s34, s17, 2", "s_load_dwordx8 s[64:71], s[20:21], s34", "s_waitcnt lgkmcnt(0)"]
      + [f"v_mov_b64 {S2(d, l)}, s[{64 + l}:{65 + l}]" for l in range(0, L, 2)])
    H(("PUSH_TMP", d), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1"]
      + [f"ds_read_b64 {S2(d, l)}, v5 offset:{256 * l}" for l in range(0, L, 2)] + ["s_waitcnt lgkmcnt(0)"])
    H(("PUSH_TMP_BOOL", d), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1", "ds_read_b32 v6, v5",
                             "s_waitcnt lgkmcnt(0)", f"v_cmp_ne_u32_e64 {B(d)}, 0, v6"])
    H(("PUSH_BOOL", d), ["s_cmp_lg_u32 s17, 0", f"s_cselect_b64 {B(d)}, -1, 0"])
H(("STORE_TMP", 0), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1"]
  + [f"ds_write_b64 v5, {S2(0, l)} offset:{256 * l}" for l in range(0, L, 2)])
H(("STORE_TMP_BOOL", 0), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1",
                          f"v_cndmask_b32_e64 v6, 0, 1, {B(0)}", "ds_write_b32 v5, v6"])

# ---------------------------------------------------------------- Bool (SALU on lane masks)
for d in range(D):
    H(("NOT", d), [f"s_not_b64 {B(d)}, {B(d)}"])
for d in range(1, D):
    a, b = B(d - 1), B(d)
    H(("AND", d), [f"s_and_b64 {a}, {a}, {b}"])
    H(("OR", d), [f"s_or_b64 {a}, {a}, {b}"])
    H(("XOR", d), [f"s_xor_b64 {a}, {a}, {b}"])
    H(("IFF", d), [f"s_xnor_b64 {a}, {a}, {b}"])
    H(("IMPLIES", d), [f"s_orn2_b64 {a}, {b}, {a}"])
for d in range(2, D):
    H(("BITE", d), [f"s_and_b64 s[34:35], {B(d - 2)}, {B(d - 1)}", f"s_andn2_b64 s[36:37], {B(d)}, {B(d - 2)}",
                    f"s_or_b64 {B(d - 2)}, s[34:35], s[36:37]"])
    H(("BITE_EF", d), [f"s_and_b64 s[34:35], {B(d - 1)}, {B(d)}", f"s_andn2_b64 s[36:37], {B(d - 2)}, {B(d - 1)}",
                       f"s_or_b64 {B(d - 2)}, s[34:35], s[36:37]"])


# ---------------------------------------------------------------- 256-bit predicates
def eq_body(d):
    """8 limb compares into 8 distinct SGPR pairs, then a SALU AND tree (every SALU read is
    >= 4 instructions after the VALU write)."""
    a, b = d - 1, d
    regs = ["s[34:35]", "s[36:37]", "s[38:39]", "s[60:61]", "s[64:65]", "s[66:67]", "s[68:69]", "s[70:71]"]
    out = [f"v_cmp_eq_u32_e64 {regs[l]}, {S(a, l)}, {S(b, l)}" for l in range(L)]
    out += ["s_nop 1",
            "s_and_b64 s[34:35], s[34:35], s[36:37]", "s_and_b64 s[38:39], s[38:39], s[60:61]",
            "s_and_b64 s[64:65], s[64:65], s[66:67]", "s_and_b64 s[68:69], s[68:69], s[70:71]",
            "s_and_b64 s[34:35], s[34:35], s[38:39]", "s_and_b64 s[64:65], s[64:65], s[68:69]",
            f"s_and_b64 {B(a)}, s[34:35], s[64:65]"]
    return out


def lt_chain(x, y, dst):
    """dst mask = (x < y) unsigned over 8 limbs (slots x, y); borrow chain with hazard nops."""
    out = [f"v_sub_co_u32_e64 v5, s[34:35], {S(x, 0)}, {S(y, 0)}"]
    cur = "s[34:35]"
    for l in range(1, L):
        nxt = dst if l == L - 1 else ("s[36:37]" if cur == "s[34:35]" else "s[34:35]")
        out.append("s_nop 1")
        out.append(f"v_subb_co_u32_e64 v5, {nxt}, {S(x, l)}, {S(y, l)}, {cur}")
        cur = nxt
    return out


def flip_signs(d):
    return [f"v_xor_b32 {S(d - 1, 7)}, 0x80000000, {S(d - 1, 7)}", f"v_xor_b32 {S(d, 7)}, 0x80000000, {S(d, 7)}"]


for d in range(1, D):
    a, b = d - 1, d
    H(("EQ", d), eq_body(d))
    for signed in (False, True):
        pre = flip_signs(d) if signed else []
        p = "S" if signed else "U"
        H((p + "LT", d), pre + lt_chain(a, b, B(a)))                       # a < b
        H((p + "GT", d), pre + lt_chain(b, a, B(a)))                       # b < a
        H((p + "LE", d), pre + lt_chain(b, a, "s[38:39]") + ["s_nop 1", f"s_not_b64 {B(a)}, s[38:39]"])  # !(b < a)
        H((p + "GE", d), pre + lt_chain(a, b, "s[38:39]") + ["s_nop 1", f"s_not_b64 {B(a)}, s[38:39]"])  # !(a < b)


# ---------------------------------------------------------------- 256-bit arithmetic
def carry_chain(first, rest, n=L):
    out = [first(0)]
    for l in range(1, n):
        out.append("s_nop 1")
        out.append(rest(l))
    return out


for d in range(1, D):
    a, b = d - 1, d
    H(("ADD", d), carry_chain(lambda l: f"v_add_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}",
                              lambda l: f"v_addc_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}, vcc"))
    H(("SUB", d), carry_chain(lambda l: f"v_sub_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}",
                              lambda l: f"v_subb_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}, vcc"))
    for nm, ins in (("BAND", "v_and_b32"), ("BOR", "v_or_b32"), ("BXOR", "v_xor_b32")):
        H((nm, d), [f"{ins} {S(a, l)}, {S(a, l)}, {S(b, l)}" for l in range(L)])
for d in range(D):
    H(("NEG", d), carry_chain(lambda l: f"v_sub_co_u32 {S(d, l)}, vcc, 0, {S(d, l)}",
                              lambda l: f"v_subb_co_u32 {S(d, l)}, vcc, 0, {S(d, l)}, vcc"))
    H(("BNOT", d), [f"v_not_b32 {S(d, l)}, {S(d, l)}" for l in range(L)])
for d in range(2, D):
    H(("ITE", d), [f"v_cndmask_b32_e64 {S(d - 2, l)}, {S(d, l)}, {S(d - 1, l)}, {B(d - 2)}" for l in range(L)])
    # else-first ternaries (gprog.h G_ITE_EF / G_BITE_EF): else at d-2, cond at d-1, then at d
    H(("ITE_EF", d), [f"v_cndmask_b32_e64 {S(d - 2, l)}, {S(d - 2, l)}, {S(d, l)}, {B(d - 1)}" for l in range(L)])


def mul_body(d):
    """S[d-1] = S[d-1] * S[d] mod 2^256: product scanning (Comba) columns 0..7, 64-bit column
    accumulator v[4:5] (v_mad_u64_u32 with carry-out) + overflow word v6; carries are added
    through three rotating SGPR pairs so every VALU carry read is >= 2 instructions after its
    write.  Column 0 has no carries; each later column's first carry-add writes the overflow word
    (no reset move); the accumulator shift (v4, v5) <- (v5, v6) is one v_pk_mov_b32; column 7's
    low word goes straight to S[d-1][7] after its last product."""
    a, b = d - 1, d
    C = ["s[34:35]", "s[36:37]", "s[38:39]"]
    out = [f"v_mad_u64_u32 v[4:5], s[60:61], {S(a, 0)}, {S(b, 0)}, 0",
           f"v_mov_b32 {T(0)}, v4", "v_mov_b32 v4, v5", "v_mov_b32 v5, 0"]
    for k in range(1, L):
        prods = [(i, k - i) for i in range(k + 1)]
        if k == L - 1:
            # last column: only the low word matters, no carry tracking
            for i, j in prods:
                out.append(f"v_mad_u64_u32 v[4:5], s[60:61], {S(a, i)}, {S(b, j)}, v[4:5]")
            break
        mads = [f"v_mad_u64_u32 v[4:5], {C[t % 3]}, {S(a, i)}, {S(b, j)}, v[4:5]" for t, (i, j) in enumerate(prods)]
        adds = [f"v_addc_co_u32_e64 v6, s[60:61], 0, {'0' if t == 0 else 'v6'}, {C[t % 3]}" for t in range(len(prods))]
        seq = []
        n = len(prods)
        # m0 m1 m2 a0 m3 a1 m4 a2 ... then flush
        for t in range(n):
            seq.append(mads[t])
            if t >= 2:
                seq.append(adds[t - 2])
        tail = [adds[t] for t in range(max(0, n - 2), n)]
        if n == 2:
            seq += ["s_nop 0"] + tail
        else:
            seq += tail
        out += seq
        out += [f"v_mov_b32 {T(k)}, v4", "v_mov_b32 v4, v5", "v_mov_b32 v5, v6"]
    out += [f"v_mov_b64 {S2(a, l)}, v[{TBASE + l}:{TBASE + l + 1}]" for l in range(0, 6, 2)]
    out += [f"v_mov_b32 {S(a, 6)}, {T(6)}", f"v_mov_b32 {S(a, 7)}, v4"]
    return out


for d in range(1, D):
    H(("MUL", d), mul_body(d))


# ---------------------------------------------------------------- kernel frame
def frame():
    P = []
    P += [
        "s_mov_b64 s[10:11], %0",
        "s_mov_b32 s96, %1",
        "s_mov_b32 s97, %2",
        "v_mov_b32 v3, %3",
        "s_load_dwordx16 s[64:79], s[10:11], 0x0",
        "s_load_dwordx8 s[80:87], s[10:11], 0x40",
        "s_waitcnt lgkmcnt(0)",
        "s_mov_b64 s[22:23], s[64:65]",
        "s_mov_b64 s[46:47], s[66:67]",
        "s_mov_b64 s[88:89], s[68:69]",
        "s_mov_b64 s[90:91], s[70:71]",
        "s_mov_b64 s[26:27], s[72:73]",
        "s_mov_b64 s[92:93], s[74:75]",
        "s_mov_b64 s[94:95], s[76:77]",
        "s_mov_b32 s29, s80",
        "s_mov_b32 s98, s81",
        "s_mov_b32 s30, s84",
        "s_mov_b32 s31, s85",
        "s_mov_b32 s99, s86",
        # handler base
        "s_getpc_b64 s[12:13]",
        ".Lqsa_pc:",
        "s_add_u32 s12, s12, .Lqsa_hbase - .Lqsa_pc",
        "s_addc_u32 s13, s13, 0",
        # mode 2: dump handler offsets (block 0, lane 0)
        "s_cmp_eq_u32 s31, 2",
        "s_cbranch_scc0 .Lqsa_main",
        "s_or_b32 s34, s96, s97",
        "s_cmp_eq_u32 s34, 0",
        "s_cbranch_scc0 .Lqsa_end",
        "v_cmp_eq_u32_e64 s[34:35], 0, v3",
        "s_nop 1",
        "s_and_saveexec_b64 s[36:37], s[34:35]",
        "v_mov_b32 v4, 0",
    ]
    for k in range(len(handlers)):
        P.append(f"v_mov_b32 v5, .Lqh_{k} - .Lqsa_hbase")
        P.append(f"global_store_dword v4, v5, s[78:79] offset:{4 * k}")
    P += [
        f"v_mov_b32 v5, {len(handlers)}",
        "s_waitcnt vmcnt(0)",
        "s_mov_b64 exec, s[36:37]",
        "s_branch .Lqsa_end",
        ".Lqsa_main:",
        # wave / lane / model index
        "v_and_b32 v4, 63, v3",
        "v_lshrrev_b32 v5, 6, v3",
        # gfx950 hazard: a VALU write of a VGPR followed by v_readfirstlane of it needs wait
        # states, or the read returns the register's previous (stale) contents
        "s_nop 1",
        "v_readfirstlane_b32 s34, v5",
        "s_nop 1",
        "s_lshl_b32 s35, s96, 8",
        "s_lshl_b32 s36, s34, 6",
        "s_add_u32 s35, s35, s36",
        "s_cmp_ge_u32 s35, s29",
        "s_cbranch_scc1 .Lqsa_end",
        "s_add_u32 s28, s98, s35",            # gfirst
        "v_add_u32 v2, s35, v4",               # m
        "v_cmp_lt_u32_e64 s[62:63], v2, s29",  # valid
        "s_sub_u32 s37, s29, 1",
        "v_min_u32 v2, s37, v2",
        "v_lshlrev_b32 v2, 2, v2",
        "s_mul_i32 s37, s34, s99",
        "v_lshlrev_b32 v1, 3, v4",
        "v_add_u32 v1, s37, v1",
        "s_mov_b64 s[40:41], 0",
        "s_mov_b64 s[42:43], 0",
        "s_mov_b64 s[44:45], 0",
        "s_mul_i32 s24, s97, s83",
        "s_add_u32 s25, s24, s83",
        "s_min_u32 s25, s25, s82",
    ]
    # preload variables: 64 limb rows (row index table at args+0x60; the host points missing
    # limbs / vars at an all-zero row)
    for c in range(4):
        P += [f"s_load_dwordx16 s[64:79], s[10:11], {0x60 + 64 * c:#x}", "s_waitcnt lgkmcnt(0)"]
        for j in range(16):
            idx = 16 * c + j
            v, l = idx // 8, idx % 8
            P += [f"s_mul_i32 s34, s{64 + j}, s29", f"s_mul_hi_u32 s35, s{64 + j}, s29",
                  "s_lshl_b64 s[34:35], s[34:35], 2", "s_add_u32 s34, s34, s90", "s_addc_u32 s35, s35, s91",
                  f"global_load_dword v{VBASE + 8 * v + l}, v2, s[34:35]"]
    P += ["s_waitcnt vmcnt(0)"]
    # tape loop
    P += [
        ".Lqsa_tape_loop:",
        "s_cmp_ge_u32 s24, s25",
        "s_cbranch_scc1 .Lqsa_tapes_done",
        "s_lshl_b32 s34, s24, 5",
        "s_add_u32 s34, s22, s34",
        "s_addc_u32 s35, s23, 0",
        "s_load_dwordx8 s[80:87], s[34:35], 0x0",
        "s_waitcnt lgkmcnt(0)",
        "s_lshl_b32 s34, s82, 2",
        "s_add_u32 s72, s26, s34",           # s[72:73] = &best[tape] (handlers never touch s72-s87)
        "s_addc_u32 s73, s27, 0",
        "s_cmp_eq_u32 s31, 1",
        "s_cbranch_scc1 .Lqsa_run",
        "s_cmp_eq_u32 s30, 0",
        "s_cbranch_scc1 .Lqsa_run",
        "s_load_dword s34, s[72:73], 0x0 glc",
        "s_waitcnt lgkmcnt(0)",
        "s_cmp_ge_i32 s28, s34",
        "s_cbranch_scc1 .Lqsa_next_tape",
        ".Lqsa_run:",
        "s_lshl_b32 s34, s83, 2",
        "s_add_u32 s20, s88, s34",
        "s_addc_u32 s21, s89, 0",
        "s_lshl_b32 s34, s80, 2",
        "s_add_u32 s14, s46, s34",
        "s_addc_u32 s15, s47, 0",
        "s_load_dword s16, s[14:15], 0x0",
        "s_add_u32 s14, s14, 4",
        "s_addc_u32 s15, s15, 0",
    ] + NEXT + [
        ".Lqsa_tape_end:",
        "s_waitcnt lgkmcnt(0)",
        "s_and_b64 s[34:35], s[48:49], s[62:63]",
        "s_bcnt1_i32_b64 s38, s[62:63]",
        "s_add_u32 s40, s40, s38",
        "s_addc_u32 s41, s41, 0",
        "s_mul_i32 s60, s38, s84",
        "s_mul_hi_u32 s61, s38, s84",
        "s_add_u32 s42, s42, s60",
        "s_addc_u32 s43, s43, s61",
        "s_mul_i32 s60, s38, s87",
        "s_mul_hi_u32 s61, s38, s87",
        "s_add_u32 s44, s44, s60",
        "s_addc_u32 s45, s45, s61",
        "s_cmp_eq_u32 s31, 1",
        "s_cbranch_scc1 .Lqsa_store_verdict",
        "s_cmp_eq_u64 s[34:35], 0",
        "s_cbranch_scc1 .Lqsa_next_tape",
        "s_ff1_i32_b64 s38, s[34:35]",
        "s_add_u32 s38, s38, s28",
        "s_mov_b64 s[60:61], exec",
        "s_mov_b64 exec, 1",
        "v_mov_b32 v5, s38",
        "v_mov_b32 v6, 0",
        "global_atomic_smin v6, v5, s[72:73]",
        "s_mov_b64 exec, s[60:61]",
        "s_branch .Lqsa_next_tape",
        ".Lqsa_store_verdict:",
        "s_mul_i32 s38, s82, s29",
        "s_mul_hi_u32 s39, s82, s29",
        "s_add_u32 s38, s38, s94",
        "s_addc_u32 s39, s39, s95",
        f"v_cndmask_b32_e64 v5, 0, 1, {B(0)}",
        "v_lshrrev_b32 v6, 2, v2",
        "s_mov_b64 s[60:61], exec",
        "s_mov_b64 exec, s[62:63]",
        "global_store_byte v6, v5, s[38:39]",
        "s_mov_b64 exec, s[60:61]",
        ".Lqsa_next_tape:",
        "s_add_u32 s24, s24, 1",
        "s_branch .Lqsa_tape_loop",
        ".Lqsa_tapes_done:",
        "s_mov_b64 s[60:61], exec",
        "s_mov_b64 exec, 1",
        "v_mov_b32 v6, 0",
        "v_mov_b32 v4, s40",
        "v_mov_b32 v5, s41",
        "global_atomic_add_x2 v6, v[4:5], s[92:93]",
        "v_mov_b32 v4, s42",
        "v_mov_b32 v5, s43",
        "global_atomic_add_x2 v6, v[4:5], s[92:93] offset:8",
        "v_mov_b32 v4, s44",
        "v_mov_b32 v5, s45",
        "global_atomic_add_x2 v6, v[4:5], s[92:93] offset:16",
        "s_waitcnt vmcnt(0)",
        "s_mov_b64 exec, s[60:61]",
        "s_branch .Lqsa_end",
        ".Lqsa_hbase:",
    ]
    for k, (key, body) in enumerate(handlers):
        P.append(f".Lqh_{k}:  ; {' '.join(map(str, key))}")
        P += body
    P.append(".Lqsa_end:")
    return P


def main():
    lines = frame()
    text = "\n".join(lines) + "\n"
    clob = [f'"v{i}"' for i in range(1, 128)] + [f'"s{i}"' for i in range(10, 100) if i not in (32, 33)]
    clob += ['"vcc"', '"scc"', '"memory"']
    with open(os.path.join(HERE, "qsa_gen.inc"), "w") as f:
        f.write("// GENERATED by gen_qsa.py — do not edit\n")
        f.write("#define QSA_ASM_TEXT \\\n")
        for ln in text.splitlines():
            f.write('  "' + ln.replace('"', '\\"') + '\\n" \\\n')
        f.write("  \"\"\n")
        f.write("#define QSA_CLOBBERS " + ", ".join(clob) + "\n")
    names = sorted({k[0] for k, _ in handlers})
    with open(os.path.join(HERE, "qsa_table.h"), "w") as f:
        f.write("// GENERATED by gen_qsa.py — handler enumeration of the QSA interpreter\n")
        f.write("#ifndef MQ_QSA_TABLE_H\n#define MQ_QSA_TABLE_H\nnamespace mq {\n")
        f.write(f"constexpr int kQsaStack = {D};\nconstexpr int kQsaVars = {NV};\nconstexpr int kQsaHandlers = {len(handlers)};\n")
        f.write("enum QsaKind {\n" + "".join(f"  QK_{n},\n" for n in names) + "  QK_COUNT\n};\n")
        f.write("struct QsaHandlerKey { int kind, d, v; };\n")
        f.write("static const QsaHandlerKey kQsaHandlerKeys[] = {\n")
        for key, _ in handlers:
            kind = key[0]
            d = key[1] if len(key) > 1 else -1
            v = key[2] if len(key) > 2 else -1
            f.write(f"  {{QK_{kind}, {d}, {v}}},\n")
        f.write("};\n}  // namespace mq\n#endif\n")
    nins = sum(1 for ln in lines if ln and not ln.startswith(".L"))
    print(f"handlers={len(handlers)} asm_lines={nins}", file=sys.stderr)


if __name__ == "__main__":
    main()
