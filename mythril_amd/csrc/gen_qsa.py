#!/usr/bin/env python3
"""Generate the gfx950 threaded-code tape interpreters ("QSA") as inline assembly.

Why assembly: the evaluator is an interpreter whose operand stack must live in statically
named VGPRs and whose dispatch must be ONE indirect jump.  Expressed in HIP C++, every dispatch
join made the register allocator shuffle the whole stack (profiles/r01_*), and the AMDGPU backend
lowers a `switch` (and computed goto) to a compare tree: the LDS-stack C++ interpreter measures
~67 SALU + 26 branches per tape node on C3 (profiles/r01_c3b_pmc.json).  Here every handler ends
with the dispatch tail NEXT (decode the prefetched word, prefetch the next, s_setpc).

Two variants are generated from the same handler code (one asm statement each, label prefixes
.Lqsa / .Lqsg):

  P ("preload", qsa_kernel):  the wave's 64 models' first 8 variables are preloaded into VGPRs
     once per workgroup; PUSH_VAR is a register copy.  C2-shaped batches.
  G ("general", qsg_kernel):  variables pushed from the model rows in HBM (PUSH_MEM: the loads
     are issued by the push and waited for by the first consumer) or from rows staged in LDS;
     table-lookup subroutine (UF1).  EVM-shaped batches and hoisted column programs (mode 3).
     The product G is the compact layout (NVG = 0, set_layout): no preloaded variables, 96 VGPRs
     so 5 waves per SIMD hide the push latency (profiles/r03u: C3 26.6 -> 23.8 ms, C4 6.0 ->
     5.8 ms, C5 69.1 -> 70.4 ms against the NVG = 4 layout, 128 VGPRs with the 4 variables the
     batch pushes most preloaded).

Register map (both):
  VGPR  v1       LDS temp address (wave base + lane*8)
        v2       model byte offset m*4 (clamped)          v3 sign mask of signed division
        v[4:7]   scratch / MUL accumulator / division step
        v[8:71]  P: preloaded variables V[v][l] = v(8+8v+l), v < 8
                 G with NVG = 4: v[8:39] preloaded variables (v < 4), v[40:63] UF1 work, v64
                 program window (the compact G map: set_layout)
        v[72:119] operand stack S[d][l] = v(72+8d+l), d < 6 (256-bit values, 8 x u32 limbs;
                 compact G: v[40:87])
        v[120:127] MUL column results / division + lookup operand (compact G: v[88:95])
  SGPR  s[48:59] Bool stack B[d] = s[48+2d : 49+2d] as 64-lane masks (Bool ops are SALU)
        s[12:13] handler base, s[14:15] program pointer, s16 next word, s17 immediate
        s[74:75] M*4 (model row stride in bytes), s[76:77] subroutine return address,
        s[78:79] / s98 / s99 subroutine scratch

Programs are direct-threaded: each 32-bit word = (handler byte offset / 4) | imm << 16.
Handler offsets are read back once per context by launching each kernel in mode 2.

gfx950 hazard rule respected throughout: a VALU that writes an SGPR/VCC is followed by >= 1 wait
state before a VALU reads it as a carry (carry and borrow chains get s_nop 0, the padding LLVM's
gfx950 hazard recognizer gives v_add_co -> v_addc; the MUL interleaves three carry registers),
>= 2 before other VALU reads of it and >= 4 before a SALU reads it.  (tools/issue_probe.py: the
s_nop 1 padding cost an ADD 45 instead of 36 SIMD cycles at 4 waves per SIMD.)

Outputs: qsa_gen.inc (the two asm texts as C string literals + clobber list) and qsa_table.h
(handler enumerations used by the host-side translator in mq_api.cpp).
"""
from __future__ import annotations

import os
import re
import sys

D = 6          # stack slots of the variant being generated (set_layout: P 6, G DG)
DP = 6         # P: C2's tapes need 5-6 slots
DG = 4         # G: 4 slots keep the compact layout at 80 VGPRs = 6 waves per SIMD; the tape
               # compiler spills deeper subtrees of G programs to LDS temps (tape_compiler.cpp)
NV = 8         # preloaded variables (P)
NVG = 0        # preloaded variables (G); 0 selects the compact G layout (set_layout): 96 VGPRs,
               # 5 waves / SIMD.  4 = v[8:39] preloaded in a 128-VGPR kernel (4 waves / SIMD)
L = 8          # limbs (256-bit)
VBASE, SBASE, TBASE = 8, 72, 120
UBASE = 40     # G: UF1 work registers v[40:63]
BBASE = 48

STG = "v65"    # G: LDS address of the staged model rows of this lane (stage base + 4 * lane)
# G early exit: a 64-desc window of the wave's tapes, lane i <-> desc s25 - 1 - 64w - i (w = the
# window of the current tape counted from the wave's LAST desc); EEA = byte offset of best[tape]
# of that desc, EEV = best[] as gathered when the window was entered (None: scalar check)
EEA, EEV = "v67", "v66"

HERE = os.path.dirname(os.path.abspath(__file__))

# QSA_PROF=1 at generation: a diagnostic G build that charges the cycles (s_memtime) since the
# previous handler's end to each handler kind, in a per-wave LDS table flushed to QArgs.prof_out
# (tools/g_profile.py).  Never the product build: it adds ~12 instructions per dispatch.
PROF = os.environ.get("QSA_PROF") == "1"
PROF_VGPR = "v70"     # G: LDS address of this wave's profile table
# profile entries past the handler kinds: the tape frame split at its waits (tape header load,
# early-exit check, window / run start) and the tape end bookkeeping
PROF_EXTRA = ("FRAME", "FRAME_LD", "FRAME3", "FRAME3_LD", "F_HDR", "F_EE", "F_ENDW", "F_END", "PRELOAD", "STAGE")


def prof_point(kind):
    """Charge the cycles since the last profile point to `kind` (offset resolved in main())."""
    if not PROF:
        return []
    return ["s_memtime s[34:35]", "s_waitcnt lgkmcnt(0)",
            "s_sub_u32 s36, s34, s100",
            "s_mov_b64 s[100:101], s[34:35]",
            "s_mov_b64 s[34:35], exec", "s_mov_b64 exec, 1",
            "v_mov_b32 v4, s36", "v_mov_b32 v5, 0",
            f"ds_add_u64 {PROF_VGPR}, v[4:5] offset:@PROF:{kind}:0@",
            "v_mov_b32 v4, 1",
            f"ds_add_u64 {PROF_VGPR}, v[4:5] offset:@PROF:{kind}:8@",
            "s_mov_b64 exec, s[34:35]"]


def frame_prof(pfx):
    """Profile build: the tape start charged by mode (3 = column programs) and by whether the
    program's first block was the prefetched successor (FRAME, FRAME3) or loaded (*_LD)."""
    if not PROF:
        return []
    out = ["s_cmp_eq_u32 s31, 3", f"s_cbranch_scc1 {pfx}_fp3", "s_cmp_eq_u32 s39, 1", f"s_cbranch_scc1 {pfx}_fp0s"]
    out += prof_point("FRAME_LD") + [f"s_branch {pfx}_fpd", f"{pfx}_fp0s:"] + prof_point("FRAME")
    out += [f"s_branch {pfx}_fpd", f"{pfx}_fp3:", "s_cmp_eq_u32 s39, 1", f"s_cbranch_scc1 {pfx}_fp3s"]
    out += prof_point("FRAME3_LD") + [f"s_branch {pfx}_fpd", f"{pfx}_fp3s:"] + prof_point("FRAME3") + [f"{pfx}_fpd:"]
    return out


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


def W(k):  # division / lookup operand registers v[120:127]
    return f"v{TBASE + k}"


def W2(k):
    return f"v[{TBASE + k}:{TBASE + k + 1}]"



# G: the tape's program is streamed through a 64-word VGPR window (lane i = word i of the
# window, one coalesced load per window) and read with v_readlane: no scalar-memory round trip
# per node.  s[14:15] = byte address of the window, s16 = lane of the next word.  The translator
# places a REFILL word wherever the window runs out (the next window starts right after it) and
# never splits a PUSH_CONSTW from its inline data words.
# The window is decoded once per load (load_window), in VALU: WINA = low 32 bits of each word's
# handler address (s12 + 4 * (word & 0xffff); the host checks the handler area does not cross a
# 4 GB boundary, so s19 = s13 throughout), WINI = its immediate (word >> 16).  A dispatch is then
# two lane reads, one SALU add and the jump: the scalar unit, shared by the CU's four SIMDs, was
# the binding issue port at six SALU per dispatch.
WIN, WINA, WINI = "v64", "v68", "v69"
NWIN = "v71"       # G: the program block after the window, prefetched (load_window)


def next_g():
    return [f"v_readlane_b32 s18, {WINA}, s16",
            f"v_readlane_b32 s17, {WINI}, s16",
            "s_add_u32 s16, s16, 1",
            "s_nop 1",                      # VALU SGPR write -> SALU read (s_setpc)
            "s_setpc_b64 s[18:19]"]


NEXT_G = next_g()


# P: three-word program entries (absolute low 32 bits of the handler address, immediate,
# constant-prefetch byte offset), prefetched one entry ahead into s[96:98] (an x4 load: the
# fourth word belongs to the next entry); s[14:15] = program base, s16 = byte offset of the next
# entry, s19 = high half of the handler addresses (the host checks they share it).
# Constant prefetch: the tail that dispatches entry k also loads the 8 words at the tape's
# constants + entry k's third word into CB = s[80:87], so the constant of entry k + 1 arrives
# while handler k runs; the PF_ handler variants read it from there instead of issuing their own
# scalar load and waiting (mq_api.cpp qsa_translate assigns them: never two in a row, and the
# entry of a PF_ handler whose successor is not one re-loads its own constant, so an in-flight
# load never changes what a running handler reads).  The frame keeps the descriptor words the
# tape end needs in s78 / s79 / s100 (s[80:87] is CB while a tape runs).
PF_CB = 80
NEXT_P = [
    "s_waitcnt lgkmcnt(0)",
    "s_mov_b32 s18, s96",
    "s_mov_b32 s17, s97",
    f"s_load_dwordx8 s[{PF_CB}:{PF_CB + 7}], s[20:21], s98",
    "s_load_dwordx4 s[96:99], s[14:15], s16",
    "s_add_u32 s16, s16, 12",
    "s_setpc_b64 s[18:19]",
]


_WIN_LABELS = [0]


def load_window(first, pfx=None):
    """Make the program's next 64-word block the window (decoded, s16 = 0) and prefetch the one
    after it into NWIN (mq_api.cpp qsa_window_layout: blocks are aligned and contiguous).
    first (tape start, s[36:37] = the program's address): the block is NWIN when the previous
    window's successor is this program (consecutive descriptors), else it is loaded.  Otherwise
    (REFILL): the block is NWIN, 256 bytes on."""
    k = _WIN_LABELS[0]
    _WIN_LABELS[0] += 1
    lane4 = LANE4 or "v5"
    out = [] if LANE4 else ["v_mbcnt_lo_u32_b32 v5, -1, 0", "v_mbcnt_hi_u32_b32 v5, -1, v5", "v_lshlrev_b32 v5, 2, v5"]
    if first:
        # A program may start inside a block (column programs are packed back to back,
        # mq_api.cpp qsa_pack_program): s16 = its word offset, s[36:37] = the block.  A program
        # starting in the current window needs no load: the window is decoded already.
        out += ["s_and_b32 s16, s36, 0xff",
                "s_lshr_b32 s16, s16, 2",
                "s_andn2_b32 s36, s36, 0xff",
                "s_cmp_eq_u64 s[36:37], s[14:15]"] + (["s_cselect_b32 s39, 1, 0"] if PROF else []) + [
                f"s_cbranch_scc1 {pfx}_wsame{k}"]
        # the prefetched window was issued before the previous tape's stores (s59 of them, column
        # rows / a verdict byte / a hit's atomic): wait for it, not for them (vector memory
        # operations complete in order)
        w = f"{pfx}_ws{k}"
        out += ["s_cmp_eq_u32 s59, 0", f"s_cbranch_scc1 {w}0",
                "s_cmp_eq_u32 s59, 1", f"s_cbranch_scc1 {w}1",
                "s_cmp_lt_u32 s59, 4", f"s_cbranch_scc1 {w}2",
                "s_cmp_lt_u32 s59, 8", f"s_cbranch_scc1 {w}4",
                "s_waitcnt vmcnt(8)", f"s_branch {w}d",
                f"{w}4:", "s_waitcnt vmcnt(4)", f"s_branch {w}d",
                f"{w}2:", "s_waitcnt vmcnt(2)", f"s_branch {w}d",
                f"{w}1:", "s_waitcnt vmcnt(1)", f"s_branch {w}d",
                f"{w}0:", "s_waitcnt vmcnt(0)",
                f"{w}d:", "s_mov_b32 s59, 0"]
        out += ["s_add_u32 s34, s14, 256", "s_addc_u32 s35, s15, 0",
                "s_cmp_eq_u64 s[34:35], s[36:37]",
                "s_mov_b64 s[14:15], s[36:37]"] + (["s_cselect_b32 s39, 1, 0"] if PROF else []) + [
                f"s_cbranch_scc1 {pfx}_win_pref",
                f"global_load_dword {NWIN}, {lane4}, s[14:15]",
                "s_waitcnt vmcnt(0)",
                f"{pfx}_win_pref:"]
    else:
        out += ["s_add_u32 s14, s14, 256", "s_addc_u32 s15, s15, 0", "s_waitcnt vmcnt(0)"]
    out += [f"v_mov_b32 {WIN}, {NWIN}",
            f"global_load_dword {NWIN}, {lane4}, s[14:15] offset:256"]
    out += [] if first else ["s_mov_b32 s16, 0"]
    out += [f"v_and_b32 v5, 0xffff, {WIN}",
            f"v_lshl_add_u32 {WINA}, v5, {3 if PROF else 2}, s12",
            f"v_lshrrev_b32 {WINI}, 16, {WIN}",
            "s_nop 1"]                      # VALU VGPR write -> v_readlane of it
    if first:
        # (the same-window path wrote s16 a few SALU instructions ago: an SGPR a SALU wrote is
        # read as v_readlane's lane select only after 4 wait states)
        out += [f"s_branch {pfx}_wdone{k}", f"{pfx}_wsame{k}:", "s_nop 3", f"{pfx}_wdone{k}:"]
    return out


# G: a handler that reads the stack first waits for the pushes in flight — global loads (PUSH_MEM)
# and LDS reads of staged model rows (PUSH_MEMS)
VMWAIT = "s_waitcnt vmcnt(0) lgkmcnt(0)"
# ... and the "_L" variant of every stack reader (and of its fused forms), which waits for LDS /
# scalar loads only: the translator picks it when no PUSH_MEM (global load) is outstanding
# (mq_api.cpp qsa_translate, final pass).  Otherwise the first stack reader of every tape also
# waited for the prefetch of the NEXT program window (load_window's NWIN), an L2 / HBM round trip
# (C4's tapes: ULTK right after a staged PUSH_MEMS at ~5 800 cycles per dispatch, profiles/r04h)
LGKMWAIT = "s_waitcnt lgkmcnt(0)"


def zero_limbs(d, lo):
    """S[d][lo..7] = 0 (64-bit moves where aligned)."""
    out = []
    l = lo
    while l < L:
        if l % 2 == 0 and l + 1 < L:
            out.append(f"v_mov_b64 {S2(d, l)}, 0")
            l += 2
        else:
            out.append(f"v_mov_b32 {S(d, l)}, 0")
            l += 1
    return out


# ---------------------------------------------------------------- handler bodies
def eq_body(d, bl=None):
    """8 limb compares into 8 distinct SGPR pairs, then a SALU AND tree (every SALU read is
    >= 4 instructions after the VALU write).  bl(l): register of the right operand's limb l
    (default: stack slot d; a preloaded variable in the fused ...V handlers)."""
    a = d - 1
    bl = bl or (lambda l: S(d, l))
    regs = ["s[34:35]", "s[36:37]", "s[38:39]", "s[60:61]", "s[64:65]", "s[66:67]", "s[68:69]", "s[70:71]"]
    out = [f"v_cmp_eq_u32_e64 {regs[l]}, {S(a, l)}, {bl(l)}" for l in range(L)]
    out += ["s_nop 1",
            "s_and_b64 s[34:35], s[34:35], s[36:37]", "s_and_b64 s[38:39], s[38:39], s[60:61]",
            "s_and_b64 s[64:65], s[64:65], s[66:67]", "s_and_b64 s[68:69], s[68:69], s[70:71]",
            "s_and_b64 s[34:35], s[34:35], s[38:39]", "s_and_b64 s[64:65], s[64:65], s[68:69]",
            f"s_and_b64 {B(a)}, s[34:35], s[64:65]"]
    return out


# inline-constant classes of the G compare-with-constant handlers: 0 = the 16-bit immediate
# (no data words), 1 = two data words (limbs 0-1), 2 = eight data words
KCLS = (0, 2, 8)


def const_words(nw):
    """Read the nw inline data words after the handler word into s64.. (s16 past them)."""
    out = []
    for i in range(nw):
        out += [f"v_readlane_b32 s{64 + i}, {WIN}, s16", "s_add_u32 s16, s16, 1"]
    return out + (["s_nop 1"] if nw else [])     # VALU SGPR write -> VALU read


def kconst(l, nw):
    """Operand for limb l of an inline constant of class nw (immediate in s17 when nw == 0)."""
    if nw == 0:
        return "s17" if l == 0 else "0"
    return f"s{64 + l}" if l < nw else "0"


def eq_const_body(xl, nw, dst):
    """dst = (value with limbs xl(l) == inline constant of class nw): one compare per constant
    limb, the limbs above it OR-reduced in VALU and compared with 0."""
    n = max(nw, 1)
    regs = ["s[34:35]", "s[36:37]", "s[38:39]", "s[60:61]", "s[64:65]", "s[66:67]", "s[68:69]", "s[70:71]"]
    # (the constant sits in s64.. for nw > 0: its compares go to the low pairs; upper limbs below)
    out = []
    for l in range(n):
        out.append(f"v_cmp_eq_u32_e64 {regs[l] if nw < 8 else regs[l]}, {xl(l)}, {kconst(l, nw)}")
    if n < L:
        up = [xl(l) for l in range(n, L)]
        acc = "v4"
        out.append(f"v_or3_b32 v4, {up[0]}, {up[1]}, {up[2]}" if len(up) >= 3 else f"v_or_b32 v4, {up[0]}, {up[1]}")
        rest = up[3:] if len(up) >= 3 else up[2:]
        while rest:
            if len(rest) >= 2:
                out.append(f"v_or3_b32 v4, v4, {rest[0]}, {rest[1]}")
                rest = rest[2:]
            else:
                out.append(f"v_or_b32 v4, v4, {rest[0]}")
                rest = []
        out.append(f"v_cmp_eq_u32_e64 {regs[n]}, 0, {acc}")
        n += 1
    out.append("s_nop 3")
    # AND tree over the n masks
    live = regs[:n]
    while len(live) > 1:
        nxt = []
        for i in range(0, len(live) - 1, 2):
            out.append(f"s_and_b64 {live[i]}, {live[i]}, {live[i + 1]}")
            nxt.append(live[i])
        if len(live) % 2:
            nxt.append(live[-1])
        live = nxt
    out.append(f"s_mov_b64 {dst}, {live[0]}")
    return out


def lt_chain(x, y, dst):
    """dst mask = (x < y) unsigned over 8 limbs; x, y are slot numbers or limb -> register
    functions; borrow chain with hazard nops."""
    xl = x if callable(x) else (lambda l, _x=x: S(_x, l))
    yl = y if callable(y) else (lambda l, _y=y: S(_y, l))
    out = [f"v_sub_co_u32_e64 v5, s[34:35], {xl(0)}, {yl(0)}"]
    cur = "s[34:35]"
    for l in range(1, L):
        nxt = dst if l == L - 1 else ("s[36:37]" if cur == "s[34:35]" else "s[34:35]")
        out.append("s_nop 0")
        out.append(f"v_subb_co_u32_e64 v5, {nxt}, {xl(l)}, {yl(l)}, {cur}")
        cur = nxt
    return out


def tl_signed(nw):
    """T = the inline constant of class nw with its sign bit (255) flipped."""
    out = [f"v_mov_b32 {T(l)}, {kconst(l, nw)}" for l in range(L - 1)]
    if nw < L:
        return out + [f"v_mov_b32 {T(L - 1)}, 0x80000000"]
    return out + [f"v_mov_b32 {T(L - 1)}, {kconst(L - 1, nw)}", f"v_xor_b32 {T(L - 1)}, 0x80000000, {T(L - 1)}"]


def flip_top(x):
    return [f"v_xor_b32 {S(x, L - 1)}, 0x80000000, {S(x, L - 1)}"]


def flip_signs(d):
    return [f"v_xor_b32 {S(d - 1, 7)}, 0x80000000, {S(d - 1, 7)}", f"v_xor_b32 {S(d, 7)}, 0x80000000, {S(d, 7)}"]


def carry_chain(first, rest, n=L):
    out = [first(0)]
    for l in range(1, n):
        out.append("s_nop 0")
        out.append(rest(l))
    return out


def mul_body(d, bl=None):
    """S[d-1] = S[d-1] * b mod 2^256 (b = slot d, or bl(j) = register of limb j): product
    scanning (Comba) columns 0..7.  A column's state is a 64-bit accumulator pair (v_mad_u64_u32
    with carry-out) plus an overflow word accumulated directly in the high word of the NEXT
    column's pair.  Even columns k accumulate in (T(k), T(k+1)), so their result word is already
    in place and only the high word moves down into v4; odd columns accumulate in v[4:5] and move
    result and high word out (T(k), T(k+1)): 16 moves per multiply instead of 20.  Carries are
    added through three rotating SGPR pairs so every VALU carry read is >= 2 instructions after
    its write; each column's first carry-add resets the overflow word; column 7 keeps only its
    low word."""
    a = d - 1
    bl = bl or (lambda j: S(d, j))
    C = ["s[34:35]", "s[36:37]", "s[38:39]"]

    def pair(k):   # (pair, lo, hi) of column k's accumulator
        if k % 2 == 0:
            return f"v[{TBASE + k}:{TBASE + k + 1}]", T(k), T(k + 1)
        return "v[4:5]", "v4", "v5"

    p0, lo0, hi0 = pair(0)
    out = [f"v_mad_u64_u32 {p0}, s[60:61], {S(a, 0)}, {bl(0)}, 0",
           f"v_mov_b32 v4, {hi0}", "v_mov_b32 v5, 0"]
    for k in range(1, L):
        pr, lo, hi = pair(k)
        prods = [(i, k - i) for i in range(k + 1)]
        if k == L - 1:
            # last column: only the low word matters, no carry tracking
            for i, j in prods:
                out.append(f"v_mad_u64_u32 {pr}, s[60:61], {S(a, i)}, {bl(j)}, {pr}")
            out += [f"v_mov_b64 {S2(a, l)}, v[{TBASE + l}:{TBASE + l + 1}]" for l in range(0, 6, 2)]
            out += [f"v_mov_b32 {S(a, 6)}, {T(6)}", f"v_mov_b32 {S(a, 7)}, {lo}"]
            break
        _, _, ohi = pair(k + 1)            # next column's pair; its high word is our overflow
        mads = [f"v_mad_u64_u32 {pr}, {C[t % 3]}, {S(a, i)}, {bl(j)}, {pr}" for t, (i, j) in enumerate(prods)]
        adds = [f"v_addc_co_u32_e64 {ohi}, s[60:61], 0, {'0' if t == 0 else ohi}, {C[t % 3]}"
                for t in range(len(prods))]
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
        if k % 2 == 0:
            out += [f"v_mov_b32 v4, {hi}"]                           # result already in T(k)
        else:
            out += [f"v_mov_b32 {T(k)}, v4", f"v_mov_b32 {T(k + 1)}, v5"]
    return out


def mul_to(al, bl, rbase, rel1=False):
    """v[rbase + k] = word k of a * b mod 2^256 (al(i) / bl(j) = registers of limb i / j; rbase
    even): mul_body's Comba columns with the even columns accumulating in the result block itself,
    for operands that are not the destination (no final copy).  rel1: the adds keep their VGPR in
    src0, so an s_set_gpr_idx_on ... gpr_idx(SRC1) that relocates b's registers leaves them alone."""
    C = ["s[34:35]", "s[36:37]", "s[38:39]"]

    def R(k):
        return f"v{rbase + k}"

    def pair(k):
        if k % 2 == 0:
            return f"v[{rbase + k}:{rbase + k + 1}]", R(k), R(k + 1)
        return "v[4:5]", "v4", "v5"

    def addc(ohi, t, c):
        if rel1:
            return f"v_addc_co_u32_e64 {ohi}, s[60:61], {'0' if t == 0 else ohi}, 0, {c}"
        return f"v_addc_co_u32_e64 {ohi}, s[60:61], 0, {'0' if t == 0 else ohi}, {c}"

    p0, lo0, hi0 = pair(0)
    out = [f"v_mad_u64_u32 {p0}, s[60:61], {al(0)}, {bl(0)}, 0",
           f"v_mov_b32 v4, {hi0}", "v_mov_b32 v5, 0"]
    for k in range(1, L):
        pr, lo, hi = pair(k)
        prods = [(i, k - i) for i in range(k + 1)]
        if k == L - 1:
            for i, j in prods:
                out.append(f"v_mad_u64_u32 {pr}, s[60:61], {al(i)}, {bl(j)}, {pr}")
            out.append(f"v_mov_b32 {R(7)}, {lo}")
            break
        _, _, ohi = pair(k + 1)
        mads = [f"v_mad_u64_u32 {pr}, {C[t % 3]}, {al(i)}, {bl(j)}, {pr}" for t, (i, j) in enumerate(prods)]
        adds = [addc(ohi, t, C[t % 3]) for t in range(len(prods))]
        n = len(prods)
        for t in range(n):
            out.append(mads[t])
            if t >= 2:
                out.append(adds[t - 2])
        out += (["s_nop 0"] if n == 2 else []) + [adds[t] for t in range(max(0, n - 2), n)]
        if k % 2 == 0:
            out += [f"v_mov_b32 v4, {hi}"]
        else:
            out += [f"v_mov_b32 {R(k)}, v4", f"v_mov_b32 {R(k + 1)}, v5"]
    return out


def lshr_body(d, q, arith):
    """S[d] >>= 32q + s in place (s = imm, 0..31): limb l = (S[l+q+1] : S[l+q]) >> s, ascending
    so every source is read before it is overwritten; ASHR fills with the sign word v4."""
    out = [f"v_ashrrev_i32 v4, 31, {S(d, 7)}"] if arith else []
    for l in range(L):
        src = l + q
        if src + 1 <= L - 1:
            out.append(f"v_alignbit_b32 {S(d, l)}, {S(d, src + 1)}, {S(d, src)}, s17")
        elif src == L - 1:
            out.append(f"v_alignbit_b32 {S(d, l)}, v4, {S(d, L - 1)}, s17" if arith
                       else f"v_lshrrev_b32 {S(d, l)}, s17, {S(d, L - 1)}")
        else:
            out.append(f"v_mov_b32 {S(d, l)}, {'v4' if arith else 0}")
    return out


def shl_body(d, q, bits):
    """S[d] <<= 32q + s in place, descending.  bits: s != 0 and imm = 32 - s
    (limb l = (S[l-q] : S[l-q-1]) >> (32 - s)); otherwise a pure word move."""
    out = []
    for l in range(L - 1, -1, -1):
        src = l - q
        if src < 0:
            out.append(f"v_mov_b32 {S(d, l)}, 0")
        elif not bits:
            if src != l:
                out.append(f"v_mov_b32 {S(d, l)}, {S(d, src)}")
        elif src >= 1:
            out.append(f"v_alignbit_b32 {S(d, l)}, {S(d, src)}, {S(d, src - 1)}, s17")
        else:
            out.append(f"v_alignbit_b32 {S(d, l)}, {S(d, 0)}, 0, s17")
    return out


def copy_to_w(d):
    return [f"v_mov_b64 {W2(l)}, {S2(d, l)}" for l in range(0, L, 2)]


def copy_from_w(d):
    return [f"v_mov_b64 {S2(d, l)}, {W2(l)}" for l in range(0, L, 2)]


def divc_body(x, kind, pfx):
    """Division of slot x by a constant divisor c (|c| < 2^32, from the tape constants at imm:
    {d_norm, v, shift, |c|}).  kinds: UDIVC UREMC SREMC SMODCP SMODCN SDIVCP SDIVCN (P/N = sign
    of c).  bvsrem / bvsmod / bvsdiv at 256 bits (SMT-LIB)."""
    out = ["s_lshl_b32 s34, s17, 2", "s_load_dwordx4 s[64:67], s[20:21], s34"] + copy_to_w(x) + ["s_waitcnt lgkmcnt(0)"]
    signed = kind not in ("UDIVC", "UREMC")
    if signed:
        out.append(f"s_call_b64 s[76:77], {pfx}_sub_abs")       # v3 = sign(a) mask, W = |a|
    out.append(f"s_call_b64 s[76:77], {pfx}_sub_udiv32")         # W = q, v4 = r
    if kind == "UDIVC":
        out += copy_from_w(x)
    elif kind == "UREMC":
        out += [f"v_mov_b32 {S(x, 0)}, v4"] + zero_limbs(x, 1)
    elif kind == "SREMC":
        # r with the dividend's sign: -r = (2^32 - r, ~0, ..) when r != 0
        out += ["v_sub_u32 v5, 0, v4",
                "v_cmp_ne_u32_e64 s[34:35], 0, v3",
                "v_cmp_ne_u32_e64 s[36:37], 0, v4",
                "s_nop 3",
                "s_and_b64 s[36:37], s[36:37], s[34:35]",
                f"v_cndmask_b32_e64 {S(x, 0)}, v4, v5, s[34:35]",
                "v_cndmask_b32_e64 v6, 0, -1, s[36:37]"]
        out += [f"v_mov_b32 {S(x, l)}, v6" for l in range(1, L)]
    elif kind == "SMODCP":
        # c > 0: t = (a < 0 && r != 0) ? c - r : r   (non-negative, < c)
        out += ["v_sub_u32 v5, s67, v4",
                "v_cmp_ne_u32_e64 s[34:35], 0, v3",
                "v_cmp_ne_u32_e64 s[36:37], 0, v4",
                "s_nop 3",
                "s_and_b64 s[36:37], s[36:37], s[34:35]",
                "s_nop 0",
                f"v_cndmask_b32_e64 {S(x, 0)}, v4, v5, s[36:37]"] + zero_limbs(x, 1)
    elif kind == "SMODCN":
        # c < 0: result = -t, t = a >= 0 ? (r != 0 ? |c| - r : 0) : r
        out += ["v_sub_u32 v5, s67, v4",
                "v_cmp_ne_u32_e64 s[36:37], 0, v4",
                "v_cmp_ne_u32_e64 s[34:35], 0, v3",
                "s_nop 1",
                "v_cndmask_b32_e64 v5, 0, v5, s[36:37]",
                "v_cndmask_b32_e64 v5, v5, v4, s[34:35]",
                "v_sub_u32 v4, 0, v5",
                "v_cmp_ne_u32_e64 s[36:37], 0, v5",
                f"v_mov_b32 {S(x, 0)}, v4",
                "s_nop 1",
                "v_cndmask_b32_e64 v6, 0, -1, s[36:37]"]
        out += [f"v_mov_b32 {S(x, l)}, v6" for l in range(1, L)]
    elif kind in ("SDIVCP", "SDIVCN"):
        # q negated when the operand signs differ
        if kind == "SDIVCN":
            out.append("v_not_b32 v3, v3")
        out.append(f"s_call_b64 s[76:77], {pfx}_sub_cneg")
        out += copy_from_w(x)
    return out


def sub_abs_cneg(pfx):
    """_sub_abs: v3 = sign mask of W, then _sub_cneg: W = (W ^ v3) - v3 (256-bit: subtracting the
    all-ones word v3 from every limb with borrow = adding 1 to ~W when v3 = ~0)."""
    out = [f"{pfx}_sub_abs:", f"v_ashrrev_i32 v3, 31, {W(7)}", f"{pfx}_sub_cneg:"]
    out += [f"v_xor_b32 {W(l)}, {W(l)}, v3" for l in range(L)]
    out += carry_chain(lambda l: f"v_sub_co_u32 {W(l)}, vcc, {W(l)}, v3",
                       lambda l: f"v_subb_co_u32 {W(l)}, vcc, {W(l)}, v3, vcc")
    out += ["s_setpc_b64 s[76:77]"]
    return out


def sub_udiv32(pfx):
    """W[0..7] = W / c, v4 = W mod c for a 32-bit divisor c (wave-uniform), by 2-by-1 word division
    with a precomputed reciprocal (Moller & Granlund, "Improved division by invariant integers",
    2011, Alg. 4): s64 = c << sh (normalised), s65 = floor((2^64-1)/s64) - 2^32, s66 = sh.
    The numerator is normalised limb by limb on the fly ((W[i]:W[i-1]) >> (32-sh)); quotient
    words overwrite W[i] (W[i-1] is still unread when step i writes).  ~14 VALU per limb."""
    out = [f"{pfx}_sub_udiv32:",
           "s_cmp_eq_u32 s66, 0",
           "s_cselect_b64 s[70:71], 0, -1",          # all lanes when sh != 0
           "s_sub_u32 s68, 32, s66",
           f"v_lshrrev_b32 v5, s68, {W(7)}",
           "v_cndmask_b32_e64 v5, 0, v5, s[70:71]"]   # r = top bits shifted out (0 when sh == 0)
    for i in range(L - 1, -1, -1):
        lo = W(i - 1) if i > 0 else "0"
        out += [f"v_alignbit_b32 v4, {W(i)}, {lo}, s68",
                f"v_cndmask_b32_e64 v4, {W(i)}, v4, s[70:71]",      # u0 = normalised limb i
                "v_mad_u64_u32 v[6:7], s[34:35], s65, v5, v[4:5]",    # (q1:q0) = v*r + (r:u0)
                "v_add_u32 v7, 1, v7",
                "v_mul_lo_u32 v5, v7, s64",
                "v_sub_u32 v5, v4, v5",                               # r = u0 - q1*d
                "v_cmp_gt_u32_e64 s[36:37], v5, v6",
                "v_add_u32 v4, s64, v5",
                "v_add_u32 v6, -1, v7",
                "s_nop 1",
                "v_cndmask_b32_e64 v5, v5, v4, s[36:37]",
                "v_cndmask_b32_e64 v7, v7, v6, s[36:37]",
                "v_cmp_le_u32_e64 s[38:39], s64, v5",
                "v_subrev_u32 v4, s64, v5",
                "v_add_u32 v6, 1, v7",
                "s_nop 1",
                "v_cndmask_b32_e64 v5, v5, v4, s[38:39]",
                f"v_cndmask_b32_e64 {W(i)}, v7, v6, s[38:39]"]
    out += ["v_lshrrev_b32 v4, s66, v5", "s_setpc_b64 s[76:77]"]
    return out


def sub_udivv(pfx):
    """G: unsigned 256-bit division by a variable divisor (bvudiv / bvurem, SMT-LIB: x / 0 = all
    ones, x % 0 = x).  In: dividend U[0:8], divisor U[16:24] (U = the UF1 work registers).  Out:
    quotient U[0:8], remainder W[0:8].  Clobbers U, W, v3-v7 and s[34:39], s[60:61], s[64:71].

    Normalised schoolbook division (Knuth, TAOCP 4.3.1 Algorithm D), per lane: the divisor is
    shifted left by s = 32k + b bits (k whole limbs in three conditional stages, then b bits) so
    its top bit is set, the dividend by the same amount into 16 limbs u'; the quotient is then
    8 base-2^32 digits, j = 7 .. 0.  Each digit is estimated from the window's top two limbs by a
    2-by-1 division with the divisor's reciprocal (Moller & Granlund 2011, Alg. 4; the reciprocal
    floor((2^64 - 1) / d1) - 2^32 comes from an fp64 estimate plus an exact integer fix-up), refined
    against the second divisor limb (step D3, <= 2 decrements), multiplied back and subtracted
    from the 9-limb window; the rare borrow adds the divisor back once.  The digit replaces the
    window's top limb (zero after the step), so u'[8:16] ends as the quotient and u'[0:8] as the
    normalised remainder.  A digit every lane's window shows to be 0 (top limb 0, next limb below
    d1) is skipped wave-uniformly.  A zero divisor divides by 1 and is patched at the end.
    ~650 VALU per call (the radix-2 loop it replaces took 32 steps per significant limb, ~58 VALU
    each).  Algorithm model: tools/udivv_model.py."""
    U = [f"v{UBASE + l}" for l in range(16)]           # u' (16 limbs)
    Vd = [f"v{UBASE + 16 + l}" for l in range(8)]      # v' (normalised divisor)
    d1, d0 = Vd[7], Vd[6]
    P, PL, PH = W2(0), W(0), W(1)                      # 64-bit products
    NR, RH = W2(2), W(3)                               # (n_, rhat) pair
    QH, INV = W(4), W(5)
    AD, ADL = W2(6), W(6)                              # multiply-subtract addend (carry, 0)
    out = [f"{pfx}_sub_udivv:"]
    out += [f"v_mov_b64 v[{UBASE + 8 + l}:{UBASE + 9 + l}], 0" for l in range(0, 8, 2)]
    # zero divisor lanes (s[64:65]) divide by 1
    out += [f"v_or3_b32 v5, {Vd[0]}, {Vd[1]}, {Vd[2]}", f"v_or3_b32 v5, v5, {Vd[3]}, {Vd[4]}",
            f"v_or3_b32 v5, v5, {Vd[5]}, {Vd[6]}", f"v_or_b32 v5, v5, {Vd[7]}",
            "v_cmp_eq_u32_e64 s[64:65], 0, v5", "s_nop 1",
            f"v_cndmask_b32_e64 {Vd[0]}, {Vd[0]}, 1, s[64:65]"]
    # v6 = top nonzero limb of the divisor, v3 = k = zero limbs above it, v7 = b = its leading zeros
    out += [f"v_mov_b32 v6, {Vd[7]}", "v_mov_b32 v3, 0"]
    for l in range(6, -1, -1):
        out += ["v_cmp_eq_u32_e64 vcc, 0, v6", "s_nop 1",
                f"v_cndmask_b32_e64 v6, v6, {Vd[l]}, vcc",
                "v_addc_co_u32_e64 v3, vcc, v3, 0, vcc"]
    out += ["v_ffbh_u32 v7, v6",
            "v_and_b32 v5, 4, v3", "v_cmp_ne_u32_e64 s[66:67], 0, v5",
            "v_and_b32 v5, 2, v3", "v_cmp_ne_u32_e64 s[68:69], 0, v5",
            "v_and_b32 v5, 1, v3", "v_cmp_ne_u32_e64 s[70:71], 0, v5",
            "v_cmp_eq_u32_e64 s[36:37], 0, v7",
            "v_sub_u32 v5, 32, v7",
            "s_nop 1"]
    # whole-limb shift left by k (stages of 4, 2, 1 limbs), highest limb first
    for st, m, hi in ((4, "s[66:67]", 11), (2, "s[68:69]", 13), (1, "s[70:71]", 14)):
        out += [f"v_cndmask_b32_e64 {U[i]}, {U[i]}, {U[i - st]}, {m}" for i in range(hi, st - 1, -1)]
        out += [f"v_cndmask_b32_e64 {U[i]}, {U[i]}, 0, {m}" for i in range(st - 1, -1, -1)]
        out += [f"v_cndmask_b32_e64 {Vd[i]}, {Vd[i]}, {Vd[i - st]}, {m}" for i in range(7, st - 1, -1)]
        out += [f"v_cndmask_b32_e64 {Vd[i]}, {Vd[i]}, 0, {m}" for i in range(st - 1, -1, -1)]
    # bit shift left by b (v_alignbit by 32 - b; b = 0 keeps the limb: s[36:37])
    for R, n in ((U, 16), (Vd, 8)):
        for i in range(n - 1, 0, -1):
            out += [f"v_alignbit_b32 v6, {R[i]}, {R[i - 1]}, v5", f"v_cndmask_b32_e64 {R[i]}, v6, {R[i]}, s[36:37]"]
        out.append(f"v_lshlrev_b32 {R[0]}, v7, {R[0]}")
    # INV = floor((2^64 - 1) / d1) - 2^32: fp64 reciprocal (one Newton step), then exact fix-up
    # with p = (INV + 2^32) * d1: p >= 2^64 -> INV - 1; p + d1 < 2^64 -> INV + 1
    out += [f"v_cvt_f64_u32 {P}, {d1}",
            f"v_rcp_f64 {NR}, {P}",
            "s_nop 1",
            f"v_fma_f64 {AD}, -{P}, {NR}, 1.0",
            f"v_fma_f64 {NR}, {NR}, {AD}, {NR}",
            f"v_ldexp_f64 {NR}, {NR}, 64",
            "s_mov_b32 s34, 0", "s_mov_b32 s35, 0xc1f00000",
            f"v_add_f64 {NR}, {NR}, s[34:35]",
            f"v_cvt_u32_f64 {INV}, {NR}",
            "v_mov_b32 v4, 0", f"v_mov_b32 v5, {d1}",
            f"v_mad_u64_u32 {P}, s[34:35], {INV}, {d1}, v[4:5]",
            f"v_add_co_u32 v4, vcc, {PL}, {d1}",
            "s_nop 0",
            f"v_addc_co_u32 v5, vcc, {PH}, 0, vcc",
            "s_nop 3",
            "s_or_b64 s[36:37], s[34:35], vcc",
            "s_not_b64 s[36:37], s[36:37]",
            f"v_add_u32 v4, -1, {INV}", f"v_add_u32 v5, 1, {INV}",
            f"v_cndmask_b32_e64 {INV}, {INV}, v4, s[34:35]",
            f"v_cndmask_b32_e64 {INV}, {INV}, v5, s[36:37]"]
    for j in range(7, -1, -1):
        n1, n0, nn = U[j + 8], U[j + 7], U[j + 6]
        lbl = f"{pfx}_udv_j{j}"
        out += [f"v_cmp_eq_u32_e64 s[34:35], 0, {n1}",
                f"v_cmp_lt_u32_e64 s[36:37], {n0}, {d1}",
                "s_nop 3",
                "s_and_b64 s[34:35], s[34:35], s[36:37]",
                "s_cmp_eq_u64 s[34:35], exec",
                f"s_cbranch_scc1 {lbl}"]
        # (QH, RH) = divmod(n1:n0, d1) for n1 < d1 (Moller-Granlund)
        out += [f"v_mov_b32 v4, {n0}", f"v_mov_b32 v5, {n1}",
                f"v_mad_u64_u32 {P}, s[38:39], {INV}, {n1}, v[4:5]",
                f"v_add_u32 {PH}, 1, {PH}",
                f"v_mul_lo_u32 v6, {PH}, {d1}",
                f"v_sub_u32 v3, {n0}, v6",
                f"v_cmp_gt_u32_e64 s[34:35], v3, {PL}",
                f"v_add_u32 v6, {d1}, v3",
                f"v_add_u32 {QH}, -1, {PH}",
                f"v_cndmask_b32_e64 v3, v3, v6, s[34:35]",
                f"v_cndmask_b32_e64 {QH}, {PH}, {QH}, s[34:35]",
                f"v_cmp_le_u32_e64 s[36:37], {d1}, v3",
                f"v_subrev_u32 v6, {d1}, v3",
                f"v_add_u32 {PH}, 1, {QH}",
                f"v_cndmask_b32_e64 {RH}, v3, v6, s[36:37]",
                f"v_cndmask_b32_e64 {QH}, {QH}, {PH}, s[36:37]"]
        # n1 == d1: QH = 2^32 - 1, RH = n0 + d1 (s[60:61] = lanes where that overflowed)
        out += [f"v_cmp_eq_u32_e64 s[34:35], {n1}, {d1}",
                f"v_add_co_u32 v6, s[36:37], {n0}, {d1}",
                "s_nop 1",
                f"v_cndmask_b32_e64 {QH}, {QH}, -1, s[34:35]",
                f"v_cndmask_b32_e64 {RH}, {RH}, v6, s[34:35]",
                "s_nop 2",
                "s_and_b64 s[60:61], s[34:35], s[36:37]",
                f"v_mov_b32 {W(2)}, {nn}"]
        # D3: while RH < 2^32 and QH * d0 > (RH : n_): QH -= 1, RH += d1 (at most twice)
        for it in range(2):
            out += [f"v_mad_u64_u32 {P}, s[38:39], {QH}, {d0}, 0",
                    f"v_cmp_gt_u64_e64 s[34:35], {P}, {NR}",
                    "s_nop 3",
                    "s_andn2_b64 s[34:35], s[34:35], s[60:61]",
                    "s_cmp_eq_u64 s[34:35], 0",
                    f"s_cbranch_scc1 {pfx}_udv_d3_{j}",
                    f"v_add_u32 v6, -1, {QH}",
                    f"v_add_co_u32 v3, s[36:37], {RH}, {d1}",
                    f"v_cndmask_b32_e64 {QH}, {QH}, v6, s[34:35]",
                    f"v_cndmask_b32_e64 {RH}, {RH}, v3, s[34:35]",
                    "s_nop 2",
                    "s_and_b64 s[36:37], s[36:37], s[34:35]",
                    "s_or_b64 s[60:61], s[60:61], s[36:37]"]
        out += [f"{pfx}_udv_d3_{j}:"]
        # window u'[j .. j+8] -= QH * v'; vcc = lanes that borrowed
        out += [f"v_mov_b64 {AD}, 0"]
        for i in range(8):
            out.append(f"v_mad_u64_u32 {P}, s[38:39], {QH}, {Vd[i]}, {AD}")
            out.append(f"v_sub_co_u32 {U[j + i]}, vcc, {U[j + i]}, {PL}" if i == 0
                       else f"v_subb_co_u32 {U[j + i]}, vcc, {U[j + i]}, {PL}, vcc")
            out.append(f"v_mov_b32 {ADL}, {PH}")
        out += [f"v_subb_co_u32 v6, vcc, {n1}, {ADL}, vcc",
                "s_nop 3",
                "s_cmp_eq_u64 vcc, 0",
                f"s_cbranch_scc1 {pfx}_udv_ok{j}",
                "s_mov_b64 s[34:35], vcc",
                f"v_add_u32 v6, -1, {QH}",
                f"v_cndmask_b32_e64 {QH}, {QH}, v6, s[34:35]"]
        for i in range(8):
            out += [f"v_cndmask_b32_e64 v3, 0, {Vd[i]}, s[34:35]",
                    f"v_add_co_u32 {U[j]}, vcc, {U[j]}, v3" if i == 0
                    else f"v_addc_co_u32 {U[j + i]}, vcc, {U[j + i]}, v3, vcc"]
        out += [f"{pfx}_udv_ok{j}:", f"v_mov_b32 {n1}, {QH}", f"{lbl}:"]
    # remainder = u'[0:8] >> (32k + b): bits first, then whole limbs
    out += [f"v_alignbit_b32 {W(i)}, {U[i + 1]}, {U[i]}, v7" for i in range(7)]
    out += [f"v_lshrrev_b32 {W(7)}, v7, {U[7]}"]
    for st, m in ((4, "s[66:67]"), (2, "s[68:69]"), (1, "s[70:71]")):
        out += [f"v_cndmask_b32_e64 {W(i)}, {W(i)}, {W(i + st) if i + st < L else 0}, {m}" for i in range(L)]
    out += [f"v_mov_b64 v[{UBASE + l}:{UBASE + l + 1}], v[{UBASE + 8 + l}:{UBASE + 9 + l}]" for l in range(0, L, 2)]
    # divisor 0: quotient all ones, remainder the dividend (= the quotient by 1)
    out += ["s_cmp_eq_u64 s[64:65], 0", f"s_cbranch_scc1 {pfx}_udv_nz"]
    out += [f"v_cndmask_b32_e64 {W(l)}, {W(l)}, {U[l]}, s[64:65]" for l in range(L)]
    out += [f"v_cndmask_b32_e64 {U[l]}, {U[l]}, -1, s[64:65]" for l in range(L)]
    out += [f"{pfx}_udv_nz:", "s_setpc_b64 s[76:77]"]
    return out


def shiftv_body(x, kind):
    """G: S[x] shifted by the variable amount S[x + 1] (per lane; imm = the width W): amounts
    >= W (or with high limbs) give 0 (ASHR, at 256 bits only: the sign fill).  A barrel shift:
    whole limbs in three conditional stages (4, 2, 1 limbs), then the bit shift with per-lane
    v_alignbit / 64-bit shifts."""
    X = [S(x, l) for l in range(L)]
    amt = [S(x + 1, l) for l in range(L)]
    right = kind != "SHLV"
    fill = "v6" if kind == "ASHRV" else "0"
    out = [f"v_or3_b32 v5, {amt[1]}, {amt[2]}, {amt[3]}", f"v_or3_b32 v5, v5, {amt[4]}, {amt[5]}",
           f"v_or3_b32 v5, v5, {amt[6]}, {amt[7]}",
           "v_cmp_ne_u32_e64 s[34:35], 0, v5", f"v_cmp_le_u32_e64 s[36:37], s17, {amt[0]}",
           f"v_bfe_u32 v7, {amt[0]}, 5, 3", f"v_and_b32 v3, 31, {amt[0]}"]
    if kind == "ASHRV":
        out.append(f"v_ashrrev_i32 v6, 31, {X[L - 1]}")
    for k in (4, 2, 1):
        out += [f"v_and_b32 v5, {k}, v7", "v_cmp_ne_u32_e64 vcc, 0, v5", "s_nop 1"]
        order = range(L) if right else range(L - 1, -1, -1)
        for i in order:
            j = i + k if right else i - k
            src = X[j] if 0 <= j < L else fill
            out.append(f"v_cndmask_b32_e64 {X[i]}, {X[i]}, {src}, vcc")
    if right:
        for i in range(L):
            hi = X[i + 1] if i + 1 < L else ("v6" if kind == "ASHRV" else "0")
            out.append(f"v_alignbit_b32 {X[i]}, {hi}, {X[i]}, v3")
    else:
        for i in range(L - 1, 0, -1):
            out += [f"v_mov_b32 v4, {X[i - 1]}", f"v_mov_b32 v5, {X[i]}", "v_lshlrev_b64 v[4:5], v3, v[4:5]",
                    f"v_mov_b32 {X[i]}, v5"]
        out.append(f"v_lshlrev_b32 {X[0]}, v3, {X[0]}")
    out += ["s_nop 1", "s_or_b64 s[38:39], s[34:35], s[36:37]"]
    out += [f"v_cndmask_b32_e64 {X[i]}, {X[i]}, {fill}, s[38:39]" for i in range(L)]
    return out


def cneg(regs, m):
    """regs (a 256-bit value, limbs) = -regs where the lane mask VGPR m is all ones: (x ^ m) - m."""
    return [f"v_xor_b32 {r}, {r}, {m}" for r in regs] + carry_chain(
        lambda l: f"v_sub_co_u32 {regs[l]}, vcc, {regs[l]}, {m}",
        lambda l: f"v_subb_co_u32 {regs[l]}, vcc, {regs[l]}, {m}, vcc")


def sdivv_body(x, kind, cin_call):
    """G: bvsdiv / bvsrem / bvsmod at 256 bits by a variable divisor (slots x, x + 1): the
    unsigned division of |a| by |b| (sub_udivv), then the SMT-LIB sign rules; v6 / v7 = sign
    masks of a / b (slots x / x + 1 still hold a and b).  A zero divisor needs no case of its own: |a| / 0 = all ones gives -1 or 1,
    |a| % 0 = |a| gives a back."""
    A = [f"v{UBASE + l}" for l in range(L)]
    Bv = [f"v{UBASE + 16 + l}" for l in range(L)]
    Tv = [f"v{UBASE + 16 + l}" for l in range(L)]
    cin, call = cin_call[:-1], cin_call[-1:]
    out = cin + [f"v_ashrrev_i32 v6, 31, {A[L - 1]}", f"v_ashrrev_i32 v7, 31, {Bv[L - 1]}"]
    # (sub_udivv clobbers v6 / v7: the sign masks are re-read from the operand slots after it)
    out += cneg(A, "v6") + cneg(Bv, "v7") + call
    out += [f"v_ashrrev_i32 v6, 31, {S(x, L - 1)}", f"v_ashrrev_i32 v7, 31, {S(x + 1, L - 1)}"]
    Wr = [W(l) for l in range(L)]
    if kind == "SDIVV":
        out += ["v_xor_b32 v6, v6, v7"] + cneg(A, "v6")
        out += [f"v_mov_b64 {S2(x, l)}, v[{UBASE + l}:{UBASE + l + 1}]" for l in range(0, L, 2)]
    elif kind == "SREMV":
        out += cneg(Wr, "v6") + copy_from_w(x)
    else:
        # t = sa ? -u : u, plus b (the original divisor, slot x + 1) when the signs differ and u != 0
        out += [f"v_or3_b32 v5, {Wr[0]}, {Wr[1]}, {Wr[2]}", f"v_or3_b32 v5, v5, {Wr[3]}, {Wr[4]}",
                f"v_or3_b32 v5, v5, {Wr[5]}, {Wr[6]}", f"v_or_b32 v5, v5, {Wr[7]}",
                "v_cmp_ne_u32_e64 s[34:35], 0, v5",
                "v_xor_b32 v7, v6, v7",
                "v_cmp_ne_u32_e64 s[36:37], 0, v7"]
        out += cneg(Wr, "v6")
        out += ["s_nop 3", "s_and_b64 s[38:39], s[34:35], s[36:37]"]
        out += [f"v_cndmask_b32_e64 {Tv[l]}, 0, {S(x + 1, l)}, s[38:39]" for l in range(L)]
        out += carry_chain(lambda l: f"v_add_co_u32 {Wr[l]}, vcc, {Wr[l]}, {Tv[l]}",
                           lambda l: f"v_addc_co_u32 {Wr[l]}, vcc, {Wr[l]}, {Tv[l]}, vcc")
        out += copy_from_w(x)
    return out


def sub_uf1(pfx):
    """Arity-1 model function lookup (UF / as-array select, z3 completion: the else value when no
    entry matches): key W[0..7] (canonical), s98 = function id; result in v[UBASE:UBASE+7].
    FuncDev (qs_launch.h) of the function gives nl_a0 / nl_res / stride and the offsets of its
    entry rows, per-model entry ranges (entry_ptr) and SoA else block.  Per lane the entries are
    scanned in order and the first match wins (mq.h model layout); the wave loops over the
    longest list with finished lanes masked off."""
    P = pfx
    out = [f"{P}_sub_uf1:"]
    out += [f"v_mov_b64 v[{UBASE + l}:{UBASE + 1 + l}], 0" for l in range(0, 8, 2)]
    out += ["s_load_dwordx8 s[64:71], s[10:11], 0x160",       # funcs, entry_ptr, entry_words, else_words
            "s_load_dword s99, s[10:11], 0x180",             # n_funcs
            "s_waitcnt lgkmcnt(0)",
            "s_cmp_ge_u32 s98, s99",
            f"s_cbranch_scc1 {P}_uf_ret",
            "s_mul_i32 s34, s98, 56",                         # sizeof(FuncDev)
            "s_add_u32 s78, s64, s34",
            "s_addc_u32 s79, s65, 0",
            "s_load_dword s36, s[78:79], 0x4",                # nl_a0
            "s_load_dword s37, s[78:79], 0xc",                # nl_res
            "s_load_dword s38, s[78:79], 0x10",               # stride (words)
            "s_load_dword s99, s[78:79], 0x14",               # dense_e
            "s_load_dwordx2 s[64:65], s[78:79], 0x18",        # entry_base
            "s_load_dwordx2 s[60:61], s[78:79], 0x20",        # ptr_base
            "s_load_dwordx2 s[34:35], s[78:79], 0x28",        # else_base
            "s_load_dwordx2 s[78:79], s[78:79], 0x30",        # dense_base
            "s_waitcnt lgkmcnt(0)",
            "s_lshl_b64 s[34:35], s[34:35], 2",
            "s_add_u32 s70, s70, s34",
            "s_addc_u32 s71, s71, s35",                       # else rows
            "s_lshl_b64 s[60:61], s[60:61], 3",
            "s_add_u32 s66, s66, s60",
            "s_addc_u32 s67, s67, s61",                       # this function's entry_ptr[M+1]
            "s_lshl_b64 s[64:65], s[64:65], 2",
            "s_add_u32 s68, s68, s64",
            "s_addc_u32 s69, s69, s65",                       # entry 0 of the function
            "s_lshl_b32 s39, s38, 2",                         # stride bytes
            "s_lshl_b32 s98, s36, 2",                        # value offset in an entry
            "s_cmp_lg_u32 s99, 0",
            f"s_cbranch_scc1 {P}_uf_dense"]
    # The scan: eight entries per memory round trip by their first key limb (keys are hashes or
    # small integers: a limb-0 match is nearly always the entry), a full key compare for the
    # candidates only; then one round trip for the value (matched lanes) or the else value.
    # Entry offsets are 32-bit, relative to the function's entry 0 (mq_api.cpp keeps
    # entry_words under 4 GB for G and pads it: limb-0 reads run up to 7 entries past a lane's
    # last one).  U[0:8] hold the eight limb-0 words during the scan, the result after it.
    # SGPRs: s36 nl_a0, s37 nl_res, s39 stride bytes, s98 value offset, s[68:69] entry 0,
    # s[70:71] else rows, s[60:61] exec at entry, s[64:65] matched lanes, s[66:67] lanes still
    # scanning, s[34:35] / s[78:79] / s99 scratch.
    out += ["v_lshlrev_b32 v4, 1, v2",                        # m*8
            "global_load_dword v5, v4, s[66:67]",             # first entry of (f, m)
            "global_load_dword v6, v4, s[66:67] offset:8",    # end
            "s_waitcnt vmcnt(0)",
            "v_mul_lo_u32 v136, v5, s39",                      # byte offset of entry lo
            "s_mov_b64 s[60:61], exec",
            "s_mov_b64 s[64:65], 0",
            f"{P}_uf_loop:",
            "v_cmp_lt_u32_e64 s[66:67], v5, v6",
            "s_nop 3",
            "s_and_b64 exec, exec, s[66:67]",
            f"s_cbranch_execz {P}_uf_done"]
    for j in range(8):
        out += [f"s_mul_i32 s99, s39, {j}", "v_add_u32 v137, s99, v136",
                f"global_load_dword v{UBASE + j}, v137, s[68:69]"]
    out += ["s_mov_b64 s[66:67], exec", "s_waitcnt vmcnt(0)"]
    for j in range(8):
        nj = f"{P}_uf_nj{j}"
        out += [f"v_cmp_eq_u32_e64 s[34:35], v{UBASE + j}, {W(0)}",
                f"v_add_u32 v139, {j}, v5",
                "v_cmp_lt_u32_e64 s[78:79], v139, v6",
                "s_nop 3",
                "s_and_b64 s[34:35], s[34:35], s[78:79]",
                "s_and_b64 s[34:35], s[34:35], s[66:67]",      # (scc: any candidate)
                f"s_cbranch_scc0 {nj}",
                "s_mov_b64 exec, s[34:35]",
                f"s_mul_i32 s99, s39, {j}", "v_add_u32 v137, s99, v136"]
        for l in range(1, L):
            out += [f"s_cmp_le_u32 s36, {l}", f"s_cbranch_scc1 {P}_uf_kl{j}",
                    f"global_load_dword v{UBASE + 12 + l}, v137, s[68:69] offset:{4 * l}"]
        out += [f"{P}_uf_kl{j}:", "s_waitcnt vmcnt(0)", "v_mov_b32 v148, 0"]
        for l in range(1, L):
            out += [f"s_cmp_le_u32 s36, {l}", f"s_cbranch_scc1 {P}_uf_kc{j}",
                    f"v_xor_b32 v149, v{UBASE + 12 + l}, {W(l)}", "v_or_b32 v148, v148, v149"]
        out += [f"{P}_uf_kc{j}:",
                "v_cmp_eq_u32_e64 s[34:35], 0, v148",
                "s_nop 3",
                "s_and_b64 s[34:35], s[34:35], exec",
                "s_or_b64 s[64:65], s[64:65], s[34:35]",
                "s_mov_b64 exec, s[34:35]",
                "v_mov_b32 v138, v137",                          # matched entry's offset
                "s_andn2_b64 s[66:67], s[66:67], s[34:35]",     # matched lanes are done
                "s_mov_b64 exec, s[66:67]",
                f"{nj}:"]
    out += ["s_mov_b64 exec, s[66:67]",
            "v_add_u32 v5, 8, v5",
            "s_lshl_b32 s99, s39, 3",
            "v_add_u32 v136, s99, v136",
            f"s_branch {P}_uf_loop",
            f"{P}_uf_done:",
            "s_mov_b64 exec, s[60:61]"]
    out += [f"v_mov_b64 v[{UBASE + l}:{UBASE + 1 + l}], 0" for l in range(0, 8, 2)]
    # matched lanes: the value after the key; the others: the else value (SoA rows)
    out += ["s_and_b64 exec, s[60:61], s[64:65]",
            f"s_cbranch_execz {P}_uf_vl_issued",
            "v_add_u32 v150, s98, v138"]
    for l in range(L):
        out += [f"s_cmp_le_u32 s37, {l}", f"s_cbranch_scc1 {P}_uf_vl_issued",
                f"global_load_dword v{UBASE + l}, v150, s[68:69] offset:{4 * l}"]
    out += [f"{P}_uf_vl_issued:",
            "s_andn2_b64 exec, s[60:61], s[64:65]",
            f"s_cbranch_execz {P}_uf_else_done",
            "s_mov_b64 s[34:35], s[70:71]"]
    for l in range(L):
        out += [f"s_cmp_le_u32 s37, {l}", f"s_cbranch_scc1 {P}_uf_else_done",
                f"global_load_dword v{UBASE + l}, v2, s[34:35]",
                "s_add_u32 s34, s34, s74", "s_addc_u32 s35, s35, s75"]
    out += [f"{P}_uf_else_done:",
            "s_waitcnt vmcnt(0)",
            "s_mov_b64 exec, s[60:61]",
            f"{P}_uf_ret:",
            "s_setpc_b64 s[76:77]"]
    # Dense slots (FuncDev dense_e > 0, mq_api.cpp mq_models_upload): key limb l of entry slot e
    # of every model is one SoA row, so the wave's probe of slot e is one coalesced 256-byte read
    # per limb.  Same scan as above (first key limb of eight slots per round trip, full compare
    # of candidates); a lane stops at its model's entry count.  SGPRs: s38 dense_e, s98 slot,
    # s[68:69] the keys block, s39 / s[78:79] / s[34:35] scratch.
    out += [f"{P}_uf_dense:",
            "s_mov_b32 s38, s99",
            "s_load_dwordx2 s[68:69], s[10:11], 0x1b0",      # dense_words
            "s_waitcnt lgkmcnt(0)",
            "s_lshl_b64 s[78:79], s[78:79], 2",
            "s_add_u32 s68, s68, s78",
            "s_addc_u32 s69, s69, s79",
            "v_lshlrev_b32 v4, 1, v2",
            "global_load_dword v5, v4, s[66:67]",
            "global_load_dword v6, v4, s[66:67] offset:8",
            "s_mov_b64 s[60:61], exec",
            "s_mov_b64 s[64:65], 0",
            "s_mov_b32 s98, 0"]
    # round 0's key limbs are requested together with the entry counts (one round trip less;
    # a slot past a model's count is read but never matched)
    for j in range(8):
        out += [f"s_add_u32 s39, s98, {j}", "s_cmp_ge_u32 s39, s38", f"s_cbranch_scc1 {P}_ufd_ld0",
                "s_mul_i32 s39, s39, s36",
                "s_mul_i32 s78, s39, s74", "s_mul_hi_u32 s79, s39, s74",
                "s_add_u32 s78, s78, s68", "s_addc_u32 s79, s79, s69",
                f"global_load_dword v{UBASE + j}, v2, s[78:79]"]
    out += [f"{P}_ufd_ld0:",
            "s_waitcnt vmcnt(0)",
            "v_sub_u32 v6, v6, v5",                          # this model's entries
            "v_cmp_lt_u32_e64 s[66:67], s98, v6",
            "s_nop 3",
            "s_and_b64 exec, exec, s[66:67]",
            f"s_cbranch_execz {P}_ufd_done",
            f"s_branch {P}_ufd_ld",
            f"{P}_ufd_loop:",
            "v_cmp_lt_u32_e64 s[66:67], s98, v6",
            "s_nop 3",
            "s_and_b64 exec, exec, s[66:67]",
            f"s_cbranch_execz {P}_ufd_done"]
    for j in range(8):
        out += [f"s_add_u32 s39, s98, {j}", "s_cmp_ge_u32 s39, s38", f"s_cbranch_scc1 {P}_ufd_ld",
                "s_mul_i32 s39, s39, s36",
                "s_mul_i32 s78, s39, s74", "s_mul_hi_u32 s79, s39, s74",
                "s_add_u32 s78, s78, s68", "s_addc_u32 s79, s79, s69",
                f"global_load_dword v{UBASE + j}, v2, s[78:79]"]
    out += [f"{P}_ufd_ld:", "s_mov_b64 s[66:67], exec", "s_waitcnt vmcnt(0)"]
    def dense_values(lbl):
        # the value limbs of the matched lanes' slots (v138) into U[0 .. nl_res): value limb l of
        # slot e at keys + (dense_e * nl_a0 + e * nl_res + l) * M * 4 (exec = the lanes to load)
        o = ["s_mul_i32 s99, s38, s36",                      # dense_e * nl_a0
             "s_mul_i32 s78, s99, s74", "s_mul_hi_u32 s79, s99, s74",
             "s_add_u32 s78, s78, s68", "s_addc_u32 s79, s79, s69",
             "s_mul_i32 s39, s37, s74",                      # nl_res * M * 4
             "v_mov_b32 v149, s39",                          # (one SGPR operand per VALU)
             "v_mad_u64_u32 v[150:151], s[34:35], v138, v149, s[78:79]",
             "v_add_co_u32 v150, vcc, v150, v2",
             "v_addc_co_u32 v151, vcc, 0, v151, vcc"]
        for l in range(L):
            o += [f"s_cmp_le_u32 s37, {l}", f"s_cbranch_scc1 {lbl}",
                  f"global_load_dword v{UBASE + l}, v[150:151], off"]
            if l < L - 1:
                o += ["v_add_co_u32 v150, vcc, s74, v150", "v_addc_co_u32 v151, vcc, 0, v151, vcc"]
        return o + [f"{lbl}:"]

    # Fast path: each lane's candidate = its lowest slot of the round whose key limb 0 matches
    # (v137, -1: none), then ONE round trip for the candidates' other key limbs (a per-lane
    # gather) and the full compare.  The per-slot path below took one round trip per slot that
    # any lane matched -- up to 8 a round, since 64 lanes are 64 models with their own tables.
    # Lanes whose limb 0 matched but whose key did not (a false candidate: another slot of the
    # round may still match) send the round to the per-slot path.
    out += ["v_mov_b32 v137, -1"]
    for j in reversed(range(8)):
        out += [f"s_add_u32 s39, s98, {j}", "s_cmp_ge_u32 s39, s38", f"s_cbranch_scc1 {P}_ufc_s{j}",
                f"v_cmp_eq_u32_e64 s[34:35], v{UBASE + j}, {W(0)}",
                "v_cmp_lt_u32_e64 s[78:79], s39, v6",
                "s_nop 3",
                "s_and_b64 s[34:35], s[34:35], s[78:79]",
                "v_mov_b32 v139, s39",
                "v_cndmask_b32 v137, v137, v139, s[34:35]",
                f"{P}_ufc_s{j}:"]
    out += ["v_cmp_ne_u32_e64 s[34:35], -1, v137",
            "s_nop 3",
            "s_and_b64 exec, s[34:35], s[66:67]",
            f"s_cbranch_execz {P}_ufc_none",
            "s_mul_i32 s39, s36, s74",                        # nl_a0 * M * 4: one slot's key rows
            "v_mov_b32 v149, s39",
            "v_mad_u64_u32 v[150:151], s[34:35], v137, v149, s[68:69]",
            "v_add_co_u32 v150, vcc, v150, v2",
            "v_addc_co_u32 v151, vcc, 0, v151, vcc"]
    for l in range(1, L):
        out += [f"s_cmp_le_u32 s36, {l}", f"s_cbranch_scc1 {P}_ufc_kl",
                "v_add_co_u32 v150, vcc, s74, v150", "v_addc_co_u32 v151, vcc, 0, v151, vcc",
                f"global_load_dword v{UBASE + 12 + l}, v[150:151], off"]
    # ... and the candidate slot's value limbs in the same round trip (into U, whose limb-0 words
    # the candidate choice has consumed; a false candidate reloads them on the per-slot path)
    out += [f"{P}_ufc_kl:", "v_mov_b32 v138, v137"] + dense_values(f"{P}_ufc_vl")
    out += ["s_waitcnt vmcnt(0)", "v_mov_b32 v148, 0"]
    for l in range(1, L):
        out += [f"s_cmp_le_u32 s36, {l}", f"s_cbranch_scc1 {P}_ufc_kc",
                f"v_xor_b32 v149, v{UBASE + 12 + l}, {W(l)}", "v_or_b32 v148, v148, v149"]
    out += [f"{P}_ufc_kc:",
            "v_cmp_eq_u32_e64 s[34:35], 0, v148",
            "s_nop 3",
            "s_and_b64 s[34:35], s[34:35], exec",
            "s_andn2_b64 s[78:79], exec, s[34:35]",           # false candidates
            "s_or_b64 s[64:65], s[64:65], s[34:35]",
            "s_mov_b64 exec, s[34:35]",
            "v_mov_b32 v138, v137",                           # matched slot
            "s_andn2_b64 s[66:67], s[66:67], s[34:35]",
            "s_mov_b64 exec, s[66:67]",
            "s_cmp_lg_u64 s[78:79], 0",
            f"s_cbranch_scc1 {P}_ufd_slow",
            f"s_branch {P}_ufd_next",
            f"{P}_ufc_none:",
            "s_mov_b64 exec, s[66:67]",
            f"s_branch {P}_ufd_next",
            f"{P}_ufd_slow:"]
    for j in range(8):
        out += [f"s_add_u32 s39, s98, {j}", "s_cmp_ge_u32 s39, s38", f"s_cbranch_scc1 {P}_ufs_ld",
                "s_mul_i32 s39, s39, s36",
                "s_mul_i32 s78, s39, s74", "s_mul_hi_u32 s79, s39, s74",
                "s_add_u32 s78, s78, s68", "s_addc_u32 s79, s79, s69",
                f"global_load_dword v{UBASE + j}, v2, s[78:79]"]
    out += [f"{P}_ufs_ld:", "s_waitcnt vmcnt(0)"]
    for j in range(8):
        nj = f"{P}_ufd_nj{j}"
        out += [f"s_add_u32 s39, s98, {j}", "s_cmp_ge_u32 s39, s38", f"s_cbranch_scc1 {P}_ufs_end",
                f"v_cmp_eq_u32_e64 s[34:35], v{UBASE + j}, {W(0)}",
                "v_cmp_lt_u32_e64 s[78:79], s39, v6",
                "s_nop 3",
                "s_and_b64 s[34:35], s[34:35], s[78:79]",
                "s_and_b64 s[34:35], s[34:35], s[66:67]",
                f"s_cbranch_scc0 {nj}",
                "s_mov_b64 exec, s[34:35]",
                "s_mul_i32 s99, s39, s36",
                "s_mul_i32 s78, s99, s74", "s_mul_hi_u32 s79, s99, s74",
                "s_add_u32 s78, s78, s68", "s_addc_u32 s79, s79, s69"]
        for l in range(1, L):
            out += [f"s_cmp_le_u32 s36, {l}", f"s_cbranch_scc1 {P}_ufd_kl{j}",
                    "s_add_u32 s78, s78, s74", "s_addc_u32 s79, s79, 0",
                    f"global_load_dword v{UBASE + 12 + l}, v2, s[78:79]"]
        out += [f"{P}_ufd_kl{j}:", "s_waitcnt vmcnt(0)", "v_mov_b32 v148, 0"]
        for l in range(1, L):
            out += [f"s_cmp_le_u32 s36, {l}", f"s_cbranch_scc1 {P}_ufd_kc{j}",
                    f"v_xor_b32 v149, v{UBASE + 12 + l}, {W(l)}", "v_or_b32 v148, v148, v149"]
        out += [f"{P}_ufd_kc{j}:",
                "v_cmp_eq_u32_e64 s[34:35], 0, v148",
                "s_nop 3",
                "s_and_b64 s[34:35], s[34:35], exec",
                "s_or_b64 s[64:65], s[64:65], s[34:35]",
                "s_mov_b64 exec, s[34:35]",
                "v_mov_b32 v138, s39",                           # matched slot
                "s_andn2_b64 s[66:67], s[66:67], s[34:35]",
                "s_mov_b64 exec, s[66:67]",
                f"{nj}:"]
    # (per-slot path only) the values of every lane matched so far, then scan on
    out += [f"{P}_ufs_end:",
            "s_and_b64 exec, s[60:61], s[64:65]",
            f"s_cbranch_execz {P}_ufs_vd"] + dense_values(f"{P}_ufs_vl") + [
            "s_waitcnt vmcnt(0)",
            f"{P}_ufs_vd:"]
    out += [f"{P}_ufd_next:",
            "s_mov_b64 exec, s[66:67]",
            "s_add_u32 s98, s98, 8",
            f"s_branch {P}_ufd_loop",
            f"{P}_ufd_done:",
            "s_mov_b64 exec, s[60:61]"]
    # matched lanes hold their values in U[0 .. nl_res); limbs past nl_res are zero for every lane
    for l in range(L):
        out += [f"s_cmp_le_u32 s37, {l}", f"s_cbranch_scc0 {P}_ufz{l}", f"v_mov_b32 v{UBASE + l}, 0", f"{P}_ufz{l}:"]
    out += [f"s_branch {P}_uf_vl_issued"]
    # the lookup's pointer / match registers were written as v128..v151: move them to UBASE + k
    def remap(line):
        line = re.sub(r"v\[(\d+):(\d+)\]", lambda m: f"v[{fix(int(m.group(1)))}:{fix(int(m.group(2)))}]", line)
        return re.sub(r"\bv(\d+)\b", lambda m: f"v{fix(int(m.group(1)))}", line)
    return [remap(x) for x in out]


def fix(r):
    return UBASE + r - 128 if 128 <= r < 152 else r


# ---------------------------------------------------------------- handler table
# Bool producers with fused AND / OR forms (make_handlers); ACC_UNARY leave their result at their
# own slot d, the others (binary) at d - 1
ACC_UNARY = ("PUSH_VARB", "PUSH_MEMB", "PUSH_MEMSB", "PUSH_PKB", "PUSH_TMP_BOOL", "NOT")
ACC_KINDS = ACC_UNARY + ("AND", "OR", "EQ", "EQV", "EQC", "EQK", "EQVK") + tuple(
    p + c + sfx for p in "US" for c in ("LT", "GT", "LE", "GE") for sfx in ("", "V", "C", "K") if not (p == "S" and sfx))
# binary kinds whose result lands at their own slot x (the constant is not on the stack)
ACC_AT_X = ("EQK", "EQVK", "ULTK", "UGTK", "ULEK", "UGEK")
# a compare followed by NOT becomes the complementary compare (translator peephole)
NOT_OF = {"LT": "GE", "GE": "LT", "GT": "LE", "LE": "GT"}


_LONG_CALLS = [0]


def long_calls(body):
    """Profile build only: its longer handlers put the subroutines out of s_call's 16-bit reach,
    so a handler's ``s_call_b64 s[76:77], sub`` becomes a 64-bit pc-relative call through the
    subroutine scratch s[78:79] (the subroutines sit before the handlers: a negative offset)."""
    out = []
    for ln in body:
        if ln.startswith("s_call_b64 s[76:77], "):
            target = ln.split(", ", 1)[1]
            k = _LONG_CALLS[0]
            _LONG_CALLS[0] += 1
            out += ["s_getpc_b64 s[78:79]", f".Llc{k}:", f"s_add_u32 s78, s78, {target} - .Llc{k}",
                    "s_addc_u32 s79, s79, 0xffffffff", "s_swappc_b64 s[76:77], s[78:79]"]
        else:
            out.append(ln)
    return out


def handler_data_words(body):
    """Inline program words a G handler body reads past its own word: every window read
    advances s16, and the dispatch tail's advance is the next handler word."""
    adv = sum(1 for ln in body if ln == "s_add_u32 s16, s16, 1")
    tail = sum(1 for ln in body if ln.startswith("s_setpc_b64 s[18:19]"))
    return adv - tail


def make_handlers(variant, pfx):
    """(key, body lines) for the variant; key = (kind, d, v)."""
    G = variant == "g"
    hs = []
    acc = []   # (key, body without the dispatch tail) of the Bool producers that get _A/_O forms

    def H(key, body, tail=True, reads_stack=True):
        pre = [VMWAIT] if (G and reads_stack) else []
        prof = prof_point(key[0]) if G else []
        if tail:
            hs.append((key, pre + list(body) + prof + (NEXT_G if G else NEXT_P)))
            if pre:
                hs.append(((key[0] + "_L",) + tuple(key[1:]), [LGKMWAIT] + list(body) + prof_point(key[0] + "_L") + NEXT_G))
        else:
            hs.append((key, prof + pre + list(body)))
        if key[0] in ACC_KINDS and tail:
            acc.append((key, list(body), bool(pre)))

    H(("END",), [f"s_branch {pfx}_tape_end"], tail=False, reads_stack=False)
    if G:
        # a program whose last push (PUSH_MEM) may still be in flight (mq_api.cpp final pass):
        # the tape end waits for it here, so the column store needs no vector wait of its own
        H(("END_V",), ["s_waitcnt vmcnt(0)", f"s_branch {pfx}_tape_end"], tail=False, reads_stack=False)
        H(("REFILL",), load_window(False, pfx), reads_stack=False)
    # ---- leaves
    for d in range(D):
        # preloaded variables (P: the batch's first 8; G: the 8 its tapes push most)
        for v in range(NVG if G else NV):
            H(("PUSH_VAR", d, v), [f"v_mov_b64 {S2(d, l)}, {V2(v, l)}" for l in range(0, L, 2)], reads_stack=False)
            H(("PUSH_VARB", d, v), [f"v_cmp_ne_u32_e64 {B(d)}, 0, v{VBASE + 8 * v}", "s_nop 3"], reads_stack=False)
        if G:
            # variable row imm: loads in flight until the next stack reader's vmcnt wait
            for n in range(1, L + 1):
                body = ["s_mul_i32 s34, s17, s29", "s_mul_hi_u32 s35, s17, s29", "s_lshl_b64 s[34:35], s[34:35], 2",
                        "s_add_u32 s34, s34, s90", "s_addc_u32 s35, s35, s91"]
                for l in range(n):
                    body.append(f"global_load_dword {S(d, l)}, v2, s[34:35]")
                    if l < n - 1:
                        body += ["s_add_u32 s34, s34, s74", "s_addc_u32 s35, s35, s75"]
                body += zero_limbs(d, n)
                H(("PUSH_MEM", d, n - 1), body, reads_stack=False)
            H(("PUSH_MEMB", d), ["s_mul_i32 s34, s17, s29", "s_mul_hi_u32 s35, s17, s29", "s_lshl_b64 s[34:35], s[34:35], 2",
                                 "s_add_u32 s34, s34, s90", "s_addc_u32 s35, s35, s91",
                                 "global_load_dword v4, v2, s[34:35]", "s_waitcnt vmcnt(0)",
                                 f"v_cmp_ne_u32_e64 {B(d)}, 0, v4", "s_nop 3"], reads_stack=False)
            # staged rows (imm = LDS slot of the variable's first limb row, the tile's 64 words of
            # a row at STAGE + 256 * slot; v65 = STAGE + 4 * lane): LDS reads instead of global
            # loads, waited for by the next stack reader
            for n in range(1, L + 1):
                H(("PUSH_MEMS", d, n - 1), ["s_lshl_b32 s34, s17, 8", f"v_add_u32 v5, s34, {STG}"]
                  + [f"ds_read_b32 {S(d, l)}, v5 offset:{256 * l}" for l in range(n)] + zero_limbs(d, n),
                  reads_stack=False)
            H(("PUSH_MEMSB", d), ["s_lshl_b32 s34, s17, 8", f"v_add_u32 v5, s34, {STG}", "ds_read_b32 v4, v5",
                                  "s_waitcnt lgkmcnt(0)", f"v_cmp_ne_u32_e64 {B(d)}, 0, v4", "s_nop 3"], reads_stack=False)
            # Bool variable imm as the tile's packed lane mask (QArgs bool_masks; s[96:97] = this
            # tile's masks): one scalar load straight into the Bool stack
            H(("PUSH_PKB", d), ["s_lshl_b32 s34, s17, 3", f"s_load_dwordx2 {B(d)}, s[96:97], s34", "s_waitcnt lgkmcnt(0)"],
              reads_stack=False)
        if G:
            # a run of n + 1 packed Bool masks (the translator merges consecutive PUSH_PKB_A at
            # slot d, after a PUSH_PKB at d - 1 or not): PKBN_A AND-s them into B(d - 1), PKBP
            # pushes their AND as B(d) (at most six masks a word).  imm = the first mask, n inline
            # data words the others;
            # all n + 1 scalar loads are in flight behind one wait.  (lowering puts the Bool
            # columns of a conjunction first, so C4's ~11 column conjuncts are one or two words)
            # (mask pairs: never s[72:75] — &best[tape], M * 4 — nor s[80:87], live across handlers)
            idx = ["s35", "s36", "s37", "s38", "s39"]
            mr = ["s[64:65]", "s[66:67]", "s[68:69]", "s[70:71]", "s[76:77]", "s[78:79]"]
            for n in range(1, len(mr)):
                body = ["s_lshl_b32 s34, s17, 3", f"s_load_dwordx2 {mr[0]}, s[96:97], s34"]
                for i in range(n):
                    body += [f"v_readlane_b32 {idx[i]}, {WIN}, s16", "s_add_u32 s16, s16, 1"]
                body += ["s_nop 3"]
                for i in range(n):
                    body += [f"s_lshl_b32 {idx[i]}, {idx[i]}, 3",
                             f"s_load_dwordx2 {mr[i + 1]}, s[96:97], {idx[i]}"]
                body += ["s_waitcnt lgkmcnt(0)"]
                if d >= 1:
                    H(("PKBN_A", d, n), body + [f"s_and_b64 {B(d - 1)}, {B(d - 1)}, {mr[i]}" for i in range(n + 1)],
                      reads_stack=False)
                H(("PKBP", d, n), body + [f"s_and_b64 {B(d)}, {mr[0]}, {mr[1]}"]
                  + [f"s_and_b64 {B(d)}, {B(d)}, {mr[i]}" for i in range(2, n + 1)],
                  reads_stack=False)
        H(("PUSH_CONST", d), ["s_lshl_b32 s34, s17, 2", "s_load_dwordx8 s[64:71], s[20:21], s34", "s_waitcnt lgkmcnt(0)"]
          + [f"v_mov_b64 {S2(d, l)}, s[{64 + l}:{65 + l}]" for l in range(0, L, 2)], reads_stack=False)
        if G:
            # constants inline in the program stream: imm16 (PUSH_CONSTI) or n+1 data words
            H(("PUSH_CONSTI", d), [f"v_mov_b32 {S(d, 0)}, s17"] + zero_limbs(d, 1), reads_stack=False)
            for n in range(L):
                body = []
                for l in range(n + 1):
                    body += [f"v_readlane_b32 s{64 + l}, {WIN}, s16", "s_add_u32 s16, s16, 1"]
                body += ["s_nop 1"] + [f"v_mov_b32 {S(d, l)}, s{64 + l}" for l in range(n + 1)] + zero_limbs(d, n + 1)
                H(("PUSH_CONSTW", d, n), body, reads_stack=False)
        H(("PUSH_TMP", d), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1"]
          + [f"ds_read_b64 {S2(d, l)}, v5 offset:{256 * l}" for l in range(0, L, 2)] + ["s_waitcnt lgkmcnt(0)"],
          reads_stack=False)
        H(("PUSH_TMP_BOOL", d), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1", "ds_read_b32 v6, v5",
                                 "s_waitcnt lgkmcnt(0)", f"v_cmp_ne_u32_e64 {B(d)}, 0, v6", "s_nop 3"], reads_stack=False)
        H(("PUSH_BOOL", d), ["s_cmp_lg_u32 s17, 0", f"s_cselect_b64 {B(d)}, -1, 0"], reads_stack=False)
    H(("STORE_TMP", 0), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1"]
      + [f"ds_write_b64 v5, {S2(0, l)} offset:{256 * l}" for l in range(0, L, 2)])
    H(("STORE_TMP_BOOL", 0), ["s_lshl_b32 s34, s17, 11", "v_add_u32 v5, s34, v1",
                              f"v_cndmask_b32_e64 v6, 0, 1, {B(0)}", "ds_write_b32 v5, v6"], reads_stack=False)
    # ---- Bool (SALU on lane masks)
    for d in range(D):
        H(("NOT", d), [f"s_not_b64 {B(d)}, {B(d)}"], reads_stack=False)
    for d in range(1, D):
        a, b = B(d - 1), B(d)
        H(("AND", d), [f"s_and_b64 {a}, {a}, {b}"], reads_stack=False)
        H(("OR", d), [f"s_or_b64 {a}, {a}, {b}"], reads_stack=False)
        H(("XOR", d), [f"s_xor_b64 {a}, {a}, {b}"], reads_stack=False)
        H(("IFF", d), [f"s_xnor_b64 {a}, {a}, {b}"], reads_stack=False)
        H(("IMPLIES", d), [f"s_orn2_b64 {a}, {b}, {a}"], reads_stack=False)
    for d in range(2, D):
        H(("BITE", d), [f"s_and_b64 s[34:35], {B(d - 2)}, {B(d - 1)}", f"s_andn2_b64 s[36:37], {B(d)}, {B(d - 2)}",
                        f"s_or_b64 {B(d - 2)}, s[34:35], s[36:37]"], reads_stack=False)
        H(("BITE_EF", d), [f"s_and_b64 s[34:35], {B(d - 1)}, {B(d)}", f"s_andn2_b64 s[36:37], {B(d - 2)}, {B(d - 1)}",
                           f"s_or_b64 {B(d - 2)}, s[34:35], s[36:37]"], reads_stack=False)
    # ---- 256-bit predicates (unsigned compares are exact on canonical values of any width)
    for d in range(1, D):
        a, b = d - 1, d
        H(("EQ", d), eq_body(d))
        for signed in (False, True):
            pre = flip_signs(d) if signed else []
            p = "S" if signed else "U"
            H((p + "LT", d), pre + lt_chain(a, b, B(a)))
            H((p + "GT", d), pre + lt_chain(b, a, B(a)))
            H((p + "LE", d), pre + lt_chain(b, a, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(a)}, s[38:39]"])
            H((p + "GE", d), pre + lt_chain(a, b, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(a)}, s[38:39]"])
        # signed compare below 256 bits: flip bit W-1 of both operands, then compare unsigned
        for p in range(L):
            H(("FLIP2", d, p), ["s_lshl_b32 s34, 1, s17", f"v_xor_b32 {S(d - 1, p)}, s34, {S(d - 1, p)}",
                                f"v_xor_b32 {S(d, p)}, s34, {S(d, p)}"])
    # ---- 256-bit arithmetic (results below 256 bits are re-masked by MASK*)
    for d in range(1, D):
        a, b = d - 1, d
        H(("ADD", d), carry_chain(lambda l: f"v_add_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}",
                                  lambda l: f"v_addc_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}, vcc"))
        H(("SUB", d), carry_chain(lambda l: f"v_sub_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}",
                                  lambda l: f"v_subb_co_u32 {S(a, l)}, vcc, {S(a, l)}, {S(b, l)}, vcc"))
        for nm, ins in (("BAND", "v_and_b32"), ("BOR", "v_or_b32"), ("BXOR", "v_xor_b32")):
            H((nm, d), [f"{ins} {S(a, l)}, {S(a, l)}, {S(b, l)}" for l in range(L)])
        H(("MUL", d), mul_body(d))
    for d in range(D):
        H(("NEG", d), carry_chain(lambda l: f"v_sub_co_u32 {S(d, l)}, vcc, 0, {S(d, l)}",
                                  lambda l: f"v_subb_co_u32 {S(d, l)}, vcc, 0, {S(d, l)}, vcc"))
        H(("BNOT", d), [f"v_not_b32 {S(d, l)}, {S(d, l)}" for l in range(L)])
    for d in range(2, D):
        H(("ITE", d), [f"v_cndmask_b32_e64 {S(d - 2, l)}, {S(d, l)}, {S(d - 1, l)}, {B(d - 2)}" for l in range(L)])
        # else-first ternaries (gprog.h G_ITE_EF / G_BITE_EF): else at d-2, cond at d-1, then at d
        H(("ITE_EF", d), [f"v_cndmask_b32_e64 {S(d - 2, l)}, {S(d - 2, l)}, {S(d, l)}, {B(d - 1)}" for l in range(L)])
    # ---- width handling, constant shifts, sign extension (any slot, in place)
    for d in range(D):
        for n in range(1, L + 1):
            # keep n limbs, the top one masked to imm bits (MASKP) or whole (MASKZ)
            H(("MASKP", d, n - 1), ["s_lshl_b32 s34, 1, s17", "s_add_u32 s34, s34, -1",
                                    f"v_and_b32 {S(d, n - 1)}, s34, {S(d, n - 1)}"] + zero_limbs(d, n))
            if n < L:
                H(("MASKZ", d, n - 1), zero_limbs(d, n))
        for q in range(L):
            H(("LSHRI", d, q), lshr_body(d, q, False))
            H(("ASHRI", d, q), lshr_body(d, q, True))
            H(("SHLI", d, q), shl_body(d, q, True))
            if q:
                H(("SHLW", d, q), shl_body(d, q, False))
        for p in range(L):
            fill = [f"v_ashrrev_i32 v4, 31, {S(d, p)}"] + [f"v_mov_b32 {S(d, l)}, v4" for l in range(p + 1, L)]
            H(("SEXTB", d, p), [f"v_bfe_i32 {S(d, p)}, {S(d, p)}, 0, s17"] + fill)
            if p < L - 1:
                H(("SEXTA", d, p), fill)
    # ---- division by a constant (operand slot x = d - 1 of the binary op)
    for x in range(D - 1):
        for kind in ("UDIVC", "UREMC", "SREMC", "SMODCP", "SMODCN", "SDIVCP", "SDIVCN"):
            H((kind, x), divc_body(x, kind, pfx))
    # ---- G: division by a variable divisor (operand slots x, x + 1; sub_udivv)
    if G:
        for x in range(D - 1):
            cin = [f"v_mov_b64 v[{UBASE + l}:{UBASE + l + 1}], {S2(x, l)}" for l in range(0, L, 2)]
            cin += [f"v_mov_b64 v[{UBASE + 16 + l}:{UBASE + 17 + l}], {S2(x + 1, l)}" for l in range(0, L, 2)]
            call = [f"s_call_b64 s[76:77], {pfx}_sub_udivv"]
            H(("UDIVV", x), cin + call + [f"v_mov_b64 {S2(x, l)}, v[{UBASE + l}:{UBASE + l + 1}]" for l in range(0, L, 2)])
            H(("UREMV", x), cin + call + copy_from_w(x))
            for kind in ("SDIVV", "SREMV", "SMODV"):
                H((kind, x), sdivv_body(x, kind, cin + call))
            for kind in ("SHLV", "LSHRV", "ASHRV"):
                H((kind, x), shiftv_body(x, kind))
    # ---- model function lookup (G: uses v[8:31])
    if G:
        for d in range(D):
            H(("UF1", d), copy_to_w(d) + ["s_mov_b32 s98, s17", f"s_call_b64 s[76:77], {pfx}_sub_uf1"]
              + [f"v_mov_b64 {S2(d, l)}, v[{UBASE + l}:{UBASE + 1 + l}]" for l in range(0, L, 2)])
            H(("UF1B", d), copy_to_w(d) + ["s_mov_b32 s98, s17", f"s_call_b64 s[76:77], {pfx}_sub_uf1",
                                            f"v_and_b32 v4, 1, v{UBASE}", f"v_cmp_ne_u32_e64 {B(d)}, 0, v4", "s_nop 3"])
    # ---- P: right operand a constant, used straight from SGPRs (one SGPR source per VALU
    # instruction; ADD/SUB/compares would need a second one for the carry and keep the push)
    if not G:
        for d in range(1, D):
            a = d - 1
            ld = ["s_lshl_b32 s34, s17, 2", "s_load_dwordx8 s[64:71], s[20:21], s34", "s_waitcnt lgkmcnt(0)"]
            cl = (lambda l: f"s{64 + l}")
            for nm, ins in (("BANDC", "v_and_b32"), ("BORC", "v_or_b32"), ("BXORC", "v_xor_b32")):
                H((nm, d), ld + [f"{ins} {S(a, l)}, {cl(l)}, {S(a, l)}" for l in range(L)])
            H(("MULC", d), ld + mul_body(d, cl))
            H(("EQC", d), ld + eq_body(d, cl))
            # carry chains and compares read VCC / a carry SGPR besides their operands: the
            # constant goes to T first (one dispatch and no stack copy instead of PUSH_CONST)
            tl = [f"v_mov_b64 v[{TBASE + l}:{TBASE + l + 1}], s[{64 + l}:{65 + l}]" for l in range(0, L, 2)]
            H(("ADDC", d), ld + tl + carry_chain(lambda l: f"v_add_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}",
                                                 lambda l: f"v_addc_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}, vcc"))
            H(("SUBC", d), ld + tl + carry_chain(lambda l: f"v_sub_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}",
                                                 lambda l: f"v_subb_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}, vcc"))
            xa = (lambda l: S(a, l))
            H(("ULTC", d), ld + tl + lt_chain(xa, T, B(a)))
            H(("UGTC", d), ld + tl + lt_chain(T, xa, B(a)))
            H(("ULEC", d), ld + tl + lt_chain(T, xa, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(a)}, s[38:39]"])
            H(("UGEC", d), ld + tl + lt_chain(xa, T, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(a)}, s[38:39]"])
    # ---- G: compares against a constant carried inline (the translator drops the constant's
    # push): EQK / ULTK / UGTK / ULEK / UGEK (x, cls) compare slot x with it, EQVK (x, 2v + c)
    # compares preloaded variable v with it; the result lands in B(x).  cls: KCLS
    if G:
        for x in range(D - 1):
            for cls, nw in enumerate(KCLS):
                kread = const_words(nw)
                H(("EQK", x, cls), kread + eq_const_body(lambda l, _x=x: S(_x, l), nw, B(x)))
                tl = [f"v_mov_b32 {T(l)}, {kconst(l, nw)}" for l in range(L)]
                xa = (lambda l, _x=x: S(_x, l))
                H(("ULTK", x, cls), kread + tl + lt_chain(xa, T, B(x)))
                H(("UGTK", x, cls), kread + tl + lt_chain(T, xa, B(x)))
                H(("ULEK", x, cls), kread + tl + lt_chain(T, xa, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(x)}, s[38:39]"])
                H(("UGEK", x, cls), kread + tl + lt_chain(xa, T, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(x)}, s[38:39]"])
                # signed at 256 bits (SLT / SGT with a constant operand): both sign bits flipped,
                # then the unsigned borrow chain (calldata bytes: ite(k <s size, cd_k, 0))
                H(("SLTK", x, cls), kread + tl_signed(nw) + flip_top(x) + lt_chain(xa, T, B(x)))
                H(("SGTK", x, cls), kread + tl_signed(nw) + flip_top(x) + lt_chain(T, xa, B(x)))
            for v in range(NVG):
                for c, nw in enumerate(KCLS[1:]):
                    H(("EQVK", x, 2 * v + c), const_words(nw) + eq_const_body(lambda l, _v=v: f"v{VBASE + 8 * _v + l}", nw, B(x)),
                      reads_stack=False)
        # "push model variable row imm (n limbs) at x; compare it with an inline constant; AND
        # into B(x - 1)" as one handler (the translator merges PUSH_MEM / PUSH_MEMS + EQK_A): the
        # value goes to T, never to the stack, and the load wait is the handler's own
        tl = lambda l: T(l)
        for x in range(1, D):
            for n in range(1, L + 1):
                mem = ["s_mul_i32 s34, s17, s29", "s_mul_hi_u32 s35, s17, s29", "s_lshl_b64 s[34:35], s[34:35], 2",
                       "s_add_u32 s34, s34, s90", "s_addc_u32 s35, s35, s91"]
                for l in range(n):
                    mem.append(f"global_load_dword {T(l)}, v2, s[34:35]")
                    if l < n - 1:
                        mem += ["s_add_u32 s34, s34, s74", "s_addc_u32 s35, s35, s75"]
                lds = ["s_lshl_b32 s34, s17, 8", f"v_add_u32 v5, s34, {STG}"] + \
                      [f"ds_read_b32 {T(l)}, v5 offset:{256 * l}" for l in range(n)]
                zero = [f"v_mov_b32 {T(l)}, 0" for l in range(n, L)]
                for src, load, wait in (("M", mem, "s_waitcnt vmcnt(0)"), ("S", lds, "s_waitcnt lgkmcnt(0)")):
                    for nw in (2, 8):
                        H((f"{src}EQK{nw}_A", x, n - 1),
                          load + zero + const_words(nw) + [wait] + eq_const_body(tl, nw, B(x))
                          + [f"s_and_b64 {B(x - 1)}, {B(x - 1)}, {B(x)}"], reads_stack=False)
        # "push staged variable row imm (n limbs) at x; unsigned-compare it with an inline
        # constant; AND into B(x - 1)" (PUSH_MEMS + ULTK_A / UGTK_A: C4's balance checks): the
        # value goes to the free slot x, the constant to T (a borrow chain reads one SGPR only)
        for x in range(1, D):
            for n in (1, 2, 8):
                lds = ["s_lshl_b32 s34, s17, 8", f"v_add_u32 v5, s34, {STG}"] + \
                      [f"ds_read_b32 {S(x, l)}, v5 offset:{256 * l}" for l in range(n)]
                for nw in (2, 8):
                    pre = lds + zero_limbs(x, n) + const_words(nw) + \
                        [f"v_mov_b32 {T(l)}, {kconst(l, nw)}" for l in range(L)] + ["s_waitcnt lgkmcnt(0)"]
                    xs = (lambda l, _x=x: S(_x, l))
                    for nm, a_, b_ in (("ULTK", xs, T), ("UGTK", T, xs)):
                        H((f"S{nm}{nw}_A", x, n - 1), pre + lt_chain(a_, b_, B(x))
                          + [f"s_and_b64 {B(x - 1)}, {B(x - 1)}, {B(x)}"], reads_stack=False)
        # "push staged variable row imm (n limbs) at x; signed-compare it (256 bits) with an
        # inline constant" (PUSH_MEMS + SLTK / SGTK; the Bool stays at B(x))
        for x in range(D - 1):
            for n in (1, 2, 8):
                lds = ["s_lshl_b32 s34, s17, 8", f"v_add_u32 v5, s34, {STG}"] + \
                      [f"ds_read_b32 {S(x, l)}, v5 offset:{256 * l}" for l in range(n)]
                for nw in (2, 8):
                    pre = lds + zero_limbs(x, n) + const_words(nw) + tl_signed(nw) + ["s_waitcnt lgkmcnt(0)"] + flip_top(x)
                    xs = (lambda l, _x=x: S(_x, l))
                    for nm, a_, b_ in (("SLTK", xs, T), ("SGTK", T, xs)):
                        H((f"S{nm}{nw}", x, n - 1), pre + lt_chain(a_, b_, B(x)), reads_stack=False)
        # ite(c, x, 0) (the translator drops the zero's push): then-value at t, condition B(t - 1)
        for t in range(1, D - 1):
            H(("ITEZ", t), [f"v_cndmask_b32_e64 {S(t - 1, l)}, 0, {S(t, l)}, {B(t - 1)}" for l in range(L)])
            # ... its then-value a staged row (n limbs) pushed right before: read into the
            # result slot (its own value is the dead condition's) and masked there
            for n in range(1, L + 1):
                H(("ITEZS", t, n - 1), ["s_lshl_b32 s34, s17, 8", f"v_add_u32 v5, s34, {STG}"]
                  + [f"ds_read_b32 {S(t - 1, l)}, v5 offset:{256 * l}" for l in range(n)] + zero_limbs(t - 1, n)
                  + ["s_waitcnt lgkmcnt(0)"]
                  + [f"v_cndmask_b32_e64 {S(t - 1, l)}, 0, {S(t - 1, l)}, {B(t - 1)}" for l in range(n)],
                  reads_stack=False)
        # concat: S[d-1] = S[d-1] << (32q + s) | S[d] (s != 0, imm = 32 - s; SHLI + BOR in one):
        # the low operand is narrower than 32q + s bits, so only limbs 0..q take it
        for d in range(1, D):
            for q in range(L):
                H(("SHLOR", d, q), shl_body(d - 1, q, True) + [f"v_or_b32 {S(d - 1, l)}, {S(d - 1, l)}, {S(d, l)}"
                                                              for l in range(q + 1)])
    # ---- (last: these handlers never branch, so the subroutine calls above stay in s_call range)
    # ---- binary ops whose right operand is a preloaded variable (the translator fuses
    # PUSH_VAR v at slot d with the consuming op at d: no stack copy, one dispatch less)
    if True:
        for d in range(1, D):
            a = d - 1
            for v in range(NVG if G else NV):
                def vl(l, v=v):
                    return f"v{VBASE + 8 * v + l}"
                H(("ADDV", d, v), carry_chain(lambda l: f"v_add_co_u32 {S(a, l)}, vcc, {S(a, l)}, {vl(l)}",
                                              lambda l: f"v_addc_co_u32 {S(a, l)}, vcc, {S(a, l)}, {vl(l)}, vcc"))
                H(("SUBV", d, v), carry_chain(lambda l: f"v_sub_co_u32 {S(a, l)}, vcc, {S(a, l)}, {vl(l)}",
                                              lambda l: f"v_subb_co_u32 {S(a, l)}, vcc, {S(a, l)}, {vl(l)}, vcc"))
                for nm, ins in (("BANDV", "v_and_b32"), ("BORV", "v_or_b32"), ("BXORV", "v_xor_b32")):
                    H((nm, d, v), [f"{ins} {S(a, l)}, {S(a, l)}, {vl(l)}" for l in range(L)])
                H(("MULV", d, v), mul_body(d, vl))
                H(("EQV", d, v), eq_body(d, vl))
                xa = (lambda l: S(a, l))
                H(("ULTV", d, v), lt_chain(xa, vl, B(a)))
                H(("UGTV", d, v), lt_chain(vl, xa, B(a)))
                H(("ULEV", d, v), lt_chain(vl, xa, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(a)}, s[38:39]"])
                H(("UGEV", d, v), lt_chain(xa, vl, "s[38:39]") + ["s_nop 3", f"s_not_b64 {B(a)}, s[38:39]"])
    # ---- P: binary ops whose BOTH operands are leaves (the translator fuses "PUSH_VAR v1 / PUSH_CONST
    # c at slot x; PUSH_VAR v2; OP" into one handler at slot x): the right variable v2 is addressed
    # through M0 (s_set_gpr_idx_on, imm = 8 * v2 in the low byte of an index word), so one handler
    # serves every v2; no operand copies and one dispatch instead of two
    #   kindVV (x, v1): S[x] = V[v1] OP V[v2]            imm = 8 * v2
    #   MULVV (x):      S[x] = V[v1] * V[v2]              imm = 8 * v1 | (8 * v2) << 16
    #   kindCV (x):     S[x] = C OP V[v2]                 imm = const word offset | (8 * v2) << 16
    if not G:
        def vr(l):   # limb l of the M0-relocated variable (V[0] + 8 * v2)
            return f"v{VBASE + l}"
        on1 = ["s_set_gpr_idx_on s17, gpr_idx(SRC1)"]
        off = ["s_set_gpr_idx_off"]
        for x in range(D - 1):
            for v1 in range(NV):
                def v1l(l, v1=v1):
                    return f"v{VBASE + 8 * v1 + l}"
                H(("ADDVV", x, v1), on1 + carry_chain(lambda l: f"v_add_co_u32 {S(x, l)}, vcc, {v1l(l)}, {vr(l)}",
                                                      lambda l: f"v_addc_co_u32 {S(x, l)}, vcc, {v1l(l)}, {vr(l)}, vcc") + off)
                H(("SUBVV", x, v1), on1 + carry_chain(lambda l: f"v_sub_co_u32 {S(x, l)}, vcc, {v1l(l)}, {vr(l)}",
                                                      lambda l: f"v_subb_co_u32 {S(x, l)}, vcc, {v1l(l)}, {vr(l)}, vcc") + off)
                for nm, ins in (("BANDVV", "v_and_b32"), ("BORVV", "v_or_b32"), ("BXORVV", "v_xor_b32")):
                    H((nm, x, v1), on1 + [f"{ins} {S(x, l)}, {v1l(l)}, {vr(l)}" for l in range(L)] + off)
            # MULVV: V[v1] copied into S[x] through an SRC0-relocated index, then the MULV body
            H(("MULVV", x), ["s_set_gpr_idx_on s17, gpr_idx(SRC0)"] + [f"v_mov_b64 {S2(x, l)}, {V2(0, l)}" for l in range(0, L, 2)]
              + ["s_set_gpr_idx_off", "s_lshr_b32 s35, s17, 16", "s_set_gpr_idx_on s35, gpr_idx(SRC1)"]
              + mul_to(lambda i: S(x, i), vr, TBASE, rel1=True)
              + [f"v_mov_b64 {S2(x, l)}, v[{TBASE + l}:{TBASE + l + 1}]" for l in range(0, L, 2)] + off)
            ld = ["s_and_b32 s34, s17, 0xffff", "s_lshl_b32 s34, s34, 2", "s_load_dwordx8 s[64:71], s[20:21], s34",
                  "s_lshr_b32 s35, s17, 16", "s_set_gpr_idx_on s35, gpr_idx(SRC1)", "s_waitcnt lgkmcnt(0)"]
            # carry chains read VCC besides their operands (one SGPR per VALU): the constant goes to
            # T first, as in ADDC
            tl = [f"v_mov_b64 v[{TBASE + l}:{TBASE + l + 1}], s[{64 + l}:{65 + l}]" for l in range(0, L, 2)]
            H(("ADDCV", x), ld + tl + carry_chain(lambda l: f"v_add_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}",
                                                  lambda l: f"v_addc_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}, vcc") + off)
            H(("SUBCV", x), ld + tl + carry_chain(lambda l: f"v_sub_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}",
                                                  lambda l: f"v_subb_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}, vcc") + off)
            for nm, ins in (("BANDCV", "v_and_b32"), ("BORCV", "v_or_b32"), ("BXORCV", "v_xor_b32")):
                H((nm, x), ld + [f"{ins} {S(x, l)}, s{64 + l}, {vr(l)}" for l in range(L)] + off)
            H(("MULCV", x), ld + mul_to(lambda i: f"s{64 + i}", vr, SBASE + 8 * x, rel1=True) + off)
            # prefetched-constant variants: the constant is already in CB (see NEXT_P)
            cb = (lambda l: f"s{PF_CB + l}")
            pfo = ["s_lshr_b32 s35, s17, 16", "s_set_gpr_idx_on s35, gpr_idx(SRC1)"]
            tlb = [f"v_mov_b64 v[{TBASE + l}:{TBASE + l + 1}], s[{PF_CB + l}:{PF_CB + 1 + l}]" for l in range(0, L, 2)]
            H(("PF_ADDCV", x), pfo + tlb + carry_chain(lambda l: f"v_add_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}",
                                                       lambda l: f"v_addc_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}, vcc") + off)
            H(("PF_SUBCV", x), pfo + tlb + carry_chain(lambda l: f"v_sub_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}",
                                                       lambda l: f"v_subb_co_u32 {S(x, l)}, vcc, {T(l)}, {vr(l)}, vcc") + off)
            for nm, ins in (("PF_BANDCV", "v_and_b32"), ("PF_BORCV", "v_or_b32"), ("PF_BXORCV", "v_xor_b32")):
                H((nm, x), pfo + [f"{ins} {S(x, l)}, {cb(l)}, {vr(l)}" for l in range(L)] + off)
            H(("PF_MULCV", x), pfo + mul_to(cb, vr, SBASE + 8 * x, rel1=True) + off)
        for d in range(D):
            H(("PF_PUSH_CONST", d), [f"v_mov_b64 {S2(d, l)}, s[{PF_CB + l}:{PF_CB + 1 + l}]" for l in range(0, L, 2)],
              reads_stack=False)
        for d in range(1, D):
            a = d - 1
            cb = (lambda l: f"s{PF_CB + l}")
            for nm, ins in (("PF_BANDC", "v_and_b32"), ("PF_BORC", "v_or_b32"), ("PF_BXORC", "v_xor_b32")):
                H((nm, d), [f"{ins} {S(a, l)}, {cb(l)}, {S(a, l)}" for l in range(L)])
            H(("PF_MULC", d), mul_body(d, cb))
            tlb = [f"v_mov_b64 v[{TBASE + l}:{TBASE + l + 1}], s[{PF_CB + l}:{PF_CB + 1 + l}]" for l in range(0, L, 2)]
            H(("PF_ADDC", d), tlb + carry_chain(lambda l: f"v_add_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}",
                                                lambda l: f"v_addc_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}, vcc"))
            H(("PF_SUBC", d), tlb + carry_chain(lambda l: f"v_sub_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}",
                                                lambda l: f"v_subb_co_u32 {S(a, l)}, vcc, {S(a, l)}, {T(l)}, vcc"))
    # ---- Bool producers fused with the AND / OR that consumes their result (kind_A / kind_O):
    # the translator rewrites "X; AND" into "X_A" when X leaves its result at the AND's right
    # slot, one dispatch instead of two (AND / OR are ~30 % of the dispatches of EVM-shaped tapes)
    for key, body, waits in acc:
        kind, d = key[0], key[1]
        r = d if (kind in ACC_UNARY or kind in ACC_AT_X) else d - 1
        if r < 1:
            continue
        for suf, ins, ins_n in (("_A", "s_and_b64", "s_andn2_b64"), ("_O", "s_or_b64", "s_orn2_b64")):
            if kind == "NOT":   # the consumer takes the complement directly
                fused = [f"{ins_n} {B(r - 1)}, {B(r - 1)}, {B(r)}"]
            else:
                fused = list(body) + (["s_nop 3"] if body[-1].startswith("v_") else []) + [f"{ins} {B(r - 1)}, {B(r - 1)}, {B(r)}"]
            pre = [VMWAIT] if waits else []
            hs.append(((kind + suf,) + tuple(key[1:]), pre + fused + (prof_point(kind + suf) if G else []) + (NEXT_G if G else NEXT_P)))
            if waits:
                hs.append(((kind + suf + "_L",) + tuple(key[1:]), [LGKMWAIT] + fused + prof_point(kind + suf + "_L") + NEXT_G))
    subs = sub_abs_cneg(pfx) + sub_udiv32(pfx) + (sub_uf1(pfx) + sub_udivv(pfx) if G else [])
    return hs, subs


# ---------------------------------------------------------------- kernel frame
def store_column(pfx):
    """G mode 3 (hoisted column programs, mq_api.cpp cq_prepare): write the program's value into
    the model variable rows of the column, valid lanes only.  Descriptor: s82 = first row of the
    target variable, s85 = its limbs, s86 = 0 for a BV root, else 1 | (j + 1) << 1 for a Bool
    root whose packed lane-mask index is j (j + 1 = 0: none).  A Bool root's valid-lane mask
    B(0) goes straight to the tile's packed masks (s[96:97] + 8 j; one 8-byte vector store by
    lane 0, so no qs_pack_bool pass reads the rows back); its 0/1 row is written only when
    QArgs.bool_rows asks for it (a HIP C++ kernel of the launch reads rows).  A column is not a
    (tape, model) pair: the pair count the tape end added is taken back."""
    out = [f"{pfx}_store_column:",
           "s_sub_u32 s40, s40, 1",
           LGKMWAIT,                                    # (a vector push in flight: END_V waited)
           "s_mov_b32 s59, 0",                          # stores issued (load_window's wait)
           "s_mul_i32 s38, s82, s29", "s_mul_hi_u32 s39, s82, s29", "s_lshl_b64 s[38:39], s[38:39], 2",
           "s_add_u32 s38, s38, s90", "s_addc_u32 s39, s39, s91",
           "s_mov_b64 s[60:61], exec", "s_mov_b64 exec, s[62:63]",
           "s_cmp_eq_u32 s86, 0", f"s_cbranch_scc1 {pfx}_col_value",
           "s_lshr_b32 s36, s86, 1",
           "s_cmp_eq_u32 s36, 0",
           f"s_cbranch_scc1 {pfx}_col_row",
           "s_lshl_b32 s36, s36, 3",
           "s_sub_u32 s36, s36, 8",
           f"s_and_b64 s[34:35], {B(0)}, s[62:63]",
           "s_mov_b64 exec, 1",
           "v_mov_b32 v6, s36", "v_mov_b32 v4, s34", "v_mov_b32 v5, s35",
           "global_store_dwordx2 v6, v[4:5], s[96:97]",
           "s_add_u32 s59, s59, 1",
           "s_mov_b64 exec, s[62:63]",
           "s_load_dword s36, s[10:11], 0x18c",        # QArgs.bool_rows
           "s_waitcnt lgkmcnt(0)",
           "s_cmp_eq_u32 s36, 0",
           f"s_cbranch_scc1 {pfx}_col_done",
           f"{pfx}_col_row:",
           f"v_cndmask_b32_e64 v5, 0, 1, {B(0)}",
           "global_store_dword v2, v5, s[38:39]",
           "s_add_u32 s59, s59, 1",
           f"s_branch {pfx}_col_done",
           f"{pfx}_col_value:"]
    for l in range(L):
        out += [f"s_cmp_le_u32 s85, {l}", f"s_cbranch_scc1 {pfx}_col_done",
                f"global_store_dword v2, {S(0, l)}, s[38:39]", "s_add_u32 s59, s59, 1"]
        if l < L - 1:
            out += ["s_add_u32 s38, s38, s74", "s_addc_u32 s39, s39, s75"]
    out += [f"{pfx}_col_done:", "s_mov_b64 exec, s[60:61]", f"s_branch {pfx}_next_tape"]
    return out


STAGE_CHUNKS = 4   # G: 8-row chunks per wave per staging round (4 waves: 128 rows a round)


def stage_rows(pfx):
    """G: copy the model rows the batch's tapes push most (QArgs stage_rows[0..n_stage), a
    multiple of 8, padded with the zero row) for this workgroup's 64-model tile into LDS at
    stage_base + 256 * slot, 32 rows per wave per round (32 loads in flight), then s_barrier: the
    4 waves of the workgroup share the tile, so each row is fetched once per workgroup and every
    PUSH_MEMS of its tapes is an LDS read."""
    out = ["s_load_dwordx2 s[64:65], s[10:11], 0x184",     # n_stage, stage_base
           "s_load_dwordx2 s[66:67], s[10:11], 0x190",     # stage_rows
           "v_and_b32 v4, 63, v3",
           "v_lshlrev_b32 v4, 2, v4",
           "v_lshrrev_b32 v5, 6, v3",
           "s_nop 1",
           "v_readfirstlane_b32 s60, v5",                  # wave
           "s_waitcnt lgkmcnt(0)",
           f"v_add_u32 {STG}, s65, v4",
           "s_lshl_b32 s61, s60, 3",                        # first row of this wave's rounds
           f"{pfx}_stage_loop:",
           "s_cmp_ge_u32 s61, s64",
           f"s_cbranch_scc1 {pfx}_stage_done"]
    # a round: up to STAGE_CHUNKS chunks of 8 rows per wave (rows s61 + 32 c ..), every load
    # issued before the one wait (the UF1 work registers are free before the first tape)
    regs = [[T(j) for j in range(8)]] + [[f"v{UBASE + 8 * (c - 1) + j}" for j in range(8)] for c in range(1, STAGE_CHUNKS)]
    for c in range(STAGE_CHUNKS):
        if c:
            out += [f"s_add_u32 s70, s61, {32 * c}", "s_cmp_ge_u32 s70, s64", f"s_cbranch_scc1 {pfx}_stage_wait",
                    "s_lshl_b32 s70, s70, 2"]
        else:
            out += ["s_lshl_b32 s70, s61, 2"]
        out += ["s_load_dwordx8 s[80:87], s[66:67], s70", "s_waitcnt lgkmcnt(0)"]
        for j in range(8):
            out += [f"s_mul_i32 s68, s{80 + j}, s29", f"s_mul_hi_u32 s69, s{80 + j}, s29", "s_lshl_b64 s[68:69], s[68:69], 2",
                    "s_add_u32 s68, s68, s90", "s_addc_u32 s69, s69, s91",
                    f"global_load_dword {regs[c][j]}, v2, s[68:69]"]
    out += [f"{pfx}_stage_wait:", "s_lshl_b32 s70, s61, 8", f"v_add_u32 v5, s70, {STG}", "s_waitcnt vmcnt(0)"]
    for c in range(STAGE_CHUNKS):
        if c:
            out += [f"s_add_u32 s71, s61, {32 * c}", "s_cmp_ge_u32 s71, s64", f"s_cbranch_scc1 {pfx}_stage_next"]
        out += [f"ds_write_b32 v5, {regs[c][j]} offset:{8192 * c + 256 * j}" for j in range(8)]
    out += [f"{pfx}_stage_next:", f"s_add_u32 s61, s61, {32 * STAGE_CHUNKS}", f"s_branch {pfx}_stage_loop",
            f"{pfx}_stage_done:"]
    out += ["s_waitcnt lgkmcnt(0)",
            "s_barrier"]
    return out


# G (product build): 4 * lane, kept in v39 (the profile build's table register)
LANE4 = None


def ee_window():
    """G: load the early-exit window of the tape with s34 = s25 - 1 - s24 (tapes of the wave
    after it): EEA[i] = 4 * descs[s25 - 1 - 64 * (s34 / 64) - i].tape (clamped at desc 0),
    EEV[i] = best[] there, for all 64 lanes whatever exec holds.  Clobbers s35, s[60:61]; waits
    for both loads."""
    return ["s_mov_b64 s[60:61], exec",
            "s_mov_b64 exec, -1",
            "s_andn2_b32 s35, s34, 63",
            "s_sub_u32 s35, s25, s35",
            "s_sub_u32 s35, s35, 1",
            f"v_mbcnt_lo_u32_b32 {EEA}, -1, 0",
            f"v_mbcnt_hi_u32_b32 {EEA}, -1, {EEA}",
            f"v_sub_u32 {EEA}, s35, {EEA}",
            f"v_max_i32 {EEA}, 0, {EEA}",
            f"v_lshlrev_b32 {EEA}, 5, {EEA}",
            f"global_load_dword {EEA}, {EEA}, s[22:23] offset:8",
            "s_waitcnt vmcnt(0)",
            f"v_lshlrev_b32 {EEA}, 2, {EEA}",
            f"global_load_dword {EEV}, {EEA}, s[26:27] sc1",
            "s_waitcnt vmcnt(0)",
            "s_mov_b64 exec, s[60:61]"]


def frame(variant, pfx, handlers, subs):
    G = variant == "g"
    # descriptor words the tape end reads: node count, algorithmic ops, tape index (P: copies)
    DN, DA, DT = ("s84", "s87", "s82") if G else ("s78", "s79", "s100")
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
        # s30 = early exit on AND first-hit mode: the tape loop's one test
        "s_cmp_lg_u32 s31, 0",
        "s_cselect_b32 s30, 0, s30",
        # handler base
        "s_getpc_b64 s[12:13]",
        f"{pfx}_pc:",
        f"s_add_u32 s12, s12, {pfx}_hbase - {pfx}_pc",
        "s_addc_u32 s13, s13, 0",
        "s_mov_b32 s19, s13",
        # mode 2: dump handler offsets (block 0, lane 0)
        "s_cmp_eq_u32 s31, 2",
        f"s_cbranch_scc0 {pfx}_main",
        "s_or_b32 s34, s96, s97",
        "s_cmp_eq_u32 s34, 0",
        f"s_cbranch_scc0 {pfx}_exit",
        "v_cmp_eq_u32_e64 s[34:35], 0, v3",
        "s_nop 3",
        "s_and_saveexec_b64 s[36:37], s[34:35]",
        "v_mov_b32 v4, 0",
    ]
    for k in range(len(handlers)):
        if k % 1000 == 0 and k:
            P.append(f"v_mov_b32 v4, {4 * k}")   # global offsets are 13-bit signed
        P.append(f"v_mov_b32 v5, {pfx}_h{k} - {pfx}_hbase")
        P.append(f"global_store_dword v4, v5, s[78:79] offset:{4 * (k % 1000)}")
    nh = len(handlers)
    P += [f"v_mov_b32 v4, {4 * nh}",     # then the absolute handler base (s[12:13])
          "v_mov_b32 v5, s12", "global_store_dword v4, v5, s[78:79]",
          "v_mov_b32 v5, s13", "global_store_dword v4, v5, s[78:79] offset:4"]
    P += [
        "s_waitcnt vmcnt(0)",
        "s_mov_b64 exec, s[36:37]",
        f"s_branch {pfx}_exit",
        f"{pfx}_main:",
    ] + ([
        "v_mbcnt_lo_u32_b32 v39, -1, 0", "v_mbcnt_hi_u32_b32 v39, -1, v39", "v_lshlrev_b32 v39, 2, v39",
    ] if G and LANE4 else []) + [
        # wave / lane / model index
        "v_and_b32 v4, 63, v3",
        "v_lshrrev_b32 v5, 6, v3",
        # gfx950 hazard: a VALU write of a VGPR followed by v_readfirstlane of it needs wait
        # states, or the read returns the register's previous (stale) contents
        "s_nop 1",
        "v_readfirstlane_b32 s34, v5",
        "s_nop 1",
    ] + ([
        # G: the workgroup's 4 waves share one 64-model tile (s96) and take tape groups
        # 4*s97 + wave, so the model rows they push are fetched once per CU (qsa.hip remaps
        # the grid so the groups of a tile run together on one XCD and share its L2)
        "s_lshl_b32 s35, s96, 6",
        "s_lshl_b32 s97, s97, 2",
        "s_add_u32 s97, s97, s34",
    ] if G else [
        "s_lshl_b32 s35, s96, 8",
        "s_lshl_b32 s36, s34, 6",
        "s_add_u32 s35, s35, s36",
    ]) + [
        "s_cmp_ge_u32 s35, s29",
        f"s_cbranch_scc1 {pfx}_exit",
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
    ] + ([
        # G mode 3: a column level's groups are uneven (balanced by cost, mq_api.cpp
        # balance_groups): group g spans descriptors [t[g], t[g+1]) of the u32 table t at
        # args+0x38 (table_out, which only mode 2 writes)
        "s_cmp_eq_u32 s31, 3",
        f"s_cbranch_scc0 {pfx}_groups_done",
        "s_lshl_b32 s68, s97, 2",
        "s_load_dwordx2 s[24:25], s[78:79], s68",
        "s_waitcnt lgkmcnt(0)",
        "s_min_u32 s25, s25, s82",
        f"{pfx}_groups_done:",
    ] if G else []) + ([
        # G: s[96:97] = this tile's packed Bool masks, bool_masks + 8 * tile * n_bool_masks
        "s_load_dwordx2 s[64:65], s[10:11], 0x198",
        "s_load_dword s66, s[10:11], 0x1a0",
        "s_waitcnt lgkmcnt(0)",
        "s_mul_i32 s68, s96, s66",
        "s_mul_hi_u32 s69, s96, s66",
        "s_lshl_b64 s[68:69], s[68:69], 3",
        "s_add_u32 s96, s64, s68",
        "s_addc_u32 s97, s65, s69",
    ] if G else [])
    if G and PROF:
        # profile table of this wave, zeroed; the clock starts here (PRELOAD, STAGE: the prologue)
        P += ["s_load_dwordx2 s[64:65], s[10:11], 0x184",   # n_stage, stage_base
              "s_waitcnt lgkmcnt(0)",
              "s_lshl_b32 s64, s64, 8",
              "s_add_u32 s64, s64, s65",
              "v_lshrrev_b32 v4, 6, v3",
              "v_mul_u32_u24 v4, @PROFBYTES@, v4",
              f"v_add_u32 {PROF_VGPR}, s64, v4",
              "v_mbcnt_lo_u32_b32 v6, -1, 0", "v_mbcnt_hi_u32_b32 v6, -1, v6", "v_lshlrev_b32 v6, 3, v6",
              f"v_add_u32 v6, {PROF_VGPR}, v6", "v_mov_b32 v4, 0", "v_mov_b32 v5, 0",
              "@PROFZERO@",
              "s_waitcnt lgkmcnt(0)",
              "s_memtime s[100:101]", "s_waitcnt lgkmcnt(0)"]
    if G:
        # mode 3 (hoisted column programs) is translated without preloaded variables
        P += ["s_cmp_eq_u32 s31, 3", f"s_cbranch_scc1 {pfx}_preload_done"]
    if True:
        # preload variables: 64 limb rows (row index table at args+0x60; the host points missing
        # limbs / vars at an all-zero row)
        for c in range(NVG * L // 16 if G else NV * L // 16):
            P += [f"s_load_dwordx16 s[64:79], s[10:11], {0x60 + 64 * c:#x}", "s_waitcnt lgkmcnt(0)"]
            for j in range(16):
                idx = 16 * c + j
                v, l = idx // 8, idx % 8
                P += [f"s_mul_i32 s34, s{64 + j}, s29", f"s_mul_hi_u32 s35, s{64 + j}, s29",
                      "s_lshl_b64 s[34:35], s[34:35], 2", "s_add_u32 s34, s34, s90", "s_addc_u32 s35, s35, s91",
                      f"global_load_dword v{VBASE + 8 * v + l}, v2, s[34:35]"]
        P += ["s_waitcnt vmcnt(0)"]
    if G:
        P += [f"{pfx}_preload_done:"] + prof_point("PRELOAD")
    P += ["s_lshl_b32 s74, s29, 2", "s_lshr_b32 s75, s29, 30"]   # M*4 (after the preload's s[64:79] use)
    if G:
        P += stage_rows(pfx)
        P += prof_point("STAGE")
    if G:
        P += ["s_mov_b64 s[14:15], 0",   # no window yet (load_window's successor test fails)
              "s_mov_b32 s59, 0"]        # vector stores issued by the previous tape (none)
    ee = G and EEV is not None
    if ee:
        P += ["s_cmp_eq_u32 s30, 0",
              f"s_cbranch_scc1 {pfx}_ee_init_done",
              "s_cmp_ge_u32 s24, s25",
              f"s_cbranch_scc1 {pfx}_ee_init_done",
              "s_sub_u32 s34, s25, s24",
              "s_sub_u32 s34, s34, 1"] + ee_window() + [f"{pfx}_ee_init_done:"]
    # tape loop
    P += [
        f"{pfx}_tape_loop:",
        "s_cmp_ge_u32 s24, s25",
        f"s_cbranch_scc1 {pfx}_tapes_done",
        f"{pfx}_tape_body:",
    ] + [
        # descriptor s24 (32 bytes) through the load's SGPR offset
        "s_lshl_b32 s34, s24, 5",
        "s_load_dwordx8 s[80:87], s[22:23], s34",
        "s_waitcnt lgkmcnt(0)",
    ] + (prof_point("F_HDR") if G else []) + ([] if G else [
        # P: &best[tape] (G computes it on a hit only; handlers never touch s72-s73, s80-s87)
        "s_lshl_b32 s34, s82, 2",
        "s_add_u32 s72, s26, s34",
        "s_addc_u32 s73, s27, 0",
        # P: the first program entry is requested together with best[tape] (one round trip for
        # both; a skipped tape wasted a scalar load)
        "s_lshl_b32 s34, s80, 2",
        "s_add_u32 s14, s46, s34",
        "s_addc_u32 s15, s47, 0",
        "s_load_dwordx4 s[96:99], s[14:15], 0x0",
    ]) + [
        # s30: early exit on and the mode first-hit (set at the prologue)
        "s_cmp_eq_u32 s30, 0",
        f"s_cbranch_scc1 {pfx}_run",
    ] + ([
        # best[tape] from the window gathered when the wave entered it (a stale value only
        # costs a tape that a fresher one would have skipped); a new window every 64 tapes
        "s_sub_u32 s34, s25, s24",
        "s_sub_u32 s34, s34, 1",
        "s_and_b32 s35, s34, 63",
        "s_cmp_lg_u32 s35, 63",
        f"s_cbranch_scc1 {pfx}_ee_have",
    ] + ee_window() + [
        f"{pfx}_ee_have:",
    ] + prof_point("F_EE") + [
        "s_and_b32 s35, s34, 63",
        f"v_readlane_b32 s36, {EEV}, s35",
        "s_nop 3",                      # VALU SGPR write -> SALU read
        "s_cmp_ge_i32 s28, s36",
        f"s_cbranch_scc1 {pfx}_next_tape",
        # (no per-tape refresh: vector loads complete in order, so a refresh in flight would hold
        # up the tape's first operand wait by a coherent round trip; the window is re-gathered
        # every 64 tapes, and hits found meanwhile only cost tapes a fresher value would skip)
    ] if ee else [
        # best[tape] through the scalar cache, NOT glc: a coherent read is an L2 round trip per
        # tape that every wave waits for (C2 28.3 -> 24.1 ms without it).  A stale value only
        # skips less: best[] only decreases within a launch (atomicMin from INT32_MAX, set by
        # qs_init_best before it), and the dispatch's acquire invalidates the scalar cache
        "s_load_dword s34, s[72:73], 0x0",
        "s_waitcnt lgkmcnt(0)",
        "s_cmp_ge_i32 s28, s34",
        f"s_cbranch_scc1 {pfx}_next_tape",
    ]) + [
        f"{pfx}_run:",
        "s_lshl_b32 s34, s83, 2",
        "s_add_u32 s20, s88, s34",
        "s_addc_u32 s21, s89, 0",
    ] + (["s_lshl_b32 s34, s80, 2", "s_add_u32 s36, s46, s34", "s_addc_u32 s37, s47, 0"]
         + load_window(True, pfx) + frame_prof(pfx) + NEXT_G if G else [
        "s_mov_b32 s16, 12",
        # the tape end's descriptor words, out of CB (s[80:87]) before the first prefetch
        "s_mov_b32 s78, s84",
        "s_mov_b32 s79, s87",
        "s_mov_b32 s100, s82",
    ] + NEXT_P) + [
        f"{pfx}_tape_end:",
        "s_waitcnt lgkmcnt(0)",
    ] + (prof_point("F_ENDW") if G else []) + [
        "s_and_b64 s[34:35], s[48:49], s[62:63]",
        # counters per wave: tapes run, their node counts and algorithmic ops; multiplied by the
        # tile's valid lanes once, when the wave's tapes are done
        "s_add_u32 s40, s40, 1",
        f"s_add_u32 s42, s42, {DN}",
        "s_addc_u32 s43, s43, 0",
        f"s_add_u32 s44, s44, {DA}",
        "s_addc_u32 s45, s45, 0",
    ] + ([
        "s_cmp_eq_u32 s31, 3",
        f"s_cbranch_scc1 {pfx}_store_column",
    ] if G else []) + [
        "s_cmp_eq_u32 s31, 1",
        f"s_cbranch_scc1 {pfx}_store_verdict",
        "s_cmp_eq_u64 s[34:35], 0",
        f"s_cbranch_scc1 {pfx}_next_tape",
        "s_ff1_i32_b64 s38, s[34:35]",
        "s_add_u32 s38, s38, s28",
    ] + ([
        "s_lshl_b32 s39, s82, 2",            # G: &best[tape]
        "s_add_u32 s72, s26, s39",
        "s_addc_u32 s73, s27, 0",
    ] if G else []) + [
        "s_mov_b64 s[60:61], exec",
        "s_mov_b64 exec, 1",
        "v_mov_b32 v5, s38",
        "v_mov_b32 v6, 0",
        "global_atomic_smin v6, v5, s[72:73]",
    ] + (["s_mov_b32 s59, 1"] if G else []) + [
        "s_mov_b64 exec, s[60:61]",
        f"s_branch {pfx}_next_tape",
        f"{pfx}_store_verdict:",
        f"s_mul_i32 s38, {DT}, s29",
        f"s_mul_hi_u32 s39, {DT}, s29",
        "s_add_u32 s38, s38, s94",
        "s_addc_u32 s39, s39, s95",
        f"v_cndmask_b32_e64 v5, 0, 1, {B(0)}",
        "v_lshrrev_b32 v6, 2, v2",
        "s_mov_b64 s[60:61], exec",
        "s_mov_b64 exec, s[62:63]",
        "global_store_byte v6, v5, s[38:39]",
    ] + (["s_mov_b32 s59, 1"] if G else []) + [
        "s_mov_b64 exec, s[60:61]",
    ] + ([f"s_branch {pfx}_next_tape"] + store_column(pfx) if G else []) + [
        f"{pfx}_next_tape:",
    ] + (prof_point("F_END") if G else []) + [
        "s_add_u32 s24, s24, 1",
        "s_cmp_lt_u32 s24, s25",
        f"s_cbranch_scc1 {pfx}_tape_body",
        f"{pfx}_tapes_done:",
    ] + ([
        "v_mbcnt_lo_u32_b32 v6, -1, 0", "v_mbcnt_hi_u32_b32 v6, -1, v6", "v_lshlrev_b32 v6, 3, v6",
        f"v_add_u32 v7, {PROF_VGPR}, v6",
        "s_load_dwordx2 s[64:65], s[10:11], 0x1a8",
        "s_waitcnt lgkmcnt(0)",
        "@PROFFLUSH@",
        "s_waitcnt vmcnt(0)",
    ] if (G and PROF) else []) + [
        # counters x the tile's valid lanes: pairs = tapes run x valid, nodes and ops likewise
        "s_bcnt1_i32_b64 s38, s[62:63]",
        "s_mul_hi_u32 s41, s40, s38",
        "s_mul_i32 s40, s40, s38",
        "s_mul_i32 s43, s43, s38",
        "s_mul_hi_u32 s34, s42, s38",
        "s_add_u32 s43, s43, s34",
        "s_mul_i32 s42, s42, s38",
        "s_mul_i32 s45, s45, s38",
        "s_mul_hi_u32 s34, s44, s38",
        "s_add_u32 s45, s45, s34",
        "s_mul_i32 s44, s44, s38",
        # the wave's counters go to slot (tile ^ last tape) mod 256 of the slotted counter array
        # (qs_launch.h kCounterSlots): 10^6 waves adding into one cache line serialise in L2
        "s_lshr_b32 s34, s28, 6",
        "s_xor_b32 s34, s34, s25",
        "s_and_b32 s34, s34, 255",
        "s_lshl_b32 s34, s34, 7",
        "s_mov_b64 s[60:61], exec",
        "s_mov_b64 exec, 1",
        "v_mov_b32 v6, s34",
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
        f"s_branch {pfx}_exit",
    ]
    # the handler area exceeds the 128 KB reach of s_branch: leave through s_setpc
    P += [f"{pfx}_exit:", "s_getpc_b64 s[34:35]", f"{pfx}_exit_pc:",
          f"s_add_u32 s34, s34, {pfx}_end - {pfx}_exit_pc", "s_addc_u32 s35, s35, 0", "s_setpc_b64 s[34:35]"]
    P += subs
    if PROF and G:
        P.append(".p2align 3")
    P.append(f"{pfx}_hbase:")
    for k, (key, body) in enumerate(handlers):
        if PROF and G:
            P.append(".p2align 3")
        P.append(f"{pfx}_h{k}:  ; {' '.join(map(str, key))}")
        P += body
    P.append(f"{pfx}_end:")
    return P


VARIANTS = (("p", ".Lqsa", "QSA_ASM_TEXT_P", "P"), ("g", ".Lqsg", "QSA_ASM_TEXT_G", "G"))


def set_layout(variant):
    """Register map of the variant being generated (the body functions read these globals).
    P and G with preloads: the map in the module docstring (G adds the early-exit window v66/v67
    and the decoded program window v68/v69).  Compact G (NVG = 0): UF1 work v[8:31], program
    window v[32:34], staging address v35, next window v36, early-exit window v37/v38 (profile
    table v39), stack v[40:40+8*DG), T/W after it -> 8 * DG + 48 VGPRs (DG = 4: 80, 6 waves
    per SIMD)."""
    global SBASE, TBASE, UBASE, WIN, WINA, WINI, NWIN, STG, NEXT_G, EEA, EEV, PROF_VGPR, D, LANE4
    D = DG if variant == "g" else DP
    LANE4 = "v39" if (variant == "g" and NVG == 0 and not PROF) else None
    if variant == "g" and NVG == 0:
        SBASE, TBASE, UBASE = 40, 40 + 8 * DG, 8
        WIN, WINA, WINI, STG, NWIN = "v32", "v33", "v34", "v35", "v36"
        EEA, EEV, PROF_VGPR = "v38", "v37", "v39"
    else:
        SBASE, TBASE, UBASE = 72, 120, 40
        WIN, WINA, WINI, STG, NWIN = "v64", "v68", "v69", "v65", "v71"
        EEA, EEV, PROF_VGPR = "v67", "v66", "v70"
    NEXT_G = next_g()


def vgprs(variant):
    return 48 + 8 * DG if (variant == "g" and NVG == 0) else 128


def source_stamp() -> str:
    """sha256 of this generator: written into both outputs, compared by build.py (regenerate on
    any change of the generator, independent of file times)."""
    import hashlib
    with open(os.path.abspath(__file__), "rb") as f:
        return hashlib.sha256(f.read() + (b"PROF" if PROF else b"")).hexdigest()[:16]


def main():
    stamp = source_stamp()
    sclob = [f'"s{i}"' for i in range(10, 102) if i not in (32, 33)] + ['"vcc"', '"scc"', '"memory"']
    clob = {v: [f'"v{i}"' for i in range(1, vgprs(v))] + sclob for v in ("p", "g")}
    gen = {}
    for variant, pfx, macro, suffix in VARIANTS:
        set_layout(variant)
        hs, subs = make_handlers(variant, pfx)
        if PROF and variant == "g":
            hs = [(k, long_calls(b)) for k, b in hs]   # per emitted copy: unique labels
        gen[variant] = (hs, frame(variant, pfx, hs, subs), macro, suffix)
    # (kinds the translator names exist in the enum even when a layout generates no handler)
    names = sorted({k[0] for hs, *_ in gen.values() for k, _ in hs} | {"EQVK", "PUSH_VAR", "PUSH_VARB"})
    prof_names = names + list(PROF_EXTRA)
    prof_bytes = -(-16 * len(prof_names) // 512) * 512 if PROF else 0

    def resolve(ln):
        if "@" not in ln:
            return [ln]
        if "@PROF:" in ln:
            return [re.sub(r"@PROF:(\w+):(\d+)@", lambda m: str(16 * prof_names.index(m.group(1)) + int(m.group(2))), ln)]
        if ln == "@PROFZERO@":
            return [f"ds_write_b64 v6, v[4:5] offset:{512 * j}" for j in range(prof_bytes // 512)]
        if ln == "@PROFFLUSH@":
            out = []
            for j in range(prof_bytes // 512):
                # (global offsets are 13-bit signed: the address advances instead)
                out += [f"ds_read_b64 v[4:5], v7 offset:{512 * j}", "s_waitcnt lgkmcnt(0)",
                        "global_atomic_add_x2 v6, v[4:5], s[64:65]", "v_add_u32 v6, 0x200, v6"]
            return out
        return [ln.replace("@PROFBYTES@", str(prof_bytes))]
    for v in gen:
        hs, lines, macro, suffix = gen[v]
        gen[v] = (hs, [r for ln in lines for r in resolve(ln)], macro, suffix)
    with open(os.path.join(HERE, "qsa_gen.inc"), "w") as f:
        f.write(f"// GENERATED by gen_qsa.py (source {stamp}) — do not edit\n")
        for variant, (hs, lines, macro, suffix) in gen.items():
            f.write(f"#define {macro} \\\n")
            for ln in lines:
                f.write('  "' + ln.replace('"', '\\"') + '\\n" \\\n')
            f.write("  \"\"\n")
        f.write("#define QSA_CLOBBERS_P " + ", ".join(clob["p"]) + "\n")
        f.write("#define QSA_CLOBBERS_G " + ", ".join(clob["g"]) + "\n")
    with open(os.path.join(HERE, "qsa_table.h"), "w") as f:
        f.write(f"// GENERATED by gen_qsa.py (source {stamp}) — handler enumerations of the QSA interpreters\n")
        f.write("#ifndef MQ_QSA_TABLE_H\n#define MQ_QSA_TABLE_H\nnamespace mq {\n")
        f.write(f"constexpr int kQsaStack = {max(DP, DG)};\nconstexpr int kQsaStackP = {DP};\nconstexpr int kQsaStackG = {DG};\nconstexpr int kQsaVars = {NV};\nconstexpr int kQsaVarsG = {NVG};\nconstexpr int kQsaSel = {L};\n")
        f.write("enum QsaKind {\n" + "".join(f"  QK_{n},\n" for n in names) + "  QK_COUNT\n};\n")
        f.write("static const char* const kQsaKindNames[] = {" + ", ".join(f'"{n}"' for n in names) + "};\n")
        idx = {n: i for i, n in enumerate(names)}

        def table(name, fn):
            f.write(f"static const short {name}[] = {{" + ", ".join(str(fn(n)) for n in names) + "};\n")
        # fused AND / OR form of a kind (-1: none); where its Bool result lands (0: slot d,
        # 1: slot d - 1, -1: not a fusable producer); the complementary compare (-1: none)
        table("kQsaKindAndForm", lambda n: idx.get(n + "_A", -1))
        table("kQsaKindOrForm", lambda n: idx.get(n + "_O", -1))
        table("kQsaKindBoolRes", lambda n: (0 if (n in ACC_UNARY or n in ACC_AT_X) else 1) if n in ACC_KINDS else -1)
        # the variant that waits for LDS / scalar loads only (-1: none; G stack readers)
        table("kQsaKindLForm", lambda n: idx.get(n + "_L", -1))

        def inv(n):
            m = re.fullmatch(r"([US])(LT|GT|LE|GE)([VCK]?)", n)
            return idx.get(m.group(1) + NOT_OF[m.group(2)] + m.group(3), -1) if m else -1
        table("kQsaKindNot", inv)
        f.write(f"constexpr int kQsaKClassWords[] = {{{', '.join(map(str, KCLS))}}};\n")
        # diagnostic profile build (QSA_PROF=1): per-wave LDS table bytes; entry i = (cycles,
        # count) of kind i, entry QK_COUNT = the tape frame
        f.write(f"constexpr int kQsaProfBytes = {prof_bytes};\n")
        f.write(f"constexpr int kQsaProfExtra = {len(PROF_EXTRA)};\n")
        f.write("static const char* const kQsaProfExtraNames[] = {" + ", ".join(f'"{n}"' for n in PROF_EXTRA) + "};\n")
        f.write(f"constexpr int kQsaHandlerShiftG = {3 if PROF else 2};\n")
        f.write("struct QsaHandlerKey { int kind, d, v; };\n")
        for variant, (hs, lines, macro, suffix) in gen.items():
            f.write(f"constexpr int kQsaHandlers{suffix} = {len(hs)};\n")
            f.write(f"static const QsaHandlerKey kQsaHandlerKeys{suffix}[] = {{\n")
            for key, _ in hs:
                kind = key[0]
                d = key[1] if len(key) > 1 else -1
                v = key[2] if len(key) > 2 else -1
                f.write(f"  {{QK_{kind}, {d}, {v}}},\n")
            f.write("};\n")
        # G: inline data words each handler consumes from the program window (its reads of the
        # window advance s16; NEXT_G's one is the next handler word) — qsa_window_layout keeps a
        # handler and its data in one window, the translator's passes step over the data
        hs_g = gen["g"][0]
        f.write("static const unsigned char kQsaHandlerDataWordsG[] = {"
                + ", ".join(str(handler_data_words(b)) for _, b in hs_g) + "};\n")
        f.write("}  // namespace mq\n#endif\n")
    for variant, (hs, lines, *_ ) in gen.items():
        nins = sum(1 for ln in lines if ln and not ln.startswith(".L"))
        print(f"{variant}: handlers={len(hs)} asm_lines={nins}", file=sys.stderr)


if __name__ == "__main__":
    main()
