"""Static checks of the generated assembly interpreters (csrc/qsa_gen.inc, written by
gen_qsa.py at build time): every register an interpreter names lies inside what its inline-asm
statement declares clobbered (so inside the kernel's VGPR / SGPR allocation — a register past it
would read or write another wave's registers), and none is one the compiler reserves (s32 / s33,
the stack and frame pointers).  No GPU needed."""
import os
import re

import pytest

INC = os.path.join(os.path.dirname(__file__), "..", "mythril_amd", "csrc", "qsa_gen.inc")


def _texts():
    if not os.path.exists(INC):
        pytest.skip("qsa_gen.inc not generated (run __graft_entry__.build())")
    src = open(INC).read()
    out = {}
    for variant in ("P", "G"):
        m = re.search(r"#define QSA_ASM_TEXT_%s \\\n(.*?)\n  \"\"\n" % variant, src, re.S)
        assert m, variant
        body = "\n".join(re.findall(r'^  "(.*)\\n" \\$', m.group(1), re.M))
        clob = re.search(r"#define QSA_CLOBBERS_%s (.*)" % variant, src).group(1)
        out[variant] = (body, set(re.findall(r'"([vs]\d+)"', clob)))
    return out


def _regs(text, kind):
    used = set()
    for a, b in re.findall(r"\b%s\[(\d+):(\d+)\]" % kind, text):
        used.update(range(int(a), int(b) + 1))
    used.update(int(x) for x in re.findall(r"\b%s(\d+)\b" % kind, text))
    return used


@pytest.mark.parametrize("variant", ["P", "G"])
def test_interpreter_registers_stay_inside_the_declared_allocation(variant):
    body, clob = _texts()[variant]
    v_decl = {int(r[1:]) for r in clob if r[0] == "v"}
    s_decl = {int(r[1:]) for r in clob if r[0] == "s"}
    v_used = _regs(body, "v") - {0}          # v0 holds the work-item id on entry
    s_used = _regs(body, "s") - set(range(0, 10))   # kernel-argument / dispatch SGPRs
    assert v_used <= v_decl, sorted(v_used - v_decl)[:10]
    assert s_used <= s_decl, sorted(s_used - s_decl)[:10]
    assert not (s_used & {32, 33})


def test_product_g_is_the_compact_layout():
    """The product G kernel fits 80 VGPRs (a 4-slot operand stack: 6 waves per SIMD, DESIGN
    §3.2); P keeps 128 and its 6-slot stack."""
    t = _texts()
    assert max(_regs(t["G"][0], "v")) < 80
    assert max(_regs(t["P"][0], "v")) < 128
    assert not re.search(r"; \S+ [4-9]\b", "\n".join(ln for ln in t["G"][0].splitlines() if ln.startswith(".Lqsg_h"))), \
        "G handlers exist only for stack slots 0-3"


def test_g_handler_data_words_match_their_kinds():
    """kQsaHandlerDataWordsG (counted from each handler body's window reads) gives every
    handler that carries inline words the count its translator form emits: a handler whose data
    is mis-counted would be split from its data by the window layout (mq_api.cpp
    qsa_window_layout) and read a wild mask index / constant."""
    tab = open(os.path.join(os.path.dirname(INC), "qsa_table.h")).read()
    keys = re.findall(r"\{QK_(\w+), (-?\d+), (-?\d+)\}", tab[tab.index("kQsaHandlerKeysG"):])
    words = [int(x) for x in re.search(r"kQsaHandlerDataWordsG\[\] = \{(.*?)\};", tab).group(1).split(", ")]
    assert len(keys) == len(words)
    kcls = [int(x) for x in re.search(r"kQsaKClassWords\[\] = \{(.*?)\};", tab).group(1).split(", ")]
    for (kind, d, v), w in zip(keys, words):
        v = int(v)
        base = kind.split("_")[0]
        if base in ("PKBN", "PKBP"):
            want = v
        elif kind.startswith("PUSH_CONSTW"):
            want = v + 1
        elif base in ("MEQK2", "SEQK2", "SULTK2", "SUGTK2", "SSLTK2", "SSGTK2"):
            want = 2
        elif base in ("MEQK8", "SEQK8", "SULTK8", "SUGTK8", "SSLTK8", "SSGTK8"):
            want = 8
        elif base in ("EQK", "ULTK", "UGTK", "ULEK", "UGEK", "SLTK", "SGTK"):
            want = kcls[v]
        else:
            want = 0
        assert w == want, (kind, d, v, w, want)


# SGPRs a G handler (or a subroutine it calls) may write: scratch, the Bool stack, the dispatch
# registers and the window (REFILL).  Everything else — &best[tape] s[72:73], M * 4 s[74:75], the
# descriptor s[80:87], counters, bases — is live across dispatches.
_G_HANDLER_WRITABLE = (set(range(34, 40)) | {60, 61} | set(range(64, 72)) | set(range(76, 80)) | {98, 99}
                       | set(range(48, 56)) | set(range(14, 20)) | {100, 101})
_NO_SDST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_setpc", "s_barrier",
            "s_endpgm", "s_sleep", "s_store", "s_dcache", "s_setprio", "s_trap")


def _sgpr_dests(line):
    ins, _, ops = line.partition(" ")
    ops = [o.strip() for o in ops.split(",")]
    if not ops or not ops[0]:
        return set()
    dst = None
    if ins.startswith("s_") and not ins.startswith(_NO_SDST):
        dst = ops[0]
    elif ins.startswith(("v_readlane", "v_readfirstlane")) or (ins.startswith("v_cmp") and ins.endswith("_e64")):
        dst = ops[0]
    elif ins.startswith(("v_add_co", "v_sub_co", "v_addc_co", "v_subb_co", "v_mad_u64_u32", "v_mad_i64_i32")):
        dst = ops[1]
    if dst is None:
        return set()
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", dst)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", dst)
    return {int(m.group(1))} if m else set()


def test_g_handlers_write_only_scratch_sgprs():
    body, _ = _texts()["G"]
    lines = body.split("\n")
    start = next(i for i, ln in enumerate(lines) if re.match(r"\.Lqsg_sub_\w+:$", ln.strip()))
    region = lines[start:]
    bad = {}
    cur = "sub"
    for ln in region:
        ln = ln.strip()
        if ln.startswith(".Lqsg_h") and ";" in ln:
            cur = ln.split(";", 1)[1].strip()
            continue
        if ln.startswith(".Lqsg_end"):
            break
        w = _sgpr_dests(ln) - _G_HANDLER_WRITABLE
        if w:
            bad.setdefault(cur, set()).update(w)
    assert not bad, {k: sorted(v) for k, v in list(bad.items())[:10]}


def test_g_staging_round_keeps_the_frame_registers():
    """The G staging round (gen_qsa.py stage_rows: 32 row loads per wave in flight) loads into
    T and the UF1 work registers only — never the program window, the staging address, the
    early-exit window or 4 * lane, which are live from the kernel prologue on."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_qsa", os.path.join(os.path.dirname(INC), "gen_qsa.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    g.set_layout("g")
    live = {g.WIN, g.WINA, g.WINI, g.STG, g.NWIN, g.EEA, g.EEV, g.LANE4, "v2", "v3"}
    body = g.stage_rows("t")
    dsts = set()
    for ln in body:
        m = re.match(r"global_load_dword (v\d+),", ln)
        if m:
            dsts.add(m.group(1))
    assert len(dsts) == 8 * g.STAGE_CHUNKS
    assert not (dsts & live), sorted(dsts & live)
    assert all(int(r[1:]) < 80 for r in dsts)
