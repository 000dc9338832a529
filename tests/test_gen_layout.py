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
