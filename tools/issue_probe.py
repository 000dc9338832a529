#!/usr/bin/env python3
"""Issue-rate probe for the P interpreter's handler bodies (diagnostic, not product code).

Generates tools/_issue_probe.hip from gen_qsa.py's own handler bodies (MUL, ADD, BAND, the
dispatch tail) and times each body in a loop at 1, 2, 4 and 8 waves per SIMD, so the VALU issue
rate of a body is measured apart from the interpreter's dispatch:
  cycles per wave-instruction at occupancy W = elapsed cycles / (bodies per wave * VALU per body)
and the same for a body preceded by the P dispatch's scalar program-entry load (s_load + wait).
usage: python tools/issue_probe.py build   (here)   |   tools/_issue_probe   (on the GPU box)
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "mythril_amd", "csrc"))
import gen_qsa as g  # noqa: E402

g.set_layout("p")


def body_lines(name):
    if name == "mul":
        return g.mul_body(2)
    if name == "mulv":
        return g.mul_body(2, lambda j: f"v{g.VBASE + j}")
    if name == "add":
        return g.carry_chain(lambda l: f"v_add_co_u32 {g.S(1, l)}, vcc, {g.S(1, l)}, {g.S(2, l)}",
                             lambda l: f"v_addc_co_u32 {g.S(1, l)}, vcc, {g.S(1, l)}, {g.S(2, l)}, vcc")
    if name == "add_nop0":
        return [ln.replace("s_nop 1", "s_nop 0") for ln in body_lines("add")]
    if name == "band":
        return [f"v_and_b32 {g.S(1, l)}, {g.S(1, l)}, {g.S(2, l)}" for l in range(8)]
    if name == "mov4":
        return [f"v_mov_b64 {g.S2(3, l)}, {g.V2(1, l)}" for l in range(0, 8, 2)]
    if name in INDEP:   # 8 independent instructions of one kind (distinct destinations)
        return [INDEP[name].format(d=f"v{80 + k}", d2=f"v[{80 + 2 * k}:{81 + 2 * k}]", a=f"v{8 + k}", b=f"v{16 + k}",
                                   c=f"v{24 + k}", sl=38 + (k % 2), c2=f"v[{24 + 2 * (k % 4)}:{25 + 2 * (k % 4)}]",
                                   sd=f"s[{34 + 2 * (k % 3)}:{35 + 2 * (k % 3)}]") for k in range(8)]
    raise KeyError(name)


# one instruction kind, independent destinations: the issue cost of the kind alone
INDEP = {
    "i_and_vv": "v_and_b32 {d}, {a}, {b}",
    "i_and_sv": "v_and_b32 {d}, s60, {b}",
    "i_add_vv": "v_add_u32 {d}, {a}, {b}",
    "i_add_sv": "v_add_u32 {d}, s60, {b}",
    "i_mov_v": "v_mov_b32 {d}, {a}",
    "i_mov_s": "v_mov_b32 {d}, s60",
    "i_or3": "v_or3_b32 {d}, {a}, {b}, {c}",
    "i_alignbit": "v_alignbit_b32 {d}, {a}, {b}, 7",
    "i_addco_vcc": "v_add_co_u32 {d}, vcc, {a}, {b}",
    "i_addco_s": "v_add_co_u32 {d}, {sd}, {a}, {b}",
    "i_addc_s": "v_addc_co_u32 {d}, {sd}, {a}, {b}, {sd}",
    "i_mad64": "v_mad_u64_u32 {d2}, s[60:61], {a}, {b}, {c2}",
    "i_mullo": "v_mul_lo_u32 {d}, {a}, {b}",
    "i_mulhi": "v_mul_hi_u32 {d}, {a}, {b}",
    "i_cmp_s": "v_cmp_eq_u32_e64 {sd}, {a}, {b}",
    "i_cndmask": "v_cndmask_b32_e64 {d}, {a}, {b}, s[60:61]",
    "i_fma_f32": "v_fma_f32 {d}, {a}, {b}, {c}",
    "i_readlane": "v_readlane_b32 s{sl}, {a}, 3",
}


BODIES = ["mul", "mulv", "add", "add_nop0", "band", "mov4"] + list(INDEP)
REPS = 16


# dispatch tails after the body (smem >= 2): an indirect jump to the next body, as the
# interpreters do it.  2: s_setpc only; 3: P tail (program-entry s_load + wait, then s_setpc);
# 4: G tail (two v_readlane of the decoded window, s_nop, s_setpc)
_uid = [0]


def tail(smem):
    _uid[0] += 1
    lab = f".Ljt{_uid[0]}"
    jump = ["s_getpc_b64 s[18:19]", f"{lab}_pc:", f"s_add_u32 s18, s18, {lab} - {lab}_pc", "s_addc_u32 s19, s19, 0"]
    if smem == 2:
        return jump + ["s_setpc_b64 s[18:19]", f"{lab}:"]
    if smem == 3:
        return ["s_waitcnt lgkmcnt(0)", "s_mov_b32 s17, s97", "s_load_dwordx2 s[96:97], s[14:15], 0x0"] + jump + \
               ["s_setpc_b64 s[18:19]", f"{lab}:"]
    return ["v_readlane_b32 s16, v8, 3", "v_readlane_b32 s17, v9, 3"] + jump + ["s_nop 1", "s_setpc_b64 s[18:19]", f"{lab}:"]


def kernel(name, smem):
    lines = []
    for _ in range(REPS):
        if smem == 1:   # the P dispatch tail's program-entry load, waited for before the body
            lines += ["s_load_dwordx2 s[96:97], s[14:15], 0x0", "s_waitcnt lgkmcnt(0)"]
        lines += body_lines(name)
        if smem >= 2:
            lines += tail(smem)
    nvalu = sum(1 for ln in body_lines(name) if ln.startswith("v_"))   # the body's own (tails excluded)
    asm = "\\n".join(lines)
    clob = ", ".join(f'"v{i}"' for i in range(8, 128)) + ', "s14", "s15", "s16", "s17", "s18", "s19", "s34", "s35", "s36", "s37", "s38", "s39", ' \
        '"s60", "s61", "s96", "s97", "vcc", "scc"'
    return nvalu, f"""
__global__ __launch_bounds__(256) void k_{name}_{int(smem)}(unsigned* out, const unsigned* prog, int iters) {{
  for (int i = 0; i < iters; i++) {{
    asm volatile("s_mov_b64 s[14:15], %0\\n{asm}" :: "s"(prog) : {clob});
  }}
  if (threadIdx.x == 1u << 30) out[0] = 1;
}}
"""


def main():
    src = ["#include <hip/hip_runtime.h>", "#include <cstdio>",
           "#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, \"%s\\n\", hipGetErrorString(e)); return 1; } } while (0)"]
    runs = []
    for name in BODIES:
        for smem in ((0,) if name in INDEP else (0, 1, 2, 3, 4)):
            nvalu, text = kernel(name, smem)
            src.append(text)
            runs.append((name, smem, nvalu))
    src.append("int main() {\n  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));\n"
               "  unsigned* out; unsigned* prog; CHK(hipMalloc(&out, 64)); CHK(hipMalloc(&prog, 64)); CHK(hipMemset(prog, 0, 64));\n"
               "  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));\n"
               "  const int iters = 2048; printf(\"[\\n\");\n  bool first = true;\n")
    for name, smem, nvalu in runs:
        src.append(f"""  for (int w : {{1, 2, 4, 8}}) {{
    int blocks = p.multiProcessorCount * w;
    for (int rep = 0; rep < 2; rep++) {{
      fprintf(stderr, "{name} {smem} %d %d\\n", w, rep);
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_{name}_{smem}, dim3(blocks), dim3(256), 0, 0, out, prog, iters);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) {{
        double cyc = ms * 1e-3 * 2.4e9;
        double insts = (double)iters * {REPS} * {nvalu} * w;   // VALU wave-instructions per SIMD
        printf("%s{{\\"body\\": \\"{name}\\", \\"smem\\": {smem}, \\"valu_per_body\\": {nvalu}, \\"waves_per_simd\\": %d, \\"cycles_per_valu\\": %.3f}}\\n",
               first ? "" : ",", w, cyc / insts);
        first = false; fflush(stdout);
      }}
    }}
  }}
""")
    src.append("  printf(\"]\\n\");\n  return 0;\n}\n")
    path = os.path.join(HERE, "_issue_probe.hip")
    with open(path, "w") as f:
        f.write("\n".join(src))
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", path, "-o", os.path.join(HERE, "_issue_probe")])


if __name__ == "__main__":
    main()
