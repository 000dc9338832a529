#!/usr/bin/env python3
"""Per-kernel roofline fractions of one C4 step (diagnostic).

Inputs: the C4 bench line (bench.py --config c4: alg ops per launch, kernel_ms over the whole step,
keccak_columns, models) and the rocprofv3 kernel trace of the same workload (tools/rocpd_summary.py
JSON; evaluation kernels only, per launch of the traced run = warmup + steps).  The keccak-f[1600] column kernel's algorithmic work is keccak_columns x M x 6 514 ops
(one 136-byte block per 64-byte key ++ slot message; tape_compiler.h kKeccakOpsPerBlock, counted from
the permutation's definition); the
other kernels ("interpreters": G column levels, the flat-conjunction kernel on tapes and Bool
columns, the bit-gather columns, Bool-mask packing) share the rest; each
class's time per step is its traced total / launches.  Peaks: 39.3 T
lane-ops/s (SIMD-16 issue of the carry / compare / multiply classes) for the
interpreters; for keccak-f, whose instructions are mostly two-operand VGPR bitwise ops, also the
measured VGPR-only issue rate (2.31 cycles per wave64 instruction at 4 waves per SIMD: 68.1 T).
usage: c4_breakdown.py BENCH_C4.json KT_C4.json [OUT.json [LAUNCHES=4]]"""
import json
import sys

PEAK = 256 * 64 * 2.4e9
PEAK_VGPR_ONLY = 256 * 4 * 64 * 2.4e9 / 2.31
KECCAK_OPS_PER_BLOCK = 6514   # tape_compiler.h kKeccakOpsPerBlock (round 5: first-principles count)


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    kt = json.load(open(sys.argv[2]))["kernel_trace"]
    cfg, rl = line["config"], line["roofline"]
    M = cfg["models_per_gpu"]
    step_ms = rl["kernel_ms"]
    ops_total = rl["alg_ops_per_launch"]
    ops_kec = cfg["keccak_columns"] * M * KECCAK_OPS_PER_BLOCK
    # evaluation kernels only (the trace also holds the workload generation: model keccaks,
    # copies, row masking at upload); launches = warmup + steps of the traced bench run
    launches = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    groups = {"keccak_column_kernel": 0.0, "qsg_kernel": 0.0, "qs_column_kernel": 0.0, "fca_kernel": 0.0,
              "fc_kernel": 0.0, "cw_column_kernel": 0.0, "qs_pack_bool": 0.0, "qs_init_best": 0.0,
              "qs_finalize_best": 0.0}
    for k in kt:
        g = next((x for x in groups if "mq::" + x in k["kernel"]), None)
        if g is not None:
            groups[g] += k["total_ns"]
    ms = {g: v / launches / 1e6 for g, v in groups.items()}
    traced_ms = sum(ms.values())
    interp_ms = traced_ms - ms["keccak_column_kernel"]
    out = {
        "step_kernel_ms": step_ms, "traced_kernel_ms_per_step": traced_ms, "alg_ops_per_step": ops_total,
        "frac_whole_step": ops_total / (step_ms * 1e-3) / PEAK,
        "kernel_ms_per_step": ms,
        "keccak_columns": {"alg_ops": ops_kec, "ms": ms["keccak_column_kernel"],
                           "achieved_T": ops_kec / (ms["keccak_column_kernel"] * 1e-3) / 1e12,
                           "frac_of_39.3T": ops_kec / (ms["keccak_column_kernel"] * 1e-3) / PEAK,
                           "frac_of_vgpr_only_68.1T": ops_kec / (ms["keccak_column_kernel"] * 1e-3) / PEAK_VGPR_ONLY},
        "interpreters": {"alg_ops": ops_total - ops_kec, "ms": interp_ms,
                         "achieved_T": (ops_total - ops_kec) / (interp_ms * 1e-3) / 1e12,
                         "frac_of_39.3T": (ops_total - ops_kec) / (interp_ms * 1e-3) / PEAK},
        "sources": [sys.argv[1], sys.argv[2]],
    }
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
