#!/usr/bin/env python3
"""Rebuild profiles/pmc_traffic.json (bench.py roofline.traffic) from the FETCH_SIZE / WRITE_SIZE
summaries one `tools/gpu_evidence3.sh TAG prof` run left in profiles/TAG/ (tools/rocpd_summary.py
JSON: per kernel and grid, the average per dispatch; FETCH_SIZE x2 gfx950 correction applied there).

Traffic per launch = the sum over the evaluation kernels (the ones a bench step launches: qsa /
qsg / HIP C++ interpreters, keccak columns, Bool packing, first-hit init/finalize) of their average
bytes per dispatch x dispatches per launch.  The PMC runs are `bench.py --steps 1 --warmup 1`:
2 launches, plus one 256-thread probe dispatch per assembly kernel at context creation (grid 256,
excluded).  The same whole-step scope as the line's `achieved` (all kernels of the step).
usage: update_traffic.py TAG [c2 c3 c4 c5]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EVAL = ("mq::qsa_kernel", "mq::qsg_kernel", "mq::qs_first_hit_kernel", "mq::qs_column_kernel", "mq::keccak_column_kernel",
        "mq::fca_kernel", "mq::fc_kernel", "mq::cw_column_kernel",
        "mq::qs_pack_bool", "mq::qs_init_best", "mq::qs_finalize_best")
SHAPES = {"c2": (10000, 100000, 2), "c3": (1000, 1000000, 3), "c4": (200, 1000000, 4), "c5": (256, 1250000, 5)}
LAUNCHES = 2


def per_launch(path, field):
    pmc = json.load(open(path))["pmc"]
    total, parts = 0.0, []
    for k, v in pmc.items():
        if not any(e in k for e in EVAL) or k.endswith(" grid=256"):
            continue
        b = v.get(field, 0.0) * v["dispatches"] / LAUNCHES
        total += b
        parts.append((k, b))
    return total, parts


def main():
    tag = sys.argv[1]
    cfgs = sys.argv[2:] or list(SHAPES)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    table = json.load(open(path)) if os.path.exists(path) else {}
    for c in cfgs:
        d = os.path.join(ROOT, "profiles", tag)
        f, fp = per_launch(os.path.join(d, f"{c}_FETCH_SIZE.json"), "fetch_bytes_corrected")
        w, wp = per_launch(os.path.join(d, f"{c}_WRITE_SIZE.json"), "write_bytes")
        n, m, s = SHAPES[c]
        table[f"{c}:n{n}:m{m}:s{s}"] = {
            "fetch_bytes": int(f), "write_bytes": int(w),
            "source": f"profiles/{tag}/{c}_FETCH_SIZE.json + {c}_WRITE_SIZE.json: rocprofv3 --pmc FETCH_SIZE and --pmc "
                      f"WRITE_SIZE in separate runs of `python3 bench.py --config {c} --steps 1 --warmup 1 --no-cpu-baseline "
                      f"--no-dropin` on MI355X (tools/gpu_evidence3.sh {tag} prof); the evaluation kernels of one launch "
                      f"(tools/update_traffic.py: average per dispatch x dispatches per launch, {len(fp)} kernel shapes); "
                      f"FETCH_SIZE x2 gfx950 wide-read correction"}
        print(c, "fetch %.3e write %.3e" % (f, w))
    with open(path, "w") as fh:
        json.dump(table, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main()
