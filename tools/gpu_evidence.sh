#!/bin/bash
# Roofline evidence on MI355X: VALU peak harness (int + fp32 controls), the
# keccak-f[1600] instruction mix, and SQ counter passes of the C4 bench.  tools/gpu_evidence.sh TAG
# rocprofv3 databases are summarised to JSON on the box (tools/rocpd_summary.py) and removed.
set -o pipefail
TAG="${1:?tag}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
summ() {  # summ NAME KIND DIR : summarise every .db under DIR into OUT/NAME.json, drop DIR
  local db; db=$(find "$3" -name '*.db' | head -1)
  [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null
  rm -rf "$3"
}
timeout -k 10 120 ./mythril_amd/valu_peak > "$OUT/valu_peak.json" || exit 11
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d /tmp/kec_pmc -o run -- python3 "$R/tools/keccak_probe.py" > "$OUT/kec_probe.txt" 2>&1 || exit 12
summ kec_pmc pmc /tmp/kec_pmc
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d /tmp/c4_pmc -o run -- python3 "$R/bench.py" --config c4 --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/c4_pmc_bench.json" 2>&1 || exit 13
summ c4_pmc pmc /tmp/c4_pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_c4 -o run -- python3 "$R/bench.py" --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/kt_c4_bench.json" 2> "$OUT/kt_c4.err" || exit 14
summ kt_c4 kt /tmp/kt_c4
cd "$R"
timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 15
echo "done $TAG"
