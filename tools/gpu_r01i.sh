#!/bin/bash
# Fused variable-operand handlers (P kernel) + 2-move Comba columns: parity first, then the C2
# line; then counters of the G kernel on a reduced C3 (where its time goes) and a C4 trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01i}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 12
cd /tmp
B="$R/bench.py --config c3 --tapes 200 --models 250000 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$OUT/p1" -o run -- python3 $B > "$OUT/p1.json" 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA -d "$OUT/p2" -o run -- python3 $B > "$OUT/p2.json" 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC -d "$OUT/p3" -o run -- python3 $B > "$OUT/p3.json" 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c4" -o run -- python3 "$R/bench.py" --config c4 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/kt_c4.json" 2> "$OUT/kt_c4.err" || exit 16
echo done
