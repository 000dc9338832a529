#!/bin/bash
# PMC passes (one counter group per run) of a short C3 bench: where the G assembly interpreter
# (qsg_kernel) and the column kernel spend their time.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-pmc_c3g}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
B="$R/bench.py --config c3 --tapes 500 --models 500000 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 $B > "$OUT/kt.json" 2>&1 || exit 10
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$OUT/p1" -o run -- python3 $B > "$OUT/p1.json" 2>&1 || exit 11
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA -d "$OUT/p2" -o run -- python3 $B > "$OUT/p2.json" 2>&1 || exit 12
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_ACTIVE_INST_MISC -d "$OUT/p3" -o run -- python3 $B > "$OUT/p3.json" 2>&1 || exit 13
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/p4" -o run -- python3 $B > "$OUT/p4.json" 2>&1 || exit 14
echo done
