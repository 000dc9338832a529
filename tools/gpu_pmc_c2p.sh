#!/bin/bash
# SQ counters of the P kernel on C2 (the headline): VALU issue, SALU dispatch, instruction fetch.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-pmc_c2p}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
B="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/p1" -o run -- python3 $B > "$OUT/p1.json" 2>&1 || exit 10
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC -d "$OUT/p2" -o run -- python3 $B > "$OUT/p2.json" 2>&1 || exit 11
echo done
