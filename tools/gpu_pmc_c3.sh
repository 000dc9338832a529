#!/bin/bash
# PMC passes (one counter group per run) of a short C3 bench: where the HIP C++ interpreter spends time.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmc_c3"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
B="$R/bench.py --config c3 --tapes 100 --models 250000 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d "$OUT/p1" -o run -- python3 $B > "$OUT/p1.json" 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_WR -d "$OUT/p2" -o run -- python3 $B > "$OUT/p2.json" 2>&1 || exit 12
echo done
