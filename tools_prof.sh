#!/bin/bash
# profiling recipe used for profiles/ (run on the GPU box from the repo root)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/bench.py --tapes 2000 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/kt_bench.json
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc1 -o run -- python3 $R/bench.py --tapes 500 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc1_bench.json
