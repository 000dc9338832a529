#!/bin/bash
# Round-1 measurement pass on the GPU box: parity tests, the default bench line, rocprofv3
# kernel-trace stats of the same bench command, and separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ VALU counters).  Every GPU step has its own limit; the chain stops at the
# first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/r01"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 12
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit 13
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.json" 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.json" 2>&1 || exit 15
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d "$OUT/pmc_sq" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_sq.json" 2>&1 || exit 16
echo done
