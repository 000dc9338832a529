#!/bin/bash
# P kernel with fused variable/constant operands: parity, the default bench line (C2, CPU
# baseline), its rocprofv3 kernel trace, and separate PMC passes (HBM traffic, SQ counters).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01l}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 12
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit 13
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.json" 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.json" 2>&1 || exit 15
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d "$OUT/pmc_sq" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_sq.json" 2>&1 || exit 16
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC -d "$OUT/pmc_sq2" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_sq2.json" 2>&1 || exit 17
echo done
