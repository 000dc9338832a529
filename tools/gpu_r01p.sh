#!/bin/bash
# Hoisted columns on the G assembly kernel (mode 3): parity, then C3 / C4 / C5 lines and a C3
# kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01p}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 12
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || exit 13
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit 14
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c3" -o run -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/kt_c3_bench.json" 2> "$OUT/kt_c3_bench.err" || exit 15
echo done
