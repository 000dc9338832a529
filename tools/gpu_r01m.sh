#!/bin/bash
# Two-word P program entries: parity first, then the C2 line and C3 (both interpreters).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01m}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 12
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 13
echo done
