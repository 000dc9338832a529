#!/bin/bash
# GPU parity (incl. hoisting) + C3/C4/C5 bench lines with batch-level hoisting.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r01f"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 12
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || exit 13
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit 14
echo done
