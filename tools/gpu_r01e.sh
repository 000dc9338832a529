#!/bin/bash
# GPU parity tests, per-op probe and a C3 bench line for the LDS-stack interpreter.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r01e"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u tools/probe_ops.py > "$OUT/probe_ops.json" 2>&1 || exit 12
timeout -k 10 400 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 13
echo done
