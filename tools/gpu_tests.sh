#!/bin/bash
# GPU parity tests only (one process, per-test timeout), results under gpurun_out/$1.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-t}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
echo done
