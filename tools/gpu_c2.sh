#!/bin/bash
# GPU parity tests, then the default C2 bench line and its rocprofv3 kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-c2}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 12
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit 13
echo done
