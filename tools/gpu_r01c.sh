#!/bin/bash
# GPU tests + C2 bench + first C3 bench and its kernel trace.  Each GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r01c"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 12
timeout -k 10 400 python -u bench.py --config c3 --steps 2 --warmup 1 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 13
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c3" -o run -- python3 "$R/bench.py" --config c3 --tapes 200 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/kt_c3.json" 2> "$OUT/kt_c3.err" || exit 14
echo done
