#!/bin/bash
# Column-size threshold for the G assembly column path (MQ_G_COL_MIN_NODES): parity, then C3 / C5
# at the default, at 12 and with G columns off.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01q}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
for c in c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_${c}.json" 2> "$OUT/bench_${c}.err" || exit 12
  MQ_G_COL_MIN_NODES=12 timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_${c}_min12.json" 2> "$OUT/bench_${c}_min12.err" || exit 13
  MQ_G_COL_MIN_NODES=1000000000 timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_${c}_off.json" 2> "$OUT/bench_${c}_off.err" || exit 14
done
echo done
