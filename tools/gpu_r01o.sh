#!/bin/bash
# G kernel with wave-shared 64-model tiles + XCD-interleaved grid: parity, then a tape-group
# size sweep on C3 / C5 (MQ_G_TPG) and a kernel trace of C3.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01o}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
for t in 4 8 16 32 64; do
  MQ_G_TPG=$t timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_tpg$t.json" 2> "$OUT/c3_tpg$t.err" || exit 12
done
for t in 4 16 64; do
  MQ_G_TPG=$t timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c5_tpg$t.json" 2> "$OUT/c5_tpg$t.err" || exit 13
done
echo done
