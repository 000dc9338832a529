#!/bin/bash
# quick C2 bench only (no CPU baseline), for A/B of the assembly interpreter
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-c2q}"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -k "asm or c2 or golden" > "$OUT/pytest.log" 2>&1 || exit 11
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 12
echo done
