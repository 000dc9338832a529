#!/bin/bash
# New P/G assembly kernels: targeted parity tests first, then the full GPU suite, then C2/C3 benches.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-qsg}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "const_ops or general_asm or asm_fuzz or c2_runs or golden" > "$OUT/pytest_new.log" 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 13
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 14
echo done
