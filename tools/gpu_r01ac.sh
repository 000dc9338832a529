#!/bin/bash
# Round-end check of the committed state on a fresh box: parity, the default bench line (C2 with
# CPU baseline), its rocprofv3 kernel trace + HBM PMC passes, and the C3/C4/C5 lines (C3 traced).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01ac}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 12
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 13
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit 14
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || exit 15
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit 16
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.json" 2>&1 || exit 17
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.json" 2>&1 || exit 18
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c3" -o run -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/kt_c3_bench.json" 2> "$OUT/kt_c3_bench.err" || exit 19
echo done
