#!/bin/bash
# Round check of the tree on a fresh MI355X box (run through gpurun from the repo root):
#   tools/gpu_round.sh TAG [STAGES]
# STAGES (default "tests bench trace pmc"): tests = pytest -m gpu; bench = the default bench line
# (C2 + CPU baseline) and the C3/C4/C5 lines; trace = rocprofv3 kernel traces of C2 and C3;
# pmc = HBM FETCH_SIZE / WRITE_SIZE passes of C2 (one counter block per pass).
# Every GPU step runs under its own time limit; the script stops at the first failing step.
set -o pipefail
TAG="${1:?tag}"; STAGES="${2:-tests bench trace pmc}"
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
has() { [[ " $STAGES " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
  tail -3 "$OUT/pytest_gpu.log"
fi
if has bench; then
  timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 12
  for c in c3 c4 c5; do
    timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit 13
  done
fi
cd /tmp
if has trace; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-dropin > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit 16
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c3" -o run -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/kt_c3_bench.json" 2> "$OUT/kt_c3_bench.err" || exit 17
fi
if has pmc; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/pmc_fetch.json" 2>&1 || exit 18
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/pmc_write.json" 2>&1 || exit 19
fi
echo "done $TAG"
