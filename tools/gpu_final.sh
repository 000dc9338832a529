#!/bin/bash
# Round evidence on the committed tree: GPU tests, the default bench line (C2 + CPU baseline +
# drop-in + keccak legs), C3/C4/C5 lines, kernel traces of C2 and C3, C2 SQ counters and HBM
# traffic.  tools/gpu_final.sh TAG
set -o pipefail
TAG="${1:?tag}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 11
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 500 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit 12
timeout -k 10 500 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || exit 13
for c in c3 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit 14
done
cd /tmp
summ() { local db; db=$(find "$3" -name '*.db' | head -1); [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null; rm -rf "$3"; }
for c in c2 c3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_$c -o run -- python3 "$R/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/kt_${c}_bench.json" 2> "$OUT/kt_$c.err" || exit 15
  summ kt_$c kt /tmp/kt_$c
done
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES -d /tmp/sq_c2 -o run -- python3 "$R/bench.py" --config c2 --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/sq_c2.log" 2>&1 || exit 16
summ sq_c2 pmc /tmp/sq_c2
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d /tmp/p_$ctr -o run -- python3 "$R/bench.py" --config c2 --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/c2_$ctr.log" 2>&1 || exit 17
  summ c2_$ctr pmc /tmp/p_$ctr
done
echo "done $TAG"
