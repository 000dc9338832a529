#!/bin/bash
# Round-3 evidence on the committed tree, in two parts (each well inside one gpurun call):
#   tools/gpu_evidence3.sh TAG lines   GPU tests, smoke, the default bench line (C2 + CPU baseline +
#                                      drop-in / stream / z3-calls / keccak legs), C3/C4/C5 lines
#                                      with their CPU baselines
#   tools/gpu_evidence3.sh TAG prof    kernel traces of C2-C5 (8 timed steps after 2 warm-up: the
#                                      average is a steady-state one), SQ counters of C3-C5,
#                                      FETCH_SIZE / WRITE_SIZE of the dominant kernels of C2-C5
set -o pipefail
TAG="${1:?tag}"; PART="${2:?part}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); c=d['config']; cb=d.get('cpu_baseline') or {}; print('$2', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'parity', d['parity_ok'], 'value %.3e' % d['value'], 'cpu %.3e' % cb.get('value', 0))"; }
if [ "$PART" = "lines" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 11; }
  tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail "$OUT/smoke.txt"; exit 12; }
  timeout -k 10 600 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail "$OUT/bench_c2.err"; exit 13; }
  line "$OUT/bench_c2.json" c2
  for c in c3 c4 c5; do
    timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 2 --no-dropin > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail "$OUT/bench_$c.err"; exit 14; }
    line "$OUT/bench_$c.json" $c
  done
elif [ "$PART" = "prof" ]; then
  cd /tmp
  summ() { local db; db=$(find "$3" -name '*.db' | head -1); [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null; rm -rf "$3"; }
  for c in c2 c3 c4 c5; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_$c -o run -- python3 "$R/bench.py" --config $c --steps 8 --warmup 2 --no-cpu-baseline --no-dropin > "$OUT/kt_${c}_bench.json" 2> "$OUT/kt_$c.err" || exit 15
    summ kt_$c kt /tmp/kt_$c
  done
  for c in ${SQ_CFGS:-c3 c4 c5}; do
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES -d /tmp/sq_$c -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/sq_$c.log" 2>&1 || exit 16
    summ sq_$c pmc /tmp/sq_$c
  done
  for c in c2 c3 c4 c5; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $ctr -d /tmp/p_${c}_$ctr -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/${c}_$ctr.log" 2>&1 || exit 17
      summ ${c}_$ctr pmc /tmp/p_${c}_$ctr
    done
  done
fi
echo "done $TAG $PART"
