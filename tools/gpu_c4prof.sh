#!/bin/bash
# C4 iteration: selected GPU tests, the C4 line, its kernel trace and one SQ counter pass.
#   tools/gpu_c4prof.sh TAG "K-EXPR" [CONFIG]
set -o pipefail
TAG="${1:?tag}"; KEXPR="$2"; CFG="${3:-c4}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd "$R"
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$KEXPR" --timeout 300 --timeout-method thread > "$OUT/pytest_sel.txt" 2>&1 || { tail -40 "$OUT/pytest_sel.txt"; exit 2; }
  tail -1 "$OUT/pytest_sel.txt"
fi
timeout -k 10 600 python -u bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > "$OUT/bench_$CFG.json" 2> "$OUT/bench_$CFG.err" || { tail -20 "$OUT/bench_$CFG.err"; exit 4; }
python3 -c "import json; d=json.loads(open('$OUT/bench_$CFG.json').read().strip().splitlines()[-1]); print('$CFG', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'parity', d['parity_ok'], d['kernel_split'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt -o run -- python3 "$R/bench.py" --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/kt_bench.json" 2> "$OUT/kt.err" || exit 5
db=$(find /tmp/kt -name '*.db' | head -1); python3 "$R/tools/rocpd_summary.py" "$OUT/kt_$CFG.json" "kt=$db" > /dev/null; rm -rf /tmp/kt
python3 - "$OUT/kt_$CFG.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ld = d["last_dispatches"]
i = max(k for k, x in enumerate(ld) if x["kernel"] == "mq::qs_init_best")
print(" ".join(f"{x['kernel'].split('mq::')[-1][:14]}:{x['ns']/1e3:.0f}" for x in ld[i:] if "mq::" in x["kernel"]))
PY
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES -d /tmp/sq -o run -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/sq.log" 2>&1 || exit 6
db=$(find /tmp/sq -name '*.db' | head -1); python3 "$R/tools/rocpd_summary.py" "$OUT/sq_$CFG.json" "pmc=$db" > /dev/null; rm -rf /tmp/sq
echo "done $TAG"
