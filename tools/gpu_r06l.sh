#!/bin/bash
# Full GPU suite, the default bench line (C2 + drop-in legs), one SQ counter pass of C2.
#   tools/gpu_r06l.sh TAG
set -o pipefail
TAG="${1:?tag}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
summ() { local db; db=$(find "$3" -name '*.db' | head -1); [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null; rm -rf "$3"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 11; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 600 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail "$OUT/bench_c2.err"; exit 13; }
python3 - "$OUT/bench_c2.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c2", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4), "parity", d["parity_ok"])
for leg in ("dropin", "dropin_stream"):
    print(leg, [(x["n_queries"], x["n_models"], round(x["ms_per_batch"], 3)) for x in d.get(leg, [])])
z = d.get("z3_calls_avoided", {})
for k in ("candidates_off", "candidates_on"):
    if k in z:
        print(k, round(z[k]["ms_per_state"], 3), "serialize", round(z[k]["engine_stage_ms_per_state"]["serialize"], 3))
PY
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES -d /tmp/sq_c2 -o run -- python3 "$R/bench.py" --config c2 --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/sq_c2.log" 2>&1 || exit 16
summ sq_c2 pmc /tmp/sq_c2
echo "done $TAG"
