#!/bin/bash
# round-6 iteration: selected GPU tests, the suite, C3/C4/C5 lines, a 1-device --context line and
# the default bench line with its drop-in legs
set -o pipefail
TAG="${1:?tag}"; SEL="${2:-unary or flat or residue or merge or z3 or multi or calldata or bool_columns or c3 or c5}"
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu_iter.sh $TAG "$SEL" "c3 c4 c5" "" || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --context --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_ctx1.json 2> $O/bench_ctx1.err || { tail -20 $O/bench_ctx1.err; exit 5; }
python -c "import json; d=json.loads(open('$O/bench_ctx1.json').read().strip().splitlines()[-1]); print('ctx1', round(d['ms_per_step'],3), d['per_rank'])"
timeout -k 10 900 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 6; }
python - $O/bench_c2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c2", round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4), d["parity_ok"])
for leg in ("dropin_stream", "dropin_stream_z3stub", "dropin"):
    for c in d[leg]:
        print(leg, c["n_queries"], c["n_models"], round(c["ms_per_batch"], 3), {k: round(v, 3) for k, v in c["stage_ms"].items()},
              c.get("z3_asts_translated"), c.get("conjuncts_cached"), c["answers_match_reference_loop"])
for k in ("candidates_off", "candidates_on"):
    z = d["z3_calls_avoided"][k]
    print(k, round(z["ms_per_state"], 3), round(z["fraction_avoided"], 3), {a: round(b, 3) for a, b in z["engine_stage_ms_per_state"].items()})
PY
