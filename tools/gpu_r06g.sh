#!/bin/bash
# GPU suite, drop-in loops, default bench line
set -o pipefail
TAG="${1:?tag}"; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 3; }
tail -1 $O/pytest.txt
timeout -k 10 200 python -u tools/stream_loop.py 1 16 300 > $O/loop_1_16.json 2>&1 || exit 4
timeout -k 10 200 python -u tools/stream_loop.py 16 100 100 > $O/loop_16_100.json 2>&1 || exit 5
cat $O/loop_1_16.json $O/loop_16_100.json
timeout -k 10 900 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 6; }
python - $O/bench_c2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c2", round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4), d["parity_ok"])
for leg in ("dropin_stream", "dropin_stream_z3stub", "dropin"):
    for c in d[leg]:
        print(leg, c["n_queries"], c["n_models"], round(c["ms_per_batch"], 3), {k: round(v, 3) for k, v in c["stage_ms"].items()}, c["answers_match_reference_loop"])
for k in ("candidates_off", "candidates_on"):
    z = d["z3_calls_avoided"][k]
    print(k, round(z["ms_per_state"], 3), round(z["fraction_avoided"], 3), {a: round(b, 3) for a, b in z["engine_stage_ms_per_state"].items()})
PY
