#!/bin/bash
# Drop-in cells (tools/dropin_probe.py) under environment knobs: tools/gpu_dropin.sh TAG "CELLS" "VAR=a ..." ...
set -o pipefail
TAG="${1:?tag}"; CELLS="$2"; shift 2; O=gpurun_out/$TAG; mkdir -p $O
i=0
for envs in "" "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python -u tools/dropin_probe.py $CELLS > $O/dropin_$i.jsonl 2> $O/dropin_$i.err || { tail -20 $O/dropin_$i.err; exit 9; }
  python - "$O/dropin_$i.jsonl" "[$envs]" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    c = json.loads(ln)
    lib = {k: round(v, 3) for k, v in c["library_phase_ms"].items() if v > 0.01}
    print(sys.argv[2], "stream" if "n_parents" in c else "fresh", c["n_queries"], c["n_models"], round(c["ms_per_batch"], 3),
          {k: round(v, 3) for k, v in c["stage_ms"].items()}, lib, "cpu1", round(c["cpu_oracle_eval_ms_1thread"], 3), c["answers_match_reference_loop"])
PY
done
