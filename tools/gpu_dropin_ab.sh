#!/bin/bash
# A/B of an environment knob on the drop-in leg (diagnostic):
#   tools/gpu_dropin_ab.sh TAG VAR "V1 V2 ..." [N:M ...]
set -o pipefail
TAG="${1:?tag}"; VAR="$2"; VALS="$3"; shift 3; O=gpurun_out/$TAG; mkdir -p $O
CELLS="${*:-1:16 1:100 32:100 256:100}"
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python -u tools/dropin_probe.py $CELLS > $O/dropin_$v.jsonl 2> $O/dropin_$v.err || { tail -5 $O/dropin_$v.err; exit 4; }
  python3 -c "
import json
for l in open('$O/dropin_$v.jsonl'):
    d = json.loads(l)
    print('$VAR=$v', d['n_queries'], d['n_models'], round(d['ms_per_batch'], 2), {k: round(x, 2) for k, x in d['stage_ms'].items()},
          round(d['kernel_ms'], 3), round(d['cpu_oracle_eval_ms_1thread'], 2), d['answers_match_reference_loop'])"
done
