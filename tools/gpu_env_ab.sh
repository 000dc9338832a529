#!/bin/bash
# A/B of an environment knob on one bench config (diagnostic): tools/gpu_env_ab.sh TAG CONFIG VAR V1 V2 ...
set -o pipefail
TAG="${1:?tag}"; CFG="$2"; VAR="$3"; shift 3; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/${CFG}_${v}_$r.json 2> $O/${CFG}_${v}_$r.err || { tail -5 $O/${CFG}_${v}_$r.err; exit 4; }
  python3 -c "
import json
d=json.loads(open('$O/${CFG}_${v}_$r.json').read().strip().splitlines()[-1])
print('$VAR=$v', '$r', round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d.get('parity_ok'))"
done; done
