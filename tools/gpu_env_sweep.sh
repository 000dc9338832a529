#!/bin/bash
# Bench configs under different environment settings.
# usage: tools/gpu_env_sweep.sh TAG "c3 c5" "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
TAG="${1:?tag}"; CFGS="$2"; shift 2
O=gpurun_out/$TAG; mkdir -p $O
i=0
for envs in "$@"; do
  i=$((i+1))
  for c in $CFGS; do
    env $envs timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_${c}_$i.json 2> $O/bench_${c}_$i.err || { tail -20 $O/bench_${c}_$i.err; exit 4; }
    python - "$O/bench_${c}_$i.json" "$c [$envs]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 4), d.get("parity_ok"))
PY
  done
done
