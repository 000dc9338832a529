#!/bin/bash
# A/B timing of library variants on the C2 bench (diagnostic): tools/gpu_ab.sh TAG CONFIG VARIANT...
# (VARIANT "base" = mythril_amd/libmq.so, else mythril_amd/exp/libmq_VARIANT.so), two rounds each
set -o pipefail
TAG="${1:?tag}"; CFG="$2"; shift 2; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/mythril_amd/libmq.so; else L=$PWD/mythril_amd/exp/libmq_$v.so; fi
  MQ_LIB=$L timeout -k 10 300 python -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/${CFG}_${v}_$r.json 2> $O/${CFG}_${v}_$r.err || { tail -5 $O/${CFG}_${v}_$r.err; exit 4; }
  python3 -c "
import json,sys
d=json.loads(open('$O/${CFG}_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', '$r', round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d.get('parity_ok'))"
done; done
