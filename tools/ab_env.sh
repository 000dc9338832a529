#!/bin/bash
# A/B bench lines of library variants x environment knobs (diagnostic):
#   tools/ab_env.sh TAG "CFGS" "VARIANT[:VAR=V[,VAR=V]]" ...   (VARIANT base = mythril_amd/libmq.so,
#   else mythril_amd/exp/libmq_VARIANT.so), two rounds each
set -o pipefail
TAG="${1:?tag}"; CFGS="$2"; shift 2; O=gpurun_out/$TAG; mkdir -p $O
for CFG in $CFGS; do for r in 1 2; do for spec in "$@"; do
  v="${spec%%:*}"; envs=""; [ "$spec" != "$v" ] && envs="${spec#*:}"
  L=$PWD/mythril_amd/libmq.so; [ "$v" = base ] || L=$PWD/mythril_amd/exp/libmq_$v.so
  name=$(echo "${CFG}_${spec}_$r" | tr ':,=' '___')
  env ${envs//,/ } MQ_LIB=$L timeout -k 10 300 python -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 4; }
  python3 -c "
import json
d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1])
print('$CFG', '$spec', '$r', round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d.get('parity_ok'))"
done; done; done
