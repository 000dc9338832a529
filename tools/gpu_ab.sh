#!/bin/bash
# A/B bench lines: each ARM is "NAME:CONFIGS:ENV=VAL,ENV=VAL" (CONFIGS comma-separated; ENV may
# name MQ_LIB=mythril_amd/exp/X/libmq.so, a generator variant from tools/build_variant.sh).
# Optional selected GPU tests first (-k EXPR; "" skips).   tools/gpu_ab.sh TAG "K-EXPR" ARM [ARM ...]
set -o pipefail
TAG="${1:?tag}"; KEXPR="$2"; shift 2; O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$KEXPR" --timeout 300 --timeout-method thread > $O/pytest_sel.txt 2>&1 || { tail -40 $O/pytest_sel.txt; exit 2; }
  tail -1 $O/pytest_sel.txt
fi
for arm in "$@"; do
  name="${arm%%:*}"; rest="${arm#*:}"; cfgs="${rest%%:*}"; envs="${rest#*:}"
  [ "$envs" = "$rest" ] && envs=""
  for c in ${cfgs//,/ }; do
    f=$O/bench_${name}_$c.json
    env ${envs//,/ } timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $f 2> $O/bench_${name}_$c.err || { tail -20 $O/bench_${name}_$c.err; exit 4; }
    python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$name', '$c', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],3), 'parity', d['parity_ok'])"
  done
done
echo "done $TAG"
