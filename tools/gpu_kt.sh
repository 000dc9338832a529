#!/bin/bash
# Kernel-trace summaries (rocprofv3 --kernel-trace --stats) of bench configs, summarised on the box.
# usage: tools/gpu_kt.sh TAG "c3 c5 ..."
set -o pipefail
TAG="${1:?tag}"; CFGS="${2:-c3}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in $CFGS; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$c -o run -- python3 "$R/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/kt_${c}_bench.json" 2> "$OUT/kt_$c.err" || exit 14
  db=$(find /tmp/kt_$c -name '*.db' | head -1)
  [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/kt_$c.json" "kt=$db" > /dev/null
  rm -rf /tmp/kt_$c
done
echo "done $TAG"
