#!/bin/bash
# One rocprofv3 counter pass per argument group over a bench config, summarised on the box:
#   tools/gpu_pmc.sh TAG CONFIG "CTR CTR ..." ["CTR ..."]...   (<= 8 SQ counters per group)
set -o pipefail
TAG="${1:?tag}"; CFG="${2:?config}"; shift 2
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp -d /tmp/pmc$i -o run -- python3 "$R/bench.py" --config "$CFG" --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/pass$i.json" 2>&1 || exit $((10+i))
  db=$(find /tmp/pmc$i -name '*.db' | head -1)
  python3 "$R/tools/rocpd_summary.py" "$OUT/${CFG}_pmc$i.json" "pmc=$db" > /dev/null || exit 30
  rm -rf /tmp/pmc$i
done
echo "done $TAG"
