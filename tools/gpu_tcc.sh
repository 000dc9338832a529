#!/bin/bash
# L2 (TCC) hit / miss counters of one config's launches (one --pmc pass): tools/gpu_tcc.sh TAG CONFIG
set -o pipefail
TAG="${1:?tag}"; c="${2:?config}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
summ() { local db; db=$(find "$3" -name '*.db' | head -1); [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null; rm -rf "$3"; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d /tmp/tcc_$c -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/tcc_$c.log" 2>&1 || exit 17
summ tcc_$c pmc /tmp/tcc_$c
echo "done $TAG $c"
