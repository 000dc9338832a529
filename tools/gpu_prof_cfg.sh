#!/bin/bash
# Kernel trace and FETCH_SIZE / WRITE_SIZE passes of one config (the gpu_evidence3.sh prof steps
# for a single config): tools/gpu_prof_cfg.sh TAG CONFIG
set -o pipefail
TAG="${1:?tag}"; c="${2:?config}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
summ() { local db; db=$(find "$3" -name '*.db' | head -1); [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null; rm -rf "$3"; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_$c -o run -- python3 "$R/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/kt_${c}_bench.json" 2> "$OUT/kt_$c.err" || exit 15
summ kt_$c kt /tmp/kt_$c
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d /tmp/p_${c}_$ctr -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/${c}_$ctr.log" 2>&1 || exit 17
  summ ${c}_$ctr pmc /tmp/p_${c}_$ctr
done
echo "done $TAG $c"
