#!/bin/bash
# HBM traffic of the dominant kernel per config (FETCH_SIZE and WRITE_SIZE, one counter per pass,
# MI355X_MICROARCH.md HBM section) and the keccak-f[1600] VALU count per block (one-block and
# two-block messages in separate runs).  tools/gpu_traffic.sh TAG "c2 c3 c5"
set -o pipefail
TAG="${1:?tag}"; CFGS="${2:-c2 c3 c5}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
summ() { local db; db=$(find "$3" -name '*.db' | head -1); [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null; rm -rf "$3"; }
for c in $CFGS; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr -d /tmp/p_${c}_$ctr -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/${c}_$ctr.log" 2>&1 || exit 11
    summ ${c}_$ctr pmc /tmp/p_${c}_$ctr
  done
done
for nb in 64 200; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU -d /tmp/kec_$nb -o run -- python3 "$R/tools/keccak_probe.py" $nb > "$OUT/kec_$nb.txt" 2>&1 || exit 12
  summ kec_$nb pmc /tmp/kec_$nb
done
echo "done $TAG"
