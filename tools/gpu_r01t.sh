#!/bin/bash
# C3 HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and SQ counters of the current G kernel, then a
# tape-group size check (MQ_G_TPG 8 / 32) on C3 and C5.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r01t}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
B="$R/bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/p_fetch" -o run -- python3 $B > "$OUT/p_fetch.json" 2>&1 || exit 10
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/p_write" -o run -- python3 $B > "$OUT/p_write.json" 2>&1 || exit 11
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d "$OUT/p_sq" -o run -- python3 $B > "$OUT/p_sq.json" 2>&1 || exit 12
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/p_tcc" -o run -- python3 $B > "$OUT/p_tcc.json" 2>&1 || exit 13
cd "$R"
for t in 8 32; do
  for c in c3 c5; do
    MQ_G_TPG=$t timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/${c}_tpg$t.json" 2> "$OUT/${c}_tpg$t.err" || exit 14
  done
done
echo done
