#!/bin/bash
# Round-6 G diagnosis on C3 and C5: SQ counter passes (two counter sets), GRBM_GUI_ACTIVE of C2 and C3 (effective clock) and the per-handler G
# profile (profile build in mythril_amd/prof, tools/build_prof.sh).   tools/gpu_r06j.sh TAG
set -o pipefail
TAG="${1:?tag}"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
summ() { local db; db=$(find "$3" -name '*.db' | head -1); [ -n "$db" ] && python3 "$R/tools/rocpd_summary.py" "$OUT/$1.json" "$2=$db" > /dev/null; rm -rf "$3"; }
cd "$R"
for c in c3 c5; do
  MQ_LIB=mythril_amd/prof/libmq.so timeout -k 10 300 python3 -u tools/g_profile.py $c > "$OUT/gprof_$c.txt" 2>&1 || { tail "$OUT/gprof_$c.txt"; exit 3; }
  head -12 "$OUT/gprof_$c.txt"
done
cd /tmp
for c in c3 c5; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES -d /tmp/sq_$c -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/sq_$c.log" 2>&1 || exit 16
  summ sq_$c pmc /tmp/sq_$c
  timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES -d /tmp/sq2_$c -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/sq2_$c.log" 2>&1 || exit 17
  summ sq2_$c pmc /tmp/sq2_$c
done
for c in c2 c3; do
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d /tmp/gr_$c -o run -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/grbm_$c.log" 2>&1 || exit 18
  summ grbm_$c pmc /tmp/gr_$c
done
echo "done $TAG"
