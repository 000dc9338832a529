#!/bin/bash
# Iteration on the GPU box: selected GPU tests (-k EXPR), the whole GPU suite, bench lines of CONFIGS
# (c2 with its drop-in / stream / z3-calls / keccak legs when named "c2full"), and the G
# per-handler profile of PROF configs (profile build, tools/build_prof.sh).
#   tools/gpu_iter.sh TAG "K-EXPR" "c2 c3 ..." "c5 ..." [ENV=VAL ...]
set -o pipefail
TAG="${1:?tag}"; KEXPR="$2"; CFGS="$3"; PROFS="$4"; shift 4; for kv in "$@"; do export "$kv"; done
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "$KEXPR" --timeout 300 --timeout-method thread > $O/pytest_sel.txt 2>&1 || { tail -40 $O/pytest_sel.txt; exit 2; }
  tail -1 $O/pytest_sel.txt
fi
if [ "$KEXPR" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 3; }
  tail -1 $O/pytest.txt
fi
for c in $CFGS; do
  if [ "$c" = "c2full" ]; then
    timeout -k 10 600 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 4; }
    f=$O/bench_c2.json
  else
    timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
    f=$O/bench_$c.json
  fi
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print('$c', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],2), 'parity', d['parity_ok'], 'nodes', round(c['avg_tape_nodes'],1), 'value', '%.3e' % d['value'], d.get('kernel_split'))"
done
for c in $PROFS; do
  MQ_LIB=mythril_amd/prof/libmq.so timeout -k 10 300 python -u tools/g_profile.py $c > $O/gprof_$c.txt 2>&1 || { tail -20 $O/gprof_$c.txt; exit 8; }
  head -16 $O/gprof_$c.txt
done
