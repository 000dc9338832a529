#!/bin/bash
# round-3 iteration: selected GPU tests (-k EXPR), the whole GPU suite, bench lines of CONFIGS
# (c2 with its legs when named "c2full"), and the G per-handler profile of PROF configs.
#   tools/gpu_iter3.sh TAG "K-EXPR" "c2 c5 ..." "c5 ..."
set -o pipefail
TAG="${1:?tag}"; KEXPR="$2"; CFGS="$3"; PROFS="$4"; O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "$KEXPR" --timeout 300 --timeout-method thread > $O/pytest_sel.txt 2>&1 || { tail -40 $O/pytest_sel.txt; exit 2; }
  tail -1 $O/pytest_sel.txt
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 3; }
tail -1 $O/pytest.txt
for c in $CFGS; do
  if [ "$c" = "c2full" ]; then
    timeout -k 10 600 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 4; }
    f=$O/bench_c2.json
  else
    timeout -k 10 600 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
    f=$O/bench_$c.json
  fi
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print('$c', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],2), 'parity', d['parity_ok'], 'nodes', c['avg_tape_nodes'], c['avg_tape_nodes_unhoisted'], 'value', '%.3e' % d['value'])"
done
for c in $PROFS; do
  MQ_LIB=mythril_amd/prof/libmq.so timeout -k 10 300 python -u tools/g_profile.py $c > $O/gprof_$c.txt 2>&1 || { tail -20 $O/gprof_$c.txt; exit 8; }
  head -16 $O/gprof_$c.txt
done
if [ "$5" = "dropin" ]; then
  timeout -k 10 300 python -u tools/dropin_probe.py 1:16 1:100 32:100 256:100 > $O/dropin.jsonl 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 9; }
  python -c "
import json
for ln in open('$O/dropin.jsonl'):
    c = json.loads(ln)
    print(c['n_queries'], c['n_models'], round(c['ms_per_batch'], 3), {k: round(v, 3) for k, v in c['stage_ms'].items()}, 'kernel', round(c['kernel_ms'], 3), 'cpu1', round(c['cpu_oracle_eval_ms_1thread'], 3), c['answers_match_reference_loop'])"
  timeout -k 10 300 rocprofv3 --hip-trace --stats -d $O/ht -o ht -- python3 tools/dropin_probe.py 1:16 32:100 > $O/dropin_ht.log 2>&1 || { tail -20 $O/dropin_ht.log; exit 10; }
  f=$(find $O/ht -name '*hip_stats.csv' | head -1); [ -n "$f" ] && head -25 "$f"
fi
