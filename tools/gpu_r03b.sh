#!/bin/bash
# round-3 check: new GPU tests, full suite, default bench (C2 + legs), one-process context rehearsal, C5 line
set -o pipefail
TAG="${1:?tag}"; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "c5_deep or z3_terms or candidates" --timeout 300 --timeout-method thread > $O/pytest_sel.txt 2>&1 || { tail -40 $O/pytest_sel.txt; exit 2; }
tail -1 $O/pytest_sel.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 3; }
tail -1 $O/pytest.txt
timeout -k 10 600 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 4; }
python -c "import json,sys; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('c2', round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d['parity_ok']); print(json.dumps(d['z3_calls_avoided']))"
timeout -k 10 300 python -u bench.py --context --no-cpu-baseline --no-dropin > $O/bench_c2_ctx.json 2> $O/bench_c2_ctx.err || { tail -20 $O/bench_c2_ctx.err; exit 5; }
python -c "import json; d=json.loads(open('$O/bench_c2_ctx.json').read().strip().splitlines()[-1]); print('ctx', d['n_gpus'], round(d['ms_per_step'],2), d['config']['parallelism'], d['config']['rccl_in_library'], d['parity_ok'])"
timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 6; }
python -c "import json; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); c=d['config']; print('c5', round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d['parity_ok'], c['avg_tape_nodes'], c['avg_tape_nodes_unhoisted'], d['value'])"
# diagnostics: handler mix and per-handler profile (profile build through MQ_LIB)
for c in c3 c5; do
  timeout -k 10 300 python -u tools/qsa_mix.py $c > $O/mix_$c.txt 2>&1 || { tail -20 $O/mix_$c.txt; exit 7; }
  MQ_LIB=mythril_amd/prof/libmq.so timeout -k 10 300 python -u tools/g_profile.py $c > $O/gprof_$c.txt 2>&1 || { tail -20 $O/gprof_$c.txt; exit 8; }
  head -25 $O/gprof_$c.txt
done
