#!/bin/bash
# drop-in A/B: fresh and fork-stream cells under engine knobs (MQ_CONJ_TAPES, MQ_SPLIT_TAPES)
set -o pipefail
TAG="${1:?tag}"; shift; O=gpurun_out/$TAG; mkdir -p $O
CELLS="${CELLS:-1:16 1:100 32:100 256:100 s1:16 s1:100 s16:100 s128:100}"
summ() {
python -c "
import json,sys
for ln in open('$1'):
    c = json.loads(ln)
    n = c.get('n_parents')
    tag = ('s%d' % n) if n is not None else ''
    print(tag, c['n_queries'], c['n_models'], round(c['ms_per_batch'], 3), {k: round(v, 3) for k, v in c['stage_ms'].items()}, 'k', round(c['kernel_ms'], 3), 'cpu1', round(c['cpu_oracle_eval_ms_1thread'], 3), c.get('conjuncts_evaluated', ''), c['answers_match_reference_loop']); print('   lib', {k: round(v, 3) for k, v in c.get('library_phase_ms', {}).items() if v > 0.005})"
}
i=0
for V in "$@"; do
  i=$((i+1))
  echo "== $V"
  env $V timeout -k 10 300 python -u tools/dropin_probe.py $CELLS > $O/v$i.jsonl 2> $O/v$i.err || { tail -20 $O/v$i.err; exit 2; }
  summ $O/v$i.jsonl
done
