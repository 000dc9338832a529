#!/bin/bash
# One P-kernel iteration on the box: GPU parity tests, C2/C3/C5 bench lines, the C2 handler mix
# with P bigrams, the P dispatch probe.  usage: bash tools/gpu_p_iter.sh TAG
set -o pipefail
TAG="${1:?tag}"; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 2; }
tail -1 $O/pytest.txt
for c in c2 c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
  python - "$O/bench_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 4), d.get("parity_ok"))
PY
done
timeout -k 10 200 python -u tools/qsa_mix.py c2 > $O/mix_c2.txt 2>&1 || exit 5
timeout -k 10 200 python -u tools/p_probe.py > $O/p_probe.txt 2>&1 || exit 6
