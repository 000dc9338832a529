#!/bin/bash
# GPU tests (optionally a -k selection first), then bench lines for the given configs.
# tools/gpu_tests.sh TAG "KSEL" "CFGS"
set -o pipefail
TAG="${1:?tag}"; KSEL="$2"; CFGS="$3"; O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$KSEL" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "$KSEL" --timeout 120 --timeout-method thread > $O/pytest_sel.txt 2>&1 || { tail -40 $O/pytest_sel.txt; exit 2; }
  tail -1 $O/pytest_sel.txt
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 3; }
tail -1 $O/pytest.txt
for c in $CFGS; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
  python - "$O/bench_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 4), d.get("parity_ok"))
PY
done
