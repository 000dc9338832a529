#!/bin/bash
# One iteration on the box: full GPU tests, C3/C5/C2 benches, then the G profile build's
# per-handler profile of C3 (mythril_amd/prof/libmq.so swapped in last).
set -o pipefail
TAG="${1:?tag}"; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 2; }
tail -1 $O/pytest.txt
for c in c3 c5 c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
  python - "$O/bench_$c.json" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 4), d.get("parity_ok"))
PY
done
if [ -f mythril_amd/prof/libmq.so ]; then
  cp mythril_amd/prof/libmq.so mythril_amd/libmq.so || exit 3
  timeout -k 10 300 python -u tools/g_profile.py c3 > $O/profile_c3.txt 2>&1 || { tail -20 $O/profile_c3.txt; exit 5; }
  head -24 $O/profile_c3.txt
fi
