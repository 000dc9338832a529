# G-kernel tuning pass: GPU tests, fixed-cost probe, then C3/C5 benches over MQ_G_TPG.
# usage: bash tools/gpu_g_tune.sh TAG "tpg values"
set -o pipefail
TAG=${1:-r02h}; TPGS=${2:-"default 32 64 128"}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 2; }
tail -2 $O/pytest.txt
timeout -k 10 300 python -u tools/g_probe2.py > $O/g_probe2.txt 2>&1 || { tail -20 $O/g_probe2.txt; exit 3; }
for tpg in $TPGS; do
  for c in c3 c5; do
    if [ "$tpg" = default ]; then unset MQ_G_TPG; else export MQ_G_TPG=$tpg; fi
    timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_${c}_tpg$tpg.json 2> $O/bench_${c}_tpg$tpg.err || { tail -20 $O/bench_${c}_tpg$tpg.err; exit 4; }
    python - "$O/bench_${c}_tpg$tpg.json" "$c tpg=$tpg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 4), d.get("parity_ok"))
PY
  done
done
