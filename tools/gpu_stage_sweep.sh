set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "staged or general_asm or asm_const" -x -q --timeout 120 --timeout-method thread > $O/staged.txt 2>&1 || { tail -30 $O/staged.txt; exit 1; }
tail -2 $O/staged.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 2; }
tail -2 $O/pytest.txt
for kb in 0 32 64; do
  for c in c3 c5; do
    MQ_G_STAGE_KB=$kb timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_${c}_kb$kb.json 2> $O/bench_${c}_kb$kb.err || exit 3
    python -c "import json,sys; d=json.load(open('$O/bench_${c}_kb$kb.json')); print('$c kb=$kb', round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d['parity_ok'])"
  done
done
