#!/bin/bash
# first GPU contact: VALU peak microbenchmark, C++ interpreter smoke, asm interpreter smoke,
# GPU parity tests, short bench.  Every GPU step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./mythril_amd/valu_peak > gpurun_out/valu_peak.json 2>&1 || exit 11
MQ_DISABLE_QSA=1 timeout -k 10 180 python -u tools/qsa_smoke.py > gpurun_out/smoke_cpp.log 2>&1 || exit 12
timeout -k 10 120 python -u tools/qsa_smoke.py > gpurun_out/smoke_qsa.log 2>&1 || exit 13
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 14
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 15
echo done
