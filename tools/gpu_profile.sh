#!/bin/bash
# G-kernel per-handler profile on the box: product GPU tests first, then the profile build
# (mythril_amd/prof/libmq.so, built here with QSA_PROF=1) swapped in for tools/g_profile.py.
set -o pipefail
TAG="${1:?tag}"; CFGS="${2:-c3 c5}"; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 2; }
tail -1 $O/pytest.txt
cp mythril_amd/prof/libmq.so mythril_amd/libmq.so || exit 3
for c in $CFGS; do
  timeout -k 10 300 python -u tools/g_profile.py $c > $O/profile_$c.txt 2>&1 || { tail -20 $O/profile_$c.txt; exit 4; }
  head -30 $O/profile_$c.txt
done
