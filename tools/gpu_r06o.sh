#!/bin/bash
# Full GPU suite on the tree, then A/B bench lines (tools/gpu_ab.sh arms).   tools/gpu_r06o.sh TAG ARM...
set -o pipefail
TAG="${1:?tag}"; shift; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 11; }
tail -1 $O/pytest.txt
bash tools/gpu_ab.sh $TAG "" "$@"
