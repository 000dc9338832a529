#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks on device 0, gloo for the reduce
# (the product path is RCCL; this checks sharding, global first hits and max-over-ranks timing).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/dist"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$R"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --dist-backend gloo --device 0 --steps 3 --warmup 1 > "$OUT/c2_n2.json" 2> "$OUT/c2_n2.err" || exit 11
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --dist-backend gloo --device 0 --config c3 --tapes 100 --models 200000 --steps 1 --warmup 1 > "$OUT/c3_n2.json" 2> "$OUT/c3_n2.err" || exit 12
echo done
