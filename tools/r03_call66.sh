#!/bin/bash
# 2-rank rehearsal of the driver's N > 1 bench at the new default B = 2048: both ranks on the box's one GPU, so the
# exchange runs over gloo (RCCL needs a GPU per rank); every other part is the N > 1 path
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c66
mkdir -p $O
YAVO_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 > $O/gloo2_b2048.log 2>&1
