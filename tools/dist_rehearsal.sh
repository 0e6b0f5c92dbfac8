#!/bin/bash
# 2-rank rehearsal of bench.py's multi-GPU flow on ONE GPU (gloo backend).
set -o pipefail
mkdir -p gpurun_out
BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --rows 2000000 \
   --formats css,csr > gpurun_out/dist_rehearsal.json 2> gpurun_out/dist_rehearsal.err
