#!/bin/bash
# 8 ranks on the one GPU (gloo) through the self-launched bench, 2 M rows per
# rank (16 M x 16 M), y verified against the oracle over the whole matrix
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_gloo8
mkdir -p $O
cd $R
BENCH_DIST_BACKEND=gloo timeout -k 10 900 python3 -u bench.py --gpus 8 --rows 2000000 --verify --no-cpu --steps 5 --warmup 2 --trials 2 \
    > $O/gloo8_c2.json 2> $O/gloo8_c2.err || exit $?
BENCH_DIST_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 4 --config c3 --rows 1000000 --verify --no-cpu --steps 5 --warmup 2 --trials 2 \
    > $O/gloo4_c3.json 2> $O/gloo4_c3.err || exit $?
