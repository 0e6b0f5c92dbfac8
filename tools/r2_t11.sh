#!/bin/bash
# full GPU suite + 8-rank / 4-rank gloo rehearsals of the driver's multi-GPU bench flow
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t11
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 8 --rows 200000 --verify --no-cpu --steps 5 --warmup 2 --trials 2 > $O/gloo8_c2.json 2> $O/gloo8_c2.err || exit $?
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 4 --config c3 --rows 300000 --verify --no-cpu --steps 5 --warmup 2 --trials 2 > $O/gloo4_c3.json 2> $O/gloo4_c3.err || exit $?
