#!/bin/bash
# round 2, GPU step 3: GPU suite, default bench, 2-rank self-launch rehearsal, C++ driver on the dist path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t3
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python3 -u bench.py --gpus 2 --rows 150000 --verify --steps 5 --warmup 2 --no-cpu > $O/bench_gloo2.json 2> $O/bench_gloo2.err || exit $?
timeout -k 10 300 ./bin/spmv gen:uniform:10000000:16 --gpus 1 --resident --placement search > $O/spmv_dist1.txt 2> $O/spmv_dist1.err || exit $?
