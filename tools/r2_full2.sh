#!/bin/bash
# round 2: full GPU suite, default bench (the driver's command), config 3/4 bench lines,
# and a 4-rank gloo rehearsal of config 3 (run path) with verify
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_full2
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 500 python3 -u bench.py --config c4 --formats auto,csr,ell > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 4 --config c3 --rows 300000 --verify --no-cpu --steps 5 --warmup 2 --trials 2 > $O/gloo4_c3.json 2> $O/gloo4_c3.err || exit $?
