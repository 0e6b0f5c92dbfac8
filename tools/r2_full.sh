#!/bin/bash
# round 2: full GPU suite, then the bench lines of configs 2 and 3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_full
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 --formats auto,csr,css > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
