#!/bin/bash
# round 2, re-entry check after the container was re-created: full GPU suite
# and the driver's default bench command
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_s4
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
