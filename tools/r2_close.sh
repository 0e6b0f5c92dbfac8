#!/bin/bash
# Closing validation after the DIA y-store change: full GPU suite, smoke,
# bench lines for config 2 (default command) and config 4, rocprof of config 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_close
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c4 --formats auto,csr,ell > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
bash tools/profile_round.sh close_c4 --config c4 --formats auto --steps 20 --warmup 5 --trials 3 > $O/prof_c4.log 2>&1 || exit $?
