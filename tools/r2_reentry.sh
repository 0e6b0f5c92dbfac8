#!/bin/bash
# Re-entry validation with the libraries rebuilt in this container: full GPU
# suite, smoke, config-2 and config-3 bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_reentry
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
