#!/bin/bash
# Nontemporal y stores as the Sum default: full GPU suite, smoke, bench lines
# (config 2, config 3, emulated rank 0 of the 8-GPU job), rocprof kernel trace
# + FETCH/WRITE passes of config 2 and the rank-0 shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/nty_final
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 400 python3 -u bench.py --sim-world 8 > $O/bench_sim8.json 2> $O/bench_sim8.err || exit $?
bash tools/profile_round.sh nty_c2 --formats auto --steps 20 --warmup 5 --trials 3 > $O/prof_c2.log 2>&1 || exit $?
bash tools/profile_round.sh nty_sim8 --sim-world 8 --formats auto --steps 20 --warmup 5 --trials 3 > $O/prof_sim8.log 2>&1 || exit $?
