#!/bin/bash
# Round-2 closing validation after the re-entry changes (graphs, small-plan
# bins, AUTO threshold, wide-plan x staging): full GPU suite, smoke, bench
# lines (c2, c3, emulated rank 0 of the 8-GPU job), kernel trace + PMC of
# c2 and the rank-0 shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_final5
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 400 python3 -u bench.py --sim-world 8 --no-cpu > $O/bench_sim8.json 2> $O/bench_sim8.err || exit $?
bash tools/profile_round.sh r2f5_c2 --formats auto --steps 20 --warmup 5 --trials 3 > $O/prof_c2.log 2>&1 || exit $?
bash tools/profile_round.sh r2f5_sim8 --sim-world 8 --formats auto --steps 20 --warmup 5 --trials 3 > $O/prof_sim8.log 2>&1 || exit $?
