#!/bin/bash
# round 2, GPU step 4: bench lines for configs 3 and 4, and rocprof kernel-trace
# + PMC passes for config 2 and the emulated N = 8 rank shape
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t4
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c4 --formats auto,csr --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
bash tools/profile_round.sh r2_c2 --formats auto --trials 2 || exit $?
bash tools/profile_round.sh r2_sim8 --formats auto --trials 2 --sim-world 8 || exit $?
