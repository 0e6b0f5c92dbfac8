#!/bin/bash
# bench lines after the unclamped Sum: config 2 (driver command), config 3,
# rank 0 of the 2/4/8-GPU jobs (emulated, default formats)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_bench4
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
for W in 8 4 2; do
  timeout -k 10 500 python3 -u bench.py --sim-world $W --steps 20 --warmup 5 --no-cpu > $O/sim$W.json 2> $O/sim$W.err || exit $?
done
