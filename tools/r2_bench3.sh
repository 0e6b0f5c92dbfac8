#!/bin/bash
# bench lines with the default format list (auto, auto@plain, ...): configs 2, 3, 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_bench3
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 500 python3 -u bench.py --config c4 --formats auto,auto@plain,csr,ell > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
