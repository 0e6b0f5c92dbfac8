#!/bin/bash
# One GPU call: full GPU tests, bench lines for configs 2-4, rocprof of config 2.
set -o pipefail
R=gpurun_out/${1:-r2}; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $R/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $R/bench_c2.json 2> $R/bench_c2.err || exit 2
timeout -k 10 300 python -u bench.py --config c3 --formats auto,css,ss,hyb,csr > $R/bench_c3.json 2> $R/bench_c3.err || exit 3
timeout -k 10 300 python -u bench.py --config c4 --formats auto,csr,ell,bin > $R/bench_c4.json 2> $R/bench_c4.err || exit 4
bash tools/profile_round.sh ${1:-r2}_c2 --formats auto > $R/prof.log 2>&1 || exit 5
