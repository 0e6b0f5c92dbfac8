#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t8
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_dist_gpu.py tests/test_gpu_parity.py -k "dist or dropin" -x -v --timeout 200 --timeout-method thread > $O/pytest_dist.log 2>&1 || exit $?
BENCH_EXTRA="--sim-world 8" bash tools/ab_bench.sh $O/wide_sumwaves.jsonl c2 1 "SPMV_BIN_SUMWAVES=2" "SPMV_BIN_SUMWAVES=3" || exit $?
BENCH_EXTRA="--sim-world 4" bash tools/ab_bench.sh $O/wide_sumwaves.jsonl c2 1 "SPMV_BIN_SUMWAVES=2" "SPMV_BIN_SUMWAVES=3" "SPMV_BIN_SUMWAVES=4" || exit $?
