#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t5
mkdir -p $O
cd $R
bash tools/ab_bench.sh $O/c3_sum_balance.jsonl c3 2 "SPMV_BIN_BPW=1" "SPMV_BIN_BPW=2" "SPMV_BIN_BPW=2 SPMV_BIN_PADLOG=3" "SPMV_BIN_BPW=4" || exit $?
