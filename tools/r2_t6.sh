#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t6
mkdir -p $O
cd $R
bash tools/ab_bench.sh $O/c3_waves_pad.jsonl c3 2 "SPMV_BIN_SUMWAVES=4" "SPMV_BIN_SUMWAVES=2" "SPMV_BIN_PADLOG=5" "SPMV_BIN_SUMWAVES=2 SPMV_BIN_PADLOG=5" || exit $?
