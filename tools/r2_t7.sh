#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t7
mkdir -p $O
cd $R
# CSR rows per lane group at configs 4 (banded, 16 lanes), 2 (uniform, 4 lanes), 3 (adaptive: unchanged)
FMT=csr bash tools/ab_bench.sh $O/csr_r.jsonl c4 2 "SPMV_CSR_R=1" "SPMV_CSR_R=2" "SPMV_CSR_R=4" || exit $?
FMT=csr bash tools/ab_bench.sh $O/csr_r.jsonl c2 1 "SPMV_CSR_R=1" "SPMV_CSR_R=2" "SPMV_CSR_R=4" || exit $?
