#!/bin/bash
# CSR rows per lane group (csr_ilp_kernel) on configs 4 and 2, y bit-equal across variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_csr_ilp
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 400 python3 -u tools/bin_phase_ab.py --fmt csr --kind banded --rows 20000000 --rounds 4 --check \
  --variants "r1:;r2:SPMV_CSR_ILP=2;r4:SPMV_CSR_ILP=4" > $O/c4.jsonl 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/bin_phase_ab.py --fmt csr --rows 10000000 --rounds 4 --check \
  --variants "r1:;r2:SPMV_CSR_ILP=2;r4:SPMV_CSR_ILP=4" > $O/c2.jsonl 2>&1 || exit $?
