#!/bin/bash
# N = 8 rank shape (10M x 80M): product store policy x padding
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_w8
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 600 python3 -u tools/bin_phase_ab.py --ncols 80000000 --placement search --rounds 4 \
  --variants "base:;plain_st:SPMV_BIN_DEBUG=1;pad16:SPMV_BIN_PADLOG=4;pad16_plain:SPMV_BIN_PADLOG=4,SPMV_BIN_DEBUG=1" > $O/w8_store.jsonl 2>&1 || exit $?
