#!/bin/bash
# config 3 run path: what slows the Mul that follows a Sum (partial stores?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_long5
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 500 python3 -u tools/bin_phase_ab.py --kind powerlaw --rows 5000000 --placement search --rounds 5 \
  --variants "auto:;plain_st:SPMV_BIN_DEBUG=2048;no_st:SPMV_BIN_DEBUG=4096;exact:bin_long_len=-1" > $O/c3_store.jsonl 2>&1 || exit $?
