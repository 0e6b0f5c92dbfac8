#!/bin/bash
# config 3: long-row threshold sweep (run path) in one process
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_long3
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 400 python3 -u tools/bin_phase_ab.py --kind powerlaw --rows 5000000 --placement search --rounds 5 \
  --variants "L96:bin_long_len=96;L128:bin_long_len=128;L176:bin_long_len=176;auto:;L320:bin_long_len=320;exact:bin_long_len=-1;auto_w8:SPMV_BIN_SUMWAVES=8" > $O/c3_sweep.jsonl 2>&1 || exit $?
