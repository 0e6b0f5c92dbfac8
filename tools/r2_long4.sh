#!/bin/bash
# config 3 with the placement search for every plan: long-row threshold sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_long4
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 500 python3 -u tools/bin_phase_ab.py --kind powerlaw --rows 5000000 --placement search --rounds 5 \
  --variants "L128:bin_long_len=128;L176:bin_long_len=176;auto:;exact:bin_long_len=-1;L128b:bin_long_len=128;autob:" > $O/c3_sweep.jsonl 2>&1 || exit $?
