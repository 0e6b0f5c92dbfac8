#!/bin/bash
# BIN long-row run path with the DPP scan: parity subset + config-3 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_long2
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bin_bit_exact or golden and bin or full_size_headline" > $O/pytest_bin.log 2>&1 || exit $?
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --kind powerlaw --rows 5000000 --placement plain \
  --variants "long:;exact:bin_long_len=-1;long_pad8:SPMV_BIN_PADLOG=3;long_1000:bin_long_len=1000" > $O/c3_long_ab.jsonl 2>&1 || exit $?
