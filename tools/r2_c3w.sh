#!/bin/bash
# config 3 (run path): Sum waves x padding, search placement; then the drop-in exact-switch test
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_c3w
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dropin" > $O/pytest.log 2>&1 || exit $?
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 500 python3 -u tools/bin_phase_ab.py --kind powerlaw --rows 5000000 --placement search --rounds 4 \
  --variants "w4p16:;w8p16:SPMV_BIN_SUMWAVES=8;w8p8:SPMV_BIN_SUMWAVES=8,SPMV_BIN_PADLOG=3;w4p8:SPMV_BIN_PADLOG=3;w2p16:SPMV_BIN_SUMWAVES=2" > $O/c3_waves.jsonl 2>&1 || exit $?
