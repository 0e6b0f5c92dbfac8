#!/bin/bash
# BIN strip-block product layout: SB strips per block (S = plain bin-major)
set -o pipefail
R=gpurun_out/${1:-b22}; mkdir -p $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bin" > $R/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bin_probe.py --env "SPMV_BIN_SB=1000000,8,32,2" --repeat 2 --dbg 16 > $R/c2.jsonl 2>>$R/err || exit 2
