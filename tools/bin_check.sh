#!/bin/bash
# BIN: parity tests, then the strip width on config 2 and the N = 8 rank shape
set -o pipefail
R=gpurun_out/${1:-b20}; mkdir -p $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bin" > $R/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bin_probe.py --grid "bin_strip_cols=16384,20480" --repeat 2 > $R/c2.jsonl 2>>$R/err || exit 2
timeout -k 10 300 python -u tools/bin_probe.py --ncols 80000000 --grid "bin_strip_cols=16384,20480" > $R/n8.jsonl 2>>$R/err || exit 3
