#!/bin/bash
# BIN: parity tests, then configs 2 and 3 per-phase
set -o pipefail
R=gpurun_out/${1:-b28}; mkdir -p $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bin" > $R/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bin_probe.py --repeat 2 > $R/c2.jsonl 2>>$R/err || exit 2
timeout -k 10 300 python -u tools/bin_probe.py --kind powerlaw --rows 5000000 --repeat 2 > $R/c3.jsonl 2>>$R/err || exit 3
