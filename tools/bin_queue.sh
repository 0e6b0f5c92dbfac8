#!/bin/bash
# BIN Sum queue: bin order (sorted by size or natural) x bins per wave
set -o pipefail
R=gpurun_out/${1:-b29}; mkdir -p $R
timeout -k 10 300 python -u tools/bin_probe.py --env "SPMV_BIN_SORT=0,1" > $R/c2.jsonl 2>>$R/err || exit 2
timeout -k 10 300 python -u tools/bin_probe.py --kind powerlaw --rows 5000000 --env "SPMV_BIN_SORT=0,1;SPMV_BIN_MINPERWAVE=1,2" > $R/c3.jsonl 2>>$R/err || exit 3
