#!/bin/bash
# BIN on a subset of the CUs (is it still HBM-bound with fewer CUs?)
set -e
R=${1:-gpurun_out/b12}; mkdir -p $R
for k in 256 192 160 128; do
  SPMV_BIN_CUS=$k timeout -k 10 200 python -u tools/bin_probe.py --repeat 2 >> $R/cus.jsonl 2>>$R/err
  echo "{\"cus\": $k}" >> $R/cus.jsonl
done
