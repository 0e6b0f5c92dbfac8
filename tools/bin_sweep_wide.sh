#!/bin/bash
# BIN vs CSS on rank 0's share of an N-GPU weak-scaled job (10M rows x N*10M columns)
set -e
R=gpurun_out/b10; mkdir -p $R
for N in 8 4 2; do
  ncols=$((N*10000000))
  timeout -k 10 300 python -u tools/bin_probe.py --rows 10000000 --ncols $ncols --env "SPMV_BIN_PADLOG=3,4;SPMV_BIN_SUMWAVES=2,4" >> $R/probe_$N.jsonl 2>>$R/err
  timeout -k 10 300 python -u tools/tune.py --fmt css --rows 10000000 --ncols $ncols --rounds 2 >> $R/css_$N.jsonl 2>>$R/err
done
