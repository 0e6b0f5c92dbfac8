#!/bin/bash
# config-3 SS kernel trace + traffic (fills its roofline.traffic key), and the
# reference-shaped drop-in driver at config 2 (-DOPT_HIP_CRS semantics via
# SPMV_HIP_FORMAT=crs, crs_exact default) with its OptimizeProblem time.
#   bash tools/r5_misc.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
bash tools/profile_round.sh ${T}_c3_ss --config c3 --only-config --formats ss --trials 3 > $R/prof_c3_ss.log 2>&1 || exit 1
SPMV_HIP_FORMAT=crs SPMV_HIP_X_RESIDENT=1 SPMV_HIP_Y_RESIDENT=1 timeout -k 10 300 ./bin/spmv gen:uniform:10000000:16 > $R/spmv_c2_crs.txt 2> $R/spmv_c2_crs.err || exit 2
echo done
