#!/bin/bash
# Same-box A/B of the SS launch kernels at the config-4 shape (probe build):
# every plan timed under every launch variant in interleaved rounds.
#   bash tools/ss_ab_c4.sh <tag> [extra launch variants]
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="k0:SPMV_LAUNCH_SS=0;k1:SPMV_LAUNCH_SS=1"
LV="$LV;r2:SPMV_LAUNCH_SS=2,SPMV_LAUNCH_SS_TPW=2;r4:SPMV_LAUNCH_SS=2,SPMV_LAUNCH_SS_TPW=4"
LV="$LV;r8:SPMV_LAUNCH_SS=2,SPMV_LAUNCH_SS_TPW=8;r4p4:SPMV_LAUNCH_SS=2,SPMV_LAUNCH_SS_TPW=4,SPMV_LAUNCH_SS_PF=4"
LV="$LV;r8l40:SPMV_LAUNCH_SS=2,SPMV_LAUNCH_SS_TPW=8,SPMV_LAUNCH_SS_LDS_KB=40"
LV="$LV;r16l40:SPMV_LAUNCH_SS=2,SPMV_LAUNCH_SS_TPW=16,SPMV_LAUNCH_SS_LDS_KB=40"
LV="$LV;r8l28:SPMV_LAUNCH_SS=2,SPMV_LAUNCH_SS_TPW=8,SPMV_LAUNCH_SS_LDS_KB=28${2:+;$2}"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;s32:ss_sigma=32;ell:fmt=ell}" --launch-variants "$LV" \
    --rounds 3 --iters 20 --check > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 1
echo done
