#!/bin/bash
# SS stream-kernel ablations at the config-4 shape (probe build; the ablated
# variants compute wrong y -- timing only).
#   bash tools/ss_ablate.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="one:SPMV_LAUNCH_SS=1;a2:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=2;a4:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=4"
LV="$LV;a6:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=6;a8:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=8"
LV="$LV;a14:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=14;nowin:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_WIN=0"
LV="$LV;nostage:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_STAGE=0;tile:SPMV_LAUNCH_SS=0${2:+;$2}"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;ell:fmt=ell}" --launch-variants "$LV" \
    --rounds 4 --iters 20 > $R/ss_ablate.jsonl 2> $R/ss_ablate.err || exit 2
echo done
