#!/bin/bash
# SS stream kernel at the config-4 shape: the cost of the per-tile y stores
# (probe build, SPMV_LAUNCH_SS_SPLIT bits: 64 nontemporal, 128 no row stores,
# 32 XCD-contiguous tiles, 8 no row starts).
#   bash tools/ss_ab5.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="fast:SPMV_LAUNCH_SS=1;full:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=256;noy:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=128"
LV="$LV;fullnt:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=320"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;ell:fmt=ell}" --launch-variants "$LV" \
    --rounds 4 --iters 20 --check > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 2
echo done
