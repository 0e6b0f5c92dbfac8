#!/bin/bash
# SS stream kernel at the config-4 shape: XCD-contiguous tile mapping
# (SPMV_LAUNCH_SS_SPLIT bit 32) vs the dispatch order (probe build).
#   bash tools/ss_ab4.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="fast:SPMV_LAUNCH_SS=1;xcd:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=32;a8:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=8;xa8:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=40"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;s32:ss_sigma=32;ell:fmt=ell}" --launch-variants "$LV" \
    --rounds 4 --iters 20 --check > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 2
echo done
