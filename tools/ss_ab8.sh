#!/bin/bash
# SS at the config-4 shape: sigma x prefetch depth (probe build), for AUTO's
# long-row sigma.
#   bash tools/ss_ab8.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="pf2:SPMV_LAUNCH_SS_PF=2;pf4:SPMV_LAUNCH_SS_PF=4;pf1:SPMV_LAUNCH_SS_PF=1"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;s32:ss_sigma=32;s48:ss_sigma=48;s64:ss_sigma=64;ell:fmt=ell}" --launch-variants "$LV" --placement auto \
    --rounds 4 --iters 20 > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 2
echo done
