#!/bin/bash
# DIA at the config-4 shape: resident workgroups walking the blocks
# (dia_run_kernel, probe SPMV_LAUNCH_DEBUG=32) vs one workgroup per block.
#   bash tools/dia_run_ab.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="base:SPMV_LAUNCH_DEBUG=0;run1:SPMV_LAUNCH_DEBUG=32;run2:SPMV_LAUNCH_DEBUG=32,SPMV_LAUNCH_DIA_RUN_WG=2;noy:SPMV_LAUNCH_DEBUG=16"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt dia --rows 20000000 --per-row 64 \
    --variants "dia1:fmt=dia;dia2:fmt=dia" --launch-variants "$LV" --placement auto --check \
    --rounds 4 --iters 20 > $R/dia_run.jsonl 2> $R/dia_run.err || exit 2
echo done
