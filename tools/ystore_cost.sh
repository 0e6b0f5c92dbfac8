#!/bin/bash
# y-store cost of DIA and ELL at the config-4 shape (probe build: SPMV_LAUNCH_DEBUG=16
# and SPMV_LAUNCH_ELL_DBG=1 drop the y stores -- wrong y, timing only).
#   bash tools/ystore_cost.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="base:SPMV_LAUNCH_ELL_DBG=0;noy:SPMV_LAUNCH_DEBUG=16,SPMV_LAUNCH_ELL_DBG=1"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt dia --rows 20000000 --per-row 64 \
    --variants "dia:fmt=dia;ell:fmt=ell" --launch-variants "$LV" --placement auto \
    --rounds 4 --iters 20 > $R/ystore.jsonl 2> $R/ystore.err || exit 2
echo done
