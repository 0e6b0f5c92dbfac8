#!/bin/bash
# The y-store cost of SS and of ELL at the config-4 shape (probe build:
# SPMV_LAUNCH_SS_SPLIT=128 / SPMV_LAUNCH_ELL_DBG=1 drop the y row stores).
#   bash tools/ss_ab6.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="fast:SPMV_LAUNCH_SS=1;noy:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=128,SPMV_LAUNCH_ELL_DBG=1"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;ell:fmt=ell;csr:fmt=csr}" --launch-variants "$LV" \
    --rounds 4 --iters 20 > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 2
echo done
