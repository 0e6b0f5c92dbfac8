#!/bin/bash
# SS stream kernel: branch-free staged sums vs the branchy direct-store path
# (SPMV_LAUNCH_SS_STAGE=0) at the config-4 shape, plus the SS GPU tests.
#   bash tools/ss_ab3.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v -k "ss or csr5 or golden or device_conversion" --timeout 300 --timeout-method thread > $R/pytest_ss.log 2>&1 || exit 1
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="fast:SPMV_LAUNCH_SS=1;direct:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_STAGE=0;a8:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=8;pf4:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_PF=4;pf1:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_PF=1"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;s32:ss_sigma=32;s16:ss_sigma=16;ell:fmt=ell}" --launch-variants "$LV" \
    --rounds 4 --iters 20 > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 2
echo done
