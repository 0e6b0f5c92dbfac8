#!/bin/bash
# SS tile epilogue A/B at the config-4 shape (probe build) + the SS GPU tests
# on the product library.
#   bash tools/ss_ab2.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v -k "ss or csr5 or golden or device_conversion" --timeout 300 --timeout-method thread > $R/pytest_ss.log 2>&1 || exit 1
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="one:SPMV_LAUNCH_SS=1;split:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=1;tile:SPMV_LAUNCH_SS=0"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;s32:ss_sigma=32;s16:ss_sigma=16;ell:fmt=ell}" --launch-variants "$LV" \
    --rounds 4 --iters 20 --check > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 2
echo done
