#!/bin/bash
# SS at the config-4 shape: DPP vs ds_bpermute wave scans at the tile end,
# with and without workgroup caps (probe build).
#   bash tools/ss_ab7.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
LV="bperm:SPMV_LAUNCH_SS_SCAN=0;dpp:SPMV_LAUNCH_SS_SCAN=1"
LV="$LV;dpp_c2:SPMV_LAUNCH_SS_SCAN=1,SPMV_LAUNCH_SS_LDS_KB=48;dpp_c3:SPMV_LAUNCH_SS_SCAN=1,SPMV_LAUNCH_SS_LDS_KB=28"
LV="$LV;dpp_pf4:SPMV_LAUNCH_SS_SCAN=1,SPMV_LAUNCH_SS_PF=4;dpp_pf4_c2:SPMV_LAUNCH_SS_SCAN=1,SPMV_LAUNCH_SS_PF=4,SPMV_LAUNCH_SS_LDS_KB=48"
timeout -k 10 900 python -u tools/bin_phase_ab.py --kind banded --fmt ss --rows 20000000 --per-row 64 \
    --variants "${VARIANTS:-s20:ss_sigma=20;s64:ss_sigma=64;ell:fmt=ell}" --launch-variants "$LV" --placement auto \
    --rounds 4 --iters 20 --check > $R/ss_ab.jsonl 2> $R/ss_ab.err || exit 2
echo done
