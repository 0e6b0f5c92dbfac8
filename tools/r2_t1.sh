#!/bin/bash
# round 2, GPU step 1: placement experiment (probe build), then the GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t1
mkdir -p $O
cd $R
SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so timeout -k 10 420 python3 -u tools/placement_probe.py \
    --modes plain@SPMV_BIN_MUL_PERM=0,plain@SPMV_BIN_MUL_PERM=1,vmm:0@SPMV_BIN_MUL_PERM=1,vmm:2@SPMV_BIN_MUL_PERM=1,search@SPMV_BIN_MUL_PERM=1,search@SPMV_BIN_MUL_PERM=0 --plans 3 --window-mb 1024 > $O/placement.jsonl 2> $O/placement.err || exit $?
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
