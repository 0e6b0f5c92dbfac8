#!/bin/bash
# round 2, GPU step 2: VMM placement in FRESH processes (probe build), then the GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t2
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
P="timeout -k 10 200 python3 -u tools/placement_probe.py --plans 3 --window-mb 4096"
$P --modes vmm:2 > $O/A_vmm2_first.jsonl 2> $O/A.err || exit $?
$P --modes vmm:2@SPMV_VMM_SHUFFLE=1 > $O/B_vmm2_shuffle_first.jsonl 2> $O/B.err || exit $?
$P --modes plain,vmm:2@SPMV_VMM_SHUFFLE=1,vmm:2 > $O/C_plain_then.jsonl 2> $O/C.err || exit $?
$P --modes vmm:2@SPMV_VMM_SHUFFLE=1 > $O/D_vmm2_shuffle_first.jsonl 2> $O/D.err || exit $?
unset SPMV_HIP_LIBRARY
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
