#!/bin/bash
# VMM placement with strided handles, FRESH processes (probe build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t9
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
P="timeout -k 10 200 python3 -u tools/placement_probe.py --plans 3 --window-mb 4096"
$P --modes plain > $O/A_plain.jsonl 2> $O/A.err || exit $?
$P --modes vmm:2@SPMV_VMM_STRIDE=2 > $O/B_stride2.jsonl 2> $O/B.err || exit $?
$P --modes vmm:2@SPMV_VMM_STRIDE=4 > $O/C_stride4.jsonl 2> $O/C.err || exit $?
$P --modes vmm:64@SPMV_VMM_STRIDE=2 > $O/D_64mb_stride2.jsonl 2> $O/D.err || exit $?
$P --modes vmm:2@SPMV_VMM_STRIDE=2,plain,vmm:2@SPMV_VMM_STRIDE=2 > $O/E_mixed.jsonl 2> $O/E.err || exit $?
