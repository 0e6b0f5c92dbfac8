#!/bin/bash
# plain placement after a held allocation of H GB, fresh processes (probe build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_t10
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
for H in 0 24 64 128 200 250; do
  timeout -k 10 200 python3 -u tools/placement_probe.py --plans 2 --window-mb 4096 --modes plain --hold-gb $H >> $O/hold.jsonl 2>> $O/hold.err || exit $?
done
