#!/bin/bash
# Verdict round 1 #3 "done when": 10 BIN plans built in one process, per
# placement mode (search: the bench's choice; plain: the library default).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/place10
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 500 python3 -u tools/placement_probe.py --modes search --plans 10 > $O/search10.jsonl 2> $O/search10.err || exit $?
timeout -k 10 300 python3 -u tools/placement_probe.py --modes plain --plans 10 > $O/plain10.jsonl 2> $O/plain10.err || exit $?
