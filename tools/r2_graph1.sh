#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/graph1
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "graph or device_pointers" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/graph_latency.py > $O/latency.jsonl 2> $O/latency.err || exit $?
