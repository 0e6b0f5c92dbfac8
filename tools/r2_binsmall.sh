#!/bin/bash
# More Sum bins for small BIN plans: BIN parity tests, small-size latency.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/binsmall
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "bin or graph or golden or integer" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/graph_latency.py --sizes 10000,100000,1000000,3000000 --formats csr,bin > $O/latency.jsonl 2> $O/latency.err || exit $?
