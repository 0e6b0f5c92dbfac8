#!/bin/bash
# A/B: x strip staged with 8 (LONG: 4) loads in flight vs one at a time
# (probe switch SPMV_BIN_DEBUG=131072), in-process, at config 2, config 3,
# the N = 8 rank shape and 1 M rows; then BIN parity with the product build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/xstage
mkdir -p $O
cd $R
V='new:;old:SPMV_BIN_DEBUG=131072'
SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --rows 1000000 --check > $O/ab_1m.jsonl 2> $O/ab.err || exit $?
SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --rows 10000000 --check > $O/ab_c2.jsonl 2>> $O/ab.err || exit $?
SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --kind powerlaw --rows 5000000 --check > $O/ab_c3.jsonl 2>> $O/ab.err || exit $?
SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 400 python3 -u tools/bin_phase_ab.py --variants "$V" --rows 10000000 --ncols 80000000 --check > $O/ab_w8.jsonl 2>> $O/ab.err || exit $?
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bin or graph" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/graph_latency.py --sizes 10000,100000,1000000,3000000 --formats bin > $O/latency.jsonl 2> $O/latency.err || exit $?
