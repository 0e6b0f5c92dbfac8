#!/bin/bash
# x strip staging chosen per plan (xburst when strips >= 4 x workgroups):
# in-process A/B auto / serial / burst at the N = 2, 4, 8 rank shapes and
# config 2; BIN parity with the product build; config 2 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/xstage2
mkdir -p $O
cd $R
V='auto:;serial:SPMV_BIN_DEBUG=131072;burst:SPMV_BIN_DEBUG=262144'
for c in 80000000 40000000 20000000 10000000; do
  SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 400 python3 -u tools/bin_phase_ab.py --variants "$V" --rows 10000000 --ncols $c --check > $O/ab_n$c.jsonl 2>> $O/ab.err || exit $?
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bin or graph or full_size" > $O/pytest.log 2>&1 || exit $?
