#!/bin/bash
# Sum over each wave's bins with one batch cursor (the next bin's loads in
# flight during the write-back): BIN parity, then an in-process A/B against one
# bin at a time (probe build, SPMV_BIN_DEBUG=65536)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_sumflat
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "bin or golden or full_size or auto or experiment or dropin" > $O/pytest.log 2>&1 || exit $?
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
V='new:;old:SPMV_BIN_DEBUG=65536;new2:;old2:SPMV_BIN_DEBUG=65536'
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/c2.jsonl 2> $O/c2.err || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind powerlaw --rows 5000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/c3.jsonl 2> $O/c3.err || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --ncols 80000000 --check \
    --placement search --rounds 3 --iters 20 --variants "$V" > $O/w8.jsonl 2> $O/w8.err || exit $?
