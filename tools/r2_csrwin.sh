#!/bin/bash
# CSR with the LDS x window: parity tests, then an in-process A/B against the
# global-gather kernel at config 4 (20 M rows, 64 diagonals)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_csrwin
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "x_window or csr_lanes or golden or device_conversion or csr_64bit or c4_banded" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 -u tools/bin_phase_ab.py --fmt csr --kind banded --rows 20000000 --placement plain --check \
    --rounds 4 --iters 20 \
    --variants "win16:;glob16:x_window=-1;win8:csr_lanes=8;glob8:csr_lanes=8,x_window=-1;win32:csr_lanes=32" \
    > $O/c4_ab.jsonl 2> $O/c4_ab.err || exit $?
timeout -k 10 600 python3 -u tools/bin_phase_ab.py --fmt ell --kind banded --rows 20000000 --placement plain --check \
    --rounds 4 --iters 20 --variants 'win:;glob:x_window=-1' > $O/c4_ell_ab.jsonl 2> $O/c4_ell_ab.err || exit $?
