#!/bin/bash
# BIN long-row run path: GPU parity of the BIN tests, then config-3 A/B (run path on / off)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_long
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bin or golden" > $O/pytest_bin.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --kind powerlaw --rows 5000000 --placement plain --check \
  --variants "long:;exact:bin_long_len=-1" > $O/c3_long_ab.jsonl 2>&1 || exit $?
