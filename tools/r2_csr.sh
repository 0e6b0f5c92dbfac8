#!/bin/bash
# CSR vec4: entry pairs a + 2t and a + 2L + 2t per lane (contiguous value
# loads): same-box A/B against prevpkg/ at config 4 and config 2, then CSR
# parity (lanes, golden, full size).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/csr_pairs
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "csr or golden or crs or dropin" > $O/pytest.log 2>&1 || exit $?
FMT=csr CFG="--kind banded --rows 20000000 --per-row 64" timeout -k 10 500 bash tools/ab_lib.sh > $O/ab_c4.jsonl 2> $O/ab.err || exit $?
FMT=csr CFG="--rows 10000000" timeout -k 10 500 bash tools/ab_lib.sh > $O/ab_c2.jsonl 2>> $O/ab.err || exit $?
