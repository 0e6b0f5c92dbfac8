#!/bin/bash
# DIA y written as one 16-byte nontemporal store per row pair: same-box A/B
# against the previous build (prevpkg/) at config 4, then DIA parity.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/dia_y
mkdir -p $O
cd $R
FMT=dia CFG="--kind banded --rows 20000000 --per-row 64 --placement search" timeout -k 10 700 bash tools/ab_lib.sh > $O/ab_c4.jsonl 2> $O/ab.err || exit $?
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "dia or golden or full_size_c4" > $O/pytest.log 2>&1 || exit $?
