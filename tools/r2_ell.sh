#!/bin/bash
# ELL values re-laid out so each 16-byte value load of a wave reads 1 KB
# contiguous: same-box A/B against prevpkg/ at config 4 and config 2, then
# ELL / HYB / JDS parity.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ell_layout
mkdir -p $O
cd $R
FMT=ell CFG="--kind banded --rows 20000000 --per-row 64" timeout -k 10 500 bash tools/ab_lib.sh > $O/ab_c4.jsonl 2> $O/ab.err || exit $?
FMT=ell CFG="--rows 10000000" timeout -k 10 500 bash tools/ab_lib.sh > $O/ab_c2.jsonl 2>> $O/ab.err || exit $?
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ell or hyb or jds or golden" > $O/pytest.log 2>&1 || exit $?
