#!/bin/bash
# AUTO crossover (CSS / BIN / CSR) after the small-BIN bin rule
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/autocross
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u tools/auto_cross.py > $O/cross.jsonl 2> $O/cross.err || exit $?
