#!/bin/bash
# CSS piece-size sweep on config 3 (SPMV_CSS_PIECE_DIV, read at plan build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in 2 4 8 16 32 64; do
  SPMV_CSS_PIECE_DIV=$d timeout -k 10 200 python $R/tools/tune.py --fmt css --kind powerlaw --rows 5000000 --max-len 10000 --rounds 3 2>/dev/null | grep '^{' | sed "s/^/{\"div\": $d, \"r\": /; s/$/}/" || exit 1
done
