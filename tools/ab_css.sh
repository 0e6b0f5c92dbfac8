#!/bin/bash
# same-box A/B of CSS variants (SPMV_CSS_DEBUG values given as arguments),
# interleaved twice to expose drift
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${CFG:-"--rows 10000000"}
for rep in 1 2; do
  for d in "$@"; do
    SPMV_CSS_DEBUG=$d timeout -k 10 200 python $R/tools/tune.py --fmt css $CFG --rounds 3 2>/dev/null | grep '^{' | sed "s/^/{\"dbg\": $d, \"rep\": $rep, \"r\": /; s/$/}/" || exit 1
  done
done
