#!/bin/bash
# same box: committed build (prevpkg/) vs current build with the contiguous
# (SPMV_CSS_LAYOUT=0) and interleaved (=1) CSS list layouts, interleaved reps
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${CFG:-"--rows 10000000"}
for rep in 1 2; do
  TUNE_PKG_ROOT=$R/prevpkg timeout -k 10 200 python $R/tools/tune.py --fmt css $CFG --rounds 3 2>/dev/null | grep '^{' | sed "s/^/{\"v\": \"prev\", \"rep\": $rep, \"r\": /; s/$/}/" || exit 1
  for L in 0 1; do
    SPMV_CSS_LAYOUT=$L timeout -k 10 200 python $R/tools/tune.py --fmt css $CFG --rounds 3 2>/dev/null | grep '^{' | sed "s/^/{\"v\": \"layout$L\", \"rep\": $rep, \"r\": /; s/$/}/" || exit 1
  done
done
