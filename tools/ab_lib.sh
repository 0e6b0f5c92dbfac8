#!/bin/bash
# same-box A/B: current package vs a previous build in prevpkg/ (interleaved)
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${CFG:-"--rows 10000000"}
for rep in 1 2 3; do
  for v in cur prev; do
    if [ $v = prev ]; then export TUNE_PKG_ROOT=$R/prevpkg; else unset TUNE_PKG_ROOT; fi
    timeout -k 10 200 python $R/tools/tune.py --fmt ${FMT:-css} $CFG --rounds 3 2>/dev/null | grep '^{' | sed "s/^/{\"v\": \"$v\", \"rep\": $rep, \"r\": /; s/$/}/" || exit 1
  done
done
