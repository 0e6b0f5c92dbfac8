#!/bin/bash
# CSS ablations (pipelined kernel), one process per debug mode (env read at
# plan build): 0 full, 1 no gathers, 2 no LDS atomics, 16 all gathers in a
# 1 MiB window (all L2 hits), 8 default cache policy on the stream.
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-"--rows 10000000"}
for d in 0 1 2 16 8; do
  SPMV_CSS_DEBUG=$d timeout -k 10 300 python $R/tools/tune.py --fmt css $CFG --grid "css_lag=0,-1" --rounds 2 2>/dev/null | grep '^{' | sed "s/^/{\"dbg\": $d, \"r\": /; s/$/}/" || exit 1
done
