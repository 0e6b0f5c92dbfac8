#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in 0 8; do
  SPMV_CSS_DEBUG=$d timeout -k 10 300 python $R/tools/tune.py --fmt css --grid "css_slab_shift=17,18,19;css_lag=2,4;css_pace=1" --rounds 2 2>/dev/null | sed "s/^/{\"dbg\": $d, \"r\": /; s/$/}/" || exit 1
done
