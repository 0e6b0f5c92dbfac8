#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in 0 16; do
  SPMV_CSS_DEBUG=$d timeout -k 10 300 python $R/tools/tune.py --fmt css --grid "css_slab_shift=18;css_lag=-1,4" --rounds 3 2>/dev/null | sed "s/^/{\"dbg\": $d, \"r\": /; s/$/}/" || exit 1
done
for d in 0 16; do
  SPMV_CSS_DEBUG=$d timeout -k 10 300 python $R/tools/tune.py --fmt css --ncols 80000000 --grid "css_slab_shift=21;css_lag=-1,4" --rounds 2 2>/dev/null | sed "s/^/{\"dbg\": $d, \"sim8\": 1, \"r\": /; s/$/}/" || exit 1
done
