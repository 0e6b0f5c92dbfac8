#!/bin/bash
# CSS ablations on c2, one process per debug mode (env read at plan build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in 0 1 2 3 4; do
  SPMV_CSS_DEBUG=$d timeout -k 10 300 python $R/tools/tune.py --fmt css --grid "css_slab_shift=17,19;css_lag=-1,2;css_pace=2" --rounds 2 | sed "s/^/{\"dbg\": $d, \"r\": /; s/$/}/" || exit 1
done
