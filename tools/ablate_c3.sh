#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in 0 1 3; do
  SPMV_CSS_DEBUG=$d timeout -k 10 300 python $R/tools/tune.py --fmt css --kind powerlaw --rows 5000000 --grid "css_slab_shift=16,17,18,19;css_lag=-1,4" --rounds 2 2>/dev/null | sed "s/^/{\"dbg\": $d, \"r\": /; s/$/}/" || exit 1
done
timeout -k 10 300 python $R/tools/tune.py --fmt ss --kind powerlaw --rows 5000000 --grid "ss_sigma=8,16,24,32" --rounds 2 2>/dev/null | sed "s/^/{\"dbg\": 99, \"r\": /; s/$/}/"
