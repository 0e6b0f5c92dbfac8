#!/bin/bash
# CSS structure vs the bare gather probe on config 2, same box, no pacing:
# 0 full, 16 all-L2-hit gathers, 18 all-hit + no LDS atomics, 3 no gathers
# and no LDS (stream only); then bin/gather_probe (e8: gathers + CSS-shaped stream)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in 0 16 18 3; do
  SPMV_CSS_DEBUG=$d timeout -k 10 300 python $R/tools/tune.py --fmt css --grid "css_lag=-1" --rounds 3 2>/dev/null | grep '^{' | sed "s/^/{\"dbg\": $d, \"r\": /; s/$/}/" || exit 1
done
timeout -k 10 300 $R/bin/gather_probe > $R/gpurun_out/gp_floor.json || exit 1
