#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the CSS kernel (MI355X_MICROARCH.md:
# counters are calibrated only for 16-B/lane streams -- calibrate on a known
# byte count of your own access pattern).  Separate --pmc passes, kernel
# trace only, on config 2: the full kernel and the no-gather ablation
# (SPMV_CSS_DEBUG=1: it streams exactly the entry arrays + writes y).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/calib
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for d in 0 1; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    SPMV_CSS_DEBUG=$d timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d $OUT/dbg${d}_$ctr -o run -- python3 $R/tools/tune.py --fmt css --rounds 1 --iters 5 \
      > $OUT/dbg${d}_$ctr.log 2>&1 || exit $?
  done
done
echo done
