#!/bin/bash
# The driver's scaling runs use bench.py's default format list: rank 0's
# share of the 2-, 4- and 8-GPU jobs (emulated on one GPU, full size) with
# every default format, as the driver would build them
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_sim_full
mkdir -p $O
cd $R
for W in 8 4 2; do
  S0=$SECONDS; timeout -k 10 500 python3 -u bench.py --sim-world $W --steps 20 --warmup 5 --no-cpu \
      > $O/sim$W.json 2> $O/sim$W.err || exit $?
  echo "sim$W wall_s $((SECONDS - S0))" >> $O/wall.txt
done
