#!/bin/bash
# kernel trace + FETCH/WRITE passes for rank 0 of the 2- and 4-GPU jobs
# (emulated), so the driver's scaling lines carry roofline.traffic
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/profile_round.sh r2_sim2 --sim-world 2 --formats auto --steps 20 --warmup 5 --trials 3 > gpurun_out/prof_r2_sim2.log 2>&1 || exit 1
bash tools/profile_round.sh r2_sim4 --sim-world 4 --formats auto --steps 20 --warmup 5 --trials 3 > gpurun_out/prof_r2_sim4.log 2>&1 || exit 2
