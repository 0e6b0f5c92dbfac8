#!/bin/bash
# rank 0 of the 2-GPU job now takes 2 Sum waves: its trace + PMC again
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/profile_round.sh r2f_sim2 --sim-world 2 --formats auto --steps 20 --warmup 5 --trials 3 > gpurun_out/prof_r2f_sim2.log 2>&1 || exit 1
