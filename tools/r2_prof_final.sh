#!/bin/bash
# round-2 final profiles with the current kernels: kernel trace + FETCH/WRITE
# passes for config 2, config 3 and rank 0 of the 8-GPU job
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/profile_round.sh r2f_c2 --formats auto --steps 20 --warmup 5 --trials 3 > gpurun_out/prof_r2f_c2.log 2>&1 || exit 1
bash tools/profile_round.sh r2f_c3 --config c3 --formats auto --steps 20 --warmup 5 --trials 3 > gpurun_out/prof_r2f_c3.log 2>&1 || exit 2
bash tools/profile_round.sh r2f_sim8 --sim-world 8 --formats auto --steps 20 --warmup 5 --trials 3 > gpurun_out/prof_r2f_sim8.log 2>&1 || exit 3
