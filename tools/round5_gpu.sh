#!/bin/bash
# Round-5 GPU calls (run on the GPU box from the repo root).
#   bash tools/round5_gpu.sh main <tag>   GPU suite, N = 1 bench line, the
#                                         emulated config-5 rank beside it, and
#                                         the config-2 AUTO kernel trace + PMC
#                                         traffic from the same tree and box
#   bash tools/round5_gpu.sh check <tag>  GPU suite, smoke, N = 1 bench line
#   bash tools/round5_gpu.sh c4ss <tag>   config-4 SS vs ELL: kernel trace,
#                                         traffic and stall counters
set -o pipefail
MODE=$1; T=$2; R=gpurun_out/$T; mkdir -p $R
case $MODE in
main)
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $R/pytest.log 2>&1 || exit 1
  timeout -k 10 600 python -u bench.py > $R/bench.json 2> $R/bench.err || exit 2
  timeout -k 10 300 python -u bench.py --sim-world 8 --no-cpu --formats auto > $R/bench_sim8.json 2> $R/bench_sim8.err || exit 3
  bash tools/profile_round.sh ${T}_c2_auto --only-config --formats auto > $R/prof_c2.log 2>&1 || exit 4
  ;;
check)
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $R/pytest.log 2>&1 || exit 1
  timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $R/smoke.log 2>&1 || exit 2
  timeout -k 10 600 python -u bench.py > $R/bench.json 2> $R/bench.err || exit 3
  ;;
c4ss)
  A="--config c4 --only-config --formats ${FMTS:-ss,ell} --trials 2 --steps 20 --warmup 3"
  # shellcheck disable=SC2086
  bash tools/profile_round.sh ${T}_c4 $A > $R/prof_c4.log 2>&1 || exit 1
  # shellcheck disable=SC2086
  bash tools/pmc_stalls.sh ${T}_c4 $A > $R/stalls_c4.log 2>&1 || exit 2
  ;;
*) echo "mode?"; exit 9 ;;
esac
echo done
