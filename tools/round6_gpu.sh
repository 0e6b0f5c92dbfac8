#!/bin/bash
# Round-6 GPU calls (run on the GPU box from the repo root).
#   bash tools/round6_gpu.sh check <tag>   GPU suite, smoke, N = 1 bench line
#   bash tools/round6_gpu.sh suite <tag>   GPU suite only
#   bash tools/round6_gpu.sh sim <tag>     the emulated rank 0 of N = 2, 4, 8
#                                          beside the N = 1 line (one box)
#   bash tools/round6_gpu.sh final <tag>   check + the 8-rank config-5 flow on
#                                          one GPU (gloo), per-rank checks on
set -o pipefail
MODE=$1; T=$2; R=gpurun_out/$T; mkdir -p $R
suite() {
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $R/pytest.log 2>&1
}
case $MODE in
suite)
  suite || exit 1
  ;;
check)
  suite || exit 1
  timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $R/smoke.log 2>&1 || exit 2
  timeout -k 10 600 python -u bench.py > $R/bench.json 2> $R/bench.err || exit 3
  ;;
sim)
  timeout -k 10 300 python -u bench.py --only-config --formats auto --no-cpu > $R/sim1.json 2> $R/sim1.err || exit 1
  for N in 2 4 8; do
    timeout -k 10 300 python -u bench.py --sim-world $N --no-cpu --formats auto > $R/sim$N.json 2> $R/sim$N.err || exit 2
  done
  timeout -k 10 300 python -u bench.py --only-config --formats auto --no-cpu > $R/sim1b.json 2> $R/sim1b.err || exit 3
  ;;
final)
  suite || exit 1
  timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $R/smoke.log 2>&1 || exit 2
  timeout -k 10 600 python -u bench.py > $R/bench.json 2> $R/bench.err || exit 3
  BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 8 --steps 5 --warmup 2 --trials 2 \
      > $R/rehearsal8.json 2> $R/rehearsal8.err || exit 4
  ;;
*) echo "unknown mode $MODE"; exit 9 ;;
esac
