#!/bin/bash
# round-2 closing measurements with the current kernels: bench lines (config 2
# driver command, config 3, config 4, emulated rank 0 of 2/4/8 GPUs) and the
# rocprofv3 trace + PMC passes behind roofline.traffic
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_final2
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 500 python3 -u bench.py --config c4 --formats auto,auto@plain,csr,ell > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
for W in 8 4 2; do
  timeout -k 10 500 python3 -u bench.py --sim-world $W --steps 20 --warmup 5 --no-cpu > $O/sim$W.json 2> $O/sim$W.err || exit $?
done
bash tools/r2_prof_final.sh || exit $?
