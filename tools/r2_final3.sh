#!/bin/bash
# after the 2-wave threshold change: BIN parity, then bench lines for
# config 3 and rank 0 of the 2/4/8-GPU jobs (config 2 keeps 4 waves)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_final3
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "bin or golden or full_size or auto or experiment or dropin" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
for W in 2 4 8; do
  timeout -k 10 500 python3 -u bench.py --sim-world $W --steps 20 --warmup 5 --no-cpu > $O/sim$W.json 2> $O/sim$W.err || exit $?
done
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
