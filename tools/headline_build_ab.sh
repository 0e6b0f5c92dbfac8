#!/bin/bash
# The config-2 headline line on ONE box, alternating the plan builders
# (bench.py --build device / host), each a fresh process
#   bash tools/headline_build_ab.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for i in 1 2 3; do
  for b in device host; do
    timeout -k 10 200 python -u bench.py --only-config --no-cpu --formats auto --build $b > $O/bench_${b}_$i.json 2> $O/bench_${b}_$i.err || exit 1
  done
done
echo done
