#!/bin/bash
# config 2: Sum-ordered vs Mul-ordered products (same process, interleaved),
# beside the default line on the same box
#   bash tools/order_ab.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python -u bench.py --only-config --no-cpu --formats auto > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python -u tools/bin_phase_ab.py --rows 10000000 --placement auto --check --rounds 5 \
    --variants "sum:bin_product_order=1;mul:bin_product_order=2;sum2:bin_product_order=1;mul2:bin_product_order=2" \
    > $O/order_ab.jsonl 2> $O/order_ab.err || exit 2
echo done
