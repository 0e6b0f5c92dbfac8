#!/bin/bash
# Sum waves per workgroup at configs 3 and 2 with the one-cursor Sum
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_c3waves
mkdir -p $O
cd $R
V='w4:;w8:bin_sum_waves=8;w2:bin_sum_waves=2;w4b:;w8b:bin_sum_waves=8;w2b:bin_sum_waves=2'
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind powerlaw --rows 5000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/c3.jsonl 2> $O/c3.err || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --placement search --check \
    --rounds 2 --iters 20 --variants "$V" > $O/c2.jsonl 2> $O/c2.err || exit $?
