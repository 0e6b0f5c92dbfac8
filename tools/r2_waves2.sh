#!/bin/bash
# 2 vs 4 Sum waves (and the padding) with the one-cursor Sum: configs 2, 3 and
# rank 0 of the 2-GPU job; every variant built twice (placement noise)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_waves2
mkdir -p $O
cd $R
V='w4:;w2p8:bin_sum_waves=2,bin_pad=8;w2p16:bin_sum_waves=2,bin_pad=16;w4b:;w2p8b:bin_sum_waves=2,bin_pad=8;w2p16b:bin_sum_waves=2,bin_pad=16'
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind powerlaw --rows 5000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/c3.jsonl 2> $O/c3.err || exit $?
timeout -k 10 400 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/c2.jsonl 2> $O/c2.err || exit $?
timeout -k 10 400 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --ncols 20000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/w2.jsonl 2> $O/w2.err || exit $?
