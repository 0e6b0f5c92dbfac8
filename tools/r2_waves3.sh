#!/bin/bash
# padding at 2 Sum waves on rank 0 of the 4-GPU job; config 3 repeated
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_waves3
mkdir -p $O
cd $R
V='auto:;w2p16:bin_sum_waves=2,bin_pad=16;autob:;w2p16b:bin_sum_waves=2,bin_pad=16;autoc:;w2p16c:bin_sum_waves=2,bin_pad=16'
timeout -k 10 400 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --ncols 40000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/w4.jsonl 2> $O/w4.err || exit $?
V='w4:;w2p16:bin_sum_waves=2,bin_pad=16;w4b:;w2p16b:bin_sum_waves=2,bin_pad=16;w4c:;w2p16c:bin_sum_waves=2,bin_pad=16'
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind powerlaw --rows 5000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/c3.jsonl 2> $O/c3.err || exit $?
