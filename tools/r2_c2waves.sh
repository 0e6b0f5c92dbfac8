#!/bin/bash
# config 2: 4 vs 2 Sum waves (16-entry padding), four plans each, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_c2waves
mkdir -p $O
cd $R
V='a4:;a2:bin_sum_waves=2;b4:;b2:bin_sum_waves=2;c4:;c2:bin_sum_waves=2;d4:;d2:bin_sum_waves=2'
timeout -k 10 500 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --placement search --check \
    --rounds 3 --iters 20 --variants "$V" > $O/c2.jsonl 2> $O/c2.err || exit $?
