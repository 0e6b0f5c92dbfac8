#!/bin/bash
# What the Sum's per-bin start/end costs: ablation without LDS zeroing and y
# write-back (SPMV_BIN_DEBUG=32768, probe build, wrong y) at configs 2, 3 and
# the 8-GPU rank shape
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_sum_tail
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
V='base:;notail:SPMV_BIN_DEBUG=32768'
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --placement search \
    --rounds 3 --iters 20 --variants "$V" > $O/c2.jsonl 2> $O/c2.err || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind powerlaw --rows 5000000 --placement search \
    --rounds 3 --iters 20 --variants "$V" > $O/c3.jsonl 2> $O/c3.err || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --ncols 80000000 \
    --placement search --rounds 3 --iters 20 --variants "$V" > $O/w8.jsonl 2> $O/w8.err || exit $?
