#!/bin/bash
# config 3 with 2 Sum waves: the LDS atomics' share of the Sum (ablation, wrong y)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_c3_noat
mkdir -p $O
cd $R
export SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
V='base:;noat:SPMV_BIN_DEBUG=8;base2:;noat2:SPMV_BIN_DEBUG=8'
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --fmt bin --kind powerlaw --rows 5000000 --placement search \
    --rounds 3 --iters 20 --variants "$V" > $O/c3.jsonl 2> $O/c3.err || exit $?
