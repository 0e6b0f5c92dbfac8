#!/bin/bash
# Sum y write-back with nontemporal stores (probe switch SPMV_BIN_DEBUG=524288):
# in-process A/B at config 2, config 3 and the N = 8 rank shape, y bit-equality.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/nty
mkdir -p $O
cd $R
V='base:;nty:SPMV_BIN_DEBUG=524288;base2:'
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --rows 10000000 --check --rounds 5 > $O/ab_c2.jsonl 2>> $O/ab.err || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --kind powerlaw --rows 5000000 --check --rounds 5 > $O/ab_c3.jsonl 2>> $O/ab.err || exit $?
timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --rows 10000000 --ncols 80000000 --check --rounds 5 > $O/ab_n8.jsonl 2>> $O/ab.err || exit $?
