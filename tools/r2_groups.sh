#!/bin/bash
# Is the Mul's slow mode about the product buffer footprint written at once?
# G row groups = G Mul launches, each writing 1/G of the buffer; plain
# allocations, interleaved plans in one process
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_groups
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u tools/bin_phase_ab.py --fmt bin --kind uniform --rows 10000000 --placement plain --check \
    --rounds 2 --iters 20 \
    --variants 'g1a:;g4a:bin_groups=4;g1b:;g4b:bin_groups=4;g1c:;g4c:bin_groups=4;g1d:;g4d:bin_groups=4;g16a:bin_groups=16;g16b:bin_groups=16' \
    > $O/c2.jsonl 2> $O/c2.err || exit $?
