#!/bin/bash
# Kernel-trace + PMC passes over bench.py (run on the GPU box from the repo root).
# Usage: tools/profile_round.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --no-cpu "$@" > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 $R/bench.py --no-cpu "$@" > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- \
    python3 $R/bench.py --no-cpu "$@" > $OUT/bench_write.json 2> $OUT/bench_write.err || exit $?
echo done
