#!/bin/bash
# host-CSR build routing (spmv_options_t::build): its GPU tests and the bench
# line's plan build times.
#   bash tools/r5_build_route.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -k "routing or device_conversion or full_size or dropin or c5" --timeout 600 --timeout-method thread > $R/pytest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $R/bench.json 2> $R/bench.err || exit 2
echo done
