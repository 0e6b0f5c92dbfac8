#!/bin/bash
# SS with AUTO sigma 32 for long rows: its GPU tests, then the config-4 SS
# kernel trace + traffic (roofline.traffic key of ss_stream_kernel<32>).
#   bash tools/r5_ss32.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -k "ss or csr5 or golden or device_conversion or routing" --timeout 600 --timeout-method thread > $R/pytest.log 2>&1 || exit 1
bash tools/profile_round.sh ${T}_c4_ss --config c4 --only-config --formats ss,ell --trials 2 --steps 20 --warmup 3 > $R/prof.log 2>&1 || exit 2
echo done
