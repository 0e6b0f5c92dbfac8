#!/bin/bash
# Config-2 BIN placement spread (VERDICT r5 "next" #2): 8 same-size AUTO plans
# in one process (tools/placement_pmc.py), profiled under one --pmc group per
# pass (kernel trace on, counters of bin_mul / bin_sum dispatches only, JSON
# output = one value per counter instance), then tools/spread_summary.py.
#   bash tools/spread_pmc.sh <tag> [placement_pmc.py args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/spread_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for CTRS in "TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_RDREQ_LEVEL GRBM_GUI_ACTIVE" \
            "TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_LEVEL" \
            "TCC_TAG_STALL TCC_EA0_WRREQ_STALL TCC_BUBBLE TCC_EA0_RDREQ_DRAM" \
            "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTRS --kernel-include-regex 'bin_(mul|sum)' \
      --output-format json -d $OUT/pass$i -o run -- \
      python3 $R/tools/placement_pmc.py "$@" > $OUT/pass$i.log 2> $OUT/pass$i.err || exit $?
done
python3 $R/tools/spread_summary.py $OUT/pass1 $OUT/pass2 $OUT/pass3 $OUT/pass4 > $OUT/summary.jsonl
