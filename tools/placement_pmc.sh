#!/bin/bash
# PMC passes over tools/placement_pmc.py (slow vs fast BIN Mul in one process):
# each pass = kernel trace + <= the per-block counter limits, its own run.
#   bash tools/placement_pmc.sh <tag> [placement_pmc.py args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for CTRS in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
            "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
            "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_MISS_sum" \
            "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/pass$i -o run -- \
      python3 $R/tools/placement_pmc.py "$@" > $OUT/pass$i.log 2> $OUT/pass$i.err || exit $?
done
python3 $R/tools/placement_pmc_summary.py $OUT/pass1 $OUT/pass2 $OUT/pass3 $OUT/pass4 > $OUT/summary.jsonl
