#!/bin/bash
# Issue / stall / memory-pipe counters over bench.py, one rocprofv3 --pmc pass
# per counter group (within gfx950's per-block slots: 8 SQ, 4 TCC, 4 TCP,
# 2 TA, 2 GRBM), each its own run under a hard time limit.
#   bash tools/pmc_stalls.sh <tag> [bench args...]
# Output: gpurun_out/stalls_<tag>/pass<i>/run_counter_collection.csv, then
# tools/pmc_stalls_summary.py -> gpurun_out/stalls_<tag>/summary.json
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stalls_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES SQ_WAIT_INST_LDS" \
            "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/pass$i -o run -- \
      python3 $R/bench.py --no-cpu "$@" > $OUT/pass$i.json 2> $OUT/pass$i.err || exit $?
done
python3 $R/tools/pmc_stalls_summary.py $OUT > $OUT/summary.json
