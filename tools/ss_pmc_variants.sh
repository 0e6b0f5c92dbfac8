#!/bin/bash
# One rocprofv3 --pmc pass per SS launch variant at the config-4 shape (probe
# build): write-path and stall counters of the stream kernel with and without
# its per-tile y row stores.
#   bash tools/ss_pmc_variants.sh <tag>
set -o pipefail
T=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sspmc_$T
mkdir -p $OUT
export SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so TMPDIR=/tmp
cd /tmp
CTRS="TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_sum SQ_WAVE_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
for V in "fast:SPMV_LAUNCH_SS=1" "noy:SPMV_LAUNCH_SS=1,SPMV_LAUNCH_SS_SPLIT=128" "ell:SPMV_LAUNCH_SS=1"; do
  name=${V%%:*}
  fmt=ss; [ $name = ell ] && fmt=ell
  # shellcheck disable=SC2086
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/pass_$name -o run -- \
      python3 $R/tools/bin_phase_ab.py --kind banded --fmt $fmt --rows 20000000 --per-row 64 \
      --variants "$name:ss_sigma=20" --launch-variants "$V" --rounds 1 --iters 20 \
      > $OUT/pass_$name.log 2> $OUT/pass_$name.err || exit $?
done
for name in fast noy ell; do
  mkdir -p $OUT/s_$name && ln -sfn $OUT/pass_$name $OUT/s_$name/pass1
  python3 $R/tools/pmc_stalls_summary.py $OUT/s_$name > $OUT/summary_$name.json || exit 1
done
echo done
