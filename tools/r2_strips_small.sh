#!/bin/bash
# Strip width for mid-size BIN plans (AUTO's new 1-3.5 M column range):
# in-process A/B of bin_strip_cols at 1, 2, 3 M rows (uniform 16 / row) and
# 2 M power-law.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/strips_small
mkdir -p $O
cd $R
V='w20480:;w10240:bin_strip_cols=10240;w5120:bin_strip_cols=5120;w2560:bin_strip_cols=2560'
for m in 1000000 2000000 3000000; do
  SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --rows $m --check --rounds 3 > $O/ab_u$m.jsonl 2>> $O/ab.err || exit $?
done
SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 300 python3 -u tools/bin_phase_ab.py --variants "$V" --kind powerlaw --max-len 2000 --rows 2000000 --check --rounds 3 > $O/ab_p2000000.jsonl 2>> $O/ab.err || exit $?
