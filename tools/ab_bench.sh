#!/bin/bash
# A/B of probe-build switches on one bench config, alternating variants:
#   tools/ab_bench.sh <outfile> <config> <reps> "<ENV=V ...>" "<ENV=V ...>" ...
# each variant: bench.py --formats ${FMT:-auto} --no-cpu --trials 3 with the probe
# library; one JSON summary line per run
set -o pipefail
OUT=$1; CFG=$2; REPS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    env SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so $v timeout -k 10 240 python3 -u bench.py --config $CFG \
        --formats ${FMT:-auto} --no-cpu --trials 3 --steps 50 --warmup 10 $BENCH_EXTRA > /tmp/ab_one.json 2> /tmp/ab_one.err || exit $?
    python3 -c "
import json,sys
d=json.loads(open('/tmp/ab_one.json').read().strip().splitlines()[-1]); a=list(d['formats'].values())[0]
print(json.dumps({'variant': sys.argv[1], 'rep': int(sys.argv[2]), 'ms': round(d['ms_per_step'],4), 'gflops': round(d['value'],1),
  'phases': {k: round(v,4) for k,v in a.get('phases_ms',{}).items()}, 'stored': a.get('stored_slots'), 'bins': a.get('bin_bins'),
  'pad': a.get('bin_pad'), 'placement': a.get('placement_candidates_ms')}))" "$v" $rep >> $OUT || exit $?
  done
done
