#!/bin/bash
# same-box A/B of an environment switch read at plan build:
#   ENVVAR=SPMV_DIA_DEBUG VALUES="0 1" FMT=dia CFG="--kind banded --rows 20000000" tools/ab_env.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  for v in $VALUES; do
    env $ENVVAR=$v timeout -k 10 300 python $R/tools/tune.py --fmt $FMT $CFG --rounds 3 2>/dev/null | grep '^{' | sed "s/^/{\"$ENVVAR\": $v, \"rep\": $rep, \"r\": /; s/$/}/" || exit 1
  done
done
