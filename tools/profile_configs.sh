#!/bin/bash
# rocprofv3 trace + FETCH/WRITE PMC passes of the headline plan of configs 2-4
set -o pipefail
bash tools/profile_round.sh ${1}_c2 --formats auto > gpurun_out/prof_${1}_c2.log 2>&1 || exit 1
bash tools/profile_round.sh ${1}_c3 --config c3 --formats auto > gpurun_out/prof_${1}_c3.log 2>&1 || exit 2
bash tools/profile_round.sh ${1}_c4 --config c4 --formats auto > gpurun_out/prof_${1}_c4.log 2>&1 || exit 3
