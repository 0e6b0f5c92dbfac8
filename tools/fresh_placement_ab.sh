#!/bin/bash
# fresh-process first-plan timing of the config-2 BIN plan under each
# placement mode (AUTO = VMM handles, SEARCH, PLAIN), alternating
#   bash tools/fresh_placement_ab.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for i in 1 2 3 4; do
  for v in auto:placement=0 search:placement=2 plain:placement=1; do
    timeout -k 10 150 python -u tools/bin_phase_ab.py --rows 10000000 --rounds 3 --variants "$v" >> $O/fresh_placement.jsonl 2>> $O/err.txt || exit 1
  done
done
echo done
