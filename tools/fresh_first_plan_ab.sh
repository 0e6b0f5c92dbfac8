#!/bin/bash
# fresh-process first-plan timing: device-built vs host-built config-2 BIN
set -o pipefail
O=gpurun_out/r5ap; mkdir -p $O
for i in 1 2 3 4 5; do
  for v in dev:build=2 host:build=1; do
    timeout -k 10 120 python -u tools/bin_phase_ab.py --rows 10000000 --placement auto --rounds 3 --variants "$v" >> $O/fresh.jsonl 2>> $O/err.txt || exit 1
  done
done
echo done
