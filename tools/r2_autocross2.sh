#!/bin/bash
# AUTO's new BIN threshold: the AUTO test, and the 4 / 8 per-row and
# max_len 500 power-law cases around it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/autocross2
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "auto_format" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/auto_cross.py --sizes 1000000,2000000 --kinds uniform --per-row 4 --formats css,bin > $O/cross_u4.jsonl 2> $O/cross.err || exit $?
timeout -k 10 300 python3 -u tools/auto_cross.py --sizes 1000000,2000000 --kinds uniform --per-row 8 --formats css,bin > $O/cross_u8.jsonl 2>> $O/cross.err || exit $?
timeout -k 10 300 python3 -u tools/auto_cross.py --sizes 1000000,2000000 --kinds powerlaw --max-len 500 --formats css,bin,auto > $O/cross_p500.jsonl 2>> $O/cross.err || exit $?
