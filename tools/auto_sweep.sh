#!/bin/bash
# AUTO crossover: every format on uniform 16/row and power-law matrices of
# growing size (x = 2 .. 32 MB), one JSON line per (size, format)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for m in 250000 500000 1000000 2000000 4000000; do
  for f in css ss csr ell; do
    timeout -k 10 200 python $R/tools/tune.py --fmt $f --rows $m --rounds 2 2>/dev/null | grep '^{' | sed "s/^/{\"m\": $m, \"kind\": \"uniform\", \"r\": /; s/$/}/" || exit 1
    timeout -k 10 200 python $R/tools/tune.py --fmt $f --kind powerlaw --max-len 2000 --rows $m --rounds 2 2>/dev/null | grep '^{' | sed "s/^/{\"m\": $m, \"kind\": \"powerlaw\", \"r\": /; s/$/}/" || exit 1
  done
done
