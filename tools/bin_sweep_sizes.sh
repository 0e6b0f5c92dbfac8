set -e
R=gpurun_out/b9; mkdir -p $R
for cfg in "--rows 1000000" "--rows 2000000" "--rows 5000000" "--kind powerlaw --rows 5000000" "--kind powerlaw --rows 2000000"; do
  timeout -k 10 300 python -u tools/tune.py --fmt bin $cfg --rounds 2 >> $R/t.jsonl 2>>$R/err
  timeout -k 10 300 python -u tools/tune.py --fmt css $cfg --rounds 2 >> $R/t.jsonl 2>>$R/err
  timeout -k 10 300 python -u tools/tune.py --fmt auto $cfg --rounds 2 >> $R/t.jsonl 2>>$R/err
  echo "$cfg done" >> $R/t.jsonl
done
