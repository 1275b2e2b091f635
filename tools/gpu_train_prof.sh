#!/bin/bash
# Train step on the tuned GEMM table: kernel stats under rocprofv3, then a retune with a longer timing
# budget per candidate and a same-box A/B of the two tables.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/trainprof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/prof_train.py 8 > $OUT/prof.log 2>&1 || exit $?
tail -1 $OUT/prof.log
T2=$PWD/$OUT/gemm_long.csv
timeout -k 10 600 python -u tools/tune_gemms.py $T2 60 > $OUT/tune_long.log 2>&1 || exit $?
tail -1 $OUT/tune_long.log
for i in 1 2; do
  for t in committed long; do
    arg=""; [ $t = long ] && arg=$T2
    timeout -k 10 200 python -u tools/prof_train.py 40 $arg > $OUT/ab_$t$i.log 2>&1 || exit $?
    echo "$t $(tail -1 $OUT/ab_$t$i.log | python3 -c 'import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
