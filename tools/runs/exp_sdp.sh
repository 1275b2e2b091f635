#!/bin/bash
# java train step: decoder SDPA on the default (aotriton) backend vs the math backend, alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sdp
mkdir -p $OUT
for i in 1 2 3; do
  for v in default math; do
    CSA_SDP=$v timeout -k 10 200 python -u tools/prof_train.py 40 > $OUT/$v$i.log 2>&1 || exit $?
    echo "$v $(tail -1 $OUT/$v$i.log | python3 -c 'import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d["ms_per_step"], d["mean_loss"])')" | tee -a $OUT/ab.txt
  done
done
