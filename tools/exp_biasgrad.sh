#!/bin/bash
# One-launch bias gradient (csa_bias_grad_fused) vs the two-launch csa_bias_grad: glue GPU tests, then the java
# train step alternating (CSA_BIAS_GRAD_FUSED=1 selects the one-launch path)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/biasgrad
mkdir -p $OUT
CSA_BIAS_GRAD_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_glue_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "tests: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in two fused; do
    if [ $v = fused ]; then export CSA_BIAS_GRAD_FUSED=1; else unset CSA_BIAS_GRAD_FUSED; fi
    timeout -k 10 200 python -u tools/prof_train.py 40 > $OUT/$v$i.log 2>&1 || exit $?
    echo "$v $(tail -1 $OUT/$v$i.log | python3 -c 'import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $OUT/ab.txt
  done
done
