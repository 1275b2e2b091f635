#!/bin/bash
# CSE: the two lgrad split sums in one launch (k_sum_splits2) vs two k_sum_splits launches (exp_base)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/cse_sums
mkdir -p $OUT
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_cse_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "cse tests: $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in exp_base hip; do
    r=$(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python -u tools/cse_bench.py 64 50 2>&1 | tail -1) || exit 1
    echo "$v $r" | tee -a $OUT/ab.txt
  done
done
