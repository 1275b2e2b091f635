#!/bin/bash
# CSE 16-row backward variants, alternating CSE layer timings on one box (java dims, B=64).
set -o pipefail
export TMPDIR=/tmp
R=${1:-3}
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_cse_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > /tmp/pt.log 2>&1; rc=$?; tail -1 /tmp/pt.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 "$R"); do
  for v in hip exp_NODEFER exp_NOSB exp_NODEFER_NOSB exp_V1 exp_REL32; do
    echo "$v $(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python tools/cse_bench.py 64 50 | tail -1)" || exit 1
  done
done
