#!/bin/bash
# Round 5: k_attn_bwd_kv experiments on one box: KA (no second-half w stores), KB (no first-half w stores), KR
# (second half's dK first, next query block's Q pieces among its dV MFMAs). SBM tests on KR first.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5f; mkdir -p $O
CSA_HIP_LIB=$LIB/libcsa_KR.so timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_kr.log 2>&1; rc=$?; tail -2 $O/pytest_kr.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  for v in OLD KA KB KR; do run $v $LIB/libcsa_$v.so || exit 1; done
done
