#!/bin/bash
# Round 5: k_attn_bwd_kv experiments (KA: no second-half w stores, KB: no first-half w stores, KR: dK first + Q
# pieces among the dV MFMAs) and the software-pipelined forward (PIPE), same box, against OLD (round-4 forward)
# and the tree (k_attn_fwd64).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5g; mkdir -p $O
for v in KR PIPE; do
CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  for v in OLD KA KB KR PIPE; do run $v $LIB/libcsa_$v.so || exit 1; done
  run tree $LIB/libcsa_hip.so || exit 1
done
