#!/bin/bash
# Round 5: prologue fixes (no load-use waits before the first tile) in k_attn_fwd and k_attn_bwd_kv. SBM GPU tests;
# same-box A/B against the round-4 kernels (R4) and the persistent forward (PER); phase stamps of the tree (ST).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_property_gpu.py tests/test_bf16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  run tree $LIB/libcsa_hip.so || exit 1
  for v in R4 PER; do run $v $LIB/libcsa_$v.so || exit 1; done
done
CSA_HIP_LIB=$LIB/libcsa_ST.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/stamps_ST.txt 2>&1 || exit 1
