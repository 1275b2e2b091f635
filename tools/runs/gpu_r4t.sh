#!/bin/bash
# k_attn_bwd_kv refill placement: same-box A/B of the rolling per-half refill (shipped) vs one refill after the
# second half (CSA_EXP_KV_LATE_REFILL), SBM GPU tests on the variant first.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
CSA_HIP_LIB=$LIB/libcsa_LATEREF.so timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_t.log 2>&1; rc=$?; tail -2 gpurun_out/pt_t.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > gpurun_out/bench_t.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_t.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  run rolling $LIB/libcsa_hip.so || exit 1
  run late $LIB/libcsa_LATEREF.so || exit 1
done
