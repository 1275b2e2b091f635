#!/bin/bash
# k_attn_fwd: same-box A/B of the unconditional o rescale (shipped) vs a rescale under a ballot (CSA_EXP_FWD_COND_RESCALE).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
CSA_HIP_LIB=$LIB/libcsa_CONDRS.so timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_u.log 2>&1; rc=$?; tail -2 gpurun_out/pt_u.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > gpurun_out/bench_u.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_u.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  run base $LIB/libcsa_hip.so || exit 1
  run condrs $LIB/libcsa_CONDRS.so || exit 1
done
