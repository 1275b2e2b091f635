#!/bin/bash
# bf16 mode: same-box A/B of the recomputing query kernel (shipped) vs the one-plane handoff in bf16 mode
# (CSA_EXP_BF_HANDOFF), stage times from bench.py --precision bf16; bf16 GPU tests on the variant first.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
CSA_HIP_LIB=$LIB/libcsa_BFHO.so timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_q.log 2>&1; rc=$?; tail -2 gpurun_out/pt_q.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --precision bf16 --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > gpurun_out/bench_q.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  run recomp $LIB/libcsa_hip.so || exit 1
  run handoff $LIB/libcsa_BFHO.so || exit 1
done
