#!/bin/bash
# Projection-backward key/query split sized for half the workgroup slots per kind: GPU tests, then same-box A/B
# against the last commit at the headline shape (d = 64, B = 256) and at java dims (d = 96, B = 64).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
python -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash, built_hash; assert source_hash() == built_hash(), 'stale libcsa_hip.so'" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_s.log 2>&1; rc=$?; tail -2 gpurun_out/pt_s.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib extra-args
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg $3 > gpurun_out/bench_s.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_s.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  run tree64 $LIB/libcsa_hip.so "" || exit 1
  run old64 $LIB/libcsa_SPLIT0.so "" || exit 1
  run tree96 $LIB/libcsa_hip.so "--head-dim 96 --batch 64" || exit 1
  run old96 $LIB/libcsa_SPLIT0.so "--head-dim 96 --batch 64" || exit 1
done
