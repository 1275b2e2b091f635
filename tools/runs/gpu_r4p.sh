#!/bin/bash
# Round 4: GPU tests (16-wave slab reduction); same-box A/B of the tree against ebb1e00 (before the k_attn_fwd
# mask-packing change and the reduction change): stage_ms separates the two.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
python -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash, built_hash; assert source_hash() == built_hash(), 'stale libcsa_hip.so'" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_p.log 2>&1; rc=$?; tail -2 gpurun_out/pt_p.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_p.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_p.json')); print('$1', d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], {k: round(v,4) for k,v in d['stage_ms'].items()}, d['bf16_mode']['ms_per_step'])"
}
for i in 1 2 3 4; do
  run tree $LIB/libcsa_hip.so || exit 1
  run pack0 $LIB/libcsa_PACK0.so || exit 1
done
