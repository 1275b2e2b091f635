#!/bin/bash
# Round 4: GPU tests on the batched mask packing / conditional rescale in k_attn_fwd; same-box A/B against a
# variant without the tile's Philox calls (timing only: how much of k_attn_fwd the RNG costs).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_k.log 2>&1; rc=$?; tail -2 gpurun_out/pt_k.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_k.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_k.json')); print('$1', d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], {k: round(v,4) for k,v in d['stage_ms'].items()}, d['bf16_mode']['ms_per_step'])"
}
for i in 1 2; do
  run hip $LIB/libcsa_hip.so || exit 1
  run fwdnorng $LIB/libcsa_FWDNORNG.so || exit 1
done
