#!/bin/bash
# Same-box A/B: working tree (k_attn_fwd: batched mask packing, conditional o rescale) vs the last commit.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_l.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_l.json')); print('$1', d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], {k: round(v,4) for k,v in d['stage_ms'].items()}, d['bf16_mode']['ms_per_step'])"
}
for i in 1 2 3; do
  run hip $LIB/libcsa_hip.so || exit 1
  run prev $LIB/libcsa_PREV.so || exit 1
done
