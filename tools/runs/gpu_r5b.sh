#!/bin/bash
# Round 5: persistent k_attn_fwd_p. SBM + model GPU tests on the tree, then same-box A/B: tree (persistent) vs PO
# (one item per wave, k_attn_fwd) vs PP (persistent, half the waves at priority 1) vs PS / PSP (MFMA + DMA skeleton).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_property_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2; do
  run tree $LIB/libcsa_hip.so || exit 1
  for v in PO PP PS PSP; do run $v $LIB/libcsa_$v.so || exit 1; done
done
