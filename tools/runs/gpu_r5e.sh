#!/bin/bash
# Round 5: k_attn_fwd64 (Philox among the S MFMAs, K / T / V pieces between the E / PV MFMAs, counted vmcnt waits,
# bias as the S chain's initial accumulator, lazy rescale). SBM / property / bf16 / model GPU tests; same-box A/B
# against the round-4 kernels (R4) and the tree with the round-4 forward (OLD).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_property_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  run tree $LIB/libcsa_hip.so || exit 1
  for v in R4 OLD; do run $v $LIB/libcsa_$v.so || exit 1; done
done
CSA_HIP_LIB=$LIB/libcsa_hip.so timeout -k 10 120 python bench.py --dense --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/dense_tree.json && CSA_HIP_LIB=$LIB/libcsa_R4.so timeout -k 10 120 python bench.py --dense --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/dense_R4.json
python3 -c "import json; [print(t, json.load(open('$O/dense_'+t+'.json'))['ms_per_step'], json.load(open('$O/dense_'+t+'.json'))['stage_ms']) for t in ('tree','R4')]"
