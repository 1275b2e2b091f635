#!/bin/bash
# One-box experiment: SBM parity tests on the current build, then alternating bench runs of
#   old  = k_proj_fwd (L2 fragments, CSA_PROJ_FWD_L=0)   new = k_proj_fwd_l (LDS fragments)
# and throw-away upper-bound variants (tools/build_variant.py exp_*), at python (d=64, B=256) and
# java (d=96, B=64) dims. usage: bash tools/exp_proj_fwd.sh [rounds]
set -o pipefail
export TMPDIR=/tmp
R=${1:-2}
OUT=gpurun_out/exp_pf
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_sbm_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-cpu-config1"
run() {  # name env lib extra-args
  out=$(env $2 CSA_HIP_LIB=$3 timeout -k 10 120 python bench.py $ARGS $4) || exit $?
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$1"
}
for i in $(seq 1 "$R"); do
  run old CSA_PROJ_FWD_L=0 $LIB/libcsa_hip.so ""
  run new CSA_PROJ_FWD_L=1 $LIB/libcsa_hip.so ""
  for v in FRAG_L1 NO_ACT NO_SHFL NO_PHILOX; do run $v CSA_PROJ_FWD_L=0 $LIB/libcsa_exp_$v.so ""; done
  run old96 CSA_PROJ_FWD_L=0 $LIB/libcsa_hip.so "--head-dim 96 --batch 64"
  run new96 CSA_PROJ_FWD_L=1 $LIB/libcsa_hip.so "--head-dim 96 --batch 64"
done
