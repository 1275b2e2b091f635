#!/bin/bash
# One-box A/B of fragment-fetch variants (tools/build_variant.py exp_*): see tools/exp_proj_fwd.sh.
set -o pipefail
export TMPDIR=/tmp
R=${1:-2}
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-cpu-config1"
run() {  # name env lib extra-args
  out=$(env $2 CSA_HIP_LIB=$3 timeout -k 10 120 python bench.py $ARGS $4) || exit $?
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$1"
}
for i in $(seq 1 "$R"); do
  run old CSA_PROJ_FWD_L=0 $LIB/libcsa_hip.so ""
  run new CSA_PROJ_FWD_L=1 $LIB/libcsa_hip.so ""
  run PF6 CSA_PROJ_FWD_L=1 $LIB/libcsa_exp_PF6.so ""
  run SPREAD CSA_PROJ_FWD_L=0 $LIB/libcsa_exp_FRAG_SPREAD.so ""
  run ACT_NT CSA_PROJ_FWD_L=1 $LIB/libcsa_exp_ACT_NT.so ""
  run L1 CSA_PROJ_FWD_L=0 $LIB/libcsa_exp_FRAG_L1.so ""
done
