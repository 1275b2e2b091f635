#!/bin/bash
# Round-3 one-box experiment: SBM GPU tests on each variant library, then alternating bench runs
#   base  = shipped build          RECOMP_PO = k_proj_bwd_s<64> recomputes po (no po store / load)
#   PRIO  = half of the attention waves at s_setprio 1
# usage: bash tools/exp_r3a.sh [rounds]
set -o pipefail
export TMPDIR=/tmp
R=${1:-3}
OUT=gpurun_out/exp_r3a
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $OUT
for v in RECOMP_PO PRIO; do
  CSA_HIP_LIB=$LIB/libcsa_exp_$v.so timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg"
run() {  # name lib
  out=$(CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py $ARGS) || exit $?
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$1"
}
for i in $(seq 1 "$R"); do
  run base $LIB/libcsa_hip.so
  run RECOMP_PO $LIB/libcsa_exp_RECOMP_PO.so
  run PRIO $LIB/libcsa_exp_PRIO.so
done
