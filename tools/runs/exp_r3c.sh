#!/bin/bash
# proj_bwd outer-product operand read-ahead (CSA_EXP_OT_LA = 2 / 4 K-groups) vs the shipped build, one box.
set -o pipefail
export TMPDIR=/tmp
R=${1:-3}
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
for v in exp_OTLA2 exp_OTLA4; do
  CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > /tmp/pt.log 2>&1; rc=$?; echo "$v $(tail -1 /tmp/pt.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in $(seq 1 "$R"); do
  for v in hip exp_OTLA2 exp_OTLA4; do
    out=$(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], d['bf16_mode']['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$v"
  done
done
