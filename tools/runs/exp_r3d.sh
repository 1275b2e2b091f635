#!/bin/bash
# proj_fwd: activation blocks stored right after they are produced (CSA_EXP_EARLY_ST) vs at the item end.
set -o pipefail
export TMPDIR=/tmp
R=${1:-3}
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
CSA_HIP_LIB=$LIB/libcsa_exp_EARLY_ST.so timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > /tmp/pt.log 2>&1; rc=$?; echo "EARLY_ST $(tail -1 /tmp/pt.log)"; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 "$R"); do
  for v in hip exp_EARLY_ST; do
    out=$(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], d['bf16_mode']['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$v"
  done
done
