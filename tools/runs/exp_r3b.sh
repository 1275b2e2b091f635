#!/bin/bash
# Round-3 one-box experiment: SBM + CSE GPU tests on the shipped build, then alternating timings of
#   CSE variants (java CSE layer, B=64) and the SBM layer with / without the two-tile forward pipeline.
set -o pipefail
export TMPDIR=/tmp
R=${1:-2}
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
OUT=gpurun_out/exp_r3b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_sbm_gpu.py tests/test_cse_gpu.py tests/test_bf16_gpu.py tests/test_property_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 "$R"); do
  for v in hip exp_NOPASSWAIT exp_NOSB exp_DEFER exp_V1; do
    echo "$v $(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python tools/cse_bench.py 64 50 | tail -1)" || exit 1
  done
  for v in hip exp_FWD_SERIAL; do
    out=$(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$v"
  done
done
