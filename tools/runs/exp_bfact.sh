#!/bin/bash
# bf16 mode: h1 | h2 | po saved as bf16 (hip) vs fp32 (exp_base): SBM / bf16 GPU tests, then alternating benches
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bfact
mkdir -p $OUT
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py tests/test_sbm_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "tests: $(tail -1 $OUT/pytest.log)"; grep -E "bf16 sbm_n(37|150).*(layer.weight|proj.0.weight)" $OUT/pytest.log | head -6; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-train"
for i in 1 2 3; do
  for v in exp_base hip; do
    out=$(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python bench.py $ARGS 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1].strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['bf16_mode']['ms_per_step'])" "$out" "$v" | tee -a $OUT/ab.txt
  done
done
for v in exp_base hip; do
  out=$(CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python bench.py --precision bf16 --head-dim 96 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-train 2>/dev/null) || exit 1
  python3 -c "import json,sys; d=json.loads(sys.argv[1].strip().splitlines()[-1]); print(sys.argv[2], 'd96 B64 bf16', d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$v" | tee -a $OUT/ab.txt
done
