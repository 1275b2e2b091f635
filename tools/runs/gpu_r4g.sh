#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_g.log 2>&1; rc=$?; tail -2 gpurun_out/pt_g.log; [ $rc -eq 0 ] || exit $rc
CSA_HIP_LIB=$LIB/libcsa_RECOMP.so timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_g2.log 2>&1; rc=$?; tail -1 gpurun_out/pt_g2.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1" bash tools/ab_multi.sh 2 $LIB/libcsa_hip.so $LIB/libcsa_RECOMP_S.so $LIB/libcsa_RECOMP.so
for v in hip RECOMP; do CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v bf16', d['bf16_mode']['ms_per_step'])" || exit 1; done
