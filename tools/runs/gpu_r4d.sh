#!/bin/bash
# Round 4: SBM GPU tests on the 4-wave bwd_qg, then same-box A/B of the ds/G store kinds with kernel traces.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_sbm_gpu.py tests/test_bf16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_d.log 2>&1; rc=$?; tail -2 gpurun_out/pt_d.log; [ $rc -eq 0 ] || exit $rc
B="--steps 10 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg"
cd /tmp
for v in hip NT_DSG; do
  CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_d_$v -o run -- python3 $R/bench.py $B > $R/gpurun_out/prof_d_$v.log 2>&1 || exit $?
done
cd $R
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1" bash tools/ab_multi.sh 2 $LIB/libcsa_hip.so $LIB/libcsa_NT_DSG.so
