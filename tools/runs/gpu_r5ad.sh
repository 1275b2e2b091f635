#!/bin/bash
# Round 5: k_attn_bwd_qg loads tile kt+1's one-plane values at the top of iteration kt (hip) vs at its end
# (QGNOPF = CSA_EXP_QG_NOPF): GPU tests on the new build, then same-box A/Bs, headline and dense
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ad; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
bash tools/ab_multi.sh 3 $L/libcsa_QGNOPF.so $L/libcsa_hip.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--dense --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-padded-leg --no-cpu-config1" bash tools/ab_multi.sh 3 $L/libcsa_QGNOPF.so $L/libcsa_hip.so > $O/ab_dense.txt 2>&1; rc=$?; grep "^libcsa" $O/ab_dense.txt; exit $rc
