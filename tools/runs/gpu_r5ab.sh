#!/bin/bash
# activation block's copy (H2TOP = CSA_EXP_HAT_ACT): full GPU tests on the new build, then a same-box A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ab; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
bash tools/ab_multi.sh 3 $L/libcsa_H2TOP.so $L/libcsa_hip.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
