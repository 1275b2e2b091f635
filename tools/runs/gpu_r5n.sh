#!/bin/bash
# Round 5: projection forward with the activation stores riding along the next chain (ActStager) vs the store
# phase after the products (CSA_EXP_STORE_PHASE): SBM parity (incl. the golden train-mode activations), same-box A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5n; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sbm_gpu.py tests/test_bf16_gpu.py > $O/pytest_sbm.txt 2>&1; rc=$?; tail -3 $O/pytest_sbm.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh $L/libcsa_STPH.so $L/libcsa_hip.so 3 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
