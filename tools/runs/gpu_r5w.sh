#!/bin/bash
# Round 5: the cluster-weight gradient from h2 (po not saved by the forward; k_cluster_grad applies W2 / b2) vs
# saving po (SAVEPO, CSA_EXP_SAVE_PO): full GPU parity of the new build, then a same-box A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5w; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
bash tools/ab_multi.sh 3 $L/libcsa_SAVEPO.so $L/libcsa_hip.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
