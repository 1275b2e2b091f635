#!/bin/bash
# Round 5: what bounds the projection forward: staged stores (main) vs no activation stores vs MFMA chains only.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5o; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
bash tools/ab_multi.sh 2 $L/libcsa_hip.so $L/libcsa_NOACT.so $L/libcsa_MONLY.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
