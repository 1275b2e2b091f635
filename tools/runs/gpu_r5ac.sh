#!/bin/bash
# Round 5: live cost of launches on the step's critical path: 4 extra empty launches (EXTRA4) and the step without
# k_sparsity_finish / k_cluster_grad (NOSMALL, wrong outputs: timing only), same box
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ac; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
bash tools/ab_multi.sh 4 $L/libcsa_hip.so $L/libcsa_EXTRA4.so $L/libcsa_NOSMALL.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt | cut -c1-60; exit $rc
