#!/bin/bash
# Round 5: bound experiment: forward refill DMA cut to ~1/5 per wave (FIFTH, wrong results) vs the real kernel
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5aa; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
bash tools/ab_multi.sh 3 $L/libcsa_hip.so $L/libcsa_FIFTH.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
