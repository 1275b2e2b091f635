#!/bin/bash
# Round 5: cache policy of the staged activation stores (nt = current, default, sc1, sc1 nt), and NOACT beside them
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5p; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
bash tools/ab_multi.sh 2 $L/libcsa_hip.so $L/libcsa_AUX0.so $L/libcsa_AUX16.so $L/libcsa_AUX18.so $L/libcsa_NOACT.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
