#!/bin/bash
# Round 5: k_attn_rowprep with eight row groups per lane in flight (RP8) or X streamed non-temporally (RPNT); the one-plane
# w tiles through the default cache policy (WRT); hip = shipped. Same box, headline bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ae; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
bash tools/ab_multi.sh 3 $L/libcsa_hip.so $L/libcsa_RP8.so $L/libcsa_RPNT.so $L/libcsa_WRT.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
