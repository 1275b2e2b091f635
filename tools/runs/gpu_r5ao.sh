#!/bin/bash
# Round 5: CSE bins scatter without the waits between passes (NPW) vs shipped (hip), 6 alternated rounds of
# cse_bench 64 on one box
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ao; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
for r in 1 2 3 4 5 6; do for lib in libcsa_hip.so libcsa_NPW.so; do
  out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python tools/cse_bench.py 64 50 in_order 2>/dev/null | grep CSE) || exit 1
  echo "$lib $out"
done; done | tee $O/ab.txt
