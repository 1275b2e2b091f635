#!/bin/bash
# Round 5: attention experiments. hip = ballots packed in two groups of 8; PACK16 = all 16 ballots first (round 4);
# WDEF = bwd_kv half-1 w parked in LDS and stored after the refill DMAs; KEARLY = fwd K image refill right after
# the S chain. Parity of WDEF / KEARLY (test_sbm_gpu), then a same-box A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5t; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
for v in hip WDEF KEARLY; do
  lib=$L/libcsa_$v.so
  CSA_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sbm_gpu.py > $O/pytest_$v.txt 2>&1; rc=$?; echo "$v: $(tail -1 $O/pytest_$v.txt)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_multi.sh 3 $L/libcsa_hip.so $L/libcsa_PACK16.so $L/libcsa_WDEF.so $L/libcsa_KEARLY.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
