#!/bin/bash
# Round 6: the CSE relation-plane prep items as extra one-wave workgroups of the logits launch (N <= 256) instead of
# their own launch; CSE / model parity tests, then the java CSE layer A/B against ab5 (the committed tree)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ad; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for i in 1 2 3 4 5; do
  for lib in libcsa_ab5.so libcsa_hip.so; do
    echo -n "$lib "; CSA_HIP_LIB=$L/$lib timeout -k 10 120 python tools/cse_bench.py 64 40 2>/dev/null | tail -1 || exit 1
  done
done 2>&1 | tee $O/ab_cse.txt
