#!/bin/bash
# Round 5: the CSE relation-plane prep as extra workgroups of the logits launch (hip) vs its own launch after the
# logits (SEPP = CSA_EXP_SEP_PREP): full GPU tests on the new build, then cse_bench alternated (java layer, B = 64)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ap; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
for r in 1 2 3 4 5 6; do for lib in libcsa_SEPP.so libcsa_hip.so; do
  out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python tools/cse_bench.py 64 50 in_order 2>/dev/null | grep CSE) || exit 1
  echo "$lib $out"
done; done | tee $O/ab.txt
