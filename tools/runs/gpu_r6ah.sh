#!/bin/bash
# Round 6: k_rel_bwd_kh walks its (b,h) blocks in reverse inside each XCD (the forward's bias tiles of the last-written
# (b,h)s in L2; k_rel_bwd_qg then walks against kh's order): khrev vs hip, CSE tests + java layer A/B, 5 rounds
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ah; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
CSA_HIP_LIB=$L/libcsa_khrev.so timeout -k 10 300 python -u -m pytest tests/test_cse_gpu.py -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4 5; do
  for lib in libcsa_khrev.so libcsa_hip.so; do
    echo -n "$lib "; CSA_HIP_LIB=$L/$lib timeout -k 10 120 python tools/cse_bench.py 64 40 2>/dev/null | tail -1 || exit 1
  done
done 2>&1 | tee $O/ab_cse.txt
