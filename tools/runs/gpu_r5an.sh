#!/bin/bash
# Round 5: CSE 16-row backward knobs on the final tree (java layer, B = 64): the bins-scatter passes without the
# lgkmcnt(0) between them (NPW = CSA_EXP_NOPASSWAIT; a wave's LDS adds still execute in issue order, so the sums and
# their order are unchanged), the scatter of tile kt deferred to the top of kt + 1 (DEFER); hip = shipped.
# CSE parity tests on both variants first, then cse_bench alternated.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5an; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
for lib in libcsa_NPW.so libcsa_DEFER.so; do
  CSA_HIP_LIB=$L/$lib timeout -k 10 300 python -u -m pytest tests/test_cse_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$lib.txt 2>&1; rc=$?; echo "$lib $(tail -1 $O/pytest_$lib.txt)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do for lib in libcsa_hip.so libcsa_NPW.so libcsa_DEFER.so; do echo -n "$lib "; CSA_HIP_LIB=$L/$lib timeout -k 10 120 python tools/cse_bench.py 64 50 in_order || exit 1; done; done 2>&1 | grep CSE | tee $O/ab.txt
