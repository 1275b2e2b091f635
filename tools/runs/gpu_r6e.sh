#!/bin/bash
# Round 6: which build fails the new dead-tile test at d = 96 (base = round start, fwdv = fused row constants, hip = +dead
# tiles); the test's other shapes too
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6e; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
for lib in libcsa_base.so libcsa_fwdv.so libcsa_hip.so; do
  echo "== $lib"
  CSA_HIP_LIB=$L/$lib timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -q --timeout 120 --timeout-method thread -k "dead" > $O/pytest_$lib.txt 2>&1
  grep -E "passed|failed" $O/pytest_$lib.txt | tail -1; grep -E "^E  +(d[QKV]|Mismatched|Max abs)|^FAILED" $O/pytest_$lib.txt | head -20
done
