#!/bin/bash
# Round 5: k_proj_bwd_s<64> issues each group's dQ / dK row stores after B6, behind the next group's hat / gin / W2
# DMAs (DXL = CSA_EXP_DXLATE), so the next group top's counted vmcnt no longer waits for the stores, vs before B6
# (hip = shipped). GPU tests on the DXL build, then a same-box A/B (headline)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5aj; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
CSA_HIP_LIB=$L/libcsa_DXL.so timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_property_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_dxl.txt 2>&1; rc=$?; tail -1 $O/pytest_dxl.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch|assert" $O/pytest_dxl.txt | head -20; exit $rc; }
bash tools/ab_multi.sh 4 $L/libcsa_hip.so $L/libcsa_DXL.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
