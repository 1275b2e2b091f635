#!/bin/bash
# Round 5: k_proj_bwd_s<64> loads the next group's hat / gin rows into VGPRs after B5 and writes them into the DS region
# after B6 (HGR = CSA_EXP_HGREG), dQ / dK row stores after that, vs the hat / gin DMA after B6 waited at the next group top
# (hip = shipped). GPU tests on the HGR build, then a same-box A/B (headline)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ak; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
CSA_HIP_LIB=$L/libcsa_HGR.so timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_property_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_dxl.txt 2>&1; rc=$?; tail -1 $O/pytest_dxl.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch|assert" $O/pytest_dxl.txt | head -20; exit $rc; }
bash tools/ab_multi.sh 4 $L/libcsa_hip.so $L/libcsa_HGR.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
