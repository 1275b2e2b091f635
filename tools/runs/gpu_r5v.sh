#!/bin/bash
# Round 5: k_proj_bwd_s outer products with the operand reads one K-group ahead (hip) vs each group waiting on its
# own reads (NOLA, round-4 form): parity, then same-box A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5v; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sbm_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_multi.sh 3 $L/libcsa_NOLA.so $L/libcsa_hip.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
