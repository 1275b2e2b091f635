#!/bin/bash
# Round 5: paired workgroups for the three attention kernels (PAIR = CSA_EXP_PAIR: two independent waves per workgroup,
# consecutive blocks of mostly one (b,h) on one CU, so they read the same K / V (Q / dX) tiles through one L1; each wave
# keeps its own LDS images, no barriers) vs one wave per workgroup (hip). GPU tests on both builds, then same-box A/Bs.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ai; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
CSA_HIP_LIB=$L/libcsa_PAIR.so timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_property_gpu.py tests/test_bf16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pair.txt 2>&1; rc=$?; tail -1 $O/pytest_pair.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch|assert" $O/pytest_pair.txt | head -20; exit $rc; }
bash tools/ab_multi.sh 3 $L/libcsa_hip.so $L/libcsa_PAIR.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--dense --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-padded-leg --no-cpu-config1" bash tools/ab_multi.sh 2 $L/libcsa_hip.so $L/libcsa_PAIR.so > $O/ab_dense.txt 2>&1; rc=$?; grep "^libcsa" $O/ab_dense.txt; exit $rc
