#!/bin/bash
# Round 5, dense FullAttention occupancy: hip = fp32 forward (d = 64) at three waves per SIMD (<= 168 VGPRs) and the query
# kernel without the T image's LDS (8 KB per wave: five waves per SIMD); DW2 = forward at two waves; QGT = query kernel
# with the T image's LDS; DOLD = both as before. GPU tests on the new build, then a same-box dense A/B and a headline check
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ag; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
BENCH_ARGS="--dense --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-padded-leg --no-cpu-config1" bash tools/ab_multi.sh 3 $L/libcsa_DOLD.so $L/libcsa_DW2.so $L/libcsa_QGT.so $L/libcsa_hip.so > $O/ab_dense.txt 2>&1; rc=$?; grep "^libcsa" $O/ab_dense.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_multi.sh 2 $L/libcsa_DOLD.so $L/libcsa_hip.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
