#!/bin/bash
# Round 5: bound on the bf16 mode's "bf16 operand images" lever: the step without the in-loop image refills of
# k_attn_fwd and k_attn_bwd_kv (NODMA = CSA_EXP_NO_LOOP_DMA + CSA_EXP_FWD_NO_LOOPDMA; wrong results, timing only) vs
# shipped, in bf16 mode and in fp32, same box. Halving the image bytes can buy at most half of the difference.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5am; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
BENCH_ARGS="--precision bf16 --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-padded-leg --no-cpu-config1" bash tools/ab_multi.sh 3 $L/libcsa_hip.so $L/libcsa_NODMA.so > $O/ab_bf16.txt 2>&1; rc=$?; grep "^libcsa" $O/ab_bf16.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_multi.sh 2 $L/libcsa_hip.so $L/libcsa_NODMA.so > $O/ab.txt 2>&1; rc=$?; grep "^libcsa" $O/ab.txt; exit $rc
