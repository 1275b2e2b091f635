#!/bin/bash
# Round 5: s_memtime phase totals of k_proj_bwd_s (CSA_PHASES, workgroup (0,0), cumulative over launches)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5u; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
CSA_HIP_LIB=$L/libcsa_PHB.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-padded-leg --no-bf16-leg --no-cpu-config1 > $O/phb.txt 2>&1; rc=$?; grep PHASES $O/phb.txt | tail -8; exit $rc
