#!/bin/bash
# Round 5: s_memtime phase stamps of the projection forward (CSA_PHASES_FWD: cumulative ticks per phase, workgroup 0)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5m; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
CSA_HIP_LIB=$L/libcsa_PHF.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-padded-leg --no-bf16-leg > $O/phf.txt 2>&1; rc=$?; grep PHF $O/phf.txt | tail -16; exit $rc
