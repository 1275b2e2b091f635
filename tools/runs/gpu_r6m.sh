#!/bin/bash
# Round 6: what a dead key block costs k_attn_bwd_kv: deadnop = dead waves skip all work (timing only), nodeadkv = no
# dead-block path (every wave runs the full loop), hip = the chunked dead path; equal-length padding n = 150 / 64 / 32
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6m; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
for lib in libcsa_deadnop.so libcsa_nodeadkv.so libcsa_hip.so; do
  echo "== $lib"
  DIAG_NS=150,64,32,150,64,32 CSA_HIP_LIB=$L/$lib timeout -k 10 300 python tools/runs/diag_dead.py 2>/dev/null || exit 1
done 2>&1 | tee $O/diag.txt
