#!/bin/bash
# Round 6: k_attn_bwd_kv's w-tile stores (a 32-B piece of a 128-B row per lane and instruction): wt = plain stores
# (L2 write-back can merge the four pieces of a row), hip = non-temporal (shipped)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6r; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
for i in 1 2 3 4; do
  for lib in libcsa_wt.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
