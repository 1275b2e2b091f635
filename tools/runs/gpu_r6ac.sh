#!/bin/bash
# Round 6: the concurrent backward schedule (the projection backward's key-block items on the side stream beside
# k_attn_bwd_qg) re-measured on the round-6 kernels against in-order (AUTO), headline, 4 rounds
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ac; mkdir -p $O
cd $R
for i in 1 2 3 4; do
  for c in 1 0; do
    out=$(CSA_BWD_CONCUR=$c timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('concur', sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$c"
  done
done 2>&1 | tee $O/ab.txt
