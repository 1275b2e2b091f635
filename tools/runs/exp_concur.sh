#!/bin/bash
# One-box A/B of the concurrent attention backward (k_attn_bwd_q beside k_attn_bwd_kv on a second stream):
# SBM layer at python (d=64) dims B=256 / B=64 and java (d=96) dims B=64, then the java train step.
# usage: bash tools/exp_concur.sh [rounds]
set -o pipefail
export TMPDIR=/tmp
R=${1:-2}
L="--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-cpu-config1"
T="--steps 5 --warmup 2 --no-cpu-baseline --no-bf16-leg --no-cpu-config1"
for i in $(seq 1 "$R"); do
  for X in "" "--batch 64" "--head-dim 96 --batch 64"; do
    for E in CSA_BWD_CONCUR=0 CSA_BWD_CONCUR=1 CSA_X=default; do
      out=$(env $E timeout -k 10 120 python bench.py $L $X) || exit $?
      python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$E $X"
    done
  done
  for E in CSA_BWD_CONCUR=0 CSA_X=default; do
    out=$(env $E timeout -k 10 300 python bench.py $T) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], 'train', d['train']['ms_per_step'])" "$out" "$E"
  done
done
