#!/bin/bash
# BASELINE.json configs 4 and 5 on one GPU: the dense FullAttention ablation at the config-2 shape
# and the long-AST stress (N = 1024, k in 16..128). One bench.py line per point (train mode).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cpu-config1 --no-train >> "$OUT/sweep.jsonl" || exit $?
timeout -k 10 200 python bench.py --dense --steps 10 --warmup 3 --no-cpu-baseline --no-cpu-config1 --no-train >> "$OUT/sweep.jsonl" || exit $?
for k in 16 32 64 128; do
  timeout -k 10 200 python bench.py --seq-len 1024 --clusters $k --batch 16 --steps 5 --warmup 2 --no-cpu-baseline --no-cpu-config1 \
    --no-train >> "$OUT/sweep.jsonl" || exit $?
  tail -1 "$OUT/sweep.jsonl" | cut -c1-200
done
