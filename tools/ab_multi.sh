#!/bin/bash
# A/B/C... timing on ONE box: alternate bench runs over several builds of libcsa_hip.so and print
# ms/step + per-stage kernel times of each run. usage: BENCH_ARGS="..." bash tools/ab_multi.sh R lib...
set -o pipefail
R=$1; shift
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-padded-leg --no-cpu-config1"}
for i in $(seq 1 "$R"); do
  for L in "$@"; do
    out=$(CSA_HIP_LIB=$L timeout -k 10 120 python bench.py $ARGS) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$L"
  done
done
