#!/bin/bash
# A/B timing on ONE box (boxes differ by a few %): alternate bench runs of two builds of
# libcsa_hip.so and print ms/step + per-stage kernel times of each run.
# usage: bash tools/ab.sh <libA.so> <libB.so> [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-2}
for i in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    out=$(CSA_HIP_LIB=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-padded-leg) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2][-40:], d['ms_per_step'], d['stage_ms'])" "$out" "$L"
  done
done
