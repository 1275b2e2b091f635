#!/bin/bash
# One-box A/B of library builds: bash tools/exp_lib_ab.sh R libA.so libB.so [bench args]
set -o pipefail
export TMPDIR=/tmp
R=$1; A=$2; B=$3; X=${4:-}
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-cpu-config1 $X"
for i in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    out=$(CSA_HIP_LIB=$L timeout -k 10 120 python bench.py $ARGS) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$L"
  done
done
