#!/bin/bash
# Same-box A/B of several library builds: alternating headline layer-bench runs (R rounds), ms/step + stage times.
# usage: bash tools/ab3.sh R libA.so libB.so [libC.so ...]
set -o pipefail
R=$1; shift
for i in $(seq 1 "$R"); do
  for L in "$@"; do
    out=$(CSA_HIP_LIB=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-padded-leg --no-bf16-leg --no-side-legs --no-cpu-config1) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$L"
  done
done
