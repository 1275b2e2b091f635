#!/bin/bash
# Same-box A/B of the java train step (tools/prof_train.py: tuned GEMM table, 50 timed steps) between two
# builds of libcsa_hip.so, alternating runs. usage: bash tools/ab_train.sh <libA.so> <libB.so> [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-3}
for i in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    out=$(CSA_HIP_LIB=$L timeout -k 10 150 python tools/prof_train.py 50 | tail -1) || exit $?
    python3 -c "import ast,sys; d=ast.literal_eval(sys.argv[1]); print(sys.argv[2][-28:], d['ms_per_step'], d['mean_loss'])" "$out" "$L"
  done
done
