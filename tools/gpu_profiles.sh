#!/bin/bash
# Round profile capture: default bench line (with CPU baselines), rocprofv3 kernel stats of the SBM
# layer bench, the CSE layer and the java train step. Each GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/p}
mkdir -p "$OUT"
timeout -k 10 500 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
cat "$OUT/bench_default.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sbm" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg > "$OUT/sbm.log" 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/cse" -o run -- python tools/cse_bench.py 64 10 > "$OUT/cse.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train" -o run -- python tools/prof_train.py 5 > "$OUT/train.log" 2>&1 || exit $?
echo done
