#!/bin/bash
# Round-3 kernel census: SBM layer bench in fp32 and in bf16 mode (stage events + rocprofv3 kernel
# stats) and the java CSE layer. Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3p}
mkdir -p "$OUT"
timeout -k 10 200 python bench.py --precision bf16 --no-train --no-cpu-baseline --steps 20 > "$OUT/bench_bf16.json" 2> "$OUT/bench_bf16.err" || exit $?
cat "$OUT/bench_bf16.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sbm" -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg > "$OUT/sbm.log" 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sbm_bf16" -o run -- python bench.py --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-train > "$OUT/sbm_bf16.log" 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/cse" -o run -- python tools/cse_bench.py 64 20 > "$OUT/cse.log" 2>&1 || exit $?
tail -2 "$OUT/cse.log"
echo done
