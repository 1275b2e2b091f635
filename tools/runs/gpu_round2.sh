#!/bin/bash
# Round-end capture: default bench line (CPU baselines, train leg), rocprofv3 kernel stats of the SBM layer
# bench / CSE layer / java train step, and the PMC traffic + MFMA passes of the SBM layer bench.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r2}
mkdir -p "$OUT"
timeout -k 10 600 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
cat "$OUT/bench_default.json"
B="--steps 5 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg --no-cpu-config1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sbm" -o run -- python bench.py $B > "$OUT/sbm.log" 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/cse" -o run -- python tools/cse_bench.py 64 10 > "$OUT/cse.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train" -o run -- python tools/prof_train.py 5 > "$OUT/train.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc1" -o run -- python bench.py $B > "$OUT/pmc1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc2" -o run -- python bench.py $B > "$OUT/pmc2.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc3" -o run -- python bench.py $B > "$OUT/pmc3.log" 2>&1 || exit $?
python tools/pmc_traffic.py "$OUT/pmc2/run_counter_collection.csv" "$OUT/pmc3/run_counter_collection.csv" > "$OUT/pmc_traffic.json" || exit $?
python tools/pmc_summary.py "$OUT"/pmc*/run_counter_collection.csv > "$OUT/pmc_summary.txt"
rm -f "$OUT"/*/run_kernel_trace.csv "$OUT"/pmc*/run_counter_collection.csv.bak
echo done
