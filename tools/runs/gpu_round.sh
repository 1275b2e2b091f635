#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile, PMC counters. Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r}
mkdir -p "$OUT"
timeout -k 10 400 python -m pytest tests -m gpu -q > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 6 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-train > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc1" -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train > "$OUT/pmc1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc2" -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train > "$OUT/pmc2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc3" -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train > "$OUT/pmc3.log" 2>&1 || exit $?
python tools/pmc_traffic.py "$OUT/pmc2/run_counter_collection.csv" "$OUT/pmc3/run_counter_collection.csv" > "$OUT/pmc_traffic.json" || exit $?
python tools/pmc_summary.py "$OUT"/pmc*/run_counter_collection.csv > "$OUT/pmc_summary.txt"
echo done
