#!/bin/bash
# Quick GPU check: SBM parity tests + one bench line (no train, no CPU baseline) + kernel-trace stats.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/q}
TESTS=${2:-tests/test_sbm_gpu.py}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-train > "$OUT/trace.log" 2>&1 || exit $?
python - "$OUT/trace/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
