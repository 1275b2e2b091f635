#!/bin/bash
# CSE parity tests + per-kernel times of the java CSE layer (B=64) under rocprofv3 kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/cse}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_cse_gpu.py tests/test_model_gpu.py tests/test_property_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python tools/cse_bench.py 64 10 > $OUT/trace.log 2>&1 || exit $?
tail -3 $OUT/trace.log
python3 - $OUT/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
